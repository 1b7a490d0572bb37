# r05 lease I: FABRIK with the loop condition from the step's own radicands
# (fabrik_step4_lazy, one error band per launch): parity (all FABRIK tests, the
# full-size ones) and the A/B against the HEAD build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py tests/test_gpu_bench.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_fab.txt 2>&1; rc=$?
tail -3 gpurun_out/pytest_fab.txt; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 bash tools/fab_ab.sh libikhip_prev.so libikhip.so libikhip_band.so libikhip_prev.so libikhip.so libikhip_band.so || exit $?
