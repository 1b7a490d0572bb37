# r05 lease P: the first carry and band flag in the preparation (libikhip.so) against HEAD:
# FABRIK parity, same-box A/B against HEAD, the diagnostic breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05p
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fabrik or FABRIK or fk_err" > gpurun_out/r05p/pytest_fab.txt 2>&1; rc=$?
tail -2 gpurun_out/r05p/pytest_fab.txt; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1000 bash tools/fab_ab.sh libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so || exit $?
timeout -k 10 300 python tools/fabrik_diag.py > gpurun_out/r05p/fabrik_diag.json 2> gpurun_out/r05p/fabrik_diag.err || exit $?
echo diag ok
