# r05 lease B: the fused-quotient bit check, the FABRIK parity tests, and a same-box
# A/B of HEAD's library (libikhip_prev.so) against the working tree's.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 tools/quot_check 36 > gpurun_out/quot_check.txt 2>&1; rc=$?
cat gpurun_out/quot_check.txt; echo "quot_check rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fabrik or FABRIK or fullsize" > gpurun_out/pytest_fab.txt 2>&1; rc=$?
tail -3 gpurun_out/pytest_fab.txt; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 bash tools/fab_ab.sh libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so || exit $?
