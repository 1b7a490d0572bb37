# r05 lease V: the FABRIK stats reset folded into the classify kernel (one launch
# fewer per call): the whole GPU suite, then the same-box A/B against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05v/pytest_gpu.txt 2>&1; rc=$?
tail -2 gpurun_out/r05v/pytest_gpu.txt; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1000 bash tools/fab_ab.sh libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so || exit $?
