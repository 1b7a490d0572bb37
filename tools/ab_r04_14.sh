# FABRIK classify: cells computed outside the per-point branches, goals read coalesced
# through LDS (IKHIP_ORD_STAGE) (working
# tree libikhip.so) against HEAD (libikhip_prev.so): FABRIK tests, bench lines with the
# per-kernel event times, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "fabrik and not calc" -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fab.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_fab.txt; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/fab_ab.sh libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so || exit $?
