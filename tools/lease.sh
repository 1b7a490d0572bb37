# One lease: the GPU tests, then the profiling lease (tools/profile_round.sh: the
# default bench line, its rocprofv3 trace and PMC passes), then the FABRIK
# process-spread probe (tools/fab_spread_probe.sh).  Stops at the first crash or
# time limit; a plain test failure (rc 1) still runs the profiling.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --maxfail=20 > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = 1 ]; then bash tools/profile_round.sh || exit $?; fi
if [ "${DIAG:-1}" = 1 ]; then
  timeout -k 10 180 python tools/fabrik_diag.py > gpurun_out/fabrik_diag.json 2> gpurun_out/fabrik_diag.err
  rc=$?; echo "fabrik_diag rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${SPREAD:-1}" = 1 ]; then bash tools/fab_spread_probe.sh || exit $?; fi
