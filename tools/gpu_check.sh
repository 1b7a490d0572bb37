# GPU tests, then the default bench line (stops after a crash / timeout of the tests;
# a plain test failure, rc 1, still runs the bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 gpurun_out/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
brc=$?
echo "bench rc=$brc"
exit $brc
