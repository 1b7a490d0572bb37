# Confirmation run of the committed build, as the driver runs it at round end: the GPU
# tests, smoke(), the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_confirm.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_confirm.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_confirm.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_confirm.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_confirm.json 2> gpurun_out/bench_confirm.err
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
# the N > 1 launcher and bookkeeping on one GPU: two gloo ranks share device 0 (RCCL
# takes one rank per GPU, so --gather 0)
# (every leg of the N > 1 line: secondaries, strong legs, end-to-end, cold calls)
IKHIP_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --gather 0 --steps 5 --warmup 2 > gpurun_out/bench_2rank_gloo.json 2> gpurun_out/bench_2rank_gloo.err
rc=$?; echo "2-rank rehearsal rc=$rc"; exit $rc
