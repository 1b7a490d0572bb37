# r06 A/B lease (ANN=0 skips the ANN runs, TESTS=0 the tests, BENCH=0 the bench): the GPU tests on the working tree's build, then FABRIK (rocprof
# kernel averages, tools/fab_ab_prof.sh) and ANN split modes (tools/ann_ab.sh)
# for libikhip_prev.so (tools/build_prev.sh: git HEAD) against libikhip.so,
# interleaved twice, then the default bench line.  Stops at the first crash.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --maxfail=20 > gpurun_out/pytest_gpu.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for rep in 1 2; do
  if [ "${FAB:-1}" = 1 ]; then bash tools/fab_ab_prof.sh gpurun_out/fabprof_$rep ${LIBS:-libikhip_prev.so libikhip.so} || exit $?; fi
  [ "${ANN:-1}" = 1 ] || continue
  for m in ${ANN_MODES:-bf16x6}; do
    MODE=$m STEPS=10 bash tools/ann_ab.sh ${ANN_SPECS:-${LIBS:-libikhip_prev.so libikhip.so}} || exit $?
  done
done
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
  rc=$?; echo "bench rc=$rc"; exit $rc
fi
