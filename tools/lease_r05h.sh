# r05 lease H: the whole GPU suite, the default bench line, the layered ANN probe
# (HEAD's build against the working tree's) and the layered GEMM's counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/annb_pmc4
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --maxfail=10 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lib in libikhip.so libikhip_prev.so libikhip.so; do
  echo "== $lib"
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 300 python tools/ann_big_probe.py 2>&1 | grep dims || exit 1
done
for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/annb_pmc4/$tag -- python tools/ann_big_probe.py 131072 2048x2 > gpurun_out/annb_pmc4/$tag.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_default.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: round(v['ms_per_step'],4) for k,v in d['secondary'].items()})"
