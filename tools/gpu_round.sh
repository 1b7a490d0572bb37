# One GPU session: parity tests, bench, rocprofv3 kernel stats + PMC traffic.
# Every GPU step has its own time limit; a crash/timeout stops the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out
step() {  # step <name> <timeout> <cmd...>; stops the script on crash/timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
: > $OUT/steps.txt
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
fi
step bench_ann 600 python bench.py --steps ${STEPS:-10} --warmup 2 --cpu-seconds ${CPUS:-10}
cp $OUT/bench_ann.log $OUT/bench_ann.json
if [ "${PROFILE:-1}" = "1" ]; then
  # MODES: a subset to re-profile; the traffic of the others is kept from profiles/
  [ -f $OUT/traffic.json ] || cp profiles/traffic.json $OUT/traffic.json
  for m in ${MODES:-ann fabrik ann_bf16x6 ann_fp16x3 fk}; do
    case $m in
      ann_bf16x6) BARGS="--method ann --ann-mode bf16x6" ;;
      ann_fp16x3) BARGS="--method ann --ann-mode fp16x3" ;;
      *) BARGS="--method $m" ;;
    esac
    step prof_stats_$m 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_stats_$m -- python bench.py $BARGS --steps 5 --warmup 1 --cpu-seconds 0 --secondary 0 --end-to-end 0
    step prof_fetch_$m 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch_$m -- python bench.py $BARGS --steps 2 --warmup 1 --cpu-seconds 0 --secondary 0 --end-to-end 0
    step prof_write_$m 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write_$m -- python bench.py $BARGS --steps 2 --warmup 1 --cpu-seconds 0 --secondary 0 --end-to-end 0
    python tools/pmc_traffic.py --stats $OUT/prof_stats_$m --fetch $OUT/prof_fetch_$m --write $OUT/prof_write_$m --out $OUT/traffic.json > $OUT/traffic_$m.log 2>&1
  done
fi
tail -3 $OUT/pytest_gpu.log 2>/dev/null; cat $OUT/steps.txt
