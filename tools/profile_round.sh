# One profiling lease on the bench's own command: the default
# bench line, then the SAME bench command (all secondaries, same order, same
# warm-up; CPU baseline, end-to-end and cold legs off, since they only add
# dispatches) under `rocprofv3 --kernel-trace --stats`, then its PMC passes (one
# counter group per pass, each with --kernel-trace so every dispatch carries its
# own duration).  tools/profile_summary.py cuts every kernel's dispatches into the
# bench's methods and keeps each method's timed window.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
: > $OUT/steps.txt
step() {  # step <name> <timeout> <cmd...>: stops the script on crash / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
STEPS=${STEPS:-20}
WARM=${WARM:-5}
step bench_default 300 python bench.py --gpus 1 --steps $STEPS --warmup $WARM
BENCH="--gpus 1 --cpu-seconds 0 --end-to-end 0 --cold 0"
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- python bench.py $BENCH --steps $STEPS --warmup $WARM
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  i=$((i+1))
  step pmc_$i 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc_$i -- python bench.py $BENCH --steps 5 --warmup $WARM
done
python tools/profile_summary.py --dir $OUT --steps $STEPS --warmup $WARM --pmc-steps 5 --out $OUT/summary > $OUT/summary.log 2>&1
cat $OUT/steps.txt
