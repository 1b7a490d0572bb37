# One profiling lease: the default bench line, then per method a kernel-trace run
# of the same timed bench command and its PMC passes (each counter pass with
# --kernel-trace so that every dispatch has its own duration; one counter group
# per pass).  tools/profile_summary.py reduces it to the timed window.
#   bash tools/profile_round.sh ann ann_fp16x3 ann_bf16x6     (methods)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>: stops the script on crash / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step bench_default 300 python bench.py --gpus 1 --steps 20 --warmup 5
for m in "$@"; do
  case $m in
    ann_bf16x6) BARGS="--method ann --ann-mode bf16x6" ;;
    ann_fp16x3) BARGS="--method ann --ann-mode fp16x3" ;;
    *) BARGS="--method $m" ;;
  esac
  COMMON="--cpu-seconds 0 --secondary 0 --end-to-end 0 --cold 0"
  step trace_$m 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$m -- python bench.py $BARGS --steps 20 --warmup 5 $COMMON
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
             "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
             "TCC_HIT_sum TCC_MISS_sum" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
    i=$((i+1))
    step pmc_${m}_$i 150 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc_${m}_$i -- python bench.py $BARGS --steps 5 --warmup 5 $COMMON
  done
done
python tools/profile_summary.py --dir $OUT --methods "$@" --window 20 --pmc-window 5 --out $OUT/summary > $OUT/summary.log 2>&1
cat $OUT/steps.txt
