# PMC diagnosis passes for one bench method ($1 = ann|fabrik|ann_bf16x6|ann_fp16x3),
# one counter group per pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
m=${1:-ann}
case $m in
  ann_bf16x6) BARGS="--method ann --ann-mode bf16x6" ;;
  ann_fp16x3) BARGS="--method ann --ann-mode fp16x3" ;;
  *) BARGS="--method $m" ;;
esac
i=0
for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
           "TCC_REQ_sum TCC_READ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_${m}_$i -- python bench.py $BARGS --steps 1 --warmup 1 --cpu-seconds 0 --secondary 0 --end-to-end 0 > gpurun_out/pmc_${m}_$i.log 2>&1
  rc=$?
  echo "pmc $m $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmc_${m}_* > gpurun_out/pmc_${m}_summary.json
