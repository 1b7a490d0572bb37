# PMC diagnosis passes for one bench method ($1 = ann|fabrik), one counter group per pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
m=${1:-ann}
i=0
for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_${m}_$i -- python bench.py --method $m --steps 1 --warmup 1 --cpu-seconds 0 --secondary 0 > gpurun_out/pmc_${m}_$i.log 2>&1
  rc=$?
  echo "pmc $m $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmc_${m}_* > gpurun_out/pmc_${m}_summary.json
