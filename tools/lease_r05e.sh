# r05 lease E: counters of both builds' layered ANN GEMM (HEAD = 128 x 128 tiles,
# B from L2 per wave; working tree = 256 x 128, A and B through LDS).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/annb_pmc
for lib in libikhip_prev.so libikhip.so; do
  for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD"; do
    tag=${lib%.so}_$(echo $grp | cut -d' ' -f1)
    IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/annb_pmc/$tag -- python tools/ann_big_probe.py 131072 4096x2 > gpurun_out/annb_pmc/$tag.log 2>&1 || exit $?
    tail -1 gpurun_out/annb_pmc/$tag.log
  done
done
echo done
