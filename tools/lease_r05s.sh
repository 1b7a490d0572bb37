# r05 lease S: counters of the layered bf16x6 GEMM (annb_gemm_x6_kernel) on the
# 2048 x 2 model: MFMA busy, wave-cycle split, LDS conflicts, clock.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05s
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d /tmp/r05s_p1 -o run -- python tools/ann_big_probe.py 131072 2048x2 bf16x6 > gpurun_out/r05s/p1.log 2>&1 || exit $?
find /tmp/r05s_p1 -name '*counter_collection.csv' -exec cp {} gpurun_out/r05s/p1_counters.csv \;
echo p1 ok
