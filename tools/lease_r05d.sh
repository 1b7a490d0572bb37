# r05 lease D: the two-step fused quotient (random, near-midpoint and FABRIK
# radicands), the FABRIK core-sequence test and A/B, and counters of both builds'
# layered ANN GEMM.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/annb_pmc
timeout -k 10 300 tools/quot_check 36 || exit $?
timeout -k 10 120 tools/quot_fab_check core_test_goals.f64 1e-3 100 || exit $?
timeout -k 10 120 tools/quot_fab_check core_test_goals.f64 1e-5 200 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "core_sequences or fabrik_vs" > gpurun_out/pytest_core.txt 2>&1; rc=$?
tail -2 gpurun_out/pytest_core.txt; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 bash tools/fab_ab.sh libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so || exit $?
for lib in libikhip_prev.so libikhip.so; do
  for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=${lib%.so}_$(echo $grp | cut -d' ' -f1)
    IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/annb_pmc/$tag -- python tools/ann_big_probe.py 131072 4096x2 > gpurun_out/annb_pmc/$tag.log 2>&1 || exit $?
  done
done
echo done
