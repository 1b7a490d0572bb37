# r05 lease T: the layered bf16x6 GEMM with the swizzled LDS rows: ANN parity, the
# probe in both modes, and the x6 kernel's counters on the 2048 x 2 model.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05t
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "ann" > gpurun_out/r05t/pytest_ann.txt 2>&1; rc=$?
tail -2 gpurun_out/r05t/pytest_ann.txt; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ann_big_probe.py 262144 all bf16x6 > gpurun_out/r05t/probe_bf16x6.txt 2>&1 || exit $?
grep dims gpurun_out/r05t/probe_bf16x6.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d /tmp/r05t_p1 -o run -- python tools/ann_big_probe.py 131072 2048x2 bf16x6 > gpurun_out/r05t/p1.log 2>&1 || exit $?
find /tmp/r05t_p1 -name '*counter_collection.csv' -exec cp {} gpurun_out/r05t/p1_counters.csv \;
echo p1 ok
