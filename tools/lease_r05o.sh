# r05 lease O: why fewer VALU per FABRIK iteration did not buy time -- the wave-cycle
# split of the iteration kernel (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY)
# and the instruction-cache counters gfx950 lists.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05o
timeout -k 10 120 rocprofv3 -L > gpurun_out/r05o/counters.txt 2>&1 || exit $?
grep -i -E "ICACHE|IFETCH|INST_CACHE|SQC_" gpurun_out/r05o/counters.txt | head -40
B="python bench.py --method fabrik --steps 5 --warmup 5 --cpu-seconds 0 --secondary 0 --end-to-end 0 --cold 0 --tol 1e-3 --max-iter 100"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d /tmp/r05o_p1 -o run -- $B > gpurun_out/r05o/p1.log 2>&1 || exit $?
find /tmp/r05o_p1 -name '*counter_collection.csv' -exec cp {} gpurun_out/r05o/p1_counters.csv \;
echo p1 ok
