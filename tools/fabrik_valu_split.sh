# FABRIK iteration kernel: VALU instructions in and out of the inner loop
# (VERDICT r05 #2).  One SQ counter pass per tolerance on the FABRIK-only bench
# (rocprofv3 --pmc, --kernel-trace), then tools/fabrik_valu_split.py combines the
# kernel's SQ_INSTS_VALU with the wave-iterations the diagnostic build counts
# (gpurun_out/fabrik_diag.json, tools/fabrik_diag.py: same batch, same tolerance)
# and the loop's VALU per iteration from the ISA (tools/isa_loop.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/valu
mkdir -p $OUT
for tm in "1e-3 100" "1e-5 200"; do
  set -- $tm
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_$1 -- python bench.py --method fabrik --steps 5 --warmup 5 --cpu-seconds 0 --secondary 0 --end-to-end 0 --cold 0 --tol $1 --max-iter $2 > $OUT/pmc_$1.log 2>&1 || exit $?
  echo "valu pass tol=$1 rc=0"
done
