# The FABRIK process-to-process spread: P processes of the same
# FABRIK-only bench command, each under rocprofv3 --kernel-trace with one
# GRBM_GUI_ACTIVE counter (the per-dispatch shader clock), each printing its bench
# line (ms_per_step, the work-order table's hash after the warm-up).
# tools/fab_spread_summary.py then lines up, per process: step time, iteration-kernel
# window average, clock, table hash.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/spread
mkdir -p $OUT
P=${P:-4}
TOL=${TOL:-1e-3}
MI=${MI:-100}
for i in $(seq 1 $P); do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE --output-format csv \
      -d $OUT/p$i -- python bench.py --method fabrik --tol $TOL --max-iter $MI --secondary 0 \
      --cpu-seconds 0 --end-to-end 0 --cold 0 --steps 20 --warmup 5 > $OUT/p$i.json 2> $OUT/p$i.err
  rc=$?
  echo "p$i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python tools/fab_spread_summary.py --dir $OUT --procs $P > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
