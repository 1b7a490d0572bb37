# One box's rocprof window averages of the bench's own command (the trace step of
# tools/profile_round.sh alone, no PMC passes): gpurun_out/box/summary/traffic.json.
# Several of these on different boxes give the cross-box spread that
# tools/merge_boxes.py folds into profiles/<round>/traffic.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/box
mkdir -p $OUT
STEPS=${STEPS:-20}
WARM=${WARM:-5}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- \
  python bench.py --gpus 1 --cpu-seconds 0 --end-to-end 0 --cold 0 --steps $STEPS --warmup $WARM \
  > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python tools/profile_summary.py --dir $OUT --steps $STEPS --warmup $WARM --out $OUT/summary > $OUT/summary.log 2>&1
rc=$?; echo "summary rc=$rc"; exit $rc
