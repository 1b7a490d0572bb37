# Copy the judged summaries of a tools/gpu_round.sh run from gpurun_out/ into
# profiles/<round>/ (gpurun_out/ is scratch): rocprofv3 --stats kernel tables,
# per-kernel FETCH_SIZE / WRITE_SIZE summaries, the bench line, traffic.json.
#   bash tools/collect_profiles.sh r01
#   MODES="ann ann_fp16x3" bash tools/collect_profiles.sh r02   # the modes a run re-profiled
set -e
R=${1:?round name}
OUT=gpurun_out
DST=profiles/$R
mkdir -p $DST/pmc
for m in ${MODES:-ann fabrik ann_bf16x6 ann_fp16x3 fk}; do
  # gpurun_out/ accumulates the runs of earlier calls: take the newest
  cp "$(ls -t $OUT/prof_stats_$m/*/*_kernel_stats.csv | head -1)" $DST/${m}_kernel_stats.csv
  for c in fetch write; do
    python - "$OUT/prof_${c}_$m" "$DST/pmc/${m}_${c}_summary.csv" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
src, dst = sys.argv[1], sys.argv[2]
tot, disp = defaultdict(float), defaultdict(set)
files = sorted(glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True),
               key=os.path.getmtime)
for f in files[-1:]:  # the newest run only
    for row in csv.DictReader(open(f)):
        key = (row["Kernel_Name"][:80], row["Counter_Name"])
        tot[key] += float(row["Counter_Value"])
        disp[key].add(row["Dispatch_Id"])
with open(dst, "w", newline="") as fh:
    w = csv.writer(fh, quoting=csv.QUOTE_MINIMAL)
    w.writerow(["kernel", "counter", "dispatches", "sum_over_dispatches", "per_dispatch"])
    for (k, c), v in sorted(tot.items()):
        w.writerow([k, c, len(disp[(k, c)]), v, v / len(disp[(k, c)])])
PY
  done
done
tail -1 $OUT/bench_ann.json > $DST/bench_ann.json
cp $OUT/traffic.json profiles/traffic.json
cp $OUT/traffic.json $DST/traffic.json
ls -la $DST $DST/pmc
