"""Average kernel durations (ms) from a rocprofv3 --stats CSV directory: the
fabrik_* kernels' averages, one line (used by tools/fab_ab_prof.sh)."""
import csv
import glob
import sys

rows = {}
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Name"].split("(")[0].split("<")[0].split("::")[-1]
        if name.startswith("fabrik") or name.startswith("fk_"):
            rows[name] = (float(r["AverageNs"]) / 1e6, int(r["Calls"]))
print(" ".join(f"{k}={v[0]:.4f}ms/{v[1]}" for k, v in sorted(rows.items())))
