"""Summary of tools/fab_trace_ab.sh: per run, the bench step and the rocprof averages of
each FABRIK kernel over the timed window (the last `steps` dispatches), and per build
the mean of the runs.

    python tools/fab_trace_summary.py --dir gpurun_out/fabtrace --steps 30
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_summary import durations  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    per = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(args.dir, "*.json"))):
        tag = os.path.basename(f)[:-5]
        build = tag.rsplit("_", 1)[0]
        with open(f) as fh:
            line = json.loads(fh.read().strip().splitlines()[-1])
        tr = durations(os.path.join(args.dir, tag))
        k = {name: statistics.mean(ms for _, ms in v[-args.steps:])
             for name, v in tr.items() if name.startswith(("fabrik", "reset"))}
        k["pipeline"] = sum(k.values())
        row = {"run": tag, "ms_per_step": round(line["ms_per_step"], 4),
               **{n: round(v, 4) for n, v in k.items()}}
        print(json.dumps(row))
        per[build].append(row)
    for b, rows in per.items():
        keys = [x for x in rows[0] if x not in ("run",)]
        print(json.dumps({"build": b, "runs": len(rows),
                          **{x: round(statistics.mean(r[x] for r in rows if x in r), 4)
                             for x in keys}}))


if __name__ == "__main__":
    main()
