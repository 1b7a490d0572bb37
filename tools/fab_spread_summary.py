"""Summary of tools/fab_spread_probe.sh: per process the bench step, the iteration
kernel's timed-window average (rocprof), its shader clock (GRBM_GUI_ACTIVE / 8 over
each dispatch) and the work-order table's hash after the warm-up.

    python tools/fab_spread_summary.py --dir gpurun_out/spread --procs 4
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_summary import counters, durations  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    rows = []
    for i in range(1, args.procs + 1):
        d = os.path.join(args.dir, f"p{i}")
        with open(os.path.join(args.dir, f"p{i}.json")) as f:
            line = json.loads(f.read().strip().splitlines()[-1])
        tr = durations(d).get("fabrik_iter_kernel", [])
        pm = counters(d).get("fabrik_iter_kernel", {})
        win = tr[-args.steps:]
        ms = [m for _, m in win]
        clk = [pm[k]["GRBM_GUI_ACTIVE"] / 8 / (m * 1e-3) / 1e9 for k, m in win
               if k in pm and "GRBM_GUI_ACTIVE" in pm[k]]
        rows.append({"proc": i, "ms_per_step": line["ms_per_step"],
                     "event_ms_per_step": line.get("event_ms_per_step"),
                     "iter_rocprof_avg_ms": statistics.mean(ms) if ms else None,
                     "iter_rocprof_min_ms": min(ms) if ms else None,
                     "iter_clock_ghz": statistics.mean(clk) if clk else None,
                     "order_table": line.get("order_table")})
    for r in rows:
        print(json.dumps(r))
    a = [r["iter_rocprof_avg_ms"] for r in rows if r["iter_rocprof_avg_ms"]]
    c = [r["iter_clock_ghz"] for r in rows if r["iter_clock_ghz"]]
    hs = {json.dumps(r["order_table"], sort_keys=True) for r in rows}
    if a:
        print(json.dumps({"iter_spread": (max(a) - min(a)) / min(a),
                          "clock_spread": (max(c) - min(c)) / min(c) if c else None,
                          "tables_identical": len(hs) == 1}))


if __name__ == "__main__":
    main()
