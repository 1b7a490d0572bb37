"""Summary of tools/ann_traffic_ab.sh: per build, the ANN fp32 kernel's timed
window (the last 5 dispatches) -- duration, HBM bytes per launch (raw FETCH+WRITE and
doubled 2 FETCH + WRITE, KiB units), L2 hit rate and clock.

    python tools/ann_traffic_summary.py --dir gpurun_out/anntraffic
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_summary import counters, durations  # noqa: E402

K = "ann_fused_kernel"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--builds", nargs="*", default=["libikhip", "libikhip_dyn0"])
    args = ap.parse_args()
    for lib in args.builds:
        fig = {"build": lib}
        vals = {}
        ms_all = []
        for i in range(1, 5):
            d = os.path.join(args.dir, f"{lib}_{i}")
            if not os.path.isdir(d):
                continue
            tr = durations(d).get(K, [])[-args.steps:]
            pm = counters(d).get(K, {})
            ms_all += [m for _, m in tr]
            for k, m in tr:
                for c, v in pm.get(k, {}).items():
                    vals.setdefault(c, []).append(v)
                    if c == "GRBM_GUI_ACTIVE":
                        vals.setdefault("_clk", []).append(v / 8 / (m * 1e-3) / 1e9)
        mean = {c: statistics.mean(v) for c, v in vals.items()}
        fig["kernel_ms"] = statistics.mean(ms_all) if ms_all else None
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            fig["raw_GB"] = (mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024 / 1e9
            fig["doubled_GB"] = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024 / 1e9
        if "TCC_HIT_sum" in mean:
            fig["l2_hit"] = mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"])
        if "_clk" in mean:
            fig["clock_ghz"] = mean["_clk"]
        print(json.dumps(fig))


if __name__ == "__main__":
    main()
