"""Summarise a rocprofv3 trace of tools/e2e_trace.py: per roctx-bracketed call,
its wall time and what filled it (HIP API calls on the calling thread, copies,
kernels), and for the slow calls (> 1.5x the median) where the time went.

    python tools/e2e_trace_summary.py gpurun_out/e2e_trace > profiles/r03/e2e_trace_summary.json
"""
import csv
import glob
import json
import os
import sys

import numpy as np


def rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def ts(r):
    return int(r["Start_Timestamp"]), int(r["End_Timestamp"])


def main(d):
    marks = rows(d, "marker_api_trace.csv")
    calls = []
    for r in marks:
        name = r.get("Function") or r.get("Message") or ""
        if name.startswith("call"):
            s, e = ts(r)
            calls.append((int(name[4:]), s, e))
    calls.sort()
    if not calls:  # no marker trace: every pinned FABRIK call is K chunks, each one
        # H2D copy (SDMA), reset / classify / scatter / iterate kernels and two D2H
        # blit kernels (__amd_rocclr_copyBuffer: stats + angles); group them in call order
        h2d = sorted(ts(r) for r in rows(d, "memory_copy_trace.csv")
                     if "HOST_TO_DEVICE" in r["Direction"])
        kr = rows(d, "kernel_trace.csv")
        it = sorted(ts(r) for r in kr if "fabrik_iter_kernel" in r["Kernel_Name"])
        blit = sorted(ts(r) for r in kr if "copyBuffer" in r["Kernel_Name"])
        K = int(os.environ.get("E2E_CHUNKS", "4"))
        n = len(it) // K
        h2d, blit = h2d[-n * K:], blit[-n * 2 * K:]
        calls = [(k, h2d[k * K][0], blit[(k + 1) * 2 * K - 1][1]) for k in range(n)][10:]
    api = [(r["Function"], *ts(r)) for r in rows(d, "hip_api_trace.csv")]
    cps = [(r.get("Direction", r.get("Kind", "copy")).replace("MEMORY_COPY_", ""), *ts(r),
            int(r.get("Bytes", 0) or 0))
           for r in rows(d, "memory_copy_trace.csv")]
    ks = [(r["Kernel_Name"][:40], *ts(r)) for r in rows(d, "kernel_trace.csv")]
    dur = np.array([(e - s) / 1e6 for _, s, e in calls])
    gaps = np.array([(calls[i + 1][1] - calls[i][2]) / 1e6 for i in range(len(calls) - 1)])
    med = float(np.median(dur)) if len(dur) else 0.0
    res = {"calls": len(calls), "median_ms": med, "mean_ms": float(dur.mean()) if len(dur) else 0,
           "max_ms": float(dur.max()) if len(dur) else 0,
           "host_gap_between_calls_ms": {"median": float(np.median(gaps)) if len(gaps) else 0,
                                         "max": float(gaps.max()) if len(gaps) else 0},
           "note": "call = first H2D copy .. last D2H copy (device-side span); without "
                   "markers the host's own time per call is the gap to the next call",
           "slow": []}

    def within(items, s, e):
        return [x for x in items if x[1] < e and x[2] > s]

    # the typical call's composition, for comparison
    def compose(s, e):
        a = within(api, s, e)
        by = {}
        for f, a0, a1 in a:
            by[f] = by.get(f, 0.0) + (min(a1, e) - max(a0, s)) / 1e6
        c = within(cps, s, e)
        k = within(ks, s, e)
        return {"api_ms": {f: round(v, 4) for f, v in sorted(by.items(), key=lambda x: -x[1])[:8]},
                "copies": [(t, round((c0 - s) / 1e6, 4), round((c1 - c0) / 1e6, 4), b)
                           for t, c0, c1, b in c],
                "kernels": [(nm, round((k0 - s) / 1e6, 4), round((k1 - k0) / 1e6, 4))
                            for nm, k0, k1 in k]}
    if calls:
        i_med = int(np.argsort(dur)[len(dur) // 2])
        _, s, e = calls[i_med]
        res["median_call"] = {"call": calls[i_med][0], "ms": dur[i_med], **compose(s, e)}
    for (k, s, e), t in zip(calls, dur):
        if t > 1.5 * med:
            res["slow"].append({"call": k, "ms": t, **compose(s, e)})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
