"""Per-kernel figures of one profiling lease (tools/profile_round.sh), over the
bench's TIMED window only -- the last `--window` dispatches of each kernel --
so that warm-up launches (a fresh context's first FABRIK call runs in point
order) do not enter the averages:

* duration: from the `--kernel-trace` run of the same bench command the line
  was timed with (average / min / max over the window);
* HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE passes: `raw` =
  (FETCH_SIZE + WRITE_SIZE) KiB, `doubled` = (2 FETCH_SIZE + WRITE_SIZE) KiB (the
  gfx950 correction MI355X_MICROARCH.md establishes for wide coalesced reads; for
  gather-pattern kernels -- FABRIK reads 24-byte points through a permutation --
  the raw figure is the one to trust, both are reported);
* the shader clock of each kernel: GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
  over the dispatch's own duration, from a pass that traced the kernels too;
* pipe occupancy (MFMA busy, VALU active, fp64 pipe) as tools/pmc_summary.py.

    python tools/profile_summary.py --dir gpurun_out/prof --methods ann fabrik \\
        --window 20 --pmc-window 5 --out profiles/r03
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import FABRIK_PIPELINE, _short  # noqa: E402


def _rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def durations(d):
    """kernel -> [(dispatch id, ms)] in dispatch order."""
    res = defaultdict(list)
    for r in _rows(d, "*kernel_trace.csv"):
        k = _short(r.get("Kernel_Name", ""))
        if k:
            res[k].append((int(r["Dispatch_Id"]),
                           (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    for k in res:
        res[k].sort()
    return res


def counters(d):
    """kernel -> {dispatch id: {counter: value}}."""
    res = defaultdict(lambda: defaultdict(dict))
    for r in _rows(d, "*counter_collection.csv"):
        k = _short(r.get("Kernel_Name", ""))
        if k:
            res[k][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return res


def window_avg(vals, n):
    v = vals[-n:] if n else vals
    return sum(v) / len(v) if v else None


def summarise(base, method, window, pmc_window):
    out = {}
    tr = durations(os.path.join(base, f"trace_{method}"))
    for k, lst in tr.items():
        w = [ms for _, ms in lst[-window:]]
        out[k] = {"rocprof_avg_ms": sum(w) / len(w), "rocprof_min_ms": min(w),
                  "rocprof_max_ms": max(w), "rocprof_window": len(w),
                  "rocprof_all_dispatches": len(lst)}
    pmc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    clocks = defaultdict(list)
    for d in sorted(glob.glob(os.path.join(base, f"pmc_{method}_*"))):
        if not os.path.isdir(d):
            continue
        cs, ds = counters(d), durations(d)
        for k, bydisp in cs.items():
            ids = sorted(bydisp)[-pmc_window:]
            dur = dict(ds.get(k, []))
            for i in ids:
                for c, v in bydisp[i].items():
                    pmc[k][c].append(v)
                if "GRBM_GUI_ACTIVE" in bydisp[i] and dur.get(i):
                    clocks[k].append(bydisp[i]["GRBM_GUI_ACTIVE"] / 8 / (dur[i] * 1e-3) / 1e9)
    for k, cs in pmc.items():
        r = out.setdefault(k, {})
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            r["fetch_kib_per_launch"] = avg["FETCH_SIZE"]
            r["write_kib_per_launch"] = avg["WRITE_SIZE"]
            r["hbm_bytes_per_launch_raw"] = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
            r["hbm_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        if clocks.get(k):
            r["clock_ghz"] = sum(clocks[k]) / len(clocks[k])
        simd_cycles = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 1024
        pipes = {}
        if simd_cycles and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            pipes["MfmaUtil_pct"] = 100 * avg["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        if simd_cycles and "SQ_ACTIVE_INST_VALU" in avg:
            pipes["ValuActive_pct"] = 100 * 4 * avg["SQ_ACTIVE_INST_VALU"] / simd_cycles
        f64 = [avg.get(f"SQ_INSTS_VALU_{o}_F64") for o in ("ADD", "MUL", "FMA")]
        if simd_cycles and all(v is not None for v in f64):
            pipes["Fp64PipeBusy_pct"] = 100 * 4 * sum(f64) / simd_cycles
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            pipes["L2_hit_pct"] = 100 * avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] +
                                                                   avg["TCC_MISS_sum"])
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg:
            pipes["LdsBankConflict_pct"] = 100 * avg["SQ_LDS_BANK_CONFLICT"] / max(
                1.0, avg["SQ_LDS_IDX_ACTIVE"])
        r["counters"] = avg
        r.update(pipes)
    if all(k in out and "hbm_bytes_per_launch" in out[k] for k in FABRIK_PIPELINE):
        out["fabrik_pipeline"] = {
            "kernels": list(FABRIK_PIPELINE),
            "rocprof_avg_ms": sum(out[k]["rocprof_avg_ms"] for k in FABRIK_PIPELINE),
            "hbm_bytes_per_launch": sum(out[k]["hbm_bytes_per_launch"] for k in FABRIK_PIPELINE),
            "hbm_bytes_per_launch_raw": sum(out[k]["hbm_bytes_per_launch_raw"]
                                            for k in FABRIK_PIPELINE)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--methods", nargs="+", required=True)
    ap.add_argument("--window", type=int, default=20)
    ap.add_argument("--pmc-window", type=int, default=5)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    os.makedirs(os.path.join(args.out, "pmc"), exist_ok=True)
    traffic_path = os.path.join(args.out, "traffic.json")
    traffic = {}
    if os.path.exists(traffic_path):
        with open(traffic_path) as f:
            traffic = json.load(f)
    for m in args.methods:
        s = summarise(args.dir, m, args.window, args.pmc_window)
        with open(os.path.join(args.out, "pmc", f"{m}_summary.json"), "w") as f:
            json.dump(s, f, indent=1, sort_keys=True)
        for k, v in s.items():
            traffic[k] = {a: b for a, b in v.items() if a != "counters"}
        print(m, json.dumps({k: {a: (round(b, 4) if isinstance(b, float) else b)
                                 for a, b in v.items() if a != "counters"}
                             for k, v in s.items()}))
    with open(traffic_path, "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
