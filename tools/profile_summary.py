"""Per-kernel figures of one profiling lease (tools/profile_round.sh), for each
bench method over its TIMED window only.

The profiled command is the bench's own (all secondaries, same order, same
warm-up), so every kernel's dispatches come in blocks of warmup + E + steps (E: the
per-kernel event step, 1; the r05 re-entry lease's bench also ran an untimed step, 2), one
block per method that launches it, in the bench's method order (ann, fabrik,
fabrik_tol1e-5, ann_bf16x6, ann_fp16x3, fk); the last `steps` dispatches of a block
are the timed ones.  Per (method, kernel):

* duration (average / min / max over the window) from the `--kernel-trace --stats`
  run;
* HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE passes: `raw` =
  (FETCH_SIZE + WRITE_SIZE) KiB and `doubled` = (2 FETCH_SIZE + WRITE_SIZE) KiB (the
  gfx950 correction MI355X_MICROARCH.md establishes for wide coalesced reads; for a
  gather-pattern kernel -- FABRIK reads 24-byte points through a permutation -- the
  raw figure is the one to trust; both are reported);
* the kernel's shader clock, GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) over the
  dispatch's own duration (kernels longer than 50 us);
* pipe occupancy (MFMA busy, VALU active, fp64 pipe), L2 hit rate and LDS bank
  conflicts, as tools/pmc_summary.py computes them.

    python tools/profile_summary.py --dir gpurun_out/prof --steps 20 --warmup 5 \\
        --pmc-steps 5 --out profiles/r03
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

# bench.py's method order with --method ann (run_ann first, then the secondaries)
ORDER = ["ann", "fabrik", "fabrik_tol1e-5", "ann_bf16x6", "ann_fp16x3", "fk"]
METHODS_OF = {"ann_fused_kernel": ["ann"],
              "ann_fused_kernel_bf16x6": ["ann_bf16x6"],
              "ann_fused_kernel_fp16x3": ["ann_fp16x3"],
              "fabrik_classify_scatter_kernel": ["fabrik", "fabrik_tol1e-5"],
              "fabrik_classify_kernel": ["fabrik", "fabrik_tol1e-5"],
              "fabrik_scatter_kernel": ["fabrik", "fabrik_tol1e-5"],
              "fabrik_iter_kernel": ["fabrik", "fabrik_tol1e-5"],
              "fabrik_fold_kernel": ["fabrik", "fabrik_tol1e-5"],
              "fk_kernel": ["fk"]}


# bench.timed(): the per-kernel event steps between the warm-up and the timed loop
# (--event-steps: bench.TIMING_REPS from r06, 1 before; profiles/r05/lease_f was
# made by a bench with one more, untimed)
EVENT_STEPS = 5


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


def windows(ids, methods, block, steps):
    """method -> the dispatch ids of its timed window (the last `steps` of its block)."""
    out = {}
    if len(ids) != len(methods) * block:
        print(f"warning: {len(ids)} dispatches for {methods} x {block}", file=sys.stderr)
    for b, m in enumerate(methods):
        blk = ids[b * block:(b + 1) * block]
        out[m] = blk[-steps:]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pmc-steps", type=int, default=5)
    ap.add_argument("--event-steps", type=int, default=EVENT_STEPS)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    res = defaultdict(dict)  # method -> kernel -> figures
    tr = durations(os.path.join(args.dir, "trace"))
    for k, methods in METHODS_OF.items():
        if k not in tr:
            continue
        ids = [i for i, _ in tr[k]]
        ms = dict(tr[k])
        for m, win in windows(ids, methods, args.warmup + args.event_steps + args.steps, args.steps).items():
            w = [ms[i] for i in win]
            if w:
                res[m][k] = {"rocprof_avg_ms": sum(w) / len(w), "rocprof_min_ms": min(w),
                             "rocprof_max_ms": max(w), "rocprof_window": len(w),
                             "rocprof_all_dispatches": len(ids)}
    if "reset_stats_kernel" in tr:  # ~4 us, one per solve: its median over the run
        v = sorted(ms for _, ms in tr["reset_stats_kernel"])
        for m in ("fabrik", "fabrik_tol1e-5"):
            res[m]["reset_stats_kernel"] = {"rocprof_avg_ms": v[len(v) // 2],
                                            "note": "median over all the run's dispatches"}
    pmc = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))
    clocks = defaultdict(lambda: defaultdict(list))
    pblock = args.warmup + args.event_steps + args.pmc_steps
    for d in sorted(glob.glob(os.path.join(args.dir, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        cs, ds = counters(d), durations(d)
        for k, methods in METHODS_OF.items():
            if k not in cs:
                continue
            dur = dict(ds.get(k, []))
            for m, win in windows(sorted(cs[k]), methods, pblock, args.pmc_steps).items():
                for i in win:
                    for c, v in cs[k][i].items():
                        pmc[m][k][c].append(v)
                    if "GRBM_GUI_ACTIVE" in cs[k][i] and dur.get(i, 0.0) > 0.05:
                        clocks[m][k].append(cs[k][i]["GRBM_GUI_ACTIVE"] / 8 / (dur[i] * 1e-3) / 1e9)
    for m, byk in pmc.items():
        for k, cs in byk.items():
            r = res[m].setdefault(k, {})
            avg = {c: sum(v) / len(v) for c, v in cs.items()}
            if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
                r["fetch_kib_per_launch"] = avg["FETCH_SIZE"]
                r["write_kib_per_launch"] = avg["WRITE_SIZE"]
                r["hbm_bytes_per_launch_raw"] = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
                r["hbm_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
            if clocks[m].get(k):
                r["clock_ghz"] = sum(clocks[m][k]) / len(clocks[m][k])
            simd = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 1024
            if simd and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                r["MfmaUtil_pct"] = 100 * avg["SQ_VALU_MFMA_BUSY_CYCLES"] / simd
            if simd and "SQ_ACTIVE_INST_VALU" in avg:  # quad-cycles
                r["ValuActive_pct"] = 100 * 4 * avg["SQ_ACTIVE_INST_VALU"] / simd
            f64 = [avg.get(f"SQ_INSTS_VALU_{o}_F64") for o in ("ADD", "MUL", "FMA")]
            if simd and all(v is not None for v in f64):
                r["Fp64PipeBusy_pct"] = 100 * 4 * sum(f64) / simd
            if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
                r["L2_hit_pct"] = 100 * avg["TCC_HIT_sum"] / max(
                    1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
            if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg:
                r["LdsBankConflict_pct"] = 100 * avg["SQ_LDS_BANK_CONFLICT"] / max(
                    1.0, avg["SQ_LDS_IDX_ACTIVE"])
            r["counters"] = avg
    for m in ("fabrik", "fabrik_tol1e-5"):
        # the build's own pipeline: fused classify + scatter (r04) or the two kernels
        ks = [k for k in FABRIK_PIPELINE if k in res[m]]
        if "fabrik_iter_kernel" in ks and "reset_stats_kernel" in ks:
            res[m]["fabrik_pipeline"] = {
                "kernels": ks,
                "rocprof_avg_ms": sum(res[m][k]["rocprof_avg_ms"] for k in ks),
                "hbm_bytes_per_launch": sum(res[m][k].get("hbm_bytes_per_launch", 0.0) for k in ks),
                "hbm_bytes_per_launch_raw": sum(res[m][k].get("hbm_bytes_per_launch_raw", 0.0)
                                                for k in ks)}
    # the bench line of the same lease beside it
    line = None
    try:
        with open(os.path.join(args.dir, "bench_default.log")) as f:
            line = json.loads([x for x in f if x.startswith("{")][-1])
    except (OSError, IndexError, ValueError):
        pass
    if line:
        steps = {"ann": (line["ms_per_step"], line["kernels_ms"])}
        for m, v in line.get("secondary", {}).items():
            steps[m] = (v["ms_per_step"], v.get("kernels_ms"))
        for m, (ms, kms) in steps.items():
            if m in res:
                res[m]["bench_line"] = {"ms_per_step": ms, "kernels_ms_events": kms}
    os.makedirs(os.path.join(args.out, "pmc"), exist_ok=True)
    traffic = {}
    for m in ORDER:
        if m not in res:
            continue
        with open(os.path.join(args.out, "pmc", f"{m}_diag_summary.json"), "w") as f:
            json.dump(res[m], f, indent=1, sort_keys=True)
        for k, v in res[m].items():
            if k == "bench_line":
                continue
            key = k if m in ("ann", "fabrik", "ann_bf16x6", "ann_fp16x3", "fk") else f"{m}/{k}"
            traffic[key] = {a: b for a, b in v.items() if a != "counters"}
        print(m, json.dumps({k: ({a: (round(b, 4) if isinstance(b, float) else b)
                                  for a, b in v.items() if a != "counters"}
                                 if isinstance(v, dict) else v) for k, v in res[m].items()}))
    with open(os.path.join(args.out, "traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
