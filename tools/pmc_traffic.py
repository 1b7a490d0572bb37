"""Summarise rocprofv3 output for the bench kernels.

    python tools/pmc_traffic.py --stats DIR --fetch DIR --write DIR --out profiles/traffic.json

* --stats: a `rocprofv3 --kernel-trace --stats --output-format csv` directory
  (per-kernel call count and average duration);
* --fetch / --write: `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes
  (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: both counters are
in KiB, and on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
read (MI355X_MICROARCH.md, HBM).  Infinity-Cache hits are counted by these
counters, so this is "bytes beyond L2", an upper bound on DRAM traffic.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = ("ann_fused_kernel", "fabrik_iter_kernel", "fabrik_classify_scatter_kernel",
           "fabrik_classify_kernel",
           "fabrik_scatter_kernel", "fabrik_fold_kernel", "fabrik_simple_kernel", "reset_stats_kernel",
           "gather_unpack_kernel", "fk_kernel")
# every kernel one FABRIK solve launches (ik_fabrik.hip): the pipeline's bytes
FABRIK_PIPELINE = ("reset_stats_kernel", "fabrik_classify_scatter_kernel",
                   "fabrik_classify_kernel", "fabrik_scatter_kernel", "fabrik_iter_kernel",
                   "fabrik_fold_kernel")


def _short(name: str) -> str | None:
    if "ann_fused_kernel<" in name:  # ann_fused_kernel<MR, X>: X = 0 fp32, 1 bf16x6, 2 fp16x3
        x = name.split("ann_fused_kernel<", 1)[1].split(">", 1)[0].split(",")[-1].strip()
        return {"1": "ann_fused_kernel_bf16x6", "2": "ann_fused_kernel_fp16x3"}.get(
            x, "ann_fused_kernel")
    for k in KERNELS:
        if k in name:
            return k
    return None


def read_counters(d: str, counter: str):
    tot = defaultdict(float)
    calls = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = _short(row.get("Kernel_Name", ""))
                if not k or row.get("Counter_Name") != counter:
                    continue
                tot[k] += float(row["Counter_Value"])
                calls[k].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    return {k: (tot[k], len(calls[k])) for k in tot}


def read_stats(d: str):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = _short(row.get("Name", ""))
                if k:
                    out[k] = {"calls": int(row["Calls"]),
                              "avg_ms": float(row["AverageNs"]) / 1e6,
                              "total_ms": float(row["TotalDurationNs"]) / 1e6}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    res = {}
    if os.path.exists(args.out):
        with open(args.out) as f:
            res = json.load(f)
    stats = read_stats(args.stats) if args.stats else {}
    fetch = read_counters(args.fetch, "FETCH_SIZE") if args.fetch else {}
    write = read_counters(args.write, "WRITE_SIZE") if args.write else {}
    for k in set(stats) | set(fetch) | set(write):
        r = res.setdefault(k, {})
        if k in stats:
            r.update({"rocprof_" + a: b for a, b in stats[k].items()})
        if k in fetch and k in write:
            (fk, fc), (wk, wc) = fetch[k], write[k]
            r["fetch_kib_per_launch"] = fk / max(fc, 1)
            r["write_kib_per_launch"] = wk / max(wc, 1)
            r["hbm_bytes_per_launch"] = (2 * fk / max(fc, 1) + wk / max(wc, 1)) * 1024
    if all(k in fetch and k in write for k in FABRIK_PIPELINE):
        # per solve: the sum over its launches (60 B per point at the API boundary,
        # SURVEY 8(d); + 8 B when the FK round-trip errors are written)
        res["fabrik_pipeline"] = {
            "kernels": list(FABRIK_PIPELINE),
            "hbm_bytes_per_launch": sum(res[k]["hbm_bytes_per_launch"] for k in FABRIK_PIPELINE)}
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
