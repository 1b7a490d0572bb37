"""Fold the cross-box rocprof spread into a round's traffic.json: for every kernel
entry with a window average, `rocprof_boxes_ms` lists the profiling lease's own
figure first, then each tools/trace_box.sh box's (profiles/<round>/boxes/*/
traffic.json), and `rocprof_median_ms` is their median.  bench.py prices
frac_rocprof on the median (a driver box is any box: the profiling lease's own
clock is one draw of several), and reports the list beside it.

    python tools/merge_boxes.py profiles/r06
"""
import glob
import json
import os
import statistics
import sys


def main():
    rd = sys.argv[1]
    path = os.path.join(rd, "traffic.json")
    t = json.load(open(path))
    boxes = [json.load(open(f)) for f in sorted(glob.glob(os.path.join(rd, "boxes", "*", "traffic.json")))]
    for k, v in t.items():
        if not isinstance(v, dict) or "rocprof_avg_ms" not in v:
            continue
        ms = [v["rocprof_avg_ms"]] + [b[k]["rocprof_avg_ms"] for b in boxes
                                      if isinstance(b.get(k), dict) and "rocprof_avg_ms" in b[k]]
        v["rocprof_boxes_ms"] = ms
        v["rocprof_median_ms"] = statistics.median(ms)
    with open(path, "w") as f:
        json.dump(t, f, indent=1, sort_keys=True)
    for k in ("ann_fused_kernel", "fabrik_iter_kernel", "fabrik_tol1e-5/fabrik_iter_kernel", "fk_kernel"):
        if k in t:
            print(k, t[k]["rocprof_boxes_ms"], "median", t[k]["rocprof_median_ms"])


if __name__ == "__main__":
    main()
