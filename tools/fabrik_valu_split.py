"""VALU instructions of the FABRIK iteration kernel in and out of its inner loop
(VERDICT r05 #2), from a rocprofv3 SQ counter pass (tools/fabrik_valu_split.sh), the
diagnostic build's wave-iteration count (tools/fabrik_diag.py) and the loop's VALU
per iteration from the ISA (tools/isa_loop.py on the production build):

    in-loop = VALU per iteration x wave-iterations;  out = SQ_INSTS_VALU - in-loop

    python tools/fabrik_valu_split.py DIR DIAG_JSON LOOP_VALU [--json OUT]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def kernel_counters(d, kernel="fabrik_iter_kernel"):
    per = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r.get("Kernel_Name", ""):
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)[-5:]  # the bench's timed steps (the last five dispatches)
    out = defaultdict(float)
    for i in ids:
        for k, v in per[i].items():
            out[k] += v / len(ids)
    return dict(out), len(ids)


def main():
    d, diag, loop = sys.argv[1], sys.argv[2], float(sys.argv[3])
    dg = json.load(open(diag))
    res = {}
    for tol, key in (("1e-3", "tol0.001"), ("1e-5", "tol1e-05")):
        c, n = kernel_counters(os.path.join(d, f"pmc_{tol}"))
        if not c:
            continue
        steps = dg[key]["steps"]
        valu = c["SQ_INSTS_VALU"]
        inl = loop * steps
        res[tol] = {"SQ_INSTS_VALU": valu, "wave_iterations": steps, "loop_valu_per_iteration": loop,
                    "in_loop": inl, "out_of_loop": valu - inl,
                    "out_of_loop_frac": (valu - inl) / valu,
                    "points": dg[key].get("sum_iters") and 1_000_000,
                    "valu_active_frac_of_wave_cycles": c.get("SQ_ACTIVE_INST_VALU", 0) / c.get("SQ_WAVE_CYCLES", 1),
                    "counters": c, "dispatches_averaged": n}
        print(f"tol {tol}: SQ_INSTS_VALU {valu / 1e6:.1f} M, in loop {inl / 1e6:.1f} M "
              f"({loop:.0f} x {steps} wave-iterations), out {(valu - inl) / 1e6:.1f} M = "
              f"{100 * (valu - inl) / valu:.1f} %")
    if "--json" in sys.argv:
        json.dump(res, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
