"""How fast would FABRIK be split in two kernels?  A probe build
(-DIKHIP_PROBE_SPLIT, optionally -DIKHIP_ITER_WAVES=3) parks a finished lane's
joints straight to HBM instead of the LDS retire ring and runs no angles step
(its angles are NOT computed: timing only).  This script times one library's
pipeline on the bench's 1M random_dist points at tol 1e-3 and 1e-5, and with
--simple the max_iter = 0 pipeline (seed + angles + FK round trip, one point per
lane: an upper bound for a separate angles kernel).  One library per process:

    IKHIP_LIB=inversekinematicsann_amd/libikhip_probe3.so python3 tools/split_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist
    probe = "probe" in os.environ.get("IKHIP_LIB", "")
    n = 1_000_000
    ctx = _native.Context(0)
    pts = torch.from_numpy(random_dist(n, seed=0)).cuda()
    ang = torch.empty((n, 4), dtype=torch.float64, device="cuda")
    it = torch.empty(n, dtype=torch.int32, device="cuda")
    jo = torch.empty((n, 4, 3), dtype=torch.float64, device="cuda") if probe else None
    fk = None if probe else torch.empty(n, dtype=torch.float64, device="cuda")
    res = {"lib": os.path.basename(os.environ.get("IKHIP_LIB", "libikhip.so"))}
    cases = [("tol1e-3", 1e-3, 100), ("tol1e-5", 1e-5, 200)]
    if "--simple" in sys.argv:
        cases.append(("simple_max_iter0", 1e-3, 0))
    for name, tol, mi in cases:
        for _ in range(5):  # warm-up; the work order learns
            ctx.fabrik_solve_device(pts, ang, it, jo, tol=tol, max_iter=mi, fk_err=fk)
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ctx.fabrik_solve_device(pts, ang, it, jo, tol=tol, max_iter=mi, fk_err=fk)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        res[name] = {"median_ms": ts[len(ts) // 2], "min_ms": ts[0],
                     "iters_sum": int(it.to(torch.int64).sum().item())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
