"""The bench's FABRIK end-to-end leg (host float64 points in, host angles out,
pinned arrays: ik_fabrik_solve's chunked copy / solve / copy pipeline) called
many times, each call bracketed by a roctx range, so that a
`rocprofv3 --hip-trace --memory-copy-trace --kernel-trace --marker-trace` run
shows what a slow call waited on.  Prints the per-call
wall times as one JSON line; tools/e2e_trace_summary.py reads the trace.

    python tools/e2e_trace.py [--calls 200] [--pageable 0|1] [--ann-first 0|1]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--pageable", type=int, default=0)
    ap.add_argument("--ann-first", type=int, default=1,
                    help="run the bench's ANN step first (what precedes the leg in bench.py)")
    args = ap.parse_args()
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist
    try:
        rtx = ctypes.CDLL("/opt/rocm/lib/libroctx64.so")
        push, pop = rtx.roctxRangePushA, rtx.roctxRangePop
        push.argtypes = [ctypes.c_char_p]
    except OSError:
        push = pop = None
    n = args.points
    pts = random_dist(n, seed=0)
    ctx = _native.Context(0)
    if args.ann_first:
        from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                             REFERENCE_Y_SCALER as YS,
                                                             glorot_model)
        m = glorot_model((3,) + (500,) * 12 + (4,), seed=0)
        ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
        dp = torch.from_numpy(pts).cuda()
        da = torch.empty((n, 4), dtype=torch.float32, device="cuda")
        for _ in range(3):
            ctx.ann_solve_device(dp, da)
        torch.cuda.synchronize()
    if args.pageable:
        hp = np.ascontiguousarray(pts)
        ang = np.empty((n, 4), np.float64)
    else:
        hp = _native.pinned_empty(pts.shape, np.float64)
        hp[:] = pts
        ang = _native.pinned_empty((n, 4), np.float64)
    s = _native.IkStats()
    L, h = ctx.lib, ctx.handle

    def call():
        ctx._check(L.ik_fabrik_solve_fk(h, hp.ctypes.data, n, 1e-3, 100, ang.ctypes.data,
                                        None, None, None, 0, ctypes.byref(s)))
    for _ in range(10):
        call()
    times = []
    for k in range(args.calls):
        if push:
            push(f"call{k}".encode())
        t0 = time.perf_counter()
        call()
        times.append((time.perf_counter() - t0) * 1e3)
        if pop:
            pop()
    t = np.array(times)
    print(json.dumps({"calls": len(t), "pageable": bool(args.pageable), "mean_ms": t.mean(),
                      "median_ms": float(np.median(t)), "max_ms": t.max(),
                      "slow_calls": [int(i) for i in np.nonzero(t > 1.5 * np.median(t))[0]],
                      "times_ms": [round(x, 4) for x in t]}), flush=True)


if __name__ == "__main__":
    main()
