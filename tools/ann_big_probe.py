"""Throughput of the ANN layered path (models past the fused kernel's caps,
csrc/ik_ann_big.hip): a few model shapes on n random_dist points, device arrays,
per-kernel HIP-event times of one call and the mean of `reps` calls; prints one JSON
line per model with the achieved TFLOP/s of the Dense layers (2 * sum in * out per point).

    python tools/ann_big_probe.py [n] [only] [mode]   (only: e.g. 4096x2 or "all";
                                                      mode: fp32 (default) / bf16x6)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    from inversekinematicsann_amd.robot.position_generator import random_dist
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    ctx = _native.Context(0)
    pts = torch.from_numpy(random_dist(n, seed=0)).cuda()
    ang = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    only = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "all" else None
    mode = sys.argv[3] if len(sys.argv) > 3 else "fp32"
    ctx.ann_set_mode(mode)
    for dims in ((3, 2048, 2048, 4), (3,) + (512,) * 30 + (4,), (3, 4096, 4096, 4),
                 (3,) + (500,) * 12 + (4,)):
        if only and only != f"{dims[1]}x{len(dims) - 2}":
            continue
        m = glorot_model(dims=dims, seed=1)
        ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
        flop = 2 * sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1)) * n
        ctx.ann_solve_device(pts, ang)
        torch.cuda.synchronize()
        ctx.set_timing(True)
        ctx.ann_solve_device(pts, ang)
        torch.cuda.synchronize()
        ks = ctx.kernel_times()
        ctx.set_timing(False)
        reps = 5
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.ann_solve_device(pts, ang)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        gemm = sum(v for k, v in ks if "gemm" in k)
        print(json.dumps({"dims": f"{dims[1]}x{len(dims) - 2}", "mode": mode, "points": n,
                          "ms_per_call": ms,
                          "tflops_call": flop / ms / 1e9,
                          "gemm_ms_events": gemm, "tflops_gemm": flop / gemm / 1e9 if gemm else None,
                          "kernels": len(ks)}), flush=True)


if __name__ == "__main__":
    main()
