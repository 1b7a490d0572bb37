"""Iteration-kernel counters of the FABRIK pipeline (diagnostic build
libikhip_diag.so, IKHIP_LIB=...): lane efficiency (useful lane-steps / 64 x
wave-steps), refills and chunk grabs per wave, the core-path fallbacks, and the
spread of wave start / end times (the launch tail).  Diagnostic only."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("IKHIP_LIB", os.path.join(ROOT, "inversekinematicsann_amd",
                                                "libikhip_diag.so"))
from inversekinematicsann_amd import _native  # noqa: E402
from inversekinematicsann_amd.robot.position_generator import random_dist  # noqa: E402

NAMES = ["loops", "steps", "lane_steps", "refills", "grabs", "fallbacks", "waves", "flushes", "flush_ticks", "prep_ticks"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
pts = torch.from_numpy(random_dist(n, seed=0)).cuda()
ang = torch.empty((n, 4), dtype=torch.float64, device="cuda")
it = torch.empty(n, dtype=torch.int32, device="cuda")
ctx = _native.Context(0)
out = {}
for tol, mi in ((1e-3, 100), (1e-5, 200)):
    for _ in range(3):  # the work order learns its cost table
        ctx.fabrik_solve_device(pts, ang, it, None, tol, mi, flags=_native.IK_F_DEVICE)
    ctx.set_debug(True)
    ctx.fabrik_solve_device(pts, ang, it, None, tol, mi, flags=_native.IK_F_DEVICE)
    w = ctx.debug_words(64 + 4 * 4000).astype(np.int64)
    ctx.set_debug(False)
    c = dict(zip(NAMES, w[:len(NAMES)].tolist()))
    nw = min(c["waves"], 4000)
    t = w[64:64 + 4 * nw].reshape(nw, 4)
    t0 = t[:, 0].min()
    us = lambda v: np.percentile((v - t0) / 100.0, [0, 1, 10, 50, 90, 99, 100]).round(1).tolist()
    c["lane_eff"] = c["lane_steps"] / (64.0 * max(c["steps"], 1))
    c["sum_iters"] = int(it.sum().item())
    c["flush_us_per_wave"] = c["flush_ticks"] / 100.0 / max(c["waves"], 1)
    c["prep_us_per_wave"] = c["prep_ticks"] / 100.0 / max(c["waves"], 1)
    c["steps_per_refill"] = c["steps"] / max(c["refills"], 1)
    c["pct"] = [0, 1, 10, 50, 90, 99, 100]
    c["wave_start_us"] = us(t[:, 0])
    c["wave_dry_us"] = us(t[:, 1])
    c["wave_end_us"] = us(t[:, 2])
    c["steps_after_dry"] = np.percentile(t[:, 3], [0, 1, 10, 50, 90, 99, 100]).tolist()
    c["us_per_step_after_dry"] = float(((t[:, 2] - t[:, 1]) / 100.0).sum() / max(t[:, 3].sum(), 1))
    out[f"tol{tol:g}"] = c
print(json.dumps(out, indent=1))
