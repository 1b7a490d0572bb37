"""In-kernel s_memtime breakdown of the fused ANN kernel (workgroup 0, tiles
1..3, every wave): cycles per phase of one tile.  Diagnostic only."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from inversekinematicsann_amd import _native  # noqa: E402
from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,  # noqa: E402
                                                     REFERENCE_Y_SCALER as YS, glorot_model)
from inversekinematicsann_amd.robot.position_generator import random_dist  # noqa: E402

n = 1_000_000
m = glorot_model(seed=0)
pts = torch.from_numpy(random_dist(n, seed=0)).cuda()
ang = torch.empty((n, 4), dtype=torch.float32, device="cuda")
err = torch.empty(n, dtype=torch.float64, device="cuda")
ctx = _native.Context(0)
ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
if __import__("os").environ.get("MODE"):  # fp32 (default) / bf16x6 / fp16x3
    ctx.ann_set_mode(__import__("os").environ["MODE"])
ctx.ann_solve_device(pts, ang, err, flags=_native.IK_F_DEVICE)
ctx.set_debug(True)
ctx.ann_solve_device(pts, ang, err, flags=_native.IK_F_DEVICE)
st = ctx.debug_stamps().astype(np.int64)  # tile, wave, slot
L = len(m.weights)
res = {"layers": L, "per_tile": []}
for t in range(1, 4):
    w = st[t]
    row = {"tile_cycles": int(w[:, 31].max() - w[:, 0].min()),
           "staging": int(np.median(w[:, 1] - w[:, 0]))}
    gemm, epi = [], []
    prev = w[:, 1]
    for l in range(L):
        g = w[:, 2 + 2 * l] - prev          # start of layer -> this wave's GEMM done
        e = w[:, 3 + 2 * l] - w[:, 2 + 2 * l]  # GEMM done -> layer done (barriers, epilogue)
        gemm.append([int(x) for x in g])
        epi.append([int(x) for x in e])
        prev = w[:, 3 + 2 * l]
    row["gemm_per_layer_per_wave"] = gemm
    row["post_gemm_per_layer_per_wave"] = epi
    row["output"] = int(np.median(w[:, 31] - w[:, 3 + 2 * (L - 1)]))
    if L > 5:  # slot 30: layer 5's first K group done (from layer 4 done)
        row["layer5_first_group"] = [int(x) for x in w[:, 30] - w[:, 3 + 2 * 4]]
    res["per_tile"].append(row)
print(json.dumps(res))
