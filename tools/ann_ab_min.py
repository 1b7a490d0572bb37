"""Same-box A/B of two libikhip builds on the ANN path through the ABI both
share (the r03 and r04 split-mode kernels on one box).  Uses
only entry points every round's library exports (ik_ctx_create, ik_ann_load,
ik_ann_set_mode, ik_ann_solve, ik_ctx_set_stream), so an older build loads too.

    python tools/ann_ab_min.py LIB MODE [STEPS] [WARMUP]

One JSON line: the library, the mode, ms per step (HIP events around STEPS
IK_F_DEVICE | IK_F_ASYNC solves of 1M random_dist points on torch's stream),
and a digest of the angles (two builds that claim the same arithmetic print the
same digest)."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib_path, mode = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    warm = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    import torch
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    from inversekinematicsann_amd.robot.position_generator import random_dist
    L = ctypes.CDLL(lib_path)
    vp = ctypes.c_void_p
    L.ik_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.ik_ctx_set_stream.argtypes = [vp, vp]
    L.ik_ann_set_mode.argtypes = [vp, ctypes.c_int]
    L.ik_ann_load.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
    L.ik_ann_solve.argtypes = [vp, vp, ctypes.c_int64, vp, vp, ctypes.c_int, vp]
    L.ik_last_error.restype = ctypes.c_char_p
    h = vp()
    assert L.ik_ctx_create(0, ctypes.byref(h)) == 0, L.ik_last_error()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    assert L.ik_ctx_set_stream(h, vp(stream.cuda_stream)) == 0
    dims = (3,) + (500,) * 12 + (4,)
    m = glorot_model(dims, seed=0)
    W = [np.ascontiguousarray(w, np.float32) for w in m.weights]
    B = [np.ascontiguousarray(b, np.float32) for b in m.biases]
    acts = np.array([{"tanh": 1, "linear": 0}[a] if isinstance(a, str) else int(a)
                     for a in m.activations], np.int32)
    d = np.array(dims, np.int32)
    Wp = (vp * len(W))(*[w.ctypes.data for w in W])
    Bp = (vp * len(B))(*[b.ctypes.data for b in B])
    sc = [np.ascontiguousarray(v, np.float64) for v in (XS.mean, XS.scale, YS.mean, YS.scale)]
    rc = L.ik_ann_load(h, len(W), d.ctypes.data, acts.ctypes.data, Wp, Bp,
                       *[v.ctypes.data for v in sc])
    assert rc == 0, L.ik_last_error()
    assert L.ik_ann_set_mode(h, {"fp32": 0, "bf16x6": 1, "fp16x3": 2}[mode]) == 0
    n = 1_000_000
    dpts = torch.from_numpy(random_dist(n, seed=0)).cuda()
    dang = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    derr = torch.empty(n, dtype=torch.float64, device="cuda")

    def step():
        rc = L.ik_ann_solve(h, dpts.data_ptr(), n, dang.data_ptr(), derr.data_ptr(), 1 | 2, None)
        assert rc == 0, L.ik_last_error()
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    dig = hashlib.sha256(dang.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": os.path.basename(lib_path), "mode": mode, "ms_per_step": ms,
                      "points": n, "steps": steps, "warmup": warm, "angles_sha16": dig}),
          flush=True)


if __name__ == "__main__":
    main()
