"""Time the fused ANN kernel (reference architecture, 1M points) under each
tile variant (IKHIP_ANN_MR=1|2) and GEMM mode (IKHIP_ANN_MODE=fp32|bf16x6), in
fresh subprocesses; checks the result against a float64 numpy forward on the
first 2048 points."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, json, torch, numpy as np
sys.path.insert(0, %r)
from inversekinematicsann_amd import _native
from inversekinematicsann_amd.kinematics.ann import glorot_model, REFERENCE_X_SCALER as XS, REFERENCE_Y_SCALER as YS
from inversekinematicsann_amd.robot.position_generator import random_dist
from oracle import oracle as O
n = int(sys.argv[1])
m = glorot_model(seed=0)
p = random_dist(n, seed=0)
pts = torch.from_numpy(p).cuda()
ang = torch.empty((n, 4), dtype=torch.float32, device="cuda")
err = torch.empty(n, dtype=torch.float64, device="cuda")
ctx = _native.Context(0)
ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
F = _native.IK_F_DEVICE
for _ in range(2): ctx.ann_solve_device(pts, ang, err, flags=F)
ctx.set_timing(True)
ts = []
for _ in range(5):
    ctx.ann_solve_device(pts, ang, err, flags=F)
    ts.append(sum(v for k, v in ctx.kernel_times()))
ref = O.ann_forward(p[:2048], m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale,
                    compute=np.float64)
d = float(np.abs(ang[:2048].cpu().numpy().astype(np.float64) - ref).max())
print(json.dumps({"ms": min(ts), "ms_med": sorted(ts)[2], "max_abs_diff": d,
                  "tflops": 5.507e6 * n / (min(ts) / 1e3) / 1e12}))
''' % ROOT

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fp32", "bf16x6", "fp16x3"]
    mrs = os.environ.get("SWEEP_MR", "1,2").split(",")
    extra = [kv.split("=", 1) for kv in os.environ.get("SWEEP_ENV", "").split(";") if kv]
    for mode in modes:
     for env in ([{}] + [{k: v} for k, v in extra]):
      for mr in mrs:
        e = dict(os.environ, IKHIP_ANN_MR=mr, IKHIP_ANN_MODE=mode, **env)
        out = subprocess.run([sys.executable, "-c", CODE, str(n)], env=e, capture_output=True,
                             text=True, timeout=600)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"MR": mr, "mode": mode, **env, **(json.loads(line[-1]) if line else
                                       {"error": out.stderr[-800:]})}), flush=True)
