"""Time the FABRIK pipeline under different persistent-grid settings.
Each setting runs in a fresh subprocess (the knobs are read once per process)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, json, torch, numpy as np
sys.path.insert(0, %r)
from inversekinematicsann_amd import _native
from inversekinematicsann_amd.robot.position_generator import random_dist
n = int(sys.argv[1]); tol = float(sys.argv[2]); mi = int(sys.argv[3])
pts = torch.from_numpy(random_dist(n, seed=0)).cuda()
ang = torch.empty((n, 4), dtype=torch.float64, device="cuda")
it = torch.empty(n, dtype=torch.int32, device="cuda")
ctx = _native.Context(0)
F = _native.IK_F_DEVICE
for _ in range(3): ctx.fabrik_solve_device(pts, ang, it, None, tol, mi, flags=F)
ctx.set_timing(True)
res = {}
for _ in range(5):
    ctx.fabrik_solve_device(pts, ang, it, None, tol, mi, flags=F)
    for k, v in ctx.kernel_times():
        res.setdefault(k, []).append(v)
print(json.dumps({k: min(v) for k, v in res.items()}))
''' % ROOT

def run(env, n, tol, mi):
    e = dict(os.environ); e.update(env)
    out = subprocess.run([sys.executable, "-c", CODE, str(n), str(tol), str(mi)], env=e,
                         capture_output=True, text=True, timeout=300)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    return json.loads(line[-1]) if line else {"error": out.stderr[-500:]}

if __name__ == "__main__":
    cases = []
    if len(sys.argv) > 1 and sys.argv[1] == "order":  # work order on/off x grid knobs
        for order in ("0", "1"):
            for bpc in ("2", "4"):
                for chunk in ("32", "64"):
                    cases.append({"IKHIP_FABRIK_ORDER": order, "IKHIP_FABRIK_BPC": bpc,
                                  "IKHIP_FABRIK_CHUNK": chunk})
    if len(sys.argv) > 1 and sys.argv[1] == "grid":  # persistent-grid size, ordered pipeline
        for bpc in ("2", "3", "4"):
            cases.append({"IKHIP_FABRIK_BPC": bpc})
    if len(sys.argv) > 1 and sys.argv[1] == "bpc":  # grid size across tolerances / sizes
        for bpc in ("2", "3", "4"):
            cases.append({"IKHIP_FABRIK_BPC": bpc})
    if len(sys.argv) > 1 and sys.argv[1] == "chunk":  # grab size x grid, twice
        for _rep in range(2):
            for ch in os.environ.get("SWEEP_CHUNKS", "64,96,128,192").split(","):
                for bpc in os.environ.get("SWEEP_BPCS", "2,3").split(","):
                    cases.append({"IKHIP_FABRIK_CHUNK": ch, "IKHIP_FABRIK_BPC": bpc})
    if len(sys.argv) > 1 and sys.argv[1] == "core":  # iteration sequences x grid, twice
        for _rep in range(2):
            for core in os.environ.get("SWEEP_CORES", "1,2").split(","):
                for bpc in os.environ.get("SWEEP_BPCS", "2,3").split(","):
                    cases.append({"IKHIP_FABRIK_CORE": core, "IKHIP_FABRIK_BPC": bpc})
    for var in (() if cases else ("1", "2", "0")):
        for bpc in ("2", "4", "8"):
            for chunk in ("64", "256"):
                if var == "0" and (bpc != "8" or chunk != "64"):
                    continue
                cases.append({"IKHIP_FABRIK_VARIANT": var, "IKHIP_FABRIK_BPC": bpc,
                              "IKHIP_FABRIK_CHUNK": chunk})
    n_pts = int(os.environ.get("SWEEP_N", "1000000"))
    tols = [(float(t.split("/")[0]), int(t.split("/")[1]))
            for t in os.environ.get("SWEEP_TOLS", "1e-3/100,1e-5/200").split(",")]
    for n, tol, mi in [(n_pts, t, m) for t, m in tols]:
        for c in cases:
            r = run(c, n, tol, mi)
            tot = sum(v for v in r.values() if isinstance(v, float))
            print(json.dumps({"n": n, "tol": tol, **c, "total_ms": tot, **r}), flush=True)
