"""bench.py's cpu_baseline leg on the CPU (no GPU): the oracle timed on a bounded
sample, its thread count, and the parity fields it computes against a GPU batch
(here the oracle's own output stands in for the GPU's)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


class _Args:
    tol = 1e-3
    max_iter = 100
    cpu_seconds = 0.2


def test_fabrik_cpu_baseline_threads_and_parity():
    import bench
    from oracle import oracle as O
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(4096, seed=0)
    ang, it, _, _ = O.fabrik_ikine(pts, 1e-3, 100)
    r = bench.cpu_baseline("fabrik", _Args(), sample_pts=pts, gpu_out={"ang": ang, "iters": it})
    assert r["kind"] == "port" and r["unit"] == "IK solutions/s" and r["value"] > 0
    assert 1 <= r["cores"] <= (os.cpu_count() or 1)
    assert r["parity"]["ok"] and r["parity"]["iters_equal"] == 4096
    assert r["parity"]["max_abs_diff"] == 0.0
    bad = it.copy()
    bad[7] += 1
    r = bench.cpu_baseline("fabrik", _Args(), sample_pts=pts, gpu_out={"ang": ang, "iters": bad})
    assert not r["parity"]["ok"] and r["parity"]["iters_equal"] == 4095


def test_ann_cpu_baseline_parity_fields():
    import bench
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(8192, seed=0)
    r = bench.cpu_baseline("ann", _Args(), sample_pts=pts)
    ref = r.pop("_ref")
    assert ref.shape == (8192, 4) and r["value"] > 0 and r["cores"] >= 1
    r = bench.cpu_baseline("ann", _Args(), sample_pts=pts,
                           gpu_out={"ang": ref.astype(np.float32)})
    assert r["parity"]["ok"] and r["parity"]["max_abs_diff_vs_oracle_fp32"] <= 1e-6
