"""The multi-GPU path on a real GPU: dist.solve_sharded over the nccl (RCCL)
backend with one rank, so the RCCL all_gather of the angle rows and the
first-failing-index all_reduce run on the device (the N > 1 bookkeeping is
covered by the world-size-2 gloo tests in test_dist_gloo.py; the 8-GPU run is
the driver's scaling bench)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                      WORLD_SIZE="1", LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    from inversekinematicsann_amd.robot.position_generator import random_dist
    try:
        D.init_from_env("nccl")
        ctx = _native.Context(0)
        pts = random_dist(5000, seed=3)
        pts[1234] = [0.0, 0.0, 2.0]  # ZeroDivisionError point (point.py:40)
        dpts = torch.from_numpy(pts).cuda()
        res = {}
        out, oob, err, code = D.solve_sharded(dpts, D.gpu_solver("fabrik", ctx), 4,
                                              torch.float64, device="cuda")
        ang, _, _, st = ctx.fabrik_solve(pts)
        res["fabrik"] = (out.cpu().numpy(), oob, err, code, ang, st.first_oob, st.first_err,
                         st.first_err_code)
        m = glorot_model(dims=(3, 64, 64, 4), seed=4)
        ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
        out, oob, err, code = D.solve_sharded(dpts, D.gpu_solver("ann", ctx), 4, torch.float32,
                                              device="cuda")
        ang, _, st = ctx.ann_solve(pts)
        res["ann"] = (out.cpu().numpy(), oob, err, code, ang, st.first_oob, st.first_err,
                      st.first_err_code)
        q.put(res)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put(repr(e))


def test_solve_sharded_over_rccl():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        res = q.get(timeout=100)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert not isinstance(res, str), res
    assert p.exitcode == 0
    for method, (out, oob, err, code, ang, r_oob, r_err, r_code) in res.items():
        assert np.array_equal(out, ang, equal_nan=True), method  # same bits as one context
        assert (oob, err, code) == (r_oob, r_err, r_code), method
    assert res["fabrik"][2] == 1234 and res["fabrik"][3] == 3  # IK_E_ZERODIV
