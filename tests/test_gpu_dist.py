"""The multi-GPU path on a real GPU, through the library's own RCCL: one rank
(ik_comm_unique_id -> ik_comm_init(1, 0)), so the sharded solves run their
pack-tail kernel, the ncclAllGather over the communicator and the unpack, and
must equal a single-context solve bit for bit (rows and stats), with device and
host outputs.  No torch.distributed: the C-ABI caller's view.
The N > 1 bookkeeping (shard split, block layout, tail reduction, lowest global
failing index) is covered by the gloo tests in test_dist_gloo.py; the 8-GPU run
is the driver's scaling bench."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _worker(q):
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    from inversekinematicsann_amd.robot.position_generator import random_dist
    try:
        ctx = _native.Context(0)
        sc = D.ShardedContext(ctx, 1, 0, D.exchange_unique_id(0, lambda uid: uid))
        pts = random_dist(5000, seed=3)
        pts[1234] = [0.0, 0.0, 2.0]  # ZeroDivisionError point (point.py:40)
        pts[2000] = [1.0, 2.0, -3.5]  # out of reach (inverse.py:26-35)
        res = {}
        # FABRIK: host arrays, then device tensors
        ang, it, err, st = sc.fabrik(pts, 1e-3, 100, want_fk_err=True)
        r_ang, r_it, r_err, r_st = ctx.fabrik_solve_fk(pts, 1e-3, 100)
        res["fabrik_host"] = (ang, it, err, st.as_dict(), r_ang, r_it, r_err, r_st.as_dict())
        dpts = torch.from_numpy(pts).cuda()
        dang = torch.empty((5000, 4), dtype=torch.float64, device="cuda")
        dit = torch.empty(5000, dtype=torch.int32, device="cuda")
        derr = torch.empty(5000, dtype=torch.float64, device="cuda")
        st = sc.fabrik_device(dpts, dang, dit, derr, 1e-3, 100)
        res["fabrik_dev"] = (dang.cpu().numpy(), dit.cpu().numpy(), derr.cpu().numpy(),
                             st.as_dict(), r_ang, r_it, r_err, r_st.as_dict())
        # ANN
        m = glorot_model(dims=(3, 64, 64, 4), seed=4)
        ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
        a_ang, a_err, st = sc.ann(pts, want_fk_err=True)
        r_ang, r_err, r_st = ctx.ann_solve(pts, want_fk_err=True)
        res["ann_host"] = (a_ang, None, a_err, st.as_dict(), r_ang, None, r_err, r_st.as_dict())
        fang = torch.empty((5000, 4), dtype=torch.float32, device="cuda")
        st = sc.ann_device(dpts, fang, derr)
        res["ann_dev"] = (fang.cpu().numpy(), None, derr.cpu().numpy(), st.as_dict(), r_ang,
                          None, r_err, r_st.as_dict())
        sc.close()
        q.put(res)
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put(repr(e))


def test_sharded_solves_over_library_rccl():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(q,))
    p.start()
    try:
        res = q.get(timeout=100)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert not isinstance(res, str), res
    assert p.exitcode == 0
    for name, (ang, it, err, st, r_ang, r_it, r_err, r_st) in res.items():
        assert np.array_equal(ang, r_ang, equal_nan=True), name  # same bits as one context
        if it is not None:
            assert np.array_equal(it, r_it), name
        assert np.array_equal(err, r_err, equal_nan=True), name
        for k in ("first_oob", "first_err", "first_err_code", "max_iters", "sum_iters",
                  "n_capped", "max_fk_err"):
            assert st[k] == r_st[k], (name, k, st[k], r_st[k])
        assert abs(st["sum_fk_err"] - r_st["sum_fk_err"]) <= 1e-9 * max(1.0, r_st["sum_fk_err"])
        assert st["gather_ms"] > 0.0, name  # the all-gather ran, timed by HIP events
        assert st["first_oob"] == 2000
    assert res["fabrik_host"][3]["first_err"] == 1234
    assert res["fabrik_host"][3]["first_err_code"] == 3  # IK_E_ZERODIV
