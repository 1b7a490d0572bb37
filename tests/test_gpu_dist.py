"""The multi-GPU path on a real GPU, through the library's own RCCL: one rank
(ik_comm_unique_id -> ik_comm_init(1, 0)), so the sharded solves run their
chunked in-place ncclAllGathers on the comm stream (with the ragged last chunk
through the stage), the per-chunk stats merge, the tail + histogram gather, and
must equal a single-context solve bit for bit (rows and stats), with device and
host outputs, and at configs[3] / configs[4]'s full 10M-point seed-1 batch.  No
torch.distributed: the C-ABI caller's view.  The N > 1
bookkeeping (the chunk plan, in-place placement, tail reduction, lowest global
failing index, histograms) is covered by the gloo tests in test_dist_gloo.py;
the 8-GPU run is the driver's scaling bench."""
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
        assert sc.info() == (1, 0, 0)
        pts = random_dist(5000, seed=3)
        pts[1234] = [0.0, 0.0, 2.0]  # ZeroDivisionError point (point.py:40)
        pts[2000] = [1.0, 2.0, -3.5]  # out of reach (inverse.py:26-35)
        pts[4100] = [1.0, 2.0, -3.5]  # ... again, in a later chunk
        res = {}
        r_ang, r_it, r_err, r_st = ctx.fabrik_solve_fk(pts, 1e-3, 100)
        dpts = torch.from_numpy(pts).cuda()
        m = glorot_model(dims=(3, 64, 64, 4), seed=4)
        ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
        a_ref, a_err, a_st = ctx.ann_solve(pts, want_fk_err=True)
        # 5000 rows in 1, 3 (ragged: 1667 + 1667 + 1666) and 8 (625 each) chunks
        for chunks in (1, 3, 8):
            sc.set_chunks(chunks)
            ang, it, err, st = sc.fabrik(pts, 1e-3, 100, want_fk_err=True)
            res[f"fabrik_host_c{chunks}"] = (ang, it, err, st.as_dict(), r_ang, r_it, r_err,
                                             r_st.as_dict(), sc.fk_err_quantile(0.99))
            assert sc.info()[2] == chunks
            dang = torch.empty((5000, 4), dtype=torch.float64, device="cuda")
            dit = torch.empty(5000, dtype=torch.int32, device="cuda")
            derr = torch.empty(5000, dtype=torch.float64, device="cuda")
            st = sc.fabrik_device(dpts, dang, dit, derr, 1e-3, 100)
            res[f"fabrik_dev_c{chunks}"] = (dang.cpu().numpy(), dit.cpu().numpy(),
                                            derr.cpu().numpy(), st.as_dict(), r_ang, r_it, r_err,
                                            r_st.as_dict(), sc.fk_err_quantile(0.99))
            ang, err, st = sc.ann(pts, want_fk_err=True)
            res[f"ann_host_c{chunks}"] = (ang, None, err, st.as_dict(), a_ref, None, a_err,
                                          a_st.as_dict(), sc.fk_err_quantile(0.99))
            fang = torch.empty((5000, 4), dtype=torch.float32, device="cuda")
            st = sc.ann_device(dpts, fang, derr)
            res[f"ann_dev_c{chunks}"] = (fang.cpu().numpy(), None, derr.cpu().numpy(),
                                         st.as_dict(), a_ref, None, a_err, a_st.as_dict(),
                                         sc.fk_err_quantile(0.99))
        # no FK error asked: no histogram, and the quantile says so
        sc.set_chunks(0)
        sc.fabrik(pts[:100], 1e-3, 100)
        try:
            sc.fk_err_quantile(0.5)
            res["no_hist"] = "quantile without fk_err did not raise"
        except _native.NativeError:
            pass
        # an empty batch: still one (tail) exchange, empty stats
        ang, it, err, st = sc.fabrik(pts[:0], 1e-3, 100)
        assert ang.shape == (0, 4) and st.first_oob == -1 and st.sum_iters == 0
        sc.close()
        q.put(res)
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        import traceback
        q.put(repr(e) + traceback.format_exc())


def _spawn(target, timeout=200):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=target, args=(q,))
    p.start()
    try:
        res = q.get(timeout=timeout)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert not isinstance(res, str), res
    assert p.exitcode == 0
    return res


def test_sharded_solves_over_library_rccl():
    from inversekinematicsann_amd import dist as D
    res = _spawn(_worker)
    assert "no_hist" not in res
    for name, (ang, it, err, st, r_ang, r_it, r_err, r_st, p99) in res.items():
        assert np.array_equal(ang, r_ang, equal_nan=True), name  # same bits as one context
        if it is not None:
            assert np.array_equal(it, r_it), name
        # one rank: every row is its own, so the local FK errors are the whole batch's
        assert np.array_equal(err, r_err, equal_nan=True), name
        for k in ("first_oob", "first_err", "first_err_code", "max_iters", "sum_iters",
                  "n_capped", "max_fk_err"):
            assert st[k] == r_st[k], (name, k, st[k], r_st[k])
        assert abs(st["sum_fk_err"] - r_st["sum_fk_err"]) <= 1e-9 * max(1.0, r_st["sum_fk_err"])
        assert st["gather_ms"] > 0.0, name  # the all-gathers ran, timed by HIP events
        assert st["first_oob"] == 2000
        # the gathered histogram's p99 = the numpy restatement's on the same errors
        assert p99 == D.hist_quantile([D.fkhist(r_err)], 0.99), (name, p99)
    assert res["fabrik_host_c3"][3]["first_err"] == 1234
    assert res["fabrik_host_c3"][3]["first_err_code"] == 3  # IK_E_ZERODIV


def _fullsize_worker(q):
    """configs[3] / configs[4]'s whole 10M-point seed-1 batch through the sharded
    solves at one rank (FABRIK in 4 chunks, set explicitly: one rank plans 1), against
    the plain solve, bit for bit."""
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    from inversekinematicsann_amd.robot.position_generator import random_dist
    try:
        n = 10_000_000
        ctx = _native.Context(0)
        sc = D.ShardedContext(ctx, 1, 0, D.exchange_unique_id(0, lambda uid: uid))
        dpts = torch.from_numpy(random_dist(n, seed=1)).cuda()
        out = {}
        # configs[4]: FABRIK tol 1e-5 / 200
        a1 = torch.empty((n, 4), dtype=torch.float64, device="cuda")
        i1 = torch.empty(n, dtype=torch.int32, device="cuda")
        e1 = torch.empty(n, dtype=torch.float64, device="cuda")
        s1 = ctx.fabrik_solve_device(dpts, a1, i1, None, 1e-5, 200, fk_err=e1)
        a2, i2, e2 = torch.empty_like(a1), torch.empty_like(i1), torch.empty_like(e1)
        sc.set_chunks(4)
        s2 = sc.fabrik_device(dpts, a2, i2, e2, 1e-5, 200)
        torch.cuda.synchronize()
        out["fabrik"] = (bool(torch.equal(a1.nan_to_num(7.0), a2.nan_to_num(7.0))),
                         bool(torch.equal(i1, i2)), bool(torch.equal(e1.nan_to_num(7.0),
                                                                     e2.nan_to_num(7.0))),
                         s1.as_dict(), s2.as_dict(), sc.info())
        del a1, i1, a2, i2
        # configs[3]: the ANN reference architecture, fp32, with the FK round trip
        m = glorot_model((3,) + (500,) * 12 + (4,), seed=0)
        ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
        f1 = torch.empty((n, 4), dtype=torch.float32, device="cuda")
        s1 = ctx.ann_solve_device(dpts, f1, e1)
        f2 = torch.empty_like(f1)
        sc.set_chunks(0)
        s2 = sc.ann_device(dpts, f2, e2)
        torch.cuda.synchronize()
        out["ann"] = (bool(torch.equal(f1, f2)), True,
                      bool(torch.equal(e1.nan_to_num(7.0), e2.nan_to_num(7.0))),
                      s1.as_dict(), s2.as_dict(), sc.info())
        sc.close()
        q.put(out)
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put(repr(e) + traceback.format_exc())


def test_sharded_full_size_10m_equals_plain_solve():
    res = _spawn(_fullsize_worker, timeout=300)
    for name, (same_ang, same_it, same_err, s1, s2, info) in res.items():
        assert same_ang and same_it and same_err, name
        for k in ("first_oob", "first_err", "max_iters", "sum_iters", "n_capped", "max_fk_err"):
            assert s1[k] == s2[k], (name, k)
        assert abs(s1["sum_fk_err"] - s2["sum_fk_err"]) <= 1e-9 * max(1.0, s1["sum_fk_err"])
        assert s2["gather_ms"] > 0
    assert res["fabrik"][5][2] == 4 and res["ann"][5][2] == 1
