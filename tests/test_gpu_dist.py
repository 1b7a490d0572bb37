"""The multi-GPU path on a real GPU, through the library's own RCCL: one rank
(ik_comm_unique_id -> ik_comm_init(1, 0)), so the sharded solves run their
chunked in-place ncclAllGathers on the comm stream (with the ragged last chunk
through the stage), the per-chunk stats merge, the tail + histogram gather, and
must equal a single-context solve bit for bit (rows and stats), with device and
host outputs, and at configs[3] / configs[4]'s full 10M-point seed-1 batch.  No
torch.distributed: the C-ABI caller's view.  The N > 1
bookkeeping (the chunk plan, in-place placement, tail reduction, lowest global
failing index, histograms) is covered by the gloo tests in test_dist_gloo.py;
the 8-GPU run is the driver's scaling bench.  The device side of g > 1 (part
placement, the ragged chunk's stage, the tail reduction) runs on one GPU through
the test-only loopback communicator (ik_comm_init_loopback)."""
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


def _loopback_worker(q):
    """One GPU as rank r of g = 2, 3 (ik_comm_init_loopback: no RCCL): the device
    code of the N > 1 path -- every part placed at its plan rows, the ragged
    chunk's stage copied out truncated at n, empty parts (n < g), the tails
    reduced -- against a single-context solve and the loopback byte pattern."""
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    from inversekinematicsann_amd.robot.position_generator import random_dist
    try:
        ctx = _native.Context(0)
        pts = random_dist(5000, seed=5)
        pts[3400] = [1.0, 2.0, -3.5]  # out of reach, in rank 1's or 2's rows
        pts[4990] = [0.0, 0.0, 2.0]   # ZeroDivisionError, in the ragged chunk
        m = glorot_model(dims=(3, 64, 64, 4), seed=4)
        ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
        out = []
        for n, cases in ((5000, ((2, 1), (2, 3), (3, 3), (3, 8))), (2, ((3, 1),)),
                         (0, ((2, 1),))):
            p = pts[:n]
            f_ang, f_it, f_err, f_st = ctx.fabrik_solve_fk(p, 1e-3, 100)
            a_ang, a_err, a_st = ctx.ann_solve(p, want_fk_err=True)
            dpts = torch.from_numpy(p).cuda()
            for g, chunks in cases:
                per_rank = []
                for r in range(g):
                    sc = D.ShardedContext.loopback(ctx, g, r)
                    sc.set_chunks(chunks)
                    own = np.zeros(n, bool)
                    C, _, _ = D.plan_of(n, g, chunks)
                    for c in range(C):
                        b, e = D.part_bounds(n, g, chunks, r, c)
                        own[b:e] = True
                    ang, it, err, st = sc.fabrik(p, 1e-3, 100, want_fk_err=True)
                    ok = {
                        "fab_ang": np.array_equal(ang.view(np.uint8).reshape(n, 32), D.loopback_expected(
                            n, g, r, chunks, 32, f_ang)),
                        "fab_it": np.array_equal(it.view(np.uint8).reshape(n, 4), D.loopback_expected(
                            n, g, r, chunks, 4, f_it)),
                        "fab_err_own": np.array_equal(err[own], f_err[own], equal_nan=True),
                        "info": sc.info() == (g, r, chunks)}
                    if n and own.any():
                        ok["p99"] = sc.fk_err_quantile(0.99) == D.hist_quantile(
                            [D.fkhist(f_err[own])], 0.99)
                    fst = st.as_dict()
                    dang = torch.full((n, 4), 7.0, dtype=torch.float64, device="cuda")
                    dit = torch.full((n,), -9, dtype=torch.int32, device="cuda")
                    derr = torch.full((n,), -1.0, dtype=torch.float64, device="cuda")
                    dst = sc.fabrik_device(dpts, dang, dit, derr, 1e-3, 100).as_dict()
                    ok["fab_dev_ang"] = np.array_equal(
                        dang.cpu().numpy().view(np.uint8).reshape(n, 32),
                        D.loopback_expected(n, g, r, chunks, 32, f_ang))
                    ok["fab_dev_it"] = np.array_equal(
                        dit.cpu().numpy().view(np.uint8).reshape(n, 4),
                        D.loopback_expected(n, g, r, chunks, 4, f_it))
                    e_dev = derr.cpu().numpy()
                    ok["fab_dev_err"] = (np.array_equal(e_dev[own], f_err[own], equal_nan=True)
                                         and bool((e_dev[~own] == -1.0).all()))
                    # (the FK-error sum is a float reduction in no fixed order)
                    exact = [k for k in fst if k not in ("gather_ms", "sum_fk_err")]
                    ok["fab_dev_stats"] = ({k: dst[k] for k in exact} == {k: fst[k] for k in exact}
                                           and abs(dst["sum_fk_err"] - fst["sum_fk_err"])
                                           <= 1e-9 * max(1.0, fst["sum_fk_err"]))
                    aang, aerr, ast = sc.ann(p, want_fk_err=True)
                    ok["ann_ang"] = np.array_equal(aang.view(np.uint8).reshape(n, 16),
                                                   D.loopback_expected(n, g, r, chunks, 16, a_ang))
                    ok["ann_err_own"] = np.array_equal(aerr[own], a_err[own], equal_nan=True)
                    fang = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
                    sc.ann_device(dpts, fang, derr)
                    ok["ann_dev_ang"] = np.array_equal(
                        fang.cpu().numpy().view(np.uint8).reshape(n, 16),
                        D.loopback_expected(n, g, r, chunks, 16, a_ang))
                    per_rank.append((ok, fst, ast.as_dict()))
                    sc.close()
                out.append(((n, g, chunks), per_rank, f_st.as_dict(), a_st.as_dict()))
        q.put(out)
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put(repr(e) + traceback.format_exc())


def test_sharded_placement_at_2_and_3_ranks_loopback():
    """the sharded path's device code at g > 1 on one GPU.  Per rank:
    the whole gathered array equals its own rows of a plain solve plus the
    loopback pattern in every other rank's rows (host and device outputs, FABRIK
    32 + 4 B rows, ANN 16 B), FK errors written for its own rows only, the quantile
    from its own histogram; over the g ranks (each tail copied g times by the
    loopback), the stats add up to the plain solve's: lowest global failing
    indices, iteration sums, FK-error max and sum."""
    res = _spawn(_loopback_worker, timeout=300)
    for (n, g, chunks), per_rank, f_st, a_st in res:
        for r, (ok, fst, ast) in enumerate(per_rank):
            bad = [k for k, v in ok.items() if not v]
            assert not bad, ((n, g, chunks, r), bad)
        for st, ref in (([x[1] for x in per_rank], f_st), ([x[2] for x in per_rank], a_st)):
            for k in ("first_oob", "first_err"):
                got = [s[k] for s in st if s[k] >= 0]
                assert (min(got) if got else -1) == ref[k], ((n, g, chunks), k)
            for k in ("sum_iters", "n_capped"):
                assert sum(s[k] for s in st) == g * ref[k], ((n, g, chunks), k)
            assert max(s["max_iters"] for s in st) == ref["max_iters"]
            assert max(s["max_fk_err"] for s in st) == ref["max_fk_err"]
            tot = sum(s["sum_fk_err"] for s in st) / g
            assert abs(tot - ref["sum_fk_err"]) <= 1e-9 * max(1.0, ref["sum_fk_err"])
        if n == 5000:
            assert f_st["first_oob"] == 3400 and f_st["first_err"] == 4990


def _stall_worker(q):
    """the deadline path, driven on one GPU.  A loopback
    communicator whose all-gathers wait for a peer that never comes
    (ik_comm_loopback_stall): the synchronous sharded call returns IK_E_RCCL
    naming the rank and the wait within the deadline, the abort releases the
    stalled gather so the GPU drains, the communicator refuses later calls, and
    after ik_comm_destroy + a new communicator the same context solves again
    (bit-exact against a plain solve).  The same for an IK_F_ASYNC call ended by
    ik_ctx_sync."""
    import time
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.robot.position_generator import random_dist
    try:
        out = {}
        ctx = _native.Context(0)
        pts = random_dist(4000, seed=9)
        r_ang, r_it, _, _ = ctx.fabrik_solve(pts, 1e-3, 100)
        for mode in ("sync", "async"):
            sc = D.ShardedContext.loopback(ctx, 2, 0)
            ctx.comm_set_timeout(2.0)
            ctx.comm_loopback_stall(True)
            t0 = time.perf_counter()
            try:
                if mode == "sync":
                    sc.fabrik(pts, 1e-3, 100)
                else:
                    dpts = torch.from_numpy(pts).cuda()
                    dang = torch.empty((4000, 4), dtype=torch.float64, device="cuda")
                    sc.fabrik_device(dpts, dang, None, None, 1e-3, 100,
                                     flags=_native.IK_F_DEVICE | _native.IK_F_ASYNC)
                    ctx.sync()
                out[mode] = ("no error", 0.0, "")
            except _native.NativeError as e:
                out[mode] = (e.code, time.perf_counter() - t0, str(e))
            torch.cuda.synchronize()  # the abort released the stalled gather
            try:
                sc.fabrik(pts[:10], 1e-3, 100)
                out[mode + "_refused"] = False
            except _native.NativeError as e:
                out[mode + "_refused"] = e.code == _native.IK_E_RCCL and "aborted" in str(e)
            sc.close()
            # a new communicator on the same context works again
            sc = D.ShardedContext.loopback(ctx, 1, 0)
            ang, it, _, _ = sc.fabrik(pts, 1e-3, 100)
            out[mode + "_after"] = bool(np.array_equal(ang, r_ang) and np.array_equal(it, r_it))
            sc.close()
        q.put(out)
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put(repr(e) + traceback.format_exc())


def test_stalled_gather_times_out_with_rccl_error():
    from inversekinematicsann_amd import _native
    res = _spawn(_stall_worker, timeout=120)
    for mode in ("sync", "async"):
        code, secs, msg = res[mode]
        assert code == _native.IK_E_RCCL, (mode, res[mode])
        assert 1.9 <= secs <= 15.0, (mode, secs)
        assert "rank 0 of 2" in msg and "did not complete within 2 s" in msg, msg
        assert res[mode + "_refused"] and res[mode + "_after"], (mode, res)
