"""world_size-2 (and 3) gloo tests of the sharded solve's protocol on the CPU:
the library's own split in chunks (ik_shard_plan_of / ik_shard_part), its
in-place chunk all-gathers with the ragged last chunk staged (dist.gather_in_place,
the host mirror of ik_shard.hip's sharded_run), the tail reduction
(ik_tail_reduce) and the FK-error histograms (ik_fkhist_bin, quantiles), with
gloo as the transport.  The per-rank solver is the C oracle (test
infrastructure, the checker's stand-in for the GPU solve); the gathered rows and
the reduced stats must equal one single-process solve of the whole batch bit for
bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _part_solve(pts, b, e, tol, mi):
    """Rows [b, e) through the oracle: angles, iterations, FK errors, and the
    stats the library's pack_tail_kernel would record (global indices)."""
    from oracle import oracle as O
    local = pts[b:e]
    ang, it, _, st = O.fabrik_ikine(local, tol, mi)
    xyz, _, _ = O.fk(np.nan_to_num(ang))
    err = np.sqrt(((xyz - local) ** 2).sum(axis=1))
    err[st != 0] = np.nan
    oob = O.check_limits(local)
    bad = np.nonzero(st)[0]
    fin = err[np.isfinite(err)]
    stats = dict(first_oob=b + oob if oob >= 0 else -1,
                 first_err=b + int(bad[0]) if len(bad) else -1,
                 first_err_code=int(st[bad[0]]) if len(bad) else 0,
                 max_iters=int(it.max()) if len(it) else 0, sum_iters=int(it.sum()),
                 n_capped=int((it >= mi).sum()),
                 max_fk_err=float(fin.max()) if len(fin) else 0.0, sum_fk_err=float(fin.sum()),
                 rows=len(local))
    return ang, it, err, stats


ANN_DIMS_SMALL = (3, 48, 48, 4)  # a small tanh MLP: the protocol, not the model, is tested


def _ann_part_solve(pts, b, e):
    """Rows [b, e) through the ANN oracle (ann.py:70-76 on a seeded Glorot model):
    float32 angles, FK errors, and the stats pack_tail_kernel would record."""
    from oracle import oracle as O
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    m = glorot_model(ANN_DIMS_SMALL, seed=4)
    local = pts[b:e]
    ang = O.ann_forward(local, m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean,
                        YS.scale, compute=np.float32).astype(np.float32)
    xyz, _, _ = O.fk(ang.astype(np.float64))
    err = np.sqrt(((xyz - local) ** 2).sum(axis=1))
    oob = O.check_limits(local) if len(local) else -1
    stats = dict(first_oob=b + oob if oob >= 0 else -1, first_err=-1, first_err_code=0,
                 max_iters=0, sum_iters=0, n_capped=0,
                 max_fk_err=float(err.max()) if len(err) else 0.0, sum_fk_err=float(err.sum()),
                 rows=len(local))
    return ang, err, stats


def _tail(parts_stats):
    """The rank's tail from its parts' stats in chunk order (pack_tail_kernel)."""
    from inversekinematicsann_amd import _native
    t = _native.ShardTail()
    t.first_oob = t.first_err = -1
    for s in parts_stats:
        if t.first_oob < 0 and s["first_oob"] >= 0:
            t.first_oob = s["first_oob"]
        if t.first_err < 0 and s["first_err"] >= 0:
            t.first_err, t.first_err_code = s["first_err"], s["first_err_code"]
        t.max_iters = max(t.max_iters, s["max_iters"])
        t.sum_iters += s["sum_iters"]
        t.n_capped += s["n_capped"]
        t.max_fk_err = max(t.max_fk_err, s["max_fk_err"])
        t.sum_fk_err += s["sum_fk_err"]
        t.rows += s["rows"]
    return t


def _worker(rank, world, port, n, chunks, bad, q, method="fabrik"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import ctypes
    import torch
    import torch.distributed as dist
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.robot.position_generator import random_dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pts = random_dist(n, seed=11)
        for i, v in bad:
            pts[i] = v
        plan = _native.shard_plan(n, world, chunks)
        assert (plan.chunks, plan.part_rows, plan.full_rows) == D.plan_of(n, world, chunks)
        ang = np.full((n, 4), -7.0, np.float32 if method == "ann" else np.float64)
        it = np.full(n, -7, np.int32)
        err = np.full(n, -7.0)  # only this rank's rows are written (stays local)
        stats = []

        def solve_part(b, e):
            assert (b, e) == _native.shard_part(plan, rank, len(stats))
            if method == "ann":  # ik_ann_solve_sharded gathers the angles only
                a, f, s = _ann_part_solve(pts, b, e)
                err[b:e] = f
                stats.append(s)
                return [a]
            a, i, f, s = _part_solve(pts, b, e, 1e-3, 100)
            err[b:e] = f
            stats.append(s)
            return [a, i]

        def all_gather(send, recv):  # ncclAllGather in place: recv = g x len(send)
            out = list(torch.from_numpy(np.ascontiguousarray(recv)).chunk(world))
            dist.all_gather(out, torch.from_numpy(np.ascontiguousarray(send)))
            recv[...] = torch.cat(out).numpy()

        outs = [ang] if method == "ann" else [ang, it]
        parts = D.gather_in_place(n, world, rank, chunks, solve_part, outs, all_gather)
        assert len(parts) == plan.chunks
        while len(stats) < len(parts):  # empty parts record zero stats
            stats.append(dict(first_oob=-1, first_err=-1, first_err_code=0, max_iters=0,
                              sum_iters=0, n_capped=0, max_fk_err=0.0, sum_fk_err=0.0, rows=0))
        # the tail block (stats record + histogram), one all-gather with the last chunk
        tb = np.concatenate([np.frombuffer(bytes(_tail(stats)), np.uint8),
                             D.fkhist(err[[i for b, e in parts for i in range(b, e)]])
                             .view(np.uint8)])
        blocks = [torch.empty(tb.size, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(blocks, torch.from_numpy(tb))
        tails, hists = [], []
        for blk in blocks:
            raw = blk.numpy()
            t = _native.ShardTail()
            ctypes.memmove(ctypes.addressof(t), raw[:64].ctypes.data, 64)
            tails.append(t)
            hists.append(raw[64:].view(np.uint32))
        st = _native.tail_reduce(tails)
        q.put((rank, ang, it, err, st.as_dict(), D.hist_quantile(hists, 0.99), parts))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


def _run(world, n, chunks=1, bad=(), method="fabrik"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, chunks, list(bad), q, method))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert len(r) == 7, r
    return sorted(res, key=lambda r: r[0])


def test_plan_matches_library_and_covers_batch():
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    for n in (0, 1, 2, 7, 64, 1000, 1001, 99_991, 1_000_000, 10_000_000):
        for w in (1, 2, 3, 5, 8):
            for c in (1, 2, 3, 4, 8):
                p = _native.shard_plan(n, w, c)
                assert (p.n, p.nranks) == (n, w)
                assert (p.chunks, p.part_rows, p.full_rows) == D.plan_of(n, w, c)
                assert p.chunks <= c
                rows = np.zeros(n, np.int32)
                for k in range(p.chunks):
                    cb = k * w * p.part_rows
                    for r in range(w):
                        b, e = _native.shard_part(p, r, k)
                        assert (b, e) == D.part_bounds(n, w, c, r, k)
                        # in-place layout: the part sits at rank offset r S of its chunk
                        assert b == min(cb + r * p.part_rows, n) and e - b <= p.part_rows
                        rows[b:e] += 1
                    # only the last chunk may be ragged (staged)
                    assert (cb + w * p.part_rows <= n) == (k < p.chunks - 1 or p.full_rows == n)
                assert (rows == 1).all()
                assert p.full_rows == n or p.full_rows == (p.chunks - 1) * w * p.part_rows
                # one chunk: ik_shard_range
                if c == 1:
                    for r in range(w):
                        assert _native.shard_range(n, w, r) == D.shard_bounds(n, w, r) == \
                            _native.shard_part(p, r, 0)


def test_fkhist_bins_match_library():
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    rng = np.random.default_rng(0)
    vals = np.concatenate([
        [0.0, -0.0, 5e-324, 2.0 ** -64, 2.0 ** -65, 1.0, 1.0625, 1.0624999, 2.0 ** 63,
         2.0 ** 64, 1e300, np.inf, -1.0, np.nan],
        10.0 ** rng.uniform(-20, 3, 2000)])
    for v in vals:
        b = _native.fkhist_bin(v)
        h = D.fkhist(np.array([v]))
        if b < 0:
            assert h.sum() == 0, v
        else:
            assert h[b] == 1 and h.sum() == 1, v
            # monotonic bins: v lies below the bin's upper edge
            assert v < _native.fkhist_upper(b) or b == _native.IK_FKHIST_BINS - 1
            if b > 0:
                assert v >= _native.fkhist_upper(b - 1)
    # quantile: an upper bound within 1/16 octave of the exact order statistic
    e = 10.0 ** rng.uniform(-12, 1, 100_000)
    for q in (0.5, 0.9, 0.99, 1.0):
        exact = np.sort(e)[int(np.ceil(q * e.size)) - 1]
        got = D.hist_quantile([D.fkhist(e[:40_000]), D.fkhist(e[40_000:])], q)
        assert exact <= got <= exact * 2 ** (1 / 16) * (1 + 1e-12), (q, exact, got)


@pytest.mark.parametrize("world,n,chunks", [(2, 1001, 1), (2, 64, 1), (3, 1000, 1), (2, 1, 1),
                                            (3, 2, 1), (2, 1001, 4), (3, 1000, 3), (2, 12, 4)])
def test_gather_matches_single_process(world, n, chunks):
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(n, seed=11)
    ref_ang, ref_it, ref_err, ref_t = _part_solve(pts, 0, n, 1e-3, 100)
    seen = np.zeros(n, np.int32)
    for rank, ang, it, err, st, p99, parts in _run(world, n, chunks):
        # every rank holds the whole batch's gathered rows, bit for bit
        assert np.array_equal(ang, ref_ang) and np.array_equal(it, ref_it)
        # FK errors: only this rank's own rows, equal to the one-process ones
        mine = np.zeros(n, bool)
        for b, e in parts:
            mine[b:e] = True
            seen[b:e] += 1
        assert np.array_equal(err[mine], ref_err[mine], equal_nan=True)
        assert (err[~mine] == -7.0).all()
        assert st["first_oob"] == -1 and st["first_err"] == -1
        assert st["sum_iters"] == ref_t["sum_iters"] and st["max_iters"] == ref_t["max_iters"]
        assert st["n_capped"] == ref_t["n_capped"]
        assert st["max_fk_err"] == ref_t["max_fk_err"]
        # per-rank partial sums in rank order vs one sum: equal up to rounding
        assert abs(st["sum_fk_err"] - ref_t["sum_fk_err"]) <= 1e-12 * max(1.0, ref_t["sum_fk_err"])
        assert p99 == D.hist_quantile([D.fkhist(ref_err)], 0.99)
    assert (seen == 1).all()  # the ranks' parts cover the batch once


def test_lowest_failing_index_across_shards():
    # an out-of-reach point on rank 1 and ZeroDivision points on both ranks: the
    # reduced stats carry the lowest GLOBAL index of each (inverse.py:117, point.py:40)
    n = 100
    for chunks in (1, 3):
        res = _run(2, n, chunks,
                   bad=[(70, [1.0, 2.0, -4.0]), (10, [0.0, 0.0, 2.0]), (80, [0.0, 0.0, 2.0])])
        for _, ang, _, err, st, _, _ in res:
            assert st["first_oob"] == 70
            assert st["first_err"] == 10 and st["first_err_code"] == 3
            assert np.isnan(ang[10]).all() and np.isnan(ang[80]).all()


# ---- world 8: the driver's N = 8 run, rehearsed on the CPU ----

def test_world8_fabrik_two_chunks_ragged():
    """8 ranks, FABRIK, C = 2 chunks (the opt-in overlap; ik_comm_set_chunks) on a
    ragged n = 10 007: S = 626, chunk 0 in place, chunk 1 staged (its last part
    ragged, one rank's part empty); every rank ends with the single-process rows
    bit for bit, the stats of the whole batch, and its own FK errors only."""
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.robot.position_generator import random_dist
    n, world, chunks = 10_007, 8, 2
    C, S, full = D.plan_of(n, world, chunks)
    assert (C, S) == (2, 626) and full < n  # a staged, ragged last chunk
    pts = random_dist(n, seed=11)
    ref_ang, ref_it, ref_err, ref_t = _part_solve(pts, 0, n, 1e-3, 100)
    seen = np.zeros(n, np.int32)
    res = _run(world, n, chunks)
    assert [r[0] for r in res] == list(range(world))
    for rank, ang, it, err, st, p99, parts in res:
        assert np.array_equal(ang, ref_ang) and np.array_equal(it, ref_it), rank
        assert len(parts) == C
        mine = np.zeros(n, bool)
        for b, e in parts:
            mine[b:e] = True
            seen[b:e] += 1
        assert np.array_equal(err[mine], ref_err[mine], equal_nan=True)
        assert (err[~mine] == -7.0).all()
        assert st["sum_iters"] == ref_t["sum_iters"] and st["max_iters"] == ref_t["max_iters"]
        assert st["n_capped"] == ref_t["n_capped"]
        assert st["max_fk_err"] == ref_t["max_fk_err"]
        assert p99 == D.hist_quantile([D.fkhist(ref_err)], 0.99)
    assert (seen == 1).all()


def test_world8_ann_one_chunk():
    """8 ranks, ANN, C = 1 (the automatic plan): float32 angle rows (16 B) gathered
    in place; every rank holds what one process computes for the same eight parts
    bit for bit (the oracle's BLAS forward is row-invariant only for equal batch
    shapes, so the reference solves the same parts)."""
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.robot.position_generator import random_dist
    n, world = 10_007, 8
    pts = random_dist(n, seed=11)
    ref_ang = np.empty((n, 4), np.float32)
    ref_err = np.empty(n)
    mx = 0.0
    for r in range(world):
        b, e = D.shard_bounds(n, world, r)
        ref_ang[b:e], ref_err[b:e], t = _ann_part_solve(pts, b, e)
        mx = max(mx, t["max_fk_err"])
    res = _run(world, n, 1, method="ann")
    for rank, ang, it, err, st, p99, parts in res:
        assert ang.dtype == np.float32 and np.array_equal(ang, ref_ang), rank
        assert len(parts) == 1 and parts[0] == D.shard_bounds(n, world, rank)
        b, e = parts[0]
        assert np.array_equal(err[b:e], ref_err[b:e])
        assert st["first_oob"] == -1 and st["max_fk_err"] == mx
        assert p99 == D.hist_quantile([D.fkhist(ref_err)], 0.99)


def test_world8_lowest_failing_index():
    """8 ranks: out-of-reach points on ranks 5 and 2 and ZeroDivision points on
    ranks 7, 3 and 6 (n = 8 000, S = 1 000 at C = 1; 500 at C = 2): every rank
    reports the lowest GLOBAL index of each kind (inverse.py:117 checks the whole
    batch first; the reference then fails at the first bad point, point.py:40)."""
    n = 8000
    bad = [(5300, [1.0, 2.0, -4.0]), (2950, [7.0, 0.0, 1.0]),      # out of reach
           (7100, [0.0, 0.0, 2.0]), (3001, [0.0, 0.0, 2.0]), (6999, [0.0, 0.0, 2.0])]
    for chunks in (1, 2):
        for _, ang, _, err, st, _, _ in _run(8, n, chunks, bad=bad):
            assert st["first_oob"] == 2950
            assert st["first_err"] == 3001 and st["first_err_code"] == 3
            assert np.isnan(ang[3001]).all() and np.isnan(ang[7100]).all()


def _fallback_worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        closed = []

        class FakeSharded:
            def __init__(self, ctx, w, r, uid):
                if case == "init_fails_on_1" and r == 1:
                    raise RuntimeError("IK_E_RCCL: ncclCommInitRankConfig timed out")
                self.uid = uid

            def close(self):
                closed.append(True)

        def uid():
            if case == "no_rccl":
                raise OSError("librccl.so: cannot open shared object file")
            return b"\x01" * 128

        sc, why = bench.open_sharded(None, world, rank, sharded=FakeSharded, unique_id=uid)
        q.put((rank, sc is not None, why, bool(closed), getattr(sc, "uid", None)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "error", repr(e), False, None))


@pytest.mark.parametrize("case", ["ok", "no_rccl", "init_fails_on_1"])
def test_bench_rccl_fallback_agreed_by_every_rank(case):
    """SURVEY §8(e)'s host-only fallback: when RCCL is missing on rank 0 or its init
    fails on one rank, bench.open_sharded gives every rank no communicator (the ranks
    agree over gloo; a rank whose own init succeeded closes it) and the reason, so
    the N > 1 line runs with no collective instead of dying; with RCCL working every
    rank gets the communicator built from rank 0's broadcast id."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fallback_worker, args=(r, world, port, case, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    assert all(r[1] != "error" for r in res), res
    if case == "ok":
        assert all(r[1] is True and r[2] is None and r[4] == b"\x01" * 128 for r in res)
    else:
        assert all(r[1] is False and r[2] for r in res), res
        if case == "no_rccl":
            assert all("librccl" in r[2] or "unique id" in r[2] for r in res)
        else:
            assert res[0][3] is True  # rank 0's own communicator was closed
            assert "timed out" in res[1][2] and "another rank" in res[0][2]
