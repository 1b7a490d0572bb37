"""world_size-2 (and 3) gloo tests of the sharded solve's gather protocol on the
CPU: the library's own shard split (ik_shard_range), block layout
(ik_gather_layout_of) and tail reduction (ik_tail_reduce), with every rank's
block built from its shard's solve and one all_gather of the blocks -- the
library's RCCL path with gloo as the transport.  The per-rank solver is the C
oracle (test infrastructure, the checker's stand-in for the GPU solve); the
gathered rows and the reduced stats must equal one single-process solve of the
whole batch bit for bit."""
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


def _shard_solve(local, lo, tol, mi):
    """One rank's shard through the oracle: the rows and the tail record the
    library's pack_tail_kernel would write (global indices)."""
    from inversekinematicsann_amd import _native
    from oracle import oracle as O
    ang, it, _, st = O.fabrik_ikine(local, tol, mi)
    xyz, _, fst = O.fk(np.nan_to_num(ang))
    err = np.sqrt(((xyz - local) ** 2).sum(axis=1))
    err[st != 0] = np.nan
    t = _native.ShardTail()
    oob = O.check_limits(local)
    t.first_oob = lo + oob if oob >= 0 else -1
    bad = np.nonzero(st)[0]
    t.first_err = lo + int(bad[0]) if len(bad) else -1
    t.first_err_code = int(st[bad[0]]) if len(bad) else 0
    t.max_iters = int(it.max()) if len(it) else 0
    t.sum_iters = int(it.sum())
    t.n_capped = int((it >= mi).sum())
    fin = err[np.isfinite(err)]
    t.max_fk_err = float(fin.max()) if len(fin) else 0.0
    t.sum_fk_err = float(fin.sum())
    t.rows = len(local)
    return ang, it, err, t


def _worker(rank, world, port, n, bad, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
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
        lo, hi = _native.shard_range(n, world, rank)
        assert (lo, hi) == D.shard_bounds(n, world, rank)
        L = _native.gather_layout(_native.IK_METHOD_FABRIK, n, world, True, True)
        ang, it, err, tail = _shard_solve(pts[lo:hi], lo, 1e-3, 100)
        blk = D.pack_block(L, [ang, it, err], tail)
        out = [torch.empty(L.block_bytes, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(out, torch.from_numpy(blk))  # the one collective
        blocks = np.stack([o.numpy() for o in out])
        (g_ang, g_it, g_err), tails = D.unpack_blocks(L, blocks, n,
                                                      [np.float64, np.int32, np.float64],
                                                      [4, 1, 1])
        st = _native.tail_reduce(tails)
        q.put((rank, g_ang, g_it[:, 0], g_err[:, 0], st.as_dict()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, repr(e)))


def _run(world, n, bad=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, list(bad), q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert len(r) == 5, r
    return sorted(res, key=lambda r: r[0])


def test_shard_bounds_match_library():
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.dist import shard_bounds
    for n in (0, 1, 7, 1000, 1_000_001, 10_000_000):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert b == [_native.shard_range(n, w, r) for r in range(w)]


def test_gather_layout():
    from inversekinematicsann_amd import _native
    L = _native.gather_layout(_native.IK_METHOD_FABRIK, 10, 3, True, True)
    assert L.shard == 4 and L.nregion == 3
    assert list(L.row_bytes) == [32, 4, 8]
    assert list(L.offset) == [0, 128, 192] and L.tail_offset == 256 and L.block_bytes == 320
    L = _native.gather_layout(_native.IK_METHOD_ANN, 1_000_000, 8)
    assert L.nregion == 1 and L.row_bytes[0] == 16 and L.block_bytes == 125_000 * 16 + 64


@pytest.mark.parametrize("world,n", [(2, 1001), (2, 64), (3, 1000), (2, 1), (3, 2)])
def test_gather_matches_single_process(world, n):
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(n, seed=11)
    ref_ang, ref_it, ref_err, ref_t = _shard_solve(pts, 0, 1e-3, 100)
    for rank, ang, it, err, st in _run(world, n):
        # every rank holds the whole batch, bit for bit
        assert np.array_equal(ang, ref_ang) and np.array_equal(it, ref_it)
        assert np.array_equal(err, ref_err, equal_nan=True)
        assert st["first_oob"] == -1 and st["first_err"] == -1
        assert st["sum_iters"] == ref_t.sum_iters and st["max_iters"] == ref_t.max_iters
        assert st["n_capped"] == ref_t.n_capped
        assert st["max_fk_err"] == ref_t.max_fk_err
        # per-rank partial sums in rank order vs one sum: equal up to rounding
        assert abs(st["sum_fk_err"] - ref_t.sum_fk_err) <= 1e-12 * max(1.0, ref_t.sum_fk_err)


def test_lowest_failing_index_across_shards():
    # an out-of-reach point on rank 1 and ZeroDivision points on both ranks: the
    # reduced stats carry the lowest GLOBAL index of each (inverse.py:117, point.py:40)
    n = 100
    res = _run(2, n, bad=[(70, [1.0, 2.0, -4.0]), (10, [0.0, 0.0, 2.0]), (80, [0.0, 0.0, 2.0])])
    for _, ang, _, err, st in res:
        assert st["first_oob"] == 70
        assert st["first_err"] == 10 and st["first_err_code"] == 3
        assert np.isnan(ang[10]).all() and np.isnan(err[80])


def test_unpack_rank_formula():
    """The device unpack kernel (ik_shard.hip gather_unpack_kernel) finds row i's
    rank as ceil((i + 1) g / n) - 1 and its local row as i - floor(r n / g): the
    same split as ik_shard_range for every row."""
    from inversekinematicsann_amd.dist import shard_bounds
    for n in (1, 2, 7, 64, 1000, 1001, 99_991):
        for g in (1, 2, 3, 5, 8):
            i = np.arange(n, dtype=np.int64)
            r = ((i + 1) * g + n - 1) // n - 1
            local = i - (n * r) // g
            lo = np.array([shard_bounds(n, g, k)[0] for k in range(g)])
            hi = np.array([shard_bounds(n, g, k)[1] for k in range(g)])
            assert ((lo[r] <= i) & (i < hi[r])).all() and (local == i - lo[r]).all()
