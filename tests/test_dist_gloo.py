"""world_size-2 gloo tests of the sharding / all-gather / error-reduction logic
(CPU; the per-rank solver is the C oracle, used here only as the checker's
stand-in for the GPU solve)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, bad, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.robot.position_generator import random_dist
    from oracle import oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pts = random_dist(n, seed=11)
    for i, v in bad:
        pts[i] = v

    def solver(local):
        ang, it, _, st = O.fabrik_ikine(local)
        oob = O.check_limits(local)
        errs = np.nonzero(st)[0]
        e = int(errs[0]) if len(errs) else -1
        return torch.from_numpy(ang), oob, e, int(st[e]) if e >= 0 else 0

    out, oob, err, code = D.solve_sharded(torch.from_numpy(pts), solver, 4, torch.float64)
    q.put((rank, out.numpy(), oob, err, code))
    dist.barrier()
    dist.destroy_process_group()


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
    return sorted(res, key=lambda r: r[0])


def test_shard_bounds_cover():
    from inversekinematicsann_amd.dist import shard_bounds
    for n in (0, 1, 7, 1000, 1_000_001):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))


@pytest.mark.parametrize("n", [1001, 64])
def test_gather_matches_single_process(n):
    from inversekinematicsann_amd.robot.position_generator import random_dist
    from oracle import oracle as O
    res = _run(2, n)
    ref, _, _, _ = O.fabrik_ikine(random_dist(n, seed=11))
    for rank, out, oob, err, code in res:
        assert np.array_equal(out, ref)  # both ranks hold the whole batch
        assert oob == -1 and err == -1


def test_lowest_failing_index_across_shards():
    # an out-of-reach point on rank 1 and a ZeroDivision point on rank 0
    n = 100
    res = _run(2, n, bad=[(70, [1.0, 2.0, -4.0]), (10, [0.0, 0.0, 2.0]), (80, [0.0, 0.0, 2.0])])
    for _, _, oob, err, code in res:
        assert oob == 70
        assert err == 10 and code == 3
