"""bench.py's N > 1 runners on one GPU, in their real order:
run_ann / run_fabrik / the strong legs through a real RCCL ShardedContext of one
rank (ik_comm_init(1, 0)) -- the timed sharded steps, the stats and the p99 from
the gathered histograms, then the gather check's plain re-solves -- so that a
plain call slipped in before the sharded-only queries fails here, not on the
driver's 8-GPU node.  Also the automatic chunk plan at g > 1 (loopback)."""
import math

import pytest

pytestmark = pytest.mark.gpu


def _bench_worker(q):
    try:
        import torch
        import bench
        from inversekinematicsann_amd import _native
        from inversekinematicsann_amd import dist as D
        from inversekinematicsann_amd.robot.position_generator import random_dist
        ctx = _native.Context(0)
        stream = torch.cuda.Stream()
        torch.cuda.set_stream(stream)
        ctx.set_stream(stream.cuda_stream)
        sc = D.ShardedContext(ctx, 1, 0, D.exchange_unique_id(0, lambda uid: uid))
        n = 20_000
        pts = random_dist(n, seed=0)
        job = bench.Job(ctx, sc, pts, torch.from_numpy(pts).cuda(), 0, n, 1)
        args = bench.parse(["--steps", "2", "--warmup", "1", "--end-to-end", "0",
                            "--cpu-seconds", "0"])
        out = {}
        r = bench.run_ann(job, args)
        out["ann"] = (r["gather_check"], r["p99_fk_err"], r["max_fk_err"], r["gather_chunks"])
        r = bench.run_fabrik(job, args)  # with the cold legs (default --cold 1)
        out["fabrik"] = (r["gather_check"], r["p99_fk_err"], r["mean_iters"],
                         r["gather_chunks"], r["roofline"]["iterations_per_launch"],
                         r.get("gathered_bytes_per_row"), "cold" in r)
        # the strong legs' machinery on a small batch
        sjob = bench.strong_job(ctx, sc, 1, 0, 30_000)
        sargs = bench.parse(["--steps", "2", "--warmup", "1", "--end-to-end", "0", "--cold", "0",
                             "--cpu-seconds", "0"])
        for key, fn in bench.strong_legs().items():
            r = fn(sjob, sargs)
            e = bench.secondary_entry(key, r, 30_000, 1, sargs)
            out[key] = (r["gather_check"], r["p99_fk_err"], e["total_points"],
                        e.get("baseline_config"))
        sc.close()
        q.put(out)
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put(repr(e) + traceback.format_exc())


def _spawn(target, timeout=240):
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


def test_bench_runners_through_a_sharded_context():
    res = _spawn(_bench_worker)
    for name, v in res.items():
        gc, p99 = v[0], v[1]
        assert gc is not None and gc["bit_exact"] and gc["rows"] > 0, (name, gc)
        assert math.isfinite(p99) and p99 > 0, (name, p99)
    assert res["ann"][3] == 1                      # ANN: one chunk
    chk, _, mean_it, chunks, iters, row_bytes, cold = res["fabrik"]
    assert chunks == 1 and mean_it > 1 and iters > 0 and row_bytes == 32 and cold
    for key in ("ann_strong10M", "fabrik_tol1e-5_strong10M"):
        assert res[key][2] == 30_000 and res[key][3] is None  # one rank: no configs[3]/[4]


def _auto_chunks_worker(q):
    try:
        from inversekinematicsann_amd import _native
        from inversekinematicsann_amd import dist as D
        from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                             REFERENCE_Y_SCALER as YS,
                                                             glorot_model)
        from inversekinematicsann_amd.robot.position_generator import random_dist
        ctx = _native.Context(0)
        m = glorot_model(dims=(3, 64, 64, 4), seed=4)
        ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
        pts = random_dist(3000, seed=8)
        out = {}
        for g in (1, 2, 8):
            sc = D.ShardedContext.loopback(ctx, g, 0)
            sc.set_chunks(0)
            sc.fabrik(pts, 1e-3, 100)
            out[f"fabrik_g{g}"] = sc.info()[2]
            sc.ann(pts)
            out[f"ann_g{g}"] = sc.info()[2]
            sc.close()
        q.put(out)
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put(repr(e) + traceback.format_exc())


def test_automatic_chunks_one_for_both_methods():
    """ikhip.h ik_comm_set_chunks: automatic = one chunk for ANN and FABRIK at any
    nranks; the chunked gather stays opt-in until a real N >= 2 run has checked it
    bit for bit."""
    res = _spawn(_auto_chunks_worker, timeout=120)
    assert res == {"fabrik_g1": 1, "ann_g1": 1, "fabrik_g2": 1, "ann_g2": 1,
                   "fabrik_g8": 1, "ann_g8": 1}, res
