"""Benchmark: IK solutions/s of the MI355X engine (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): ANN MLP forward of the reference
architecture (ann.py:46-56: 3 -> 12 x Dense(500, tanh) -> Dense(4)) over 1M
random_dist points per GPU in fp32, with the FK round-trip error fused in the
same launch.  `--method fabrik` measures configs[2] (FABRIK, tol 1e-3 /
100 iterations, float64).  One step = one solve of the whole batch with
inputs already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--method ann|fabrik]
                    [--total-points T] [--gather 0|1]

N > 1 runs one process per GPU: `python bench.py --gpus N` starts
`python -m torch.distributed.run --nproc-per-node N bench.py ...` itself as a
child process (before anything here touches the GPU) and exits with its code;
a rank that finds WORLD_SIZE != --gpus exits non-zero instead of printing a
mislabeled line.  Every rank holds the same global batch (random_dist, seed 0;
seed 1 from 10M points) and calls the library's sharded solve
(ik_*_solve_sharded): it solves its parts of the batch and the library
all-gathers them in place over RCCL, chunk by chunk under the solve, with a
tail record of every rank's stats, so the step ends with the
whole batch's angles on every rank.  Weak scaling by default (1M points per
GPU); --total-points 10000000 is configs[3] (ANN) / configs[4] (FABRIK tol
1e-5 / 200) as strong scaling.  torch.distributed (gloo) is only the control
plane: the RCCL id exchange, the barriers, the max over ranks of the step time.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import math
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "IK solutions/sec (6DOF, 1M-point batch) at 1/2/4/8 GPUs; max |FK err|"
ANN_DIMS = (3,) + (500,) * 12 + (4,)
FP32_MFMA_PEAK = 157.3e12   # MI355X_MICROARCH.md: dense fp32 matrix peak
BF16_MFMA_PEAK = 2.5e15     # dense bf16 matrix peak (no sparsity)
FP16_MFMA_PEAK = 2.5e15     # dense fp16 matrix peak (no sparsity)
SPLIT_PRODUCTS = {"bf16x6": 6, "fp16x3": 3}  # MFMA products per fp32 product
FP64_VALU_PEAK = 78.6e12    # MI355X fp64 vector peak (spec)
HBM_PEAK = 8.0e12           # bytes/s
FABRIK_FLOP_PER_ITER = 132  # per executed reference iteration
FABRIK_FLOP_PER_POINT = 150  # + the seed FK and angles, per point
TIMING_REPS = 5              # steps timed per kernel (median)
TIMING_LEAD = 2              # steps ahead of them in the same back-to-back run, not used


def launch_command(argv, gpus, port):
    """The torch.distributed.run command line that runs this script on `gpus`
    ranks of one node (the driver's N > 1 form, BASELINE.json / SURVEY 8(e))."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1",
            f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _gpus_arg(argv):
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return 1


def maybe_launch(argv=None):
    """`--gpus N > 1` without a launcher: run N ranks as a child torch.distributed.run
    (rank 0 prints the line on the inherited stdout) and return its exit code;
    None when this process is a rank itself (or N == 1).  Nothing here imports
    torch or touches the GPU: the child is a new program, not an exec."""
    argv = sys.argv[1:] if argv is None else argv
    if "WORLD_SIZE" in os.environ:
        return None
    gpus = _gpus_arg(argv)
    if gpus <= 1:
        return None
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    # the ranks' runtime must use dmabuf IPC: this pool's host driver
    # supports only that, and RCCL's peer setup fails with hipIpcGetMemHandle:
    # invalid argument under the legacy mode; the pool already exports it, and an
    # explicit value in the environment wins
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(launch_command(argv, gpus, port), env=env)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--method", choices=["ann", "fabrik", "fk"], default="ann",
                    help="fk: the batched FK kernel alone (profiling; no secondaries)")
    ap.add_argument("--points", type=int, default=1_000_000, help="points per GPU")
    ap.add_argument("--tol", type=float, default=1e-3)
    ap.add_argument("--max-iter", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU-baseline time budget (rank 0, N=1); 0 disables")
    ap.add_argument("--secondary", type=int, default=1,
                    help="also time the other method and report it under 'secondary'")
    ap.add_argument("--ann-mode", choices=["fp32", "bf16x6", "fp16x3"], default="fp32",
                    help="ANN hidden-GEMM arithmetic of the headline line (ikhip.h "
                         "ik_ann_set_mode); the other mode is reported under 'secondary'")
    ap.add_argument("--end-to-end", type=int, default=1,
                    help="also time the host-pointer (PCIe-inclusive) path; 0 for profiling "
                         "runs, whose per-kernel averages it would mix in")
    ap.add_argument("--cold", type=int, default=1,
                    help="FABRIK: also time cold calls (work order forgotten); 0 for profiling "
                         "runs, whose per-kernel averages they would mix in")
    ap.add_argument("--traffic-file",
                    default=os.path.join(ROOT, "profiles", "r06", "traffic.json"))
    ap.add_argument("--pmc-dir", default=os.path.join(ROOT, "profiles", "r06", "pmc"),
                    help="committed PMC diagnosis summaries (pipe occupancy in the roofline)")
    ap.add_argument("--gather", type=int, default=1,
                    help="N>1: the sharded solve with the library's RCCL all-gather of every "
                         "rank's rows and stats in the timed step (1); 0 = every rank solves its "
                         "shard only, no collective (also the one-GPU N>1 rehearsal mode)")
    ap.add_argument("--total-points", type=int, default=0,
                    help="global batch sharded over the ranks (strong scaling; configs[3] / "
                         "configs[4] are 10000000); 0 = --points per GPU (weak scaling)")
    ap.add_argument("--strong-legs", type=int, default=1,
                    help="N>1 with the weak headline: also time configs[3] (ANN fp32 + FK "
                         "round trip) and configs[4] (FABRIK tol 1e-5 / 200) as BASELINE.json "
                         "states them, the 10M-point seed-1 batch sharded over the N ranks, "
                         "under 'secondary' (VERDICT r04 #1)")
    return ap.parse_args(argv)


def open_sharded(ctx, world, rank, sharded=None, unique_id=None):
    """The library's RCCL communicator for the timed steps' all-gather (SURVEY
    §8(e)), or -- when RCCL is missing or its init fails (or times out) on ANY
    rank -- None on every rank, with the reason: the ranks then solve their shards
    with no collective (the survey's host-only fallback) and the line says so
    (config.all_gather_in_step false, config.rccl_fallback), instead of the run
    dying.  The ranks agree over the gloo control plane.  sharded / unique_id:
    dist.ShardedContext and _native.comm_unique_id, replaceable by tests."""
    import torch
    import torch.distributed as dist
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    sharded = sharded or D.ShardedContext
    unique_id = unique_id or _native.comm_unique_id
    sc, why = None, None
    uid = None
    if rank == 0:
        try:
            uid = unique_id()
        except Exception as e:  # (no RCCL library, or ncclGetUniqueId failed)
            why = f"{type(e).__name__}: {e}"
    uid = D.torch_broadcast(uid)  # None on every rank when rank 0 has no id
    if uid is None:
        why = why or "rank 0 has no RCCL unique id"
    else:
        try:
            sc = sharded(ctx, world, rank, uid)
        except Exception as e:  # (init failed, or the library's deadline aborted it)
            why = f"{type(e).__name__}: {e}"
    ok = torch.tensor([0 if sc is None else 1], dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        if sc is not None:
            try:
                sc.close()
            except Exception:  # (its peers never joined: nothing to tear down cleanly)
                pass
            sc = None
        why = why or "another rank's RCCL init failed"
        print(f"bench.py: rank {rank}: RCCL unavailable ({why}); the ranks solve their "
              f"shards with no collective", file=sys.stderr)
    return sc, why


def dist_setup(args):
    """One process per GPU.  torch.distributed (gloo, CPU) is the control plane
    only; the data path is the library's RCCL communicator (dist.ShardedContext)."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # IKHIP_DIST_BACKEND=gloo + more ranks than GPUs: rehearsing the N > 1
    # bookkeeping on a one-GPU box (ranks share device 0; use --gather 0 there,
    # RCCL takes one rank per GPU)
    if os.environ.get("IKHIP_DIST_BACKEND", "rccl") == "gloo":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if "WORLD_SIZE" in os.environ:  # launched by torch.distributed.run (any N)
        import datetime
        import torch.distributed as dist
        # a bounded control plane too: a rank that never reaches a barrier ends
        # the run instead of holding it to the driver's limit
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=600))
    return world, rank, local


def _dist_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def barrier(world):
    if _dist_on():
        import torch.distributed as dist
        dist.barrier()


def _reduce(v: float, op) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(v: float, world: int) -> float:
    if not _dist_on():
        return v
    import torch.distributed as dist
    return _reduce(v, dist.ReduceOp.MAX)


def sum_over_ranks(v: float, world: int) -> float:
    if not _dist_on():
        return v
    import torch.distributed as dist
    return _reduce(v, dist.ReduceOp.SUM)


def _pts(n: int) -> str:
    return f"{n // 1_000_000}M" if n % 1_000_000 == 0 else f"{n}"


def _batch_words(job) -> str:
    if job.world == 1:
        return f"{_pts(job.total)} random_dist points"
    how = ("sharded contiguously, one RCCL all-gather of rows + stats inside libikhip"
           if job.sc is not None else "sharded contiguously, no collective")
    return f"{_pts(job.total)} random_dist points over {job.world} GPUs ({how})"


def load_profile(path, kernel):
    """What the profiling lease (tools/profile_round.sh -> tools/profile_summary.py)
    recorded for `kernel` over the bench's timed window, or {}."""
    try:
        with open(path) as f:
            return json.load(f).get(kernel, {}) or {}
    except (OSError, ValueError):
        return {}


def load_traffic(path, kernel):
    """HBM bytes per launch of `kernel` from the PMC passes, FETCH_SIZE doubled per
    MI355X_MICROARCH.md §HBM; None if not collected."""
    return load_profile(path, kernel).get("hbm_bytes_per_launch")


def profile_fields(path, kernel):
    """The roofline's profile-derived extras: the raw (undoubled) HBM bytes, the
    kernel's shader clock and the rocprof window average of its duration -- the
    median over the profiling lease's box and the round's trace-only boxes when
    tools/merge_boxes.py recorded them (`rocprof_boxes_ms`, the lease's own first):
    this run's box is one more draw, and boxes differ by a few %."""
    p = load_profile(path, kernel)
    out = {k: p[k] for k in ("hbm_bytes_per_launch_raw", "clock_ghz", "rocprof_avg_ms")
           if k in p}
    if "rocprof_median_ms" in p:
        out["rocprof_avg_ms"] = p["rocprof_median_ms"]
        out["rocprof_boxes_ms"] = p.get("rocprof_boxes_ms")
        out["rocprof_basis"] = "median of the boxes' timed-window averages"
    if out:
        out["profile"] = os.path.relpath(path, ROOT)
    return out


def kernel_time_ok(kernel_ms, step_ms):
    """A kernel's measured duration can be a roofline's denominator only if it
    fits inside the step that launches it (a begin marker that
    took in the kernels ahead of it gave an iteration kernel longer than its
    whole step)."""
    return bool(kernel_ms) and bool(step_ms) and kernel_ms <= step_ms


def roofline_fracs(work, kernel_ms, peak, prof, step_ms=None, loop_ms=None):
    """The roofline's achieved rate both ways: from this run's
    HIP-event kernel time (the dispatch's own start / end stamps) and from the
    committed rocprof window average of the same kernel (`prof`:
    profile_fields); `frac` / `achieved` headline the LOWER of the two.  An
    events duration is a kernel duration only if it fits inside the step it was
    stamped in (`step_ms`, kernel_time_ok) and inside the untimed loop's step
    (`loop_ms`, 1 % for clock drift): the event-stamped launch of a short
    memory-bound kernel can run slower than the untimed loop (FK: ~9 %, r06), and
    then rocprof's window stands alone.  work: algorithmic flop (or bytes) per launch."""
    valid = kernel_time_ok(kernel_ms, step_ms) if step_ms is not None else bool(kernel_ms)
    note = None
    if valid and loop_ms is not None and kernel_ms > 1.01 * loop_ms:
        valid, note = False, ("the event-stamped launch ran longer than the untimed loop's "
                              "step: the rocprof window alone prices the roofline")
    ev = work / (kernel_ms / 1e3) if valid else None
    rp = prof.get("rocprof_avg_ms")
    rq = work / (rp / 1e3) if rp else None
    cands = [x for x in (ev, rq) if x]
    head = min(cands) if cands else None
    out = {"achieved_events": ev, "frac_events": ev / peak if ev else None,
           "achieved_rocprof": rq, "frac_rocprof": rq / peak if rq else None,
           "headline": None if head is None else ("rocprof" if head == rq else "events"),
           "kernel_ms_valid": valid, "_head": head}
    if note:
        out["kernel_ms_note"] = note
    return out


def load_pipe(path, kernel):
    """Pipe occupancy of `kernel` from the committed PMC diagnosis pass
    (tools/pmc_diag.sh -> tools/pmc_summary.py): MFMA busy, VALU active and
    fp64-pipe busy as fractions of the kernel's SIMD cycles; None if absent."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    for k, v in d.items():
        if k == kernel or k.split("<")[0] == kernel:
            out = {"mfma_busy": v.get("MfmaUtil_pct", 0.0) / 100,
                   "valu_active": v.get("ValuActive_pct", 0.0) / 100,
                   "fp64_pipe_busy": v.get("Fp64PipeBusy_pct", 0.0) / 100,
                   "source": os.path.relpath(path, ROOT)}
            if "L2_hit_pct" in v:
                out["l2_hit"] = v["L2_hit_pct"] / 100
            return out
    return None


class Job:
    """The global batch and this rank's part of it.  sc: the library's sharded
    context (N > 1 with --gather 1), else None (this rank's shard only)."""

    def __init__(self, ctx, sc, pts, dpts, lo, hi, world):
        self.ctx, self.sc, self.pts, self.dpts = ctx, sc, pts, dpts
        self.lo, self.hi, self.world = lo, hi, world
        self.total = dpts.shape[0]
        self.n_local = hi - lo
        self.n_out = self.total if sc is not None else self.n_local  # rows a step returns

    @property
    def local_pts(self):
        return self.dpts[self.lo:self.hi]


def _stats_over_ranks(job, st, res):
    """The batch's stats: already batch-wide after a sharded call (the gathered
    tails), else each rank's shard reduced over the ranks."""
    if job.sc is not None:
        return st.max_fk_err, st.sum_fk_err, st.sum_iters, st.n_capped
    w = job.world
    return (max_over_ranks(st.max_fk_err, w), sum_over_ranks(st.sum_fk_err, w),
            sum_over_ranks(st.sum_iters, w), sum_over_ranks(st.n_capped, w))


def _own_parts(job):
    """This rank's rows [(begin, end)] of the last step: its parts of the chunks
    the library planned the sharded call with (ik_comm_info), else its shard."""
    if job.sc is None:
        return [(0, job.n_local)]
    from inversekinematicsann_amd import dist as D
    _, _, chunks = job.sc.info()
    C, _, _ = D.plan_of(job.total, job.world, max(1, chunks))
    return [D.part_bounds(job.total, job.world, max(1, chunks), job.sc.rank, c) for c in range(C)]


def _check_parts(job):
    """The rows this rank re-solves after a sharded step: the first and the last
    part of rank (r + 1) % N in the plan the library used (ik_comm_info)."""
    from inversekinematicsann_amd import dist as D
    q = (job.sc.rank + 1) % job.world
    chunks = max(1, job.sc.info()[2])
    C, _, _ = D.plan_of(job.total, job.world, chunks)
    parts = [D.part_bounds(job.total, job.world, chunks, q, c) for c in range(C)]
    parts = [p for p in parts if p[1] > p[0]]
    return sorted({parts[0], parts[-1]}) if parts else []


def _as_bytes(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    x = np.ascontiguousarray(x)
    return x.view(np.uint8).reshape(x.shape[0], -1) if x.ndim else x.view(np.uint8)


def compare_rows(gathered, resolved):
    """Bit-for-bit comparison of gathered rows with a plain re-solve of the same
    rows: {output name: array} each.  Returns (rows, mismatching rows)."""
    rows, bad = 0, 0
    for k, ref in resolved.items():
        a, b = _as_bytes(gathered[k]), _as_bytes(ref)
        if a.shape != b.shape:
            return max(rows, b.shape[0]), b.shape[0]
        diff = (a != b).reshape(a.shape[0], -1).any(axis=1)
        rows = max(rows, a.shape[0])
        bad = max(bad, int(diff.sum()))
    return rows, bad


def gather_check(job, outputs, resolve):
    """N > 1: after the timed steps each rank re-solves, plainly
    and unsharded, rank (r + 1) % N's first and last parts of the batch and
    compares them bit for bit with what the all-gather delivered into its own
    arrays (angles, and FABRIK's iteration counts).  Row counts add up and the
    verdict is AND-reduced over the ranks; None without a sharded context."""
    if job.sc is None:
        return None
    rows, bad = 0, 0
    for b, e in _check_parts(job):
        r, x = compare_rows({k: v[b:e] for k, v in outputs.items()}, resolve(b, e))
        rows, bad = rows + r, bad + x
    rows = int(sum_over_ranks(rows, job.world))
    bad = int(sum_over_ranks(bad, job.world))
    return {"rows": rows, "mismatched_rows": bad, "bit_exact": bad == 0,
            "what": "every rank re-solved rank (r+1)%N's first and last parts unsharded and "
                    "compared them bit for bit with its gathered rows"}


def gather_verdict(checks):
    """The line's config.gather_check from the methods' checks, and the exit code:
    0, or 3 when any gathered row differs from its re-solve."""
    checks = {k: v for k, v in checks.items() if v}
    if not checks:
        return None, 0
    ok = all(v["bit_exact"] for v in checks.values())
    return ({"rows": sum(v["rows"] for v in checks.values()), "bit_exact": ok,
             "per_method": checks}, 0 if ok else 3)


def _p99(job, derr, world):
    """p99 of the FK errors: after a sharded step the library's gathered
    histograms (every rank's own rows; an upper bound within 1/16 octave), else
    torch.quantile of this rank's errors, max over ranks."""
    if job.sc is not None:
        return job.sc.fk_err_quantile(0.99)
    import torch
    fin = derr[:1 << 24]
    fin = fin[torch.isfinite(fin)]
    return max_over_ranks(float(torch.quantile(fin, 0.99)) if fin.numel() else 0.0, world)


_HOST_OUT = {}


def _host_out(key, shape, dtype, pinned):
    """Output arrays of the end-to-end leg, allocated once per shape (pinned or not)."""
    from inversekinematicsann_amd import _native
    k = (key, shape, np.dtype(dtype).str, pinned)
    if k not in _HOST_OUT:
        _HOST_OUT[k] = _native.pinned_empty(shape, dtype) if pinned else np.empty(shape, dtype)
    return _HOST_OUT[k]


def _host_ann(job, hp, pinned):
    import ctypes
    from inversekinematicsann_amd import _native
    n = hp.shape[0]
    ang = _host_out("ann_ang", (n, 4), np.float32, pinned)  # the angles only (ann.py:76)
    s = _native.IkStats()
    fn = job.ctx.lib.ik_ann_solve_sharded if job.sc is not None else job.ctx.lib.ik_ann_solve
    job.ctx._check(fn(job.ctx.handle, hp.ctypes.data, n, ang.ctypes.data, None, 0,
                      ctypes.byref(s)))


def _host_fabrik(job, hp, pinned, tol, max_iter):
    import ctypes
    from inversekinematicsann_amd import _native
    n = hp.shape[0]
    ang = _host_out("fab_ang", (n, 4), np.float64, pinned)  # the angles only (inverse.py:139)
    s = _native.IkStats()
    L, h = job.ctx.lib, job.ctx.handle
    if job.sc is not None:
        rc = L.ik_fabrik_solve_sharded(h, hp.ctypes.data, n, tol, max_iter, ang.ctypes.data,
                                       None, None, 0, ctypes.byref(s))
    else:
        rc = L.ik_fabrik_solve_fk(h, hp.ctypes.data, n, tol, max_iter, ang.ctypes.data,
                                  None, None, None, 0, ctypes.byref(s))
    job.ctx._check(rc)


def run_ann(job, args, mode="fp32"):
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    ctx, world = job.ctx, job.world
    m = glorot_model(ANN_DIMS, seed=0)
    ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
    ctx.ann_set_mode(mode)
    dang = torch.empty((job.n_out, 4), dtype=torch.float32, device="cuda")
    derr = torch.empty(job.n_out, dtype=torch.float64, device="cuda")
    flags = _native.IK_F_DEVICE | _native.IK_F_ASYNC

    if job.sc is not None:
        def step():  # solve the shard + the library's one RCCL all-gather
            job.sc.ann_device(job.dpts, dang, derr, flags=flags)
    else:
        def step():
            ctx.ann_solve_device(job.local_pts, dang, derr, flags=flags)

    res = timed(ctx, step, args, world)
    st = ctx.stats_fetch()
    mx, sm, _, _ = _stats_over_ranks(job, st, res)
    # the p99 from the last sharded step's gathered histograms, BEFORE the gather
    # check's plain re-solves (a plain call ends the sharded call's state: ADVICE r04)
    res["p99_fk_err"] = _p99(job, derr, world)
    if job.sc is not None:
        res["gather_chunks"] = job.sc.info()[2]
        res["gather_ms"] = st.gather_ms

        def resolve(b, e):
            a = torch.empty((e - b, 4), dtype=torch.float32, device="cuda")
            ctx.ann_solve_device(job.dpts[b:e], a, torch.empty(e - b, dtype=torch.float64,
                                                               device="cuda"))
            return {"ang": a}
        res["gather_check"] = gather_check(job, {"ang": dang}, resolve)
    res["max_fk_err"] = mx
    res["mean_fk_err"] = sm / job.total
    res["fk_err_note"] = ("random Glorot weights (the reference .h5 is not shipped): the FK "
                          "round trip is computed in the same launch; not model accuracy")
    res["outputs"] = {"ang": dang}
    if args.end_to_end:
        res["end_to_end"] = end_to_end(job, lambda hp, pinned: _host_ann(job, hp, pinned), args)
    ctx.ann_set_mode("fp32")
    flop_pt = m.flops_per_point()
    kname = "ann_fused_kernel" if mode == "fp32" else f"ann_fused_kernel_{mode}"
    k = res["kernels"].get(kname)
    n = job.n_local
    # split modes: k bf16 / fp16 MFMA products per fp32 product, so the
    # fp32-equivalent matrix peak is the 16-bit peak / k (the input and output
    # layers stay fp32)
    peak = (FP32_MFMA_PEAK if mode == "fp32" else
            (BF16_MFMA_PEAK if mode == "bf16x6" else FP16_MFMA_PEAK) / SPLIT_PRODUCTS[mode])
    traffic = load_traffic(args.traffic_file, kname)
    prof = profile_fields(args.traffic_file, kname)
    fr = roofline_fracs(flop_pt * n, k, peak, prof, res["event_step_ms"], res["ms_per_step"])
    achieved = fr.pop("_head")
    res["roofline"] = {"bound": "mfma", "achieved": achieved / 1e12 if achieved else None,
                       "peak": peak / 1e12, "unit": "TFLOP/s",
                       "frac": achieved / peak if achieved else None,
                       "frac_events": fr["frac_events"], "frac_rocprof": fr["frac_rocprof"],
                       "frac_headline": fr["headline"], "kernel_ms_valid": fr["kernel_ms_valid"],
                       "event_step_ms": res["event_step_ms"],
                       **({"kernel_ms_note": fr["kernel_ms_note"]} if "kernel_ms_note" in fr else {}),
                       "traffic": traffic, "kernel": kname,
                       "kernel_ms": k, "algorithmic_flop_per_point": flop_pt,
                       "points_per_launch": n, **prof}
    diag = "ann_diag_summary.json" if mode == "fp32" else f"ann_{mode}_diag_summary.json"
    res["roofline"]["pipes"] = load_pipe(os.path.join(args.pmc_dir, diag), kname)
    if mode == "fp32":
        res["dtype"] = "fp32"
        res["workload"] = ("ANN MLP forward (3-12x500tanh-4, fp32) + fused FK round-trip error, "
                           + _batch_words(job))
    else:
        res["dtype"] = {"bf16x6": "fp32 via bf16x6 (3-way bf16 split, 6 MFMA products, fp32 "
                                  "accumulate)",
                        "fp16x3": "fp32 via fp16x3 (2-way fp16 split of power-of-two-scaled "
                                  "operands, 3 MFMA products, fp32 accumulate)"}[mode]
        res["workload"] = (f"ANN MLP forward (3-12x500tanh-4), hidden GEMMs in the {mode} mode "
                           "(accuracy: tests/test_gpu_parity.py::test_ann_split_modes and "
                           "cpu_baseline.parity) + fused FK round-trip error, " + _batch_words(job))
    return res


def run_fabrik(job, args, tol=None, max_iter=None):
    import torch
    tol = args.tol if tol is None else tol
    max_iter = args.max_iter if max_iter is None else max_iter
    from inversekinematicsann_amd import _native
    ctx, world = job.ctx, job.world
    dang = torch.empty((job.n_out, 4), dtype=torch.float64, device="cuda")
    dit = torch.empty(job.n_out, dtype=torch.int32, device="cuda")
    derr = torch.empty(job.n_out, dtype=torch.float64, device="cuda")
    flags = _native.IK_F_DEVICE | _native.IK_F_ASYNC

    # the --verbose FK round trip (cli.py:54-72) in the same launch as the angles
    if job.sc is not None:
        def solve(p, a, i, e):  # solve the shard + the library's RCCL all-gathers
            job.sc.fabrik_device(p, a, i, e, tol, max_iter, flags=flags)
        batch = job.dpts
        # the timed step gathers what the reference returns, the angles
        # (inverse.py:139: 32 B a row); the iteration counts travel only in the
        # untimed call after the timed steps
        step_it = None
    else:
        def solve(p, a, i, e):
            ctx.fabrik_solve_device(p, a, i, None, tol, max_iter, flags=flags, fk_err=e)
        batch = job.local_pts
        step_it = dit

    def step():
        solve(batch, dang, step_it, derr)

    # the warm-up steps teach the work-order table on ANOTHER batch of the same
    # distribution (seed 2), so the timed steps do not start from a table
    # learned on their own points
    wpts = torch.from_numpy(warm_batch(batch.shape[0])).cuda()
    wang, werr = torch.empty_like(dang), torch.empty_like(derr)
    wit = None if step_it is None else torch.empty_like(dit)

    def warm():
        solve(wpts, wang, wit, werr)

    ctx.fabrik_reset_order()  # start from a fresh context's table, whatever ran before
    table = {}

    def after_warm():
        # the work-order table the timed steps start from: the same bytes in every
        # process of the same build and batch (process spread)
        t = ctx.fabrik_order_get()
        table["sha16"] = hashlib.sha256(t.tobytes()).hexdigest()[:16]
        table["cells_seen"] = int((t > 0).sum())

    res = timed(ctx, step, args, world, warm=warm, after_warm=after_warm)
    res["order_table"] = table
    del wpts, wang, wit, werr
    if job.sc is not None:
        res["gather_chunks"] = job.sc.info()[2]
        res["gather_ms"] = ctx.stats_fetch().gather_ms  # the last timed step's gathers
        res["gathered_bytes_per_row"] = 32
        # untimed: the same sharded call with the iteration counts gathered too
        # (the rows are the timed steps' own: the solve is deterministic)
        solve(batch, dang, dit, derr)
        ctx.sync()
    st = ctx.stats_fetch()
    mx, sm, sum_iters, n_capped = _stats_over_ranks(job, st, res)
    # the p99 from the last sharded call's gathered histograms, BEFORE the gather
    # check's plain re-solves (a plain call ends the sharded call's state: ADVICE r04)
    res["p99_fk_err"] = _p99(job, derr, world)
    if job.sc is not None:
        def resolve(b, e):
            a = torch.empty((e - b, 4), dtype=torch.float64, device="cuda")
            i = torch.empty(e - b, dtype=torch.int32, device="cuda")
            ctx.fabrik_solve_device(job.dpts[b:e], a, i, None, tol, max_iter,
                                    fk_err=torch.empty(e - b, dtype=torch.float64, device="cuda"))
            return {"ang": a, "iters": i}
        res["gather_check"] = gather_check(job, {"ang": dang, "iters": dit}, resolve)
    if args.cold:
        res["cold"] = cold_steps(ctx, step)
        if job.sc is None:
            # the same cold call on batches of other distributions:
            # the built-in table was learned on random_dist only
            res["cold"]["other_distributions"] = cold_other(ctx, job.n_local, tol, max_iter)
    n = job.n_local
    res["mean_iters"] = sum_iters / job.total
    res["n_capped"] = int(n_capped)
    res["max_fk_err"] = mx
    res["mean_fk_err"] = sm / job.total
    res["outputs"] = {"ang": dang, "iters": dit}
    if args.end_to_end:
        res["end_to_end"] = end_to_end(
            job, lambda hp, pinned: _host_fabrik(job, hp, pinned, tol, max_iter), args)
    # this rank's own iterations (the kernel's work), from its shard of the rows
    local_iters = sum(int(dit[b:e].sum().item()) for b, e in _own_parts(job))
    local_points = sum(e - b for b, e in _own_parts(job))
    k = res["kernels"].get("fabrik_iter_kernel")
    # 132 flop per iteration + 150 per point (seed and angles, both in
    # this kernel)
    flops = FABRIK_FLOP_PER_ITER * local_iters + FABRIK_FLOP_PER_POINT * local_points
    pkey = "fabrik_iter_kernel" if (tol, max_iter) != (1e-5, 200) else \
        "fabrik_tol1e-5/fabrik_iter_kernel"
    traffic = load_traffic(args.traffic_file, pkey)
    prof = profile_fields(args.traffic_file, pkey)
    fr = roofline_fracs(flops, k, FP64_VALU_PEAK, prof, res["event_step_ms"], res["ms_per_step"])
    achieved = fr.pop("_head")
    res["roofline"] = {"bound": "valu_fp64", "achieved": achieved / 1e12 if achieved else None,
                       "peak": FP64_VALU_PEAK / 1e12, "unit": "TFLOP/s",
                       "frac": achieved / FP64_VALU_PEAK if achieved else None,
                       "frac_events": fr["frac_events"], "frac_rocprof": fr["frac_rocprof"],
                       "frac_headline": fr["headline"], "kernel_ms_valid": fr["kernel_ms_valid"],
                       "event_step_ms": res["event_step_ms"],
                       **({"kernel_ms_note": fr["kernel_ms_note"]} if "kernel_ms_note" in fr else {}),
                       "traffic": traffic, "kernel": "fabrik_iter_kernel", "kernel_ms": k,
                       "algorithmic_flop_per_iteration": FABRIK_FLOP_PER_ITER,
                       "algorithmic_flop_per_point": FABRIK_FLOP_PER_POINT,
                       "iterations_per_launch": local_iters,
                       "points_per_launch": local_points,
                       **prof,
                       # the flop count prices a correctly rounded sqrt / division as
                       # one flop; the pipes say how busy the SIMDs actually are
                       "pipes": load_pipe(os.path.join(
                           args.pmc_dir, "fabrik_diag_summary.json" if pkey ==
                           "fabrik_iter_kernel" else "fabrik_tol1e-5_diag_summary.json"),
                           "fabrik_iter_kernel")}
    res["dtype"] = "f64"
    res["workload"] = (f"FABRIK ikine (seed FK + loop + angles) + fused FK round-trip error, "
                       f"tol {tol:g} / {max_iter} iterations, float64, " + _batch_words(job))
    return res


FK_BYTES_PER_POINT = 32 + 24   # float64 angles in, float64 effector xyz out


FK_BATCH_FACTOR = 32  # FK angle vectors per rank = 32 x the shard's points (32M at the default)


def run_fk(job, args):
    """Batched FK (forward.py:73-94, the DH chain) on
    FK_BATCH_FACTOR times as many angle vectors as this rank's shard has points,
    drawn uniformly in [-pi, pi): its bound is HBM (56 B per point) or the float64
    sin/cos + products, whichever is longer.  32M vectors (1.8 GB per launch) make
    a launch ~0.36 ms and are ~7x the 256 MB Infinity Cache, so no step re-reads the
    last one's angles from it: at 8M (448 MB) the events-timed loop ran ~7 % faster
    than rocprof's serialized dispatches, at 1M the dispatch's fixed cost was 7 %
    (r06).  No collective (each rank its own vectors)."""
    import torch
    from inversekinematicsann_amd import _native
    ctx, world, n = job.ctx, job.world, job.n_local * FK_BATCH_FACTOR
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    dang = (torch.rand((n, 4), generator=g, dtype=torch.float64, device="cuda") * 2 - 1) * math.pi
    dxyz = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    flags = _native.IK_F_DEVICE | _native.IK_F_ASYNC

    def step():
        ctx.fk_device(dang, dxyz, flags=flags)

    res = timed(ctx, step, args, world)
    res["outputs"] = {"xyz": dxyz}
    k = res["kernels"].get("fk_kernel")
    prof = profile_fields(args.traffic_file, "fk_kernel")
    fr = roofline_fracs(FK_BYTES_PER_POINT * n, k, HBM_PEAK, prof, res["event_step_ms"],
                        res["ms_per_step"])
    achieved = fr.pop("_head")
    res["roofline"] = {"bound": "hbm", "achieved": achieved / 1e9 if achieved else None,
                       "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                       "frac": achieved / HBM_PEAK if achieved else None,
                       "frac_events": fr["frac_events"], "frac_rocprof": fr["frac_rocprof"],
                       "frac_headline": fr["headline"], "kernel_ms_valid": fr["kernel_ms_valid"],
                       "event_step_ms": res["event_step_ms"],
                       "timing_note": "events: the dispatch's own start / end stamps "
                                      "(hipExtLaunchKernel); rocprof: its kernel trace",
                       **({"kernel_ms_note": fr["kernel_ms_note"]} if "kernel_ms_note" in fr else {}),
                       "traffic": load_traffic(args.traffic_file, "fk_kernel"),
                       **prof,
                       "kernel": "fk_kernel", "kernel_ms": k,
                       "algorithmic_bytes_per_point": FK_BYTES_PER_POINT,
                       "points_per_launch": n}
    res["dtype"] = "f64"
    res["unit"] = "FK evaluations/s"
    res["workload"] = f"FK (DH chain, float64), {_pts(n)} angle vectors per GPU"
    res["total"] = n * world
    return res


def warm_batch(n):
    """The FABRIK warm-up batch: random_dist points of a seed no timed step uses."""
    from inversekinematicsann_amd.robot.position_generator import random_dist
    return random_dist(n, seed=2)


def timed(ctx, step, args, world, warm=None, after_warm=None):
    """W warm-up steps, one step timed per kernel, then K steps between barriers.
    Every wait on the steps is ctx.sync() first (ik_ctx_sync): bounded by the
    communicator's deadline at N > 1, so a stuck peer ends the run with
    IK_E_RCCL rather than hanging it; torch.cuda.synchronize() then returns at once."""
    import torch
    for _ in range(args.warmup):
        (warm or step)()
    ctx.sync()
    torch.cuda.synchronize()
    if after_warm is not None:
        after_warm()
    # per-kernel durations: the library launches each kernel of a timed call with
    # hipExtLaunchKernel's start / stop events, which the dispatch itself stamps
    # (ik_ctx_set_timing), so a kernel's interval holds neither the
    # kernels ahead of it in the step nor the host's launch latency.  TIMING_LEAD +
    # TIMING_REPS steps back to back with the timings accumulating (set_timing(2):
    # no host sync between them, so no step starts from an idle, clocked-down GPU --
    # a 0.4 ms FK step behind a single lead step still ran ~5 % slow); the median
    # of the last TIMING_REPS steps' per-kernel sums, each step's own duration from
    # the stream's events around it.
    kernels, event_step_ms = {}, None
    nsteps = TIMING_LEAD + TIMING_REPS
    ctx.set_timing(2)
    evs = []
    for _ in range(nsteps):
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        s0.record()
        step()
        s1.record()
        evs.append((s0, s1))
    ctx.sync()
    torch.cuda.synchronize()
    times = ctx.kernel_times()
    ctx.set_timing(False)
    if times and len(times) % nsteps == 0 and len(times) < 64:
        per_step = len(times) // nsteps
        per = {}
        for s_ in range(TIMING_LEAD, nsteps):
            one = {}
            for name, ms in times[s_ * per_step:(s_ + 1) * per_step]:
                one[name] = one.get(name, 0.0) + ms
            for name, ms in one.items():
                per.setdefault(name, []).append(ms)
        kernels = {name: float(np.median(v)) for name, v in per.items()}
        event_step_ms = float(np.median([a.elapsed_time(b) for a, b in evs[TIMING_LEAD:]]))
    else:  # (more kernels a step than the 64 slots hold: each step timed on its own)
        per, steps_ms = {}, []
        for _ in range(TIMING_REPS):
            step()
            ctx.set_timing(True)
            s0 = torch.cuda.Event(enable_timing=True)
            s1 = torch.cuda.Event(enable_timing=True)
            s0.record()
            step()
            s1.record()
            ctx.sync()
            torch.cuda.synchronize()
            steps_ms.append(s0.elapsed_time(s1))
            one = {}
            for name, ms in ctx.kernel_times():
                one[name] = one.get(name, 0.0) + ms
            ctx.set_timing(False)
            for name, ms in one.items():
                per.setdefault(name, []).append(ms)
        kernels = {name: float(np.median(v)) for name, v in per.items()}
        event_step_ms = float(np.median(steps_ms))
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    ctx.sync()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    wall = max_over_ranks(wall, world)
    ev_ms = ev0.elapsed_time(ev1) / args.steps
    return {"wall_s": wall, "ms_per_step": wall * 1e3 / args.steps, "event_ms_per_step": ev_ms,
            "kernels": kernels, "event_step_ms": event_step_ms}


def cold_steps(ctx, step, reps=3):
    """The FABRIK step as a fresh context's first call makes it (the CLI's and
    the RPC worker's first request, cli.py:269-287): the work-order table reset
    to the library's built-in one for SixDOFRobot (ik_fabrik_reset_order), while
    `value` is the warm steady state.  Beside it the same call from an EMPTY
    table (point order: what a robot without a built-in table gets).  Median over
    `reps` (each call teaches the table, so each is preceded by a reset); scratch
    is already sized, so this isolates the work order's effect."""
    import torch

    def run(reset):
        times = []
        for _ in range(reps):
            reset()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            step()
            e1.record()
            ctx.sync()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        return times

    prior = run(ctx.fabrik_reset_order)
    empty = run(lambda: ctx.fabrik_order_set(None))
    ctx.fabrik_reset_order()
    step()  # re-learn before anything else runs
    ctx.sync()
    torch.cuda.synchronize()
    return {"ms": float(np.median(prior)), "all_ms": prior,
            "empty_table_ms": float(np.median(empty)), "empty_table_all_ms": empty,
            "note": "fresh-context call: work-order table reset to the built-in SixDOFRobot "
                    "table before each call (ik_fabrik_reset_order); empty_table: point order; "
                    "warm = ms_per_step (its table learned on a warm-up batch of another seed)"}


def cold_batches(n):
    """The cold call's other inputs: n points of the uniform
    workspace box (the reference's random_distribution('uniform'),
    position_generator.py:91-92, drawn vectorised with a seeded generator: 37 % of
    them out of reach, capped) and an n-point spring trajectory (the CLI's
    --shape spring, position_generator.py:73-78, with the cli.py:195 example's
    shape arguments 2, 3, 6): consecutive points of one smooth curve, so point
    order runs through easy and hard stretches in long runs."""
    from inversekinematicsann_amd.robot.position_generator import spring
    from inversekinematicsann_amd.robot.robot import SixDOFRobot
    lim = SixDOFRobot.effector_workspace_limits
    rng = np.random.default_rng(5)
    box = np.stack([rng.uniform(float(lo), float(hi), n) for lo, hi in lim.values()], axis=1)
    return {"uniform_box": box, "spring": spring(n, 2, 3, 6)}


def cold_other(ctx, n, tol, max_iter, reps=3):
    """cold_steps on each of cold_batches(n): a fresh context's table (the
    built-in one) against an empty table (point order), median of `reps` each,
    with the iteration counts of both compared (the order must not change them)."""
    import torch
    out = {}
    for name, pts in cold_batches(n).items():
        dp = torch.from_numpy(pts).cuda()
        ang = torch.empty((n, 4), dtype=torch.float64, device="cuda")
        it = torch.empty(n, dtype=torch.int32, device="cuda")
        err = torch.empty(n, dtype=torch.float64, device="cuda")

        def step():
            ctx.fabrik_solve_device(dp, ang, it, None, tol, max_iter, fk_err=err)
        step()  # scratch sized for this batch
        ctx.sync()
        c = cold_steps(ctx, step, reps)
        it_prior = it.clone()
        ctx.fabrik_order_set(None)
        step()
        ctx.sync()
        same = bool(torch.equal(it, it_prior))
        ctx.fabrik_reset_order()
        out[name] = {"ms": c["ms"], "all_ms": c["all_ms"], "empty_table_ms": c["empty_table_ms"],
                     "empty_table_all_ms": c["empty_table_all_ms"],
                     "prior_over_empty": c["ms"] / c["empty_table_ms"],
                     "iters_equal_across_orders": same,
                     "mean_iters": float(it.double().mean().item())}
        del dp, ang, it, err
    return out


def end_to_end(job, solve_host, args):
    """PCIe-inclusive rate (SURVEY 8(d) "end-to-end"): host float64 points in,
    host angles out (the reference's outputs: 24 B in, 16 B (ANN) / 32 B (FABRIK)
    out per point) through the library's host-pointer path (H2D, kernels, D2H,
    stats; with N > 1 the sharded call and its all-gather).  Two host memories:
    pinned (ik_host_alloc; FABRIK: the copies of chunks overlap the kernels of
    others) and pageable numpy arrays (one shot, the driver stages them).  The
    box's PCIe moves ~55 GB/s and its two directions do not overlap
    (tools/pcie_probe.py), so 1M FABRIK points cost >= 1.02 ms of copies.
    Reported beside `value`, never as it."""
    import torch
    from inversekinematicsann_amd import _native
    pts = job.pts if job.sc is not None else job.pts[job.lo:job.hi]
    reps = max(1, min(args.steps, 10))

    def rate(host_pts, pinned):
        # untimed warm-up (10 calls): the staging scratch, the pipeline's streams,
        # and the copy engines' queues, which the runtime sets up over the first
        # calls (the first pinned calls of a process measured 19-22 / 7.7-10 /
        # 1.2-8.3 ms, steady 1.10-1.13: tools/pinned_probe.py)
        for _ in range(10):
            solve_host(host_pts, pinned)
        barrier(job.world)
        t0 = time.perf_counter()
        calls = []  # this rank's per-call times (the host path returns when D2H is done)
        for _ in range(reps):
            t1 = time.perf_counter()
            solve_host(host_pts, pinned)
            calls.append((time.perf_counter() - t1) * 1e3)
        torch.cuda.synchronize()
        barrier(job.world)
        wall = max_over_ranks(time.perf_counter() - t0, job.world)
        return wall * 1e3 / reps, float(np.median(calls)), float(max(calls))

    pp = _native.pinned_empty(pts.shape, np.float64)
    pp[:] = pts
    ms, med, mx = rate(pp, True)
    ms_pageable, med_p, mx_p = rate(np.ascontiguousarray(pts), False)
    # ms_per_step / value: the mean over the timed calls; median / max per call
    # beside it (the runtime's pinned copies have occasional multi-ms outliers)
    return {"ms_per_step": ms, "value": job.total / (ms / 1e3), "steps": reps,
            "median_ms": med, "max_ms": mx,
            "unit": "IK solutions/s",
            "path": "host pointers (ik_*_solve without IK_F_DEVICE), pinned host arrays "
                    "(ik_host_alloc; chunked copy/compute overlap)",
            "pageable": {"ms_per_step": ms_pageable,
                         "value": job.total / (ms_pageable / 1e3),
                         "median_ms": med_p, "max_ms": mx_p}}


def _host_cpu():
    """The GPU host's CPU (record the model and os.cpu_count())."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": affinity,
            "omp_num_threads": omp,
            # why `cores` is not os_cpu_count: a one-GPU box is leased one GPU's share of
            # the host (OMP_NUM_THREADS, set by the box), and the baseline uses that share
            "cores_note": ("one GPU's share of the host: OMP_NUM_THREADS=%s on this box; "
                           "os.cpu_count() counts the whole machine" % omp) if omp else
                          "all CPUs this process may use"}


# cpu_baseline samples: the first points of the GPU batch, which the oracle's output on
# them also checks (the first 100k for ANN; FABRIK: 16 x 4096)
CPU_SAMPLE = {"ann": 100_000, "fabrik": 65_536}


def cpu_baseline(method, args, sample_pts=None, gpu_out=None):
    """The oracle timed on this host (rank 0, N=1) over a bounded sample, which
    is the first points of the GPU batch: the oracle's results on it are also
    the bench's parity check of the GPU output."""
    from oracle import oracle as O
    from inversekinematicsann_amd.robot.position_generator import random_dist
    budget = args.cpu_seconds
    if method == "ann":
        try:
            from threadpoolctl import threadpool_info
            threads = max([i.get("num_threads", 1) for i in threadpool_info()
                           if i.get("user_api") == "blas"] or [1])
        except Exception:  # noqa: BLE001
            threads = os.cpu_count() or 1
        from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                             REFERENCE_Y_SCALER as YS,
                                                             glorot_model)
        m = glorot_model(ANN_DIMS, seed=0)
        chunk = CPU_SAMPLE["ann"] if sample_pts is None else min(CPU_SAMPLE["ann"],
                                                                   len(sample_pts))
        pts = sample_pts[:chunk] if sample_pts is not None else random_dist(chunk, seed=99)
        # timed in 8192-point batches (cache-sized: the numpy MLP's best rate), cycling
        # through the sample; the first full pass is the parity reference
        bs = 8192
        starts = list(range(0, chunk, bs))
        first = np.empty((chunk, 4), np.float32)
        done, t0, k = 0, time.perf_counter(), 0
        while True:
            b0 = starts[k % len(starts)]
            out = O.ann_forward(pts[b0:b0 + bs], m.weights, m.biases, m.activations, XS.mean,
                                XS.scale, YS.mean, YS.scale, compute=np.float32)
            if k < len(starts):
                first[b0:b0 + bs] = out
            done += out.shape[0]
            k += 1
            if k >= len(starts) and time.perf_counter() - t0 >= budget:
                break
        el = time.perf_counter() - t0
        res = {"value": done / el, "unit": "IK solutions/s", "cores": threads, "kind": "port",
               "host_cpu": _host_cpu(),
               "sample": f"{done} points (the GPU batch's first {chunk}, cycled) in "
                         f"{bs}-point batches, numpy fp32 MLP (oracle.ann_forward) on "
                         f"{threads} BLAS threads, {el:.1f} s"}
        if gpu_out is not None:
            d = float(np.abs(gpu_out["ang"][:chunk].astype(np.float64) - first).max())
            res["parity"] = {"points": chunk, "max_abs_diff_vs_oracle_fp32": d,
                             "tolerance": 1e-5, "ok": d <= 1e-5}
        res["_ref"] = first  # for the other ANN modes' parity (dropped before printing)
        return res
    chunk = CPU_SAMPLE["fabrik"] if sample_pts is None else min(CPU_SAMPLE["fabrik"],
                                                                  len(sample_pts))
    pts = sample_pts[:chunk] if sample_pts is not None else random_dist(chunk, seed=99)
    # the C oracle on the host's share of cores, one slice of the chunk per thread
    # (ctypes releases the GIL for the call)
    from concurrent.futures import ThreadPoolExecutor
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1),
                         os.cpu_count() or 1))
    parts = np.array_split(np.arange(chunk), threads)
    done, t0, first = 0, time.perf_counter(), None
    with ThreadPoolExecutor(threads) as pool:
        while True:
            outs = list(pool.map(lambda ix: O.fabrik_ikine(pts[ix], args.tol, args.max_iter),
                                 parts))
            out = tuple(np.concatenate([o[k] for o in outs]) for k in range(4))
            first = out if first is None else first
            done += chunk
            if time.perf_counter() - t0 >= budget:
                break
    el = time.perf_counter() - t0
    res = {"value": done / el, "unit": "IK solutions/s", "cores": threads, "kind": "port",
           "host_cpu": _host_cpu(),
           "sample": f"{done} points (the GPU batch's first {chunk}, repeated), C oracle "
                     f"(oracle/ik_oracle.c, scalar) on {threads} threads, one slice of the "
                     f"chunk each, tol {args.tol:g}/{args.max_iter}, {el:.1f} s"}
    if gpu_out is not None:
        ang_ref, it_ref = first[0], first[1]
        d = float(np.abs(gpu_out["ang"][:chunk] - ang_ref).max())
        same = int((gpu_out["iters"][:chunk] == it_ref).sum())
        res["parity"] = {"points": chunk, "max_abs_diff": d, "tolerance": 1e-5,
                         "iters_equal": same, "ok": d <= 1e-5 and same == chunk}
    return res


def _config_ref(method, total, world, tol, max_iter):
    """Which BASELINE.json config a line measures (configs[0] is the CPU plumbing)."""
    if method == "ann":
        if total >= 10_000_000 and world > 1:
            return "configs[3]"
        return "configs[1]" if total == 1_000_000 * world else None
    if method == "fabrik":
        if (tol, max_iter) == (1e-5, 200) and total >= 10_000_000 and world > 1:
            return "configs[4]"
        return "configs[2]" if (tol, max_iter) == (1e-3, 100) and total == 1_000_000 * world \
            else None
    return None


STRONG_POINTS = 10_000_000  # configs[3] / configs[4]: 10M points over the N GPUs


def strong_legs():
    """The N > 1 strong-scaling legs: secondary key -> runner.
    Their keys end in '_strong10M'; the method and settings are in the name."""
    return {"ann_strong10M": lambda j, a: run_ann(j, a, mode="fp32"),
            "fabrik_tol1e-5_strong10M": lambda j, a: run_fabrik(j, a, tol=1e-5, max_iter=200)}


def leg_settings(key, args):
    """(method, tol, max_iter) a secondary key measures."""
    method = "fabrik" if key.startswith("fabrik") else ("ann" if key.startswith("ann") else key)
    if key.startswith("fabrik_tol1e-5"):
        return method, 1e-5, 200
    return method, args.tol, args.max_iter


def secondary_entry(key, r2, total, world, args):
    """One method's entry under the line's 'secondary', labelled with the
    BASELINE.json config it measures (_config_ref), if any."""
    e = {"value": r2.get("total", total) / (r2["ms_per_step"] / 1e3),
         "unit": r2.get("unit", "IK solutions/s"),
         "ms_per_step": r2["ms_per_step"], "dtype": r2["dtype"],
         "roofline": r2["roofline"], "workload": r2["workload"],
         "kernels_ms": r2["kernels"], "total_points": r2.get("total", total),
         **{k: r2[k] for k in ("max_fk_err", "mean_fk_err", "p99_fk_err", "mean_iters",
                               "n_capped", "end_to_end", "gather_chunks", "gather_ms", "cold",
                               "gather_check", "order_table", "gathered_bytes_per_row")
            if k in r2}}
    method, tol, max_iter = leg_settings(key, args)
    if method == "ann" and key not in ("ann", "ann_strong10M"):
        return e  # the split modes: no BASELINE config names them
    cref = _config_ref(method, total, world, tol, max_iter)
    if cref:
        e["baseline_config"] = cref
    return e


DRIVER_TIMEOUT_S = 600  # the driver's limit on one bench.py run (BENCH_r05.json timeout_s)
# measured per-step times at 1M points per rank (profiles/r05/lease_bench_default.json)
LEG_STEP_MS = {"ann": 39.2, "fabrik": 0.36, "fabrik_tol1e-5": 0.51, "ann_bf16x6": 21.9,
               "ann_fp16x3": 12.7, "fk": 0.45}  # (fk: FK_BATCH_FACTOR x the points)
E2E_BYTES_PER_POINT = {"ann": 24 + 16, "fabrik": 24 + 32}
PCIE_BYTES_PER_S = 50e9   # tools/pcie_probe.py: ~55 GB/s, the directions do not overlap
STARTUP_S = 120.0         # first `import torch` + HIP init on a fresh box (1-2 min)
RCCL_INIT_S = 30.0        # communicator setup on the success path (bounded by the deadline)
BATCH_GEN_S_PER_M = 0.2   # random_dist, seconds per million points (1.4 s for 10M here)


def wall_budget(world, steps, warmup, rccl_timeout_s=120.0, points=1_000_000, cpu_seconds=10.0):
    """An upper estimate of one `bench.py --gpus N` run's wall time, in seconds,
    by leg (the driver's first N = 8 run must fit its 600 s
    limit).  Each leg: W warm-up + TIMING_LEAD + TIMING_REPS event-timed + K timed steps, the
    untimed gather check (N > 1: two parts re-solved), 20 end-to-end calls each
    way (pinned / pageable, the whole batch through PCIe), and its batch
    generation; plus start-up, RCCL init and, at N > 1, the two strong legs on
    10M points.  `stall_path_s`: the longest a run whose collective never
    completes can last before IKHIP_RCCL_TIMEOUT_S aborts it."""
    total = points * world
    per_rank_m = points / 1e6
    legs = {}
    for key, ms in LEG_STEP_MS.items():
        n_steps = warmup + TIMING_LEAD + TIMING_REPS + steps + (2 if world > 1 else 0)
        t = n_steps * ms * per_rank_m / 1e3
        method = "fabrik" if key.startswith("fabrik") else ("ann" if key.startswith("ann") else None)
        if method:
            e2e = (ms * per_rank_m / 1e3 + total * E2E_BYTES_PER_POINT[method] / PCIE_BYTES_PER_S)
            t += 2 * 20 * e2e
        if method == "fabrik":
            t += BATCH_GEN_S_PER_M * total / 1e6 + 6 * ms * per_rank_m / 1e3  # warm batch + cold
        legs[key] = t
    if world > 1:
        sm = STRONG_POINTS / world / 1e6
        for key, base in (("ann_strong10M", "ann"), ("fabrik_tol1e-5_strong10M", "fabrik_tol1e-5")):
            n_steps = warmup + TIMING_LEAD + TIMING_REPS + steps + 2
            legs[key] = (n_steps * LEG_STEP_MS[base] * sm / 1e3
                         + BATCH_GEN_S_PER_M * STRONG_POINTS / 1e6
                         + (BATCH_GEN_S_PER_M * STRONG_POINTS / 1e6 if base.startswith("fabrik")
                            else 0.0))
    fixed = {"startup": STARTUP_S, "rccl_init": RCCL_INIT_S if world > 1 else 0.0,
             "batch": BATCH_GEN_S_PER_M * total / 1e6, "model_loads": 4 * 2.0,
             # rank 0 at N = 1: the ANN and FABRIK oracles, cpu_seconds each (+ one pass)
             "cpu_baseline": 2 * (cpu_seconds + 2.0) if world == 1 else 0.0}
    total_s = sum(legs.values()) + sum(fixed.values())
    return {"legs_s": legs, "fixed_s": fixed, "total_s": total_s,
            "stall_path_s": total_s + rccl_timeout_s,
            "limit_s": DRIVER_TIMEOUT_S}


def strong_job(ctx, sc, world, rank, total):
    """The configs[3] / configs[4] batch (random_dist, seed 1) on every rank, this
    rank's shard of it, on the same context and communicator as the headline."""
    import torch
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(total, seed=1)
    lo, hi = D.shard_bounds(total, world, rank)
    return Job(ctx, sc, pts, torch.from_numpy(pts).cuda(), lo, hi, world)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        # a line labelled with one GPU count must measure that many ranks
        print(f"bench.py: --gpus {args.gpus} but {world} rank(s) (WORLD_SIZE); launch N > 1 "
              f"as `python bench.py --gpus N` (it starts the ranks itself) or with "
              f"torch.distributed.run --nproc-per-node N", file=sys.stderr)
        sys.exit(2)
    import torch
    if os.environ.get("IKHIP_DIST_BACKEND", "rccl") != "gloo" and \
            torch.cuda.device_count() < world:
        print(f"bench.py: {world} ranks but {torch.cuda.device_count()} GPU(s) visible "
              "(one rank per GPU; IKHIP_DIST_BACKEND=gloo --gather 0 rehearses more ranks "
              "than GPUs)", file=sys.stderr)
        sys.exit(2)
    world, rank, local = dist_setup(args)
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.robot.position_generator import random_dist
    strong = args.total_points > 0
    total = args.total_points if strong else args.points * world
    # the global batch, identical on every rank (seed 0; seed 1 from 10M)
    pts = random_dist(total, seed=1 if total >= 10_000_000 else 0)
    dpts = torch.from_numpy(pts).cuda()
    lo, hi = D.shard_bounds(total, world, rank)
    ctx = _native.Context(local)
    # one non-default stream shared by the library and torch's events
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    sc, rccl_fallback = None, None
    if world > 1 and args.gather:
        sc, rccl_fallback = open_sharded(ctx, world, rank)
    job = Job(ctx, sc, pts, dpts, lo, hi, world)
    other_modes = [m for m in ("fp32", "bf16x6", "fp16x3") if m != args.ann_mode]
    runners = {"ann": lambda j, a: run_ann(j, a, mode=args.ann_mode), "fabrik": run_fabrik,
               # configs[4]'s divergent-iteration stress settings on the same batch
               "fabrik_tol1e-5": lambda j, a: run_fabrik(j, a, tol=1e-5, max_iter=200),
               "fk": run_fk}
    for om in other_modes:
        runners[f"ann_{om}"] = (lambda mm: lambda j, a: run_ann(j, a, mode=mm))(om)
    res = runners[args.method](job, args)
    outputs = {args.method: res["outputs"]}
    checks = {args.method: res.get("gather_check")}
    secondary = {}
    if args.secondary and args.method != "fk":
        others = (["fabrik", "fabrik_tol1e-5"] + [f"ann_{om}" for om in other_modes] + ["fk"]
                  if args.method == "ann" else ["ann", "fabrik_tol1e-5", "fk"])
        if args.method == "fabrik" and (args.tol, args.max_iter) == (1e-5, 200):
            others.remove("fabrik_tol1e-5")
        for other in others:
            r2 = runners[other](job, args)
            checks[other] = r2.get("gather_check")
            secondary[other] = secondary_entry(other, r2, total, world, args)
            outputs[other] = r2["outputs"]
    if world > 1 and not strong and args.strong_legs and args.method != "fk":
        # configs[3] / configs[4] as BASELINE.json states them: the 10M-point seed-1
        # batch sharded over the N ranks (strong scaling), beside the weak headline
        sjob = strong_job(ctx, sc, world, rank, STRONG_POINTS)
        sargs = argparse.Namespace(**{**vars(args), "end_to_end": 0, "cold": 0})
        for key, fn in strong_legs().items():
            r2 = fn(sjob, sargs)
            checks[key] = r2.get("gather_check")
            secondary[key] = secondary_entry(key, r2, STRONG_POINTS, world, sargs)
            secondary[key]["scaling"] = "strong"
            del r2
        del sjob
    gcheck, exit_code = gather_verdict(checks)
    value = res.get("total", total) / (res["ms_per_step"] / 1e3)
    line = {
        "metric": METRIC, "value": value, "unit": res.get("unit", "IK solutions/s"), "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
        "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
        "dtype": res["dtype"],
        "data": "synthetic: random_dist points (truncated normal sd 0.5 in the workspace box; "
                "one global batch, seed 0, seed 1 from 10M points); ANN weights random "
                "Glorot-uniform of the reference architecture (the reference .h5 is not "
                "shipped); reference StandardScaler constants",
        "config": {"workload": res["workload"],
                   "baseline_config": _config_ref(args.method, total, world, args.tol,
                                                  args.max_iter),
                   "points_per_gpu": hi - lo, "total_points": total,
                   "parallelism": f"dp{world}", "method": args.method,
                   "ann_mode": args.ann_mode if args.method == "ann" else None,
                   # a gloo rehearsal with more ranks than GPUs: the ranks share a
                   # device, so per-rank kernel durations (and fracs) are not one GPU's
                   **({"devices_shared": world // max(1, torch.cuda.device_count())}
                      if world > torch.cuda.device_count() else {}),
                   "all_gather_in_step": sc is not None,
                   **({"rccl_fallback": rccl_fallback} if rccl_fallback else {}),
                   "collective": ("RCCL all-gathers inside libikhip (ik_*_solve_sharded): each "
                                  "chunk's angles (+ FABRIK iterations) gathered in place under "
                                  "the next chunk's solve; per-rank stats tail + FK-error "
                                  "histogram with the last chunk; FK errors stay local")
                   if sc is not None else None,
                   "n_ranks_rccl": sc.info()[0] if sc is not None else None,
                   "gather_chunks": res.get("gather_chunks"),
                   "gather_check": gcheck,
                   "strong_legs": ({k: secondary[k].get("baseline_config") for k in strong_legs()
                                    if k in secondary} or None),
                   "tol": args.tol if args.method == "fabrik" else None,
                   "max_iter": args.max_iter if args.method == "fabrik" else None},
        "roofline": res["roofline"],
        "event_ms_per_step": res["event_ms_per_step"],
        "kernels_ms": res["kernels"],
    }
    for k in ("max_fk_err", "mean_fk_err", "p99_fk_err", "fk_err_note", "mean_iters", "n_capped",
              "end_to_end", "gather_ms", "cold", "order_table"):
        if k in res:
            line[k] = res[k]
    if secondary:
        line["secondary"] = secondary
    if rank == 0 and world == 1 and args.cpu_seconds > 0 and args.method != "fk":
        def host(o):
            return {k: v[:max(CPU_SAMPLE.values())].cpu().numpy() for k, v in o.items()}
        line["cpu_baseline"] = cpu_baseline(args.method, args, pts, host(outputs[args.method]))
        if args.secondary:
            other = "fabrik" if args.method == "ann" else "ann"
            line["secondary"][other]["cpu_baseline"] = cpu_baseline(other, args, pts,
                                                                    host(outputs[other]))
        if args.method == "ann" and args.secondary:
            # the other ANN modes against the same oracle sample as the headline
            ref = line["cpu_baseline"].get("_ref")
            for om in other_modes:
                key = f"ann_{om}"
                if key in line["secondary"] and ref is not None:
                    d = float(np.abs(host(outputs[key])["ang"][:ref.shape[0]]
                                     .astype(np.float64) - ref).max())
                    line["secondary"][key]["parity"] = {
                        "points": int(ref.shape[0]), "max_abs_diff_vs_oracle_fp32": d,
                        "tolerance": 1e-5, "ok": d <= 1e-5}
        for v in [line["cpu_baseline"]] + [x.get("cpu_baseline") for x in
                                           line.get("secondary", {}).values()]:
            if isinstance(v, dict):
                v.pop("_ref", None)
    if sc is not None:
        sc.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
        if exit_code:
            print("bench.py: gathered rows differ from their plain re-solve "
                  f"({json.dumps(gcheck)})", file=sys.stderr)
    if _dist_on():
        import torch.distributed as dist
        dist.destroy_process_group()
    return exit_code


if __name__ == "__main__":
    rc = maybe_launch()
    if rc is not None:
        sys.exit(rc)
    sys.exit(main())
