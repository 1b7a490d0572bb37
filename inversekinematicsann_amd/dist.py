"""Multi-GPU batch sharding (one process per GPU, torch.distributed over RCCL).

The reference "scales" by running competing-consumer RPC workers, one message
at a time (rpc_broker.py:55-104, README.md:11).  Here every point is
independent, so a batch is split into contiguous shards, one per rank
(rank r owns [floor(r N / g), floor((r+1) N / g))), each rank solves its shard
on its own GPU with no communication, and -- only when the caller wants the
whole result on every rank -- one all_gather of the per-point result rows
(padded to equal shard length) reassembles the batch over xGMI.  The
per-batch error reduction (first out-of-reach / first failing index) rides on
a tiny all_reduce so the reference's "lowest index raises" rule holds across
shards.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    return (n * rank) // world, (n * (rank + 1)) // world


def max_shard(n: int, world: int) -> int:
    return max(shard_bounds(n, world, r)[1] - shard_bounds(n, world, r)[0] for r in range(world))


def gather_rows(local, n_total: int, group=None):
    """All-gather the row-blocks of every rank into the full (n_total, ...)
    tensor on every rank.  `local` holds this rank's shard_bounds rows."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    m = max_shard(n_total, world)
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = torch.empty((world * m,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    parts = []
    for r in range(world):
        lo, hi = shard_bounds(n_total, world, r)
        parts.append(out[r * m: r * m + (hi - lo)])
    return torch.cat(parts, 0)


def reduce_first_index(idx: int, group=None, device=None) -> int:
    """Global minimum of per-rank 'first failing' indices (-1 = none)."""
    import torch
    import torch.distributed as dist
    big = np.iinfo(np.int64).max
    t = torch.tensor([big if idx < 0 else idx], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    v = int(t.item())
    return -1 if v == big else v


def solve_sharded(points_global, solver: Callable, n_out: int, out_dtype, *, gather=True,
                  group=None, device=None):
    """Shard `points_global` (N x 3, identical on every rank) across the ranks,
    run `solver(local_points) -> (local_out (n_local x n_out), first_oob_local,
    first_err_local, err_code)` on this rank's shard and optionally all_gather
    the rows.  Returns (out, first_oob, first_err, err_code) with global
    indices; out is the full batch if gather else this rank's shard."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = int(points_global.shape[0])
    lo, hi = shard_bounds(n, world, rank)
    local_out, oob, err, code = solver(points_global[lo:hi])
    oob_g = reduce_first_index(oob + lo if oob >= 0 else -1, group, device)
    err_g = reduce_first_index(err + lo if err >= 0 else -1, group, device)
    # the code of the globally first error travels with its owner
    c = torch.tensor([code if (err >= 0 and err + lo == err_g) else 0], dtype=torch.int32,
                     device=device)
    dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
    if not torch.is_tensor(local_out):
        local_out = torch.as_tensor(local_out, device=device)
    if gather:
        out = gather_rows(local_out.to(out_dtype).reshape(hi - lo, n_out), n, group)
    else:
        out = local_out
    return out, oob_g, err_g, int(c.item())


def gpu_solver(method: str, ctx, tol: float = 1e-3, max_iter: int = 100,
               check_limits: bool = True) -> Callable:
    """A solver for solve_sharded backed by libikhip on this rank's GPU:
    device tensors in, device tensors out, no host round trip."""
    import torch
    from . import _native

    def run(local_pts):
        n = local_pts.shape[0]
        flags = _native.IK_F_DEVICE | (0 if check_limits else _native.IK_F_NO_LIMITS)
        if method == "fabrik":
            ang = torch.empty((n, 4), dtype=torch.float64, device=local_pts.device)
            st = ctx.fabrik_solve_device(local_pts, ang, None, None, tol, max_iter, flags=flags)
        else:
            ang = torch.empty((n, 4), dtype=torch.float32, device=local_pts.device)
            st = ctx.ann_solve_device(local_pts, ang, None, flags=flags)
        return ang, st.first_oob, st.first_err, st.first_err_code

    return run


def init_from_env(backend: Optional[str] = None):
    """torch.distributed init for torchrun-launched ranks (MASTER_ADDR etc.)."""
    import os
    import torch
    import torch.distributed as dist
    if dist.is_initialized():
        return
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
