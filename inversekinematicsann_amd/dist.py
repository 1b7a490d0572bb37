"""Multi-GPU batch sharding: one process per GPU, libikhip's own RCCL over xGMI.

The reference "scales" by running competing-consumer RPC workers, one message
at a time (rpc_broker.py:55-104, README.md:11).  Here every point is
independent, so one batch is split into contiguous shards (rank r owns
[floor(r N / g), floor((r+1) N / g)), ik_shard_range), each rank solves its
shard on its own GPU, and ONE all-gather inside the library
(ik_*_solve_sharded) delivers every rank's result rows plus a tail record of
its stats, so every rank ends with the whole batch and the whole batch's stats
(the lowest global failing index -- the reference's sequential exception
precedence -- iteration sums, FK-error max/sum) without any other collective.

torch.distributed is only the control plane here: it hands rank 0's RCCL
unique id to the other ranks (and gives bench.py its barrier); the data path
is the library's communicator, as a C-ABI caller without torch would use it
(INTEGRATION.md).

The host-side mirror of the gather protocol (pack_block / unpack_blocks, the
library's layout and tail records) is what the library does on the device and
in its host-pointer path; the CPU tests drive it over gloo with world size 2.
"""
from __future__ import annotations

import ctypes
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import _native


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Rank's rows [begin, end) of an n-point batch (= ik_shard_range)."""
    return (n * rank) // world, (n * (rank + 1)) // world


def exchange_unique_id(rank: int, broadcast: Callable[[Optional[bytes]], bytes]) -> bytes:
    """Rank 0 asks the library for an RCCL unique id; `broadcast` hands it to
    every rank (any transport: torch.distributed, MPI, a file)."""
    uid = _native.comm_unique_id() if rank == 0 else None
    return broadcast(uid)


def torch_broadcast(uid: Optional[bytes]) -> bytes:
    """exchange_unique_id's transport over an initialised torch.distributed group."""
    import torch.distributed as dist
    box = [uid]
    dist.broadcast_object_list(box, src=0)
    return box[0]


class ShardedContext:
    """A libikhip context bound to an RCCL communicator of `world` ranks.
    ann / fabrik take the WHOLE batch on every rank (host numpy arrays, or
    device tensors via the *_device methods) and return the whole batch's
    results and stats."""

    def __init__(self, ctx: _native.Context, world: int, rank: int, uid: bytes):
        self.ctx = ctx
        self.world = int(world)
        self.rank = int(rank)
        ctx.comm_init(self.world, self.rank, uid)

    def close(self):
        self.ctx.comm_destroy()

    def ann(self, pts, check_limits=True, want_fk_err=False):
        return self.ctx.ann_solve_sharded(pts, check_limits, want_fk_err)

    def fabrik(self, pts, tol=1e-3, max_iter=100, check_limits=True, want_fk_err=False):
        return self.ctx.fabrik_solve_sharded(pts, tol, max_iter, check_limits, want_fk_err)

    def ann_device(self, pts, ang, fk_err=None, flags=_native.IK_F_DEVICE):
        return self.ctx.ann_solve_sharded_device(pts, ang, fk_err, flags)

    def fabrik_device(self, pts, ang, iters=None, fk_err=None, tol=1e-3, max_iter=100,
                      flags=_native.IK_F_DEVICE):
        return self.ctx.fabrik_solve_sharded_device(pts, ang, iters, fk_err, tol, max_iter, flags)


def init_from_env(ctx: _native.Context) -> ShardedContext:
    """For torchrun-launched ranks (RANK / WORLD_SIZE / MASTER_*): a gloo control
    group for the id exchange, then the library's RCCL communicator."""
    import os
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    uid = exchange_unique_id(rank, torch_broadcast)
    return ShardedContext(ctx, world, rank, uid)


# ---- host mirror of the gather protocol ------------------------------------------
def pack_block(layout: _native.GatherLayout, regions: Sequence[np.ndarray],
               tail: _native.ShardTail) -> np.ndarray:
    """One rank's block of the all-gather (uint8): region q's rows at offset[q],
    then the tail record, as the library lays it out in its send buffer."""
    blk = np.zeros(layout.block_bytes, np.uint8)
    for q, arr in enumerate(regions):
        raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        if raw.size > layout.shard * layout.row_bytes[q]:
            raise ValueError(f"region {q}: {raw.size} bytes exceed the layout's shard")
        blk[layout.offset[q]: layout.offset[q] + raw.size] = raw
    tb = np.frombuffer(bytes(tail), np.uint8)
    blk[layout.tail_offset: layout.tail_offset + tb.size] = tb
    return blk


def unpack_blocks(layout: _native.GatherLayout, blocks: np.ndarray, n: int,
                  dtypes: Sequence[np.dtype], widths: Sequence[int]):
    """Every rank's block (world x block_bytes uint8) -> each region's rows of the
    whole batch in point order, and the tails (what the library's unpack kernel
    and per-rank D2H copies do)."""
    world = blocks.shape[0]
    outs: List[np.ndarray] = [np.empty((n, w), dt) for dt, w in zip(dtypes, widths)]
    tails = []
    for r in range(world):
        lo, hi = shard_bounds(n, world, r)
        for q, out in enumerate(outs):
            rb = layout.row_bytes[q]
            raw = blocks[r, layout.offset[q]: layout.offset[q] + (hi - lo) * rb]
            out[lo:hi] = raw.view(out.dtype).reshape(hi - lo, out.shape[1])
        t = _native.ShardTail()
        ctypes.memmove(ctypes.addressof(t),
                       blocks[r, layout.tail_offset:].ctypes.data, ctypes.sizeof(t))
        tails.append(t)
    return outs, tails
