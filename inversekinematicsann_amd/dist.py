"""Multi-GPU batch sharding: one process per GPU, libikhip's own RCCL over xGMI.

The reference "scales" by running competing-consumer RPC workers, one message
at a time (rpc_broker.py:55-104, README.md:11).  Here every point is
independent, so one batch is split over the ranks in C chunks of g parts (rank r
owns rows [(c g + r) S, (c g + r + 1) S) of chunk c, S = ceil(n / (C g)),
ik_shard_plan_of / ik_shard_part), each rank solves its parts on its own GPU
straight into their global rows of the output arrays, and the library
all-gathers every chunk IN PLACE while the next one is solved
(ik_*_solve_sharded).  Every rank ends with the whole batch's angles (and
FABRIK iteration counts) and, from a tail record that rides with the last
chunk, the whole batch's stats -- the lowest global failing index (the
reference's sequential exception precedence), iteration sums, FK-error
max / sum / histogram -- without any other collective.  Per-point FK errors
stay on their rank.

torch.distributed is only the control plane here: it hands rank 0's RCCL
unique id to the other ranks (and gives bench.py its barrier); the data path
is the library's communicator, as a C-ABI caller without torch would use it
(INTEGRATION.md).

The host-side mirror of the protocol (plan_of / part_bounds and
gather_in_place, the library's split and its in-place chunk gathers with the
ragged last chunk staged) is what the library does on the device; the CPU tests
drive it over gloo with world sizes 2 and 3.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import _native


def plan_of(n: int, world: int, chunks: int = 1) -> Tuple[int, int, int]:
    """(chunks holding rows, part rows S, rows of the full chunks) = ik_shard_plan_of."""
    cg = chunks * world
    S = -(-n // cg) if n > 0 else 0
    per = S * world
    C = -(-n // per) if n > 0 else 0
    full = (n // per) * per if per > 0 else 0
    return C, S, full


def part_bounds(n: int, world: int, chunks: int, rank: int, chunk: int) -> Tuple[int, int]:
    """Rank's rows [begin, end) of chunk `chunk` (= ik_shard_part)."""
    _, S, _ = plan_of(n, world, chunks)
    lo = (chunk * world + rank) * S
    return min(lo, n), min(lo + S, n)


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Rank's rows [begin, end) of an n-point batch in one chunk (= ik_shard_range)."""
    return part_bounds(n, world, 1, rank, 0)


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
    results and stats (fk_err: this rank's rows only)."""

    def __init__(self, ctx: _native.Context, world: int, rank: int, uid: bytes):
        self.ctx = ctx
        self.world = int(world)
        self.rank = int(rank)
        ctx.comm_init(self.world, self.rank, uid)

    @classmethod
    def loopback(cls, ctx: _native.Context, world: int, rank: int) -> "ShardedContext":
        """TEST-ONLY: rank `rank` of `world` on one GPU without RCCL
        (ik_comm_init_loopback); see loopback_bytes for the other ranks' rows."""
        self = cls.__new__(cls)
        self.ctx, self.world, self.rank = ctx, int(world), int(rank)
        ctx.comm_init_loopback(self.world, self.rank)
        return self

    def close(self):
        self.ctx.comm_destroy()

    def info(self):
        """(ranks, rank, chunks of the last call) as the library holds them."""
        return self.ctx.comm_info()

    def set_chunks(self, chunks: int):
        self.ctx.comm_set_chunks(chunks)

    def fk_err_quantile(self, q: float) -> float:
        return self.ctx.fk_err_quantile(q)

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


# ---- host mirror of the protocol ---------------------------------------------
def loopback_bytes(slot: int, offsets: np.ndarray) -> np.ndarray:
    """ik_loopback_byte for many offsets: the bytes a loopback communicator's
    all-gather writes into rank `slot`'s part (numpy restatement)."""
    o = np.asarray(offsets, np.uint64)
    v = (np.uint64(slot * 29) + o * np.uint64(13) + (o >> np.uint64(7))) & np.uint64(0xFFFFFFFF)
    return ((v ^ np.uint64(0xA5)) & np.uint64(0xFF)).astype(np.uint8)


def loopback_expected(n: int, world: int, rank: int, chunks: int, row_bytes: int,
                      own: np.ndarray) -> np.ndarray:
    """The whole gathered array (n rows of row_bytes) as rank `rank` of a loopback
    communicator holds it after a sharded call: its own parts from `own` (the
    full-batch rows a plain solve gives), every other rank's part filled with
    loopback_bytes of (that rank, byte offset within its part)."""
    own = np.ascontiguousarray(own).view(np.uint8).reshape(n, row_bytes)
    out = np.empty((n, row_bytes), np.uint8)
    C, _, _ = plan_of(n, world, chunks)
    for c in range(C):
        for r in range(world):
            b, e = part_bounds(n, world, chunks, r, c)
            if e <= b:
                continue
            if r == rank:
                out[b:e] = own[b:e]
            else:
                out[b:e] = loopback_bytes(r, np.arange((e - b) * row_bytes)).reshape(-1, row_bytes)
    return out

def fkhist(err: np.ndarray) -> np.ndarray:
    """A rank's FK-error histogram (IK_FKHIST_BINS uint32), numpy restatement of
    fkhist_bin: 16 bins per octave from the float64 exponent and top 4 mantissa
    bits; NaN / inf / negative values are not counted."""
    e = np.asarray(err, np.float64).reshape(-1)
    e = e[np.isfinite(e) & (e >= 0)]
    bits = np.abs(e).view(np.uint64)
    k = ((bits >> np.uint64(52)).astype(np.int64) - (1023 - 64)) * 16 + \
        ((bits >> np.uint64(48)) & np.uint64(15)).astype(np.int64)
    k = np.clip(k, 0, _native.IK_FKHIST_BINS - 1)
    return np.bincount(k, minlength=_native.IK_FKHIST_BINS).astype(np.uint32)


def hist_quantile(hists: Sequence[np.ndarray], q: float) -> float:
    """ik_fk_err_quantile from gathered histograms: the upper edge of the bin
    holding the ceil(q m)-th smallest of the m counted errors."""
    h = np.sum(np.stack([np.asarray(x, np.uint64) for x in hists]), axis=0)
    tot = int(h.sum())
    if tot == 0:
        return float("nan")
    want = max(1, int(np.ceil(q * tot)))
    b = int(np.searchsorted(np.cumsum(h), want))
    if b >= _native.IK_FKHIST_BINS - 1:
        return float("inf")
    return float(np.ldexp(1.0 + (b % 16 + 1) / 16.0, b // 16 - 64))


def gather_in_place(n: int, world: int, rank: int, chunks: int,
                    solve_part: Callable[[int, int], Sequence[np.ndarray]],
                    outs: List[np.ndarray], all_gather: Callable[[np.ndarray, np.ndarray], None]):
    """The library's sharded call on host arrays: for every chunk, solve_part(b,
    e) gives this rank's rows of each gathered output, written at their global
    rows (or, in the ragged last chunk, at rank offset r S of a g S-row stage),
    then all_gather(send, recv) fills in every rank's rows in place -- recv is
    the chunk's g S rows and send the rank's S of them, as ncclAllGather's
    in-place mode.  Returns this rank's parts [(b, e)]."""
    C, S, _ = plan_of(n, world, chunks)
    parts = []
    for c in range(C):
        b, e = part_bounds(n, world, chunks, rank, c)
        cb = c * world * S
        staged = cb + world * S > n
        rows = solve_part(b, e) if e > b else [np.zeros((0,) + o.shape[1:], o.dtype)
                                                for o in outs]
        for out, r in zip(outs, rows):
            if staged:
                st = np.zeros((world * S,) + out.shape[1:], out.dtype)
                st[rank * S: rank * S + (e - b)] = r
                all_gather(st[rank * S:(rank + 1) * S], st)
                out[cb:n] = st[:n - cb]
            else:
                out[b:e] = r
                all_gather(out[b:e], out[cb:cb + world * S])
        parts.append((b, e))
    return parts
