"""Collectives used by the map/reduce engine.

The reference reduces MRTask results up a binary tree of RPCs
(water/MRTask.java:reduce2 / dfork).  Here every reduce is a single
torch.distributed collective on the row-shard owners: all_reduce for
sufficient statistics (Gram matrices, centroid sums, leaf sums), a
feature-sharded reduce_scatter for tree histograms (each rank then scores
splits for its feature slice), and all_gather for small candidate records.
All helpers are no-ops at world size 1.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import cloud


def _rccl() -> bool:
    """True when the process group is NCCL (= RCCL over xGMI on ROCm); gloo
    (CPU clouds, or a one-GPU multi-rank rehearsal) lacks reduce_scatter /
    all_gather_into_tensor and takes the portable paths below."""
    return cloud.is_gpu() and dist.get_backend() == "nccl"


def allreduce_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    if not cloud.is_distributed():
        return t
    rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
    dist.all_reduce(t, op=rop)
    return t


def allreduce_many_(ts: list[torch.Tensor], op: str = "sum") -> list[torch.Tensor]:
    """Bucketed all-reduce: flatten same-dtype tensors into one buffer."""
    if not cloud.is_distributed() or not ts:
        return ts
    by_dtype: dict = {}
    for t in ts:
        by_dtype.setdefault(t.dtype, []).append(t)
    for dt, group in by_dtype.items():
        flat = torch.cat([g.reshape(-1) for g in group])
        allreduce_(flat, op)
        off = 0
        for g in group:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n
    return ts


def allreduce_scalar(x: float, op: str = "sum", dtype=torch.float64) -> float:
    if not cloud.is_distributed():
        return float(x)
    t = torch.tensor([x], dtype=dtype, device=cloud.device())
    allreduce_(t, op)
    return float(t.item())


def reduce_scatter_dim0(t: torch.Tensor) -> torch.Tensor:
    """Sum over ranks then return this rank's contiguous slice along dim 0
    (dim 0 must be divisible by world size)."""
    w = cloud.world()
    if w == 1:
        return t
    assert t.shape[0] % w == 0
    out = torch.empty((t.shape[0] // w,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if _rccl():
        dist.reduce_scatter_tensor(out, t.contiguous())
    else:  # gloo has no reduce_scatter: all_reduce + slice
        dist.all_reduce(t)
        out.copy_(t.view(w, -1, *t.shape[1:])[cloud.rank()])
    return out


def all_gather_dim0(t: torch.Tensor) -> torch.Tensor:
    w = cloud.world()
    if w == 1:
        return t
    out = torch.empty((t.shape[0] * w,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if _rccl():
        dist.all_gather_into_tensor(out, t.contiguous())
    else:
        parts = [torch.empty_like(t) for _ in range(w)]
        dist.all_gather(parts, t.contiguous())
        out = torch.cat(parts, 0)
    return out


def all_gather_var(t: torch.Tensor) -> torch.Tensor:
    """Gather variable-length dim-0 tensors from all ranks (concatenated)."""
    w = cloud.world()
    if w == 1:
        return t
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    ns = all_gather_dim0(n).tolist()
    m = max(ns)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    g = all_gather_dim0(pad)
    return torch.cat([g[i * m: i * m + ns[i]] for i in range(w)], 0)


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if cloud.is_distributed():
        dist.broadcast(t, src)
    return t


def broadcast_object(obj, src: int = 0):
    if not cloud.is_distributed():
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, device=cloud.device() if _rccl() else None)
    return lst[0]


def all_gather_object(obj) -> list:
    if not cloud.is_distributed():
        return [obj]
    out = [None] * cloud.world()
    dist.all_gather_object(out, obj)
    return out
