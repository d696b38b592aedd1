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

# Collective sequence tracing (H2O3_TRACE_COLL=<dir>): every rank appends one
# line per collective -- sequence number, op, shape, and the calling
# h2o3_amd frames -- to <dir>/coll_rank<r>.log.  Diffing two ranks' logs
# names the first call site where the SPMD sequences diverge (a rank-local
# branch around a collective), the usual cause of a multi-rank hang.
_TRACE = {"dir": None, "f": None, "seq": 0}


# Byte accounting (always on, negligible cost): payload bytes this rank hands
# to each collective, summed per (tag, op).  `tag(...)` scopes a region
# (e.g. "tree.L7"); `bytes_report()` / `reset_bytes()` read / clear the table.
# The payload is the tensor a rank contributes (all_gather: its slice;
# reduce_scatter / all_reduce: the full buffer; all_to_all: its send buffer).
_BYTES: dict = {}
_TAG = ["-"]


class tag:
    def __init__(self, name):
        self.name = str(name)

    def __enter__(self):
        _TAG.append(self.name)
        return self

    def __exit__(self, *a):
        _TAG.pop()


def bytes_report():
    return dict(_BYTES)


def reset_bytes():
    _BYTES.clear()


def _account(op, t):
    if t is None or not hasattr(t, "numel"):
        return
    k = (_TAG[-1], op)
    _BYTES[k] = _BYTES.get(k, 0) + t.numel() * t.element_size()


class CollectiveForbidden(RuntimeError):
    """A collective was issued inside `forbid()` (a read served off the
    SPMD executor must not join the cloud's collective sequence)."""


_guard = __import__("threading").local()


class forbid:
    """Thread-scoped guard: any collective issued by this thread inside the
    block raises CollectiveForbidden instead of running (rank 0's HTTP thread
    serves reads while the executor thread drives the cloud)."""

    def __enter__(self):
        self._prev = getattr(_guard, "on", False)
        _guard.on = True
        return self

    def __exit__(self, *a):
        _guard.on = self._prev


def _guard_check(op):
    if getattr(_guard, "on", False) and cloud.is_distributed():
        raise CollectiveForbidden(op)


def _trace(op, t=None):
    _guard_check(op)
    _account(op, t)
    d = _TRACE["dir"]
    if d is None:
        import os
        d = _TRACE["dir"] = os.environ.get("H2O3_TRACE_COLL", "")
    if not d:
        return
    import os
    import traceback
    if _TRACE["f"] is None:
        os.makedirs(d, exist_ok=True)
        _TRACE["f"] = open(os.path.join(d, f"coll_rank{cloud.rank()}.log"), "w", buffering=1)
    fr = [f"{os.path.basename(x.filename)}:{x.lineno}:{x.name}" for x in traceback.extract_stack()[:-2]
          if "h2o3_amd" in x.filename and "collectives.py" not in x.filename][-6:]
    shape = tuple(t.shape) if hasattr(t, "shape") else ""
    _TRACE["f"].write(f"{_TRACE['seq']} {op} {shape} {' < '.join(reversed(fr))}\n")
    _TRACE["seq"] += 1


def _rccl() -> bool:
    """True when the process group is NCCL (= RCCL over xGMI on ROCm)."""
    return cloud.is_gpu() and dist.get_backend() == "nccl"


def _tensor_coll(t) -> bool:
    """reduce_scatter_tensor / all_gather_into_tensor: RCCL, and gloo on CPU
    tensors (so the CPU multi-rank tests run the RCCL call sequence); gloo
    with device tensors (a one-GPU multi-rank rehearsal) lacks them."""
    return _rccl() or t.device.type == "cpu"


def allreduce_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    if not cloud.is_distributed():
        return t
    rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
    _trace("all_reduce", t)
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
    _trace("reduce_scatter", t)
    if _tensor_coll(t):
        dist.reduce_scatter_tensor(out, t.contiguous())
    else:
        dist.all_reduce(t)
        out.copy_(t.view(w, -1, *t.shape[1:])[cloud.rank()])
    return out


def all_gather_dim0(t: torch.Tensor) -> torch.Tensor:
    w = cloud.world()
    if w == 1:
        return t
    out = torch.empty((t.shape[0] * w,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    _trace("all_gather", t)
    if _tensor_coll(t):
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


def all_to_all_single_(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None) -> torch.Tensor:
    """Personalised exchange along dim 0 (RCCL alltoall / gloo): rank r's
    rows in_splits[d] go to rank d, `out` receives out_splits[s] rows from
    every rank s in rank order."""
    _trace("all_to_all_single", inp)
    if not cloud.is_distributed():
        out.copy_(inp)
        return out
    if _tensor_coll(inp):
        dist.all_to_all_single(out, inp, out_splits, in_splits)
    else:   # gloo with device tensors: stage through host memory
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
        out.copy_(o)
    return out


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if cloud.is_distributed():
        _trace("broadcast", t)
        dist.broadcast(t, src)
    return t


def broadcast_object(obj, src: int = 0):
    if not cloud.is_distributed():
        return obj
    lst = [obj]
    _trace("broadcast_object")
    dist.broadcast_object_list(lst, src=src, device=cloud.device() if _rccl() else None)
    return lst[0]


def all_gather_object(obj) -> list:
    if not cloud.is_distributed():
        return [obj]
    out = [None] * cloud.world()
    _trace("all_gather_object")
    dist.all_gather_object(out, obj)
    return out
