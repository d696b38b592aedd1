"""Frame-level column ops on the HIP kernels of ops/csrc/frame.hip: batched
rollups (one launch and one host read for every column of a frame) and the
numeric block of the model matrix (tiled transpose with NA imputation and
standardization).  Reference: water/fvec/RollupStats.java, hex/DataInfo.java.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _native

_FLOATS = (torch.float32, torch.float64)


def _lib():
    lib = _native.get_lib("frame", required=False)
    if lib is not None and not getattr(lib, "_typed", False):
        P, I, LL = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
        lib.h2o_rollup_multi.argtypes = [P, I, LL, I, P, I, P, P]
        lib.h2o_expand_numeric.argtypes = [P, I, LL, P, P, P, P, I, I, I, P]
        lib._typed = True
    return lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _col_table(tensors, device):
    """FrCol {pointer, dtype, pad} per column (16 bytes, little endian)."""
    arr = np.zeros((len(tensors), 2), dtype=np.int64)
    arr[:, 0] = [t.data_ptr() for t in tensors]
    arr[:, 1] = [1 if t.dtype == torch.float64 else 0 for t in tensors]
    return torch.as_tensor(arr, device=device)


def batchable(v) -> bool:
    return (not v.on_host and v.data.is_cuda and v.data.dtype in _FLOATS and v.data.dim() == 1
            and v.data.is_contiguous())


def rollups_many(vecs) -> int:
    """Fill Vec._rollups for every eligible numeric device column of `vecs`
    (float32 / float64, row-sharded or replicated) in batched launches.
    Collective when the cloud has several ranks: every rank passes the same
    columns.  Returns the number of columns computed."""
    from ..core.vec import NUMERIC_TYPES
    from ..parallel import cloud
    from ..parallel import collectives as coll
    lib = _lib()
    if lib is None:
        return 0
    todo = [v for v in vecs if v._rollups is None and v.type in NUMERIC_TYPES and batchable(v)]
    if not todo:
        return 0
    done = 0
    # replicated columns (no collective) per length, then the row-sharded ones
    # as ONE group: every rank holds the same columns, so the batches and
    # their collectives line up even when the local lengths differ by rank
    groups = []
    rep = {}
    for v in todo:
        if v.replicated:
            rep.setdefault(int(v.data.numel()), []).append(v)
    groups += [(True, n, vs) for n, vs in sorted(rep.items())]
    sh = [v for v in todo if not v.replicated]
    uniform = len({int(v.data.numel()) for v in sh}) <= 1
    if sh and cloud.world() > 1:
        # every rank must take the same branch (the batch issues collectives);
        # replicated-only calls (possibly on one rank) issue none
        uniform = coll.allreduce_scalar(1.0 if uniform else 0.0, "min") > 0
    if sh:
        lens = {int(v.data.numel()) for v in sh}
        if uniform:
            groups.append((False, lens.pop(), sh))
        elif cloud.world() == 1:
            byn = {}
            for v in sh:
                byn.setdefault(int(v.data.numel()), []).append(v)
            groups += [(False, n, vs) for n, vs in sorted(byn.items())]
    for repl, n, vs in groups:
        for a in range(0, len(vs), 4096):
            chunk = vs[a:a + 4096]
            dev = chunk[0].data.device
            tab = _col_table([v.data for v in chunk], dev)
            nc = len(chunk)
            slices = max(1, min(128, -(-4096 // nc), -(-n // 4096)))
            part = torch.empty((nc, slices, 10), dtype=torch.float64, device=dev)
            dist = cloud.world() > 1 and not repl

            def run(pass_, mean_):
                if n > 0:
                    rc = lib.h2o_rollup_multi(_ptr(tab), nc, n, slices, None if mean_ is None else _ptr(mean_),
                                              pass_, _ptr(part), _stream())
                    if rc != 0:
                        raise RuntimeError(f"h2o_rollup_multi failed: {rc}")
                else:
                    part.zero_()
                    part[..., 8] = float(np.finfo(np.float64).max)
                    part[..., 9] = -float(np.finfo(np.float64).max)
            run(0, None)
            st = part[..., :8].sum(1)                                   # [nc, 8]: n, sum, -, counts
            mn, mx = part[..., 8].amin(1), part[..., 9].amax(1)
            if dist:
                coll.allreduce_(st)
                mm = torch.stack([mn, -mx], 1)
                coll.allreduce_(mm, "min")
                mn, mx = mm[:, 0], -mm[:, 1]
            cnt, s1, counts = st[:, 0], st[:, 1], st[:, 3:8]
            mean = torch.where(cnt > 0, s1 / torch.where(cnt > 0, cnt, torch.ones_like(cnt)), torch.zeros_like(cnt))
            mean = mean.contiguous()
            run(1, mean)                                                # exact-mean squared deviations
            m2 = part[..., 0].sum(1)
            if dist:
                coll.allreduce_(m2)
            out = torch.stack([cnt, mean, m2, mn, mx], 1)
            host = torch.cat([out, counts], 1).cpu().numpy()   # one read for the batch
            for v, h in zip(chunk, host):
                c, mu, ss, lo, hi, na, z, pi, ni_, notint = h.tolist()
                if c > 1:
                    sigma = math.sqrt(max(ss, 0.0) / (c - 1))
                else:
                    sigma = float("nan") if c == 0 else 0.0
                if c == 0:
                    lo = hi = mu = float("nan")
                v._rollups = dict(min=lo, max=hi, mean=mu, sigma=sigma, nacnt=int(na), zeros=int(z),
                                  isInt=notint == 0, nrow=v.nrow(), pinfs=int(pi), ninfs=int(ni_))
            done += nc
    return done


def expand_numeric(tensors, plug, mean, sd, X, base) -> bool:
    """X[:, base + j] = ((nan -> plug[j]) x_j - mean[j]) / sd[j] for the
    column tensors (float32 / float64, length X.shape[0]); False when the
    kernel does not apply (the caller then runs its torch loop)."""
    lib = _lib()
    if lib is None or not tensors or not X.is_cuda or X.dtype not in _FLOATS or not X.is_contiguous():
        return False
    n = X.shape[0]
    if any(not (t.is_cuda and t.dtype in _FLOATS and t.dim() == 1 and t.numel() == n and t.is_contiguous())
           for t in tensors):
        return False
    dev = X.device
    tab = _col_table(tensors, dev)
    f64 = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
    pl, mu, s_ = f64(plug), f64(mean), f64(sd)
    rc = lib.h2o_expand_numeric(_ptr(tab), len(tensors), n, _ptr(pl), _ptr(mu), _ptr(s_), _ptr(X), X.shape[1],
                                int(base), 0 if X.dtype == torch.float32 else 1, _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_expand_numeric failed: {rc}")
    # (the tables are freed after the launch: the caching allocator only hands
    # their blocks to work queued after it on this stream)
    return True
