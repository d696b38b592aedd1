"""Aggregations on the HIP kernels of ops/csrc/metrics.hip: the binomial
logit histogram plus the logloss / MSE / response sums in one pass, and
grouped f64 sums, both with wave-aggregated atomics (hex/AUC2.java AUCBuilder, ModelMetricsBinomial
MetricBuilderBinomial)."""
from __future__ import annotations

import ctypes

import torch

from . import _native


def _lib():
    lib = _native.get_lib("metrics", required=False)
    if lib is not None and not getattr(lib, "_typed", False):
        P = ctypes.c_void_p
        lib.h2o_logit_hist.argtypes = [P, P, P, ctypes.c_longlong, ctypes.c_int, P, P, P]
        lib.h2o_group_reduce.argtypes = [P, P, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P]
        lib._typed = True
    return lib


def available(t) -> bool:
    return t.is_cuda and _lib() is not None


def logit_hist(y, p1, w, nb):
    """One f64 buffer [2 nb + 5] = (positive bins, negative bins, sum w,
    sum w*logloss, sum w*(y-p)^2, sum w*y, row count) over the rows where
    neither y nor p1 is NaN.  Not yet reduced over ranks."""
    lib = _lib()
    if lib is None:
        raise RuntimeError("metrics HIP library missing")
    n = p1.numel()
    p1 = p1.reshape(-1).to(torch.float64).contiguous()
    y = y.reshape(-1).to(device=p1.device, dtype=torch.float64).contiguous()
    if y.numel() != n or (w is not None and w.numel() != n):
        raise ValueError("logit_hist: y / p1 / w lengths differ")
    w = None if w is None else w.reshape(-1).to(device=p1.device, dtype=torch.float64).contiguous()
    buf = torch.zeros(2 * nb + 5, dtype=torch.float64, device=p1.device)
    s = torch.cuda.current_stream().cuda_stream
    rc = lib.h2o_logit_hist(ctypes.c_void_p(p1.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                            ctypes.c_void_p(w.data_ptr() if w is not None else 0), n, nb,
                            ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(buf.data_ptr() + 16 * nb),
                            ctypes.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"h2o_logit_hist failed ({rc})")
    return buf


_OPS = {"sum": (0, 0.0), "min": (1, float("inf")), "max": (2, float("-inf"))}


def group_reduce(idx, vals, nbins, op="sum"):
    """f64 [nbins, C] sums / minima / maxima of vals [n, C] by idx (rows
    outside [0, nbins) skipped; empty groups hold 0 / +inf / -inf), on the
    device."""
    lib = _lib()
    if lib is None:
        raise RuntimeError("metrics HIP library missing")
    code, fill = _OPS[op]
    v = vals.to(torch.float64).contiguous()
    idx = idx.reshape(-1).to(device=v.device, dtype=torch.int64).contiguous()
    n, C = v.shape
    if idx.numel() != n:
        raise ValueError("group_reduce: idx / vals lengths differ")
    out = torch.full((nbins, C), fill, dtype=torch.float64, device=v.device)
    if n == 0 or nbins == 0 or C == 0:
        return out
    rc = lib.h2o_group_reduce(ctypes.c_void_p(idx.data_ptr()), ctypes.c_void_p(v.data_ptr()), n, C, nbins, code,
                              ctypes.c_void_p(out.data_ptr()),
                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"h2o_group_reduce failed ({rc})")
    return out


def group_sum(idx, vals, nbins):
    return group_reduce(idx, vals, nbins, "sum")
