"""Dense linear-algebra entry points for GLM / PCA / KMeans.

`weighted_gram(X, w)` = X^T diag(w) X in float64, computed by the HIP
f32-MFMA kernel (ops/csrc/gram.hip) on GPU, torch float64 on CPU.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native

_pairs_cache = {}


def _lib():
    lib = _native.get_lib("gram")
    if lib is not None and not getattr(lib, "_typed", False):
        lib.h2o_gram.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        lib._typed = True
    return lib


def weighted_gram(X: torch.Tensor, w: torch.Tensor | None = None, use_native=None, target_blocks=2048):
    """X: [N, P] f32 row-major (P multiple of 32 on GPU).  Returns [P, P] f64."""
    N, P = X.shape
    native = X.device.type == "cuda" if use_native is None else use_native
    if not native or P % 32 != 0 or X.dtype != torch.float32:
        Xd = X.to(torch.float64)
        if w is None:
            return Xd.T @ Xd
        return Xd.T @ (Xd * w.to(torch.float64).view(-1, 1))
    lib = _lib()
    T = P // 32
    key = (T, X.device)
    if key not in _pairs_cache:
        pr = [(i, j) for i in range(T) for j in range(i, T)]
        _pairs_cache[key] = (torch.tensor(pr, dtype=torch.int32, device=X.device), pr)
    pairs_t, pr = _pairs_cache[key]
    npairs = len(pr)
    splits = max(1, min(target_blocks // npairs, N // 2048))
    rpb = -(-N // splits)
    rpb = ((rpb + 7) // 8) * 8
    splits = -(-N // rpb)
    out = torch.empty((splits, npairs, 32, 32), dtype=torch.float64, device=X.device)
    X = X.contiguous()
    wt = None if w is None else w.to(torch.float32).contiguous()
    rc = lib.h2o_gram(ctypes.c_void_p(X.data_ptr()), ctypes.c_void_p(wt.data_ptr() if wt is not None else 0), N, P,
                      ctypes.c_void_p(pairs_t.data_ptr()), npairs, splits, rpb, ctypes.c_void_p(out.data_ptr()),
                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"h2o_gram failed: {rc}")
    tiles = out.sum(0)  # [npairs, 32, 32]
    ii, jj = pairs_t[:, 0].long(), pairs_t[:, 1].long()
    Gb = torch.zeros((T, T, 32, 32), dtype=torch.float64, device=X.device)
    Gb[jj, ii] = tiles.transpose(1, 2)
    Gb[ii, jj] = tiles
    return Gb.permute(0, 2, 1, 3).reshape(P, P)
