"""K-Means Lloyd pass entry point: the fused HIP kernel (ops/csrc/kmeans.hip)
on the GPU, an equivalent torch path on the CPU.

`lloyd_pass(X, C, ...)` assigns every row of X [N, P] to its closest center
of C [k, P] (squared euclidean, ties to the lowest index) and, with
``accumulate=True``, returns the per-cluster statistics of the pass in f64:
column sums, weights, within-cluster SS (distances to the *input* centers,
like the reference LloydsIterationTask's _cSqr) and the number of rows
whose assignment changed.  Reference: hex/kmeans/KMeans.java:731
(LloydsIterationTask.map).
"""
from __future__ import annotations

import ctypes
import torch

from . import _native

_cv, _ci, _cll, _cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float


def _lib():
    lib = _native.get_lib("kmeans")
    if lib is not None and not getattr(lib, "_typed", False):
        lib.h2o_kmeans_lloyd.argtypes = [_cv, _cv, _cll, _ci, _cv, _cv, _ci, _cv, _cv, _cv, _cv, _ci, _ci, _cf, _cv]
        lib.h2o_kmeans_reduce.argtypes = [_cv, _ci, _cll, _cv, _cv]
        lib.h2o_kmeans_max_k.argtypes = [_ci, _ci]
        lib.h2o_kmeans_part_stride.argtypes = [_ci, _ci]
        lib.h2o_kmeans_part_stride.restype = _cll
        lib.h2o_kmeans_resident_per_cu.argtypes = [_ci, _ci, _ci, _cf]
        lib.h2o_kmeans_sums.argtypes = [_cv, _cv, _cll, _ci, _ci, _cv, _cv, _cv, _cv, _ci, _cf, _cv]
        lib.h2o_kmeans_sums_resident_per_cu.argtypes = [_ci, _ci]
        lib.h2o_kmeans_assign.argtypes = [_cv, _cll, _ci, _cv, _cv, _ci, _cv, _cv, _ci, _cv]
        lib.h2o_kmeans_assign_resident_per_cu.argtypes = [_ci, _ci]
        lib.h2o_xv.argtypes = [_cv, _cll, _ci, _cv, _ci, _cv, _ci, _cv]
        lib.h2o_xv_resident_per_cu.argtypes = [_ci, _ci]
        lib._typed = True
    return lib


_CU = {}


def _cu_count(dev):
    if dev not in _CU:
        _CU[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return _CU[dev]


def _ptr(t):
    return _cv(0 if t is None else t.data_ptr())


class LloydStats:
    """Per-cluster statistics of one pass, packed in ONE f64 vector
    [k*P sums | k weights | k withinss | changed] so a multi-GPU reduce is
    a single all-reduce of `vec`."""

    def __init__(self, vec, k, P):
        self.vec, self.k, self.P = vec, k, P

    @property
    def sums(self):
        return self.vec[:self.k * self.P].view(self.k, self.P)

    @property
    def weights(self):
        return self.vec[self.k * self.P:self.k * self.P + self.k]

    @property
    def withinss(self):
        return self.vec[self.k * self.P + self.k:self.k * self.P + 2 * self.k]

    @property
    def changed(self):
        return float(self.vec[-1])


def native_ok(X, k, accumulate=True):
    """The fused kernel takes f32 row-major X with P % 4 == 0, P <= 256 and
    k up to an LDS-dependent bound (h2o_kmeans_max_k)."""
    if X.device.type != "cuda" or X.dtype != torch.float32 or X.dim() != 2:
        return False
    P = X.shape[1]
    lib = _lib()
    return lib is not None and 0 < k <= int(lib.h2o_kmeans_max_k(P, 1 if accumulate else 0))


def abs_bound(X, w=None):
    """max |w x| over the matrix (one pass; callers cache it per X): bounds
    the 64-bit fixed-point cluster sums of the kernel."""
    m = float(X.abs().max()) if X.numel() else 0.0
    if w is not None and w.numel():
        m *= float(w.abs().max())
    return m


def lloyd_pass(X, C, w=None, assign=None, accumulate=True, dmin=None, use_native=None, n_groups=None,
               xabs_max=None):
    """One pass over X.  assign: int32 [N] buffer, read as the previous
    assignment (changed count) and overwritten with the new one (may be
    None).  dmin: f32 [N] buffer for per-row squared distances to the
    closest center (may be None).  xabs_max: max |w x| (abs_bound) enables
    the kernel's 64-bit fixed-point cluster sums.  Returns LloydStats
    (accumulate=True) or None."""
    N, P = X.shape
    k = C.shape[0]
    native = native_ok(X, k, accumulate) if use_native is None else use_native
    C32 = C.to(device=X.device, dtype=torch.float32).contiguous()
    if not native:
        return _lloyd_torch(X, C32, w, assign, accumulate, dmin)
    lib = _lib()
    cn = (C.to(torch.float64) ** 2).sum(1).to(device=X.device, dtype=torch.float32).contiguous()
    X = X.contiguous()
    wt = None if w is None else w.to(device=X.device, dtype=torch.float32).contiguous()
    ntiles = (N + 63) // 64
    fx = 0.0
    if accumulate and xabs_max is not None:
        # per-workgroup |sum| < 2^62 for any grid up to one workgroup per CU
        rows_wg = 64 * (-(-ntiles // _cu_count(X.device)))
        fx = float(2.0 ** 62 / (max(xabs_max, 1e-30) * rows_wg)) if xabs_max > 0 else 1.0
        fx = min(fx, 2.0 ** 100)
    stride = int(lib.h2o_kmeans_part_stride(k, P))
    stream = _cv(torch.cuda.current_stream().cuda_stream)
    if accumulate and fx > 0 and n_groups is None and _split_ok(lib, k, P, fx):
        return _lloyd_split(lib, X, C32, cn, wt, k, P, ntiles, assign, dmin, xabs_max, stride, stream)
    if n_groups is None:
        # persistent grid = exactly the resident workgroups (no tail wave)
        per_cu = int(lib.h2o_kmeans_resident_per_cu(k, P, 1 if accumulate else 0, fx))
        n_groups = max(1, min(ntiles, max(per_cu, 1) * _cu_count(X.device)))
    part = None
    if accumulate:
        part = torch.empty((n_groups, stride), dtype=torch.float64, device=X.device)
    rc = lib.h2o_kmeans_lloyd(_ptr(X), _ptr(wt), N, P, _ptr(C32), _ptr(cn), k, _ptr(assign), _ptr(assign), _ptr(dmin),
                              _ptr(part), n_groups, 1 if accumulate else 0, fx, stream)
    if rc != 0:
        raise RuntimeError(f"h2o_kmeans_lloyd failed: {rc}")
    if not accumulate:
        return None
    out = torch.empty(stride, dtype=torch.float64, device=X.device)
    rc = lib.h2o_kmeans_reduce(_ptr(part), n_groups, stride, _ptr(out), stream)
    if rc != 0:
        raise RuntimeError(f"h2o_kmeans_reduce failed: {rc}")
    return LloydStats(out, k, P)


def _split_ok(lib, k, P, fx):
    """Large-k split path (assignment pass + sums pass) when the fused kernel
    would run one workgroup per CU (its LDS holds X tile + centers + sums)
    and the sums kernel fits; H2O3_KM_SPLIT=1 / 0 forces it on / off."""
    import os
    mode = os.environ.get("H2O3_KM_SPLIT", "auto")
    if mode == "0":
        return False
    if int(lib.h2o_kmeans_sums_resident_per_cu(k, P)) < 1:
        return False
    # 100M x 100 (profiles/kmeans_split_ab_r3.txt): k = 64 94 -> 41 ms, k = 128
    # 119 -> 91 ms; at k = 16 the fused kernel (2+ workgroups per CU) stays ahead
    return mode == "1" or int(lib.h2o_kmeans_resident_per_cu(k, P, 1, fx)) <= 1


def _lloyd_split(lib, X, C32, cn, wt, k, P, ntiles, assign, dmin, xabs_max, stride, stream):
    """Two HIP passes: the Lloyd kernel in assignment-only mode (new
    assignment + per-row d2, X tile and centers in LDS) then
    kmeans_sums_kernel (64-bit fixed-point per-cluster sums, weights,
    within-SS, changed count) -- see kmeans.hip."""
    N = X.shape[0]
    dev = X.device
    cus = _cu_count(dev)
    asg_new = torch.empty(N, dtype=torch.int32, device=dev)
    d2 = dmin if (dmin is not None and dmin.dtype == torch.float32 and dmin.is_contiguous()) else \
        torch.empty(N, dtype=torch.float32, device=dev)
    import os
    per_cu = int(lib.h2o_kmeans_assign_resident_per_cu(k, P))
    if per_cu > 0 and os.environ.get("H2O3_KM_ASSIGN", "wave") == "wave":
        # wave-persistent assignment kernel: X rows in registers, only the
        # centers in LDS (kmeans_assign_kernel)
        g1 = max(1, min(-(-N // 64), per_cu * cus))
        rc = lib.h2o_kmeans_assign(_ptr(X), N, P, _ptr(C32), _ptr(cn), k, _ptr(asg_new), _ptr(d2), g1, stream)
        if rc != 0:
            raise RuntimeError(f"h2o_kmeans_assign failed: {rc}")
    else:
        per_cu = int(lib.h2o_kmeans_resident_per_cu(k, P, 0, 0.0))
        g1 = max(1, min(ntiles, max(per_cu, 1) * cus))
        rc = lib.h2o_kmeans_lloyd(_ptr(X), _ptr(wt), N, P, _ptr(C32), _ptr(cn), k, _ptr(asg_new), None, _ptr(d2),
                                  None, g1, 0, 0.0, stream)
        if rc != 0:
            raise RuntimeError(f"h2o_kmeans_lloyd (assignment pass) failed: {rc}")
    g2 = max(1, min(ntiles, max(int(lib.h2o_kmeans_sums_resident_per_cu(k, P)), 1) * cus))
    rows_wg = 64 * (-(-ntiles // g2))
    fx = float(2.0 ** 62 / (max(xabs_max, 1e-30) * rows_wg)) if xabs_max > 0 else 1.0
    fx = min(fx, 2.0 ** 100)
    part = torch.empty((g2, stride), dtype=torch.float64, device=dev)
    rc = lib.h2o_kmeans_sums(_ptr(X), _ptr(wt), N, P, k, _ptr(asg_new), _ptr(assign), _ptr(d2), _ptr(part), g2, fx,
                             stream)
    if rc != 0:
        raise RuntimeError(f"h2o_kmeans_sums failed: {rc}")
    out = torch.empty(stride, dtype=torch.float64, device=dev)
    rc = lib.h2o_kmeans_reduce(_ptr(part), g2, stride, _ptr(out), stream)
    if rc != 0:
        raise RuntimeError(f"h2o_kmeans_reduce failed: {rc}")
    if assign is not None:
        assign.copy_(asg_new)
    if dmin is not None and d2 is not dmin:
        dmin.copy_(d2)
    return LloydStats(out, k, P)


def _lloyd_torch(X, C, w, assign, accumulate, dmin, chunk=1 << 20):
    """Reference path (CPU / unsupported shapes): same outputs, f64 sums."""
    N, P = X.shape
    k = C.shape[0]
    dev = X.device
    cn = (C.to(torch.float64) ** 2).sum(1).to(torch.float32)
    out = torch.zeros(k * P + 2 * k + 1, dtype=torch.float64, device=dev)
    st = LloydStats(out, k, P)
    sums, wsum, wss = st.sums, st.weights, st.withinss
    for a in range(0, N, chunk):
        Xc = X[a:a + chunk].to(torch.float32)
        d = cn.view(1, -1) - 2.0 * (Xc @ C.T)
        best, idx = d.min(1)
        d2 = ((Xc.to(torch.float64) ** 2).sum(1) + best.to(torch.float64)).clamp_min(0)
        idx32 = idx.to(torch.int32)
        if assign is not None:
            if accumulate:
                out[-1] += (assign[a:a + chunk] != idx32).sum().to(torch.float64)
            assign[a:a + chunk] = idx32
        if dmin is not None:
            dmin[a:a + chunk] = d2.to(dmin.dtype)
        if accumulate:
            wc = torch.ones(Xc.shape[0], dtype=torch.float64, device=dev) if w is None else \
                w[a:a + chunk].to(torch.float64)
            sums.index_add_(0, idx, Xc.to(torch.float64) * wc.view(-1, 1))
            wsum.index_add_(0, idx, wc)
            wss.index_add_(0, idx, wc * d2)
    return st if accumulate else None


# rows below which projections stay on the f64 torch path (small frames keep
# f64 parity with the CPU reference; large ones take the MFMA kernel)
XV_MIN_ROWS = 65536


def xv(X, V, min_rows=None):
    """X [N, W] @ V [W, k] -> [N, k] (f32 on the GPU kernel, else f64): the
    PCA / SVD projections.  On the GPU (W % 4 == 0, W, k <= 256, N >=
    min_rows) one pass of kmeans.hip's MFMA tile kernel in skinny-GEMM mode
    (exact f32 products, f32 sums over the W columns; X read once, no
    library GEMM); otherwise an f64 GEMM."""
    N, W = X.shape
    k = V.shape[1]
    lim = XV_MIN_ROWS if min_rows is None else min_rows
    lib = _lib() if X.is_cuda else None
    if (lib is None or X.dtype != torch.float32 or W % 4 or W > 256 or k > 256 or k < 1 or N < lim):
        return X.to(torch.float64) @ V.to(device=X.device, dtype=torch.float64)
    Xc = X.contiguous()
    Vt = V.to(device=X.device, dtype=torch.float32).t().contiguous()      # [k, W]
    out = torch.empty((N, k), dtype=torch.float32, device=X.device)
    per_cu = int(lib.h2o_xv_resident_per_cu(k, W))
    if per_cu < 1:
        return X.to(torch.float64) @ V.to(device=X.device, dtype=torch.float64)
    G = max(1, min(-(-N // 64), per_cu * _cu_count(X.device)))
    rc = lib.h2o_xv(_ptr(Xc), N, W, _ptr(Vt), k, _ptr(out), G, _cv(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"h2o_xv failed: {rc}")
    return out
