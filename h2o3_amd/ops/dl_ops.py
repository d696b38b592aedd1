"""Deep Learning step kernels (ops/csrc/dl.hip) with torch fallbacks of the
same semantics (CPU, and the reference for the GPU numerics tests).

fwd:     A = act(Z + b) with hashed unit dropout (train) / activation scaling
         by (1 - ratio) (test) — Neurons.fprop + Dropout.fillBytes;
bwd:     dZ = dA * act'(A) * mask, db = column sums of dZ;
update:  per neuron row: grad + L1/L2, ADADELTA or momentum / Nesterov,
         max_w2 rescale, bias update — Neurons.bprop / update_bias;
softmax: probabilities + CrossEntropy / Quadratic output gradient —
         Neurons.Softmax.setOutputLayerGradient.
mlp_step: the whole training step of a dense MLP in three hand-written
         kernels (f32 MFMA forward + backward per 16-row tile, dW tiles,
         per-row updates of every layer) — no library GEMM.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native

ACT = {"linear": 0, "tanh": 1, "rectifier": 2, "exprectifier": 3, "maxout": 4}
_cv, _ci, _cf, _cull = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_ulonglong


def _lib():
    lib = _native.get_lib("dl")
    if lib is not None and not getattr(lib, "_typed", False):
        lib.h2o_dl_fwd.argtypes = [_cv, _cv, _cv, _ci, _ci, _ci, _cf, _cull, _cv, _ci, _cf, _cv]
        lib.h2o_dl_bwd.argtypes = [_cv, _cv, _cv, _cv, _cv, _ci, _ci, _ci, _cf, _cull, _cv, _cv]
        lib.h2o_dl_seed_advance.argtypes = [_cv, _cv]
        lib.h2o_dl_update.argtypes = [_cv] * 9 + [_ci, _ci] + [_cf] * 7 + [_ci] * 3 + [_cf, _cf, _cv]
        lib.h2o_dl_softmax.argtypes = [_cv] * 7 + [_ci, _ci, _cf, _ci, _cv]
        lib.h2o_dl_mlp_step.argtypes = [_ci] + [_cv] * 15 + [_ci] + [_cv] * 4 + [_ci, _ci, _cf, _cull, _cv, _ci,
                                                                            _cv]
        lib.h2o_dl_gemm.argtypes = [_ci, _ci, _ci, _cv, ctypes.c_longlong, ctypes.c_longlong, _cv,
                                    ctypes.c_longlong, ctypes.c_longlong, _cv, _cv, ctypes.c_longlong, _cv]
        lib.h2o_dl_gemm_ws.argtypes = [_ci, _ci, _ci]
        lib.h2o_dl_gemm_ws.restype = ctypes.c_longlong
        lib._typed = True
    return lib


def _p(t):
    return _cv(0 if t is None else t.data_ptr())


def _s():
    return _cv(torch.cuda.current_stream().cuda_stream)


def _native_ok(t, use_native):
    return (t.device.type == "cuda") if use_native is None else use_native


def _check(rc, name):
    if rc != 0:
        raise RuntimeError(f"{name} failed: {rc}")


# ---------------------------------------------------------------- dropout hash
_M = (1 << 64) - 1


def _i64(c):
    return c - (1 << 64) if c >= (1 << 63) else c


def _lsr(x, s):
    return (x >> s) & ((1 << (64 - s)) - 1)


def keep_mask(seed: int, B: int, U: int, ratio: float, device) -> torch.Tensor:
    """[B, U] bool: units kept by the hashed dropout (same bits as dl.hip)."""
    if ratio <= 0:
        return torch.ones((B, U), dtype=torch.bool, device=device)
    thr = min(int(ratio * 4294967296.0), 4294967295)
    row = torch.arange(B, dtype=torch.int64, device=device).view(-1, 1)
    unit = torch.arange(U, dtype=torch.int64, device=device).view(1, -1)
    x = _i64(seed & _M) ^ ((row << 32) | unit)
    x = x + _i64(0x9E3779B97F4A7C15)
    x = (x ^ _lsr(x, 30)) * _i64(0xBF58476D1CE4E5B9)
    x = (x ^ _lsr(x, 27)) * _i64(0x94D049BB133111EB)
    x = x ^ _lsr(x, 31)
    h = _lsr(x, 32)
    return h >= thr


# ---------------------------------------------------------------- forward
def seed_advance(seed_dev, use_native=None):
    """One LCG step of a device-resident step seed (int64 [1]); the training
    step graph captures it so every replay draws new dropout masks."""
    if _native_ok(seed_dev, use_native):
        _check(_lib().h2o_dl_seed_advance(_p(seed_dev), _s()), "h2o_dl_seed_advance")
        return
    v = (int(seed_dev.item()) * 6364136223846793005 + 1442695040888963407) & _M
    seed_dev.fill_(_i64(v))


def _eff_seed(seed, seed_dev):
    return (seed + (int(seed_dev.item()) & _M)) & _M if seed_dev is not None else seed


def fwd(Z, bias, act: str, drop_ratio=0.0, seed=0, train=True, test_scale=1.0, use_native=None, seed_dev=None):
    """Z [B, U*k] (bias added in place; bias may be None), returns A [B, U].
    seed_dev: optional device int64 [1] added to `seed` inside the kernel."""
    a = ACT[act]
    B = Z.shape[0]
    U = Z.shape[1] // (2 if a == 4 else 1)
    if _native_ok(Z, use_native):
        A = torch.empty((B, U), dtype=torch.float32, device=Z.device)
        _check(_lib().h2o_dl_fwd(_p(Z), _p(bias), _p(A), B, U, a, float(drop_ratio), seed & _M, _p(seed_dev),
                                 0 if train else 1, float(test_scale), _s()), "h2o_dl_fwd")
        return A
    seed = _eff_seed(seed, seed_dev)
    if bias is not None:
        Z += bias.view(1, -1)
    if a == 4:
        A = Z.view(B, U, 2).max(2).values
    elif a == 1:
        A = torch.tanh(Z)
    elif a == 2:
        A = torch.relu(Z)
    elif a == 3:
        A = torch.where(Z > 0, Z, torch.expm1(Z))
    else:
        A = Z.clone()
    if train:
        if drop_ratio > 0:
            A = A * keep_mask(seed, B, U, drop_ratio, Z.device)
    else:
        A = A * test_scale
    return A


def bwd(dA, A, Z, act: str, drop_ratio=0.0, seed=0, use_native=None, seed_dev=None):
    """Returns (dZ [B, U*k], db [U*k])."""
    a = ACT[act]
    B, U = dA.shape
    k = 2 if a == 4 else 1
    if _native_ok(dA, use_native):
        dZ = torch.empty((B, U * k), dtype=torch.float32, device=dA.device)
        db = torch.zeros(U * k, dtype=torch.float32, device=dA.device)
        _check(_lib().h2o_dl_bwd(_p(dA.contiguous()), _p(A), _p(Z), _p(dZ), _p(db), B, U, a, float(drop_ratio),
                                 seed & _M, _p(seed_dev), _s()), "h2o_dl_bwd")
        return dZ, db
    seed = _eff_seed(seed, seed_dev)
    g = dA * keep_mask(seed, B, U, drop_ratio, dA.device) if drop_ratio > 0 else dA
    if a == 4:
        z = Z.view(B, U, 2)
        first = z[..., 0] >= z[..., 1]
        dZ = torch.stack([torch.where(first, g, 0.0), torch.where(first, 0.0, g)], 2).view(B, 2 * U)
    elif a == 1:
        dZ = g * (1 - A * A)
    elif a == 2:
        dZ = g * (A > 0)
    elif a == 3:
        dZ = g * torch.where(A > 0, torch.ones_like(A), A + 1)
    else:
        dZ = g.clone()
    return dZ, dZ.sum(0)


class UpdateParams:
    def __init__(self, ada=True, rho=0.99, eps=1e-8, rate=0.005, momentum=0.0, nesterov=True, has_momenta=False,
                 l1=0.0, l2=0.0, max_w2=float("inf"), sparsity_beta=0.0, average_activation=0.0):
        self.__dict__.update(locals())
        del self.__dict__["self"]


def update(W, dW, bias, dbias, state, p: UpdateParams, avg_act=None, use_native=None):
    """In-place per-neuron-row update of W [U, I] and bias [U]; state holds
    the ADADELTA / momentum buffers (created on first use)."""
    U, I = W.shape
    if "ada" not in state:
        state["ada"] = torch.zeros((U, I, 2), dtype=torch.float32, device=W.device)
        state["ada_b"] = torch.zeros((U, 2), dtype=torch.float32, device=W.device)
        state["mom"] = torch.zeros((U, I), dtype=torch.float32, device=W.device) if p.has_momenta else None
        state["mom_b"] = torch.zeros(U, dtype=torch.float32, device=W.device) if p.has_momenta else None
    max_w2 = float(p.max_w2) if p.max_w2 is not None and p.max_w2 < 3.0e38 else 3.4e38
    if _native_ok(W, use_native):
        _check(_lib().h2o_dl_update(_p(W), _p(dW), _p(state["ada"]), _p(state["mom"]), _p(bias), _p(dbias),
                                    _p(state["ada_b"]), _p(state["mom_b"]), _p(avg_act), U, I, p.rho, p.eps, p.rate,
                                    p.momentum, p.l1, p.l2, max_w2, int(p.ada), int(p.nesterov), int(p.has_momenta),
                                    p.sparsity_beta, p.average_activation, _s()), "h2o_dl_update")
        return
    grad = dW + torch.sign(W) * p.l1 + W * p.l2
    if p.ada:
        ada = state["ada"]
        g2 = grad * grad
        eg2 = p.rho * ada[..., 1] + (1 - p.rho) * g2
        rate = torch.sqrt((ada[..., 0] + p.eps) / (eg2 + p.eps))
        ada[..., 1] = eg2
        ada[..., 0] = p.rho * ada[..., 0] + (1 - p.rho) * rate * rate * g2
        W -= rate * grad
        avg_g2 = g2.sum(1) / max(I, 1)
    else:
        if not p.nesterov:
            delta = -p.rate * grad
            W += delta
            if p.has_momenta:
                W += p.momentum * state["mom"]
                state["mom"].copy_(delta)
        else:
            tmp = -grad
            if p.has_momenta:
                state["mom"].mul_(p.momentum).add_(tmp)
                tmp = state["mom"]
            W += p.rate * tmp
        avg_g2 = None
    if max_w2 < 3.0e38:
        r2 = (W * W).sum(1)
        scale = torch.where(r2 > max_w2, torch.sqrt(max_w2 / r2.clamp_min(1e-30)), torch.ones_like(r2))
        W *= scale.view(-1, 1)
    pg = dbias + torch.sign(bias) * p.l1 + bias * p.l2
    if p.ada:
        ab = state["ada_b"]
        ab[:, 1] = p.rho * ab[:, 1] + (1 - p.rho) * avg_g2
        rate = torch.sqrt((ab[:, 0] + p.eps) / (ab[:, 1] + p.eps))
        ab[:, 0] = p.rho * ab[:, 0] + (1 - p.rho) * rate * rate * avg_g2
    else:
        rate = torch.full_like(bias, p.rate)
    if not p.nesterov or p.ada:
        delta = -rate * pg
        nb = bias + delta
        if p.has_momenta and not p.ada:
            nb = nb + p.momentum * state["mom_b"]
            state["mom_b"].copy_(delta)
    else:
        d = -pg
        if p.has_momenta:
            state["mom_b"].mul_(p.momentum).add_(d)
            d = state["mom_b"]
        nb = bias + rate * d
    if avg_act is not None and p.sparsity_beta > 0:
        nb = nb - rate * p.sparsity_beta * (avg_act - p.average_activation)
    bias.copy_(nb)


def softmax(Z, bias, y=None, w=None, inv_n=1.0, loss="crossentropy", want_grad=True, use_native=None):
    """Z [B, K] (bias added in place).  Returns (P, dZ or None, per-row loss or None)."""
    B, K = Z.shape
    lcode = 1 if loss == "quadratic" else 0
    if _native_ok(Z, use_native):
        P = torch.empty_like(Z)
        dZ = torch.empty_like(Z) if (want_grad and y is not None) else None
        lo = torch.zeros(B, dtype=torch.float32, device=Z.device) if y is not None else None
        yy = None if y is None else y.to(torch.int64).contiguous()
        ww = None if w is None else w.to(torch.float32).contiguous()
        _check(_lib().h2o_dl_softmax(_p(Z), _p(bias), _p(P), _p(yy), _p(ww), _p(dZ), _p(lo), B, K, float(inv_n),
                                     lcode, _s()), "h2o_dl_softmax")
        return P, dZ, lo
    Z += bias.view(1, -1)
    P = torch.softmax(Z, 1)
    if y is None:
        return P, None, None
    yl = y.to(torch.int64)
    valid = yl >= 0
    wr = torch.where(valid, torch.ones(B, device=Z.device) if w is None else w.to(torch.float32),
                     torch.zeros(B, device=Z.device))
    T = torch.zeros_like(P)
    T[valid, yl[valid]] = 1.0
    g = (P - T) if lcode == 0 else (P - T) * (1 - P) * P
    dZ = g * (wr * inv_n).view(-1, 1) if want_grad else None
    py = P.gather(1, yl.clamp_min(0).view(-1, 1)).view(-1)
    lo = -wr * torch.log(py.clamp_min(1e-30))
    return P, dZ, lo


# ---------------------------------------------------------------- fused step
class _DLUpdate(ctypes.Structure):
    _fields_ = [("rho", _cf), ("eps", _cf), ("rate", _cf), ("momentum", _cf), ("l1", _cf), ("l2", _cf),
                ("max_w2", _cf), ("ada", _ci), ("nesterov", _ci), ("has_momenta", _ci),
                ("sparsity_beta", _cf), ("average_activation", _cf)]


MLP_MAX_LAYERS = 8
_FUSED_ACTS = ("tanh", "rectifier", "exprectifier", "linear")


def mlp_fits(widths) -> bool:
    """The fused step keeps one 16-row tile of every layer's input plus two
    gradient buffers in LDS (160 KB per workgroup); <= 8 layers, <= 64
    outputs."""
    nl = len(widths) - 1
    if nl < 1 or nl > MLP_MAX_LAYERS or widths[-1] > 64:
        return False
    pad = [((w + 15) // 16) * 16 + 4 for w in widths]
    floats = 16 * sum(pad) + 2 * 16 * (max(pad[1:]))
    return floats * 4 <= 160 * 1024


def _ensure_state(W, state, has_momenta):
    U, I = W.shape
    if "ada" not in state:
        state["ada"] = torch.zeros((U, I, 2), dtype=torch.float32, device=W.device)
        state["ada_b"] = torch.zeros((U, 2), dtype=torch.float32, device=W.device)
        state["mom"] = torch.zeros((U, I), dtype=torch.float32, device=W.device) if has_momenta else None
        state["mom_b"] = torch.zeros(U, dtype=torch.float32, device=W.device) if has_momenta else None


def mlp_step(X, idx, y, w, layers, acts, drops, in_drop, out_kind, inv_n, ups, seed=0, seed_dev=None,
             advance=False, bufs=None):
    """One fused training step (dl.hip dl_mlp_*).  X [n, P] f32 (rows idx
    [B] int64, or the first B = len(X) rows when idx is None); y int64 labels
    (out_kind 0 CrossEntropy / 1 Quadratic softmax) or f32 [n(,1)] targets
    (out_kind 2, linear output + quadratic loss); w row weights or None.
    layers: objects with W [U, I], b [U], state; acts / drops per hidden
    layer; ups: UpdateParams per layer.  Weights, biases and ADADELTA /
    momentum state are updated in place.  bufs: optional dict reused across
    calls for the A / dZ / dW / db scratch.  seed_dev + advance: the device
    step seed is advanced (LCG) and the new value used, as seed_advance()
    followed by the unfused step."""
    lib = _lib()
    nl = len(layers)
    B = int(idx.shape[0]) if idx is not None else int(X.shape[0])
    widths = [int(layers[0].W.shape[1])] + [int(L.W.shape[0]) for L in layers]
    dev = X.device
    bufs = {} if bufs is None else bufs
    key = (B, tuple(widths))
    if bufs.get("key") != key:
        bufs.clear()
        bufs["key"] = key
        bufs["A"] = [torch.empty((B, widths[l]), dtype=torch.float32, device=dev) for l in range(nl)]
        bufs["dZ"] = [torch.empty((B, widths[l + 1]), dtype=torch.float32, device=dev) for l in range(nl)]
        bufs["dW"] = [torch.empty_like(L.W) for L in layers]
        bufs["db"] = [torch.empty_like(L.b) for L in layers]
    for L, up in zip(layers, ups):
        _ensure_state(L.W, L.state, up.has_momenta)
    arr = lambda ts: (_cv * nl)(*[0 if t is None else t.data_ptr() for t in ts])
    wid = (_ci * (nl + 1))(*widths)
    actc = (_ci * max(1, nl - 1))(*([ACT[a] for a in acts] or [0]))
    dropc = (_cf * nl)(*([float(in_drop)] + [float(d) for d in drops]))
    upc = (_DLUpdate * nl)(*[_DLUpdate(up.rho, up.eps, up.rate, up.momentum, up.l1, up.l2,
                                       float(up.max_w2) if up.max_w2 is not None and up.max_w2 < 3.0e38 else 3.4e38,
                                       int(up.ada), int(up.nesterov), int(up.has_momenta), up.sparsity_beta,
                                       up.average_activation) for up in ups])
    Xc = X if X.is_contiguous() else X.contiguous()
    ycls = y if out_kind < 2 else None
    yreg = y.reshape(-1) if out_kind == 2 else None
    rc = lib.h2o_dl_mlp_step(nl, wid, actc, dropc, arr([L.W for L in layers]), arr([L.b for L in layers]),
                             arr(bufs["A"]), arr(bufs["dZ"]), arr(bufs["dW"]), arr(bufs["db"]),
                             arr([L.state["ada"] for L in layers]), arr([L.state["mom"] for L in layers]),
                             arr([L.state["ada_b"] for L in layers]), arr([L.state["mom_b"] for L in layers]),
                             upc, _p(Xc), int(Xc.shape[1]), _p(idx), _p(ycls), _p(yreg), _p(w), B, int(out_kind),
                             float(inv_n), seed & _M, _p(seed_dev), int(bool(advance)), _s())
    _check(rc, "h2o_dl_mlp_step")


# ---------------------------------------------------------------- GEMM
def gemm(A, B, out=None):
    """A @ B for 2-D f32 tensors (any strides: transposed views included) on
    the hand-written MFMA tile kernel (dl.hip dl_gemm_kernel) on the GPU, a
    torch matmul on the CPU.  The DL layers the fused step does not cover
    (wide hidden layers, maxout, autoencoders) run their three products per
    step -- Z = A W^T, dA = dZ W, dW = dZ^T A -- through it."""
    import os
    if A.device.type != "cuda" or A.dtype != torch.float32 or B.dtype != torch.float32 or \
            os.environ.get("H2O3_DL_GEMM", "mfma") != "mfma":
        return A @ B
    M, K = A.shape
    K2, N = B.shape
    assert K == K2, (A.shape, B.shape)
    C = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=A.device)
    if M == 0 or N == 0:
        return C
    if K == 0:
        return C.zero_()
    lib = _lib()
    # split-K workspace (thin products: few output tiles, long K), summed in
    # slice order by a second kernel -- deterministic, no float atomics
    nws = int(lib.h2o_dl_gemm_ws(M, N, K))
    ws = torch.empty(nws, dtype=torch.float32, device=A.device) if nws > 0 else None
    _check(lib.h2o_dl_gemm(M, N, K, _p(A), A.stride(0), A.stride(1), _p(B), B.stride(0), B.stride(1), _p(C),
                           _p(ws), nws, _s()), "h2o_dl_gemm")
    return C
