"""Dense linear-algebra entry points for GLM / PCA / KMeans.

`weighted_gram(X, w)` = X^T diag(w) X in float64, computed by the HIP
f32-MFMA kernel (ops/csrc/gram.hip) on GPU, torch float64 on CPU.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _native

_pairs_cache = {}


def _lib():
    lib = _native.get_lib("gram")
    if lib is not None and not getattr(lib, "_typed", False):
        lib.h2o_gram.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        P, I, LL, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float
        lib.h2o_glm_irls.argtypes = [P, LL, I, I, P, I, I, I, P, F, P, P, P, I, I, F, F, P, P, I, I, P, P, P, I, I, P]
        lib.h2o_glm_irls_chunk.argtypes = [I]
        lib.h2o_gram_split.argtypes = [P, I, I, I, P, P, LL, P, P]
        lib.h2o_glm_wide_split.argtypes = [P, I, I, I, LL, P, F, P, P, P, I, I, F, F, P, P, I, P, P, P]
        lib.h2o_glm_wide_gram.argtypes = [P, I, I, LL, P, I, I, P, I, P]
        lib.h2o_glm_wide_split_grid.argtypes = [I]
        lib.h2o_glm_wide_gram256.argtypes = [P, I, I, LL, P, I, I, P, I, I, P]
        lib.h2o_gram_f64.argtypes = [P, I, I, LL, P, P, I, I, LL, P, P]
        lib.h2o_xv_f64.argtypes = [P, I, I, LL, P, ctypes.c_double, P, P]
        lib.h2o_xtr_f64.argtypes = [P, I, I, LL, P, I, LL, P, P]
        lib._typed = True
    return lib


def _pairs(T, device):
    key = (T, device)
    if key not in _pairs_cache:
        pr = [(i, j) for i in range(T) for j in range(i, T)]
        _pairs_cache[key] = (torch.tensor(pr, dtype=torch.int32, device=device), pr)
    return _pairs_cache[key]


def _assemble(tiles, pairs_t, T):
    """[npairs, t, t] upper-triangle tiles -> symmetric [tT, tT]."""
    t = tiles.shape[-1]
    ii, jj = pairs_t[:, 0].long(), pairs_t[:, 1].long()
    Gb = torch.zeros((T, T, t, t), dtype=torch.float64, device=tiles.device)
    Gb[jj, ii] = tiles.transpose(1, 2)
    Gb[ii, jj] = tiles
    return Gb.permute(0, 2, 1, 3).reshape(t * T, t * T)


_LINK = {"identity": 0, "logit": 1, "log": 2, "inverse": 3}
_VAR = {"gaussian": 0, "binomial": 1, "quasibinomial": 1, "fractionalbinomial": 1, "poisson": 2, "gamma": 3,
        "tweedie": 4, "negativebinomial": 5}


def glm_fused_codes(family, link, tlp=1.0):
    """(link, var) codes of the fused IRLS kernel, or None when unsupported."""
    if link == "tweedie":
        link = "log" if tlp == 0 else ("identity" if tlp == 1 else None)
    if link not in _LINK or family not in _VAR:
        return None
    return _LINK[link], _VAR[family]


def _f32(t):
    return None if t is None else t.to(torch.float32).contiguous()


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def glm_irls(X, aug=-1, beta=None, b0=0.0, y=None, wprior=None, offset=None, codes=(0, 0), tvp=0.0, theta=1e-10,
             W=None, z=None, signed=None, target_blocks=1024, width=None, grad=False, bf3=None, grad_f64=True):
    """One pass of the fused IRLS kernel (ops/csrc/gram.hip glm_irls_kernel).

    Fused mode (beta given): per row eta = x.beta + b0 + offset, the family's
    IRLS weight / working response, deviance.  External mode: W, z given.
    `signed`: external W may hold negative values (default: checked).
    Returns (G [Pp, Pp] f64 — columns `aug` / `aug+1` hold X'W / X'Wz and
    their cross terms when aug >= 0 — and the f64 deviance, or None).
    `width`: logical padded width Pp when X is stored narrower (X [N, ldx],
    ldx % 4 == 0, columns ldx..Pp-1 implicitly zero; Pp = 128 ws path only).
    `grad=True` (fused mode, Pp in 32 / 64 / 128): also return the exact
    gradient channel g [Pp + 1] f64 = X'r, r = w (y - mu) dmu/deta / var
    (exact f64 products of the f32 values, f64 sums -- or, grad_f64=False,
    f32 products summed over a lane's rows of a chunk, f64 beyond; g[Pp] =
    sum r) as a third element.
    `bf3`: override H2O3_GLM_BF3 for this call (False: f32 MFMA Gram;
    "bf16": one bf16 MFMA per product, fused passes with grad=True only).
    """
    N, ldx = X.shape
    P = int(width) if width else ldx
    lib = _lib()
    if lib is None:
        raise RuntimeError("gram extension not built (run __graft_entry__.build())")
    T = P // 16  # 16x16 MFMA tiles
    pairs_t, pr = _pairs(T, X.device)
    npairs = len(pr)
    groups = -(-npairs // 36)
    target_blocks = int(os.environ.get("H2O3_GI_BLOCKS", target_blocks))   # A/B knob
    splits = max(1, min(max(1, target_blocks // groups), N // 4096))
    rpb = -(-N // splits)
    rc = lib.h2o_glm_irls_chunk(P)
    rpb = ((rpb + rc - 1) // rc) * rc
    splits = -(-N // rpb)
    out = torch.zeros((splits, npairs, 16, 16), dtype=torch.float64, device=X.device)
    dev = torch.zeros(splits, dtype=torch.float64, device=X.device)
    gout = torch.empty((splits, P + 1), dtype=torch.float64, device=X.device) if grad else None
    X = X.contiguous()
    bt = _f32(beta)
    keep = [_f32(y), _f32(wprior), _f32(offset), _f32(W), _f32(z)]
    if signed is None:
        signed = beta is None and keep[3] is not None and bool((keep[3] < 0).any())
    rc = lib.h2o_glm_irls(_ptr(X), N, P, ldx, _ptr(pairs_t), npairs, splits, rpb, _ptr(bt), float(b0),
                          _ptr(keep[0]), _ptr(keep[1]), _ptr(keep[2]), int(codes[0]), int(codes[1]), float(tvp),
                          float(theta), _ptr(keep[3]), _ptr(keep[4]), int(aug), int(bool(signed)), _ptr(out),
                          _ptr(dev), _ptr(gout), -1 if bf3 is None else (2 if bf3 == "bf16" else int(bool(bf3))),
                          int(bool(grad_f64)),
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"h2o_glm_irls failed: {rc}")
    G = _assemble(out.sum(0), pairs_t, T)
    if grad:
        return G, dev.sum(), gout.sum(0)
    return G, (dev.sum() if beta is not None else None)


def glm_grad_supported(width):
    """True when glm_irls(grad=True) runs at this padded width (the fused
    warp-specialised kernel: Pp in 32 / 64 / 128).  H2O3_GLM_EXACT_GRAD=0
    turns the channel off (A/B only: the IRLS right-hand side then comes from
    the Gram's own X'Wz column)."""
    return int(width) in (32, 64, 128) and os.environ.get("H2O3_GLM_EXACT_GRAD", "1") != "0"


def glm_irls_reference(X, aug=-1, beta=None, b0=0.0, y=None, wprior=None, offset=None, fam=None, W=None, z=None):
    """fp64 torch reference of glm_irls (tests / CPU)."""
    Xd = X.to(torch.float64).clone()
    dev = None
    if beta is not None:
        eta = Xd @ beta.to(torch.float64) + b0
        off = offset.to(torch.float64) if offset is not None else 0.0
        eta = eta + off
        mu = fam.linkinv(eta)
        pw = wprior.to(torch.float64) if wprior is not None else torch.ones_like(eta)
        yd = y.to(torch.float64)
        if fam.family == "gaussian" and fam.link == "identity":
            W, z = pw, yd - off
        else:
            d = fam.dmu_deta(eta, mu)
            W = pw * d * d / fam.variance(mu)
            z = (eta - off) + (yd - mu) / d
        dev = (pw * fam.deviance(yd, mu)).sum()
    W = torch.ones(X.shape[0], dtype=torch.float64) if W is None else W.to(torch.float64)
    if aug >= 0:
        Xd[:, aug] = 1.0
        Xd[:, aug + 1] = 0.0 if z is None else z.to(torch.float64)
    return Xd.T @ (Xd * W.view(-1, 1)), dev


def weighted_gram(X: torch.Tensor, w: torch.Tensor | None = None, use_native=None, target_blocks=2048):
    """X: [N, P] f32 row-major (P multiple of 32 on GPU).  Returns [P, P] f64."""
    N, P = X.shape
    native = X.device.type == "cuda" if use_native is None else use_native
    if not native or P % 32 != 0 or X.dtype != torch.float32:
        Xd = X.to(torch.float64)
        if w is None:
            return Xd.T @ Xd
        return Xd.T @ (Xd * w.to(torch.float64).view(-1, 1))
    if P <= 512:
        # f32 MFMA (f64 across row blocks): PCA / SVD / GLRM-init and p-values
        # read these values directly, so no bf16x3 products here
        return glm_irls(X, W=w, bf3=False)[0]
    if w is None or bool((w >= 0).all()):
        # wide designs: f32 products (PCA / SVD / GLRM-init / p-values read these
        # values directly -- the bf16x3 and bf16 Grams serve only the IRLS
        # Hessian): a plain library GEMM (rocBLAS/hipBLASLt fp32, 136 TFLOP/s at
        # N=12.5M, P=1024 vs 24 for the 32x32 tile-pair kernel, scripts/glm_wide_mb.py)
        # over 1M-row chunks of sqrt(W)-scaled rows, accumulated in f64
        G = torch.zeros((P, P), dtype=torch.float64, device=X.device)
        step = 1 << 20
        for a in range(0, N, step):
            Xc = X[a:a + step]
            if w is not None:
                Xc = Xc * w[a:a + step].to(torch.float32).sqrt().view(-1, 1)
            G += (Xc.T @ Xc).to(torch.float64)
        return G
    lib = _lib()
    T = P // 32
    pairs_t, pr = _pairs(T, X.device)
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
    return _assemble(out.sum(0), pairs_t, T)


def tmm(A: torch.Tensor, B: torch.Tensor, chunk: int = 4096) -> torch.Tensor:
    """A.T @ B for tall A [n, p], B [n, q] (B may be 1-D).  With a small
    output on the GPU the long inner dimension is split into chunks of ONE
    batched GEMM, summed after: the library tiles a [p, n] x [n, q] product
    with p, q <= 128 onto one or two workgroups that walk all n rows
    serially (a 10 x 10 f64 output over 500k rows: 40 ms; ~2 s at 20M)."""
    vec = B.dim() == 1
    Bm = B.view(-1, 1) if vec else B
    n, p = A.shape
    q = Bm.shape[1]
    if not A.is_cuda or n < 4 * chunk or max(p, q) > 256:
        out = A.T @ Bm
    else:
        S = -(-n // chunk)
        pad = S * chunk - n
        if pad:
            A = torch.cat([A, A.new_zeros((pad, p))])
            Bm = torch.cat([Bm, Bm.new_zeros((pad, q))])
        out = torch.bmm(A.reshape(S, chunk, p).transpose(1, 2), Bm.reshape(S, chunk, q)).sum(0)
    return out.view(-1) if vec else out


def gram_f64_aug(X: torch.Tensor, P: int, W: torch.Tensor, part_budget: int = 1 << 28) -> torch.Tensor:
    """[P+1, P+1] f64 Gram of [X[:, :P] | 1] weighted by W (f64 [N]), exact
    f64 products on the f64 matrix cores (ops/csrc/gram.hip gram_f64_kernel):
    the GLM top precision tier without an f64 copy of X.  X: f32 [N, ldx]
    with unit column stride."""
    N = X.shape[0]
    Pa = P + 1
    T = -(-Pa // 64)
    if N == 0:
        return torch.zeros((Pa, Pa), dtype=torch.float64, device=X.device)
    if X.dtype != torch.float32 or X.stride(1) != 1:
        raise ValueError("gram_f64_aug: X must be f32 with unit column stride")
    lib = _lib()
    pairs_t, pr = _pairs(T, X.device)
    npairs = len(pr)
    # enough slabs for ~2048 workgroups, partials within the budget
    slabs = max(1, min(-(-2048 // npairs), N // 256, part_budget // (npairs * 64 * 64 * 8)))
    rps = -(-N // slabs)
    rps = ((rps + 15) // 16) * 16
    slabs = -(-N // rps)
    part = torch.empty((slabs, npairs, 64, 64), dtype=torch.float64, device=X.device)
    Wd = W.to(torch.float64).contiguous()
    if Wd.numel() != N:
        raise ValueError("gram_f64_aug: W length differs from X rows")
    rc = lib.h2o_gram_f64(ctypes.c_void_p(X.data_ptr()), X.stride(0), P, N, ctypes.c_void_p(Wd.data_ptr()),
                          ctypes.c_void_p(pairs_t.data_ptr()), npairs, slabs, rps, ctypes.c_void_p(part.data_ptr()),
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"h2o_gram_f64 failed: {rc}")
    return _assemble(part.sum(0), pairs_t, T)[:Pa, :Pa]


def xv_f64(X: torch.Tensor, P: int, beta: torch.Tensor, b0: float = 0.0) -> torch.Tensor:
    """f64 [N] = X[:, :P] beta + b0 with f64 products from the f32 rows."""
    N = X.shape[0]
    out = torch.empty(N, dtype=torch.float64, device=X.device)
    if N == 0:
        return out
    if X.dtype != torch.float32 or X.stride(1) != 1:
        raise ValueError("xv_f64: X must be f32 with unit column stride")
    bt = beta.to(device=X.device, dtype=torch.float64).contiguous()
    if bt.numel() < P:
        raise ValueError("xv_f64: beta shorter than P")
    rc = _lib().h2o_xv_f64(ctypes.c_void_p(X.data_ptr()), X.stride(0), P, N, ctypes.c_void_p(bt.data_ptr()),
                           float(b0), ctypes.c_void_p(out.data_ptr()),
                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"h2o_xv_f64 failed: {rc}")
    return out


def xtr_f64(X: torch.Tensor, P: int, r: torch.Tensor) -> torch.Tensor:
    """f64 [P] = X[:, :P]' r (r f64 [N]) with f64 products, slab partials
    summed in a fixed order."""
    N = X.shape[0]
    if N == 0 or P == 0:
        return torch.zeros(P, dtype=torch.float64, device=X.device)
    if X.dtype != torch.float32 or X.stride(1) != 1:
        raise ValueError("xtr_f64: X must be f32 with unit column stride")
    rv = r.to(torch.float64).contiguous()
    if rv.numel() != N:
        raise ValueError("xtr_f64: r length differs from X rows")
    cb = -(-P // 256)
    slabs = max(1, min(65535, N // 512, -(-4096 // cb)))
    rps = -(-N // slabs)
    slabs = -(-N // rps)
    part = torch.empty((slabs, P), dtype=torch.float64, device=X.device)
    rc = _lib().h2o_xtr_f64(ctypes.c_void_p(X.data_ptr()), X.stride(0), P, N, ctypes.c_void_p(rv.data_ptr()), slabs,
                            rps, ctypes.c_void_p(part.data_ptr()),
                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"h2o_xtr_f64 failed: {rc}")
    return part.sum(0)


# Row chunks per batched Gram GEMM: C_b = hi_b^T [hi_b | lo_b] for g chunks of
# 512K rows in ONE strided-batched bf16 GEMM (f32 out, each chunk's f32
# accumulation stays 512K rows long; chunks summed in f64).  One GEMM per
# chunk has only 4 x 8 output tiles of 256 x 256 -- scripts/glm_wide_bmm_mb.py
# at 12.5M x 1024: 66.7 ms per pass per chunk vs 45.9 ms batched by 4
# (1142 TFLOP/s bf16).
_WIDE_GROUP = int(os.environ.get("H2O3_WIDE_GROUP", 4))


def _gram_group(H, st, Pa, G):
    """G += sum over the row chunks of H [g*st, 2Pa] of hi'hi + hi'lo + lo'hi."""
    g = H.shape[0] // st
    H3 = H.view(g, st, 2 * Pa)
    C = torch.bmm(H3[:, :, :Pa].transpose(1, 2), H3, out_dtype=torch.float32).to(torch.float64).sum(0)
    G += C[:, :Pa]
    cross = C[:, Pa:]
    G += cross + cross.T


def _overlap_ok(X, nch, grp):
    """Split / GEMM overlap (opt-in, H2O3_WIDE_OVERLAP=1: measured slower at 12.5M x 1000, the split
    kernels steal CUs from the GEMM -- profiles/glm_wide_overlap_ab_r4.txt); needs > 1 group of chunks."""
    return X.device.type == "cuda" and nch > grp and os.environ.get("H2O3_WIDE_OVERLAP", "0") == "1"


def _pipelined_groups(split, HL, N, st, grp, Pa, G):
    """Double-buffered row-chunk groups: the memory-bound split kernels of
    group g+1 run on a side stream while the compute-bound batched GEMM of
    group g runs on the current stream; events order each buffer's reuse
    (split g+2 waits for GEMM g) and the GEMM of g for its splits."""
    main = torch.cuda.current_stream()
    side = _side_stream(HL.device)
    bufs = [HL, torch.empty_like(HL)]
    side.wait_stream(main)                       # inputs written on the main stream
    gemm_done = [None, None]
    nch = -(-N // st)
    groups = [list(range(g0, min(g0 + grp, nch))) for g0 in range(0, nch, grp)]
    for gi, chunks in enumerate(groups):
        b = gi & 1
        buf = bufs[b]
        with torch.cuda.stream(side):
            if gemm_done[b] is not None:
                side.wait_event(gemm_done[b])
            sid = ctypes.c_void_p(side.cuda_stream)
            for j, i in enumerate(chunks):
                a = i * st
                r = min(st, N - a)
                split(i, a, r, buf, j, sid)
                if r < st:
                    buf[j * st + r:(j + 1) * st].zero_()
            ready = torch.cuda.Event()
            ready.record(side)
        main.wait_event(ready)
        _gram_group(buf[:len(chunks) * st], st, Pa, G)
        ev = torch.cuda.Event()
        ev.record(main)
        gemm_done[b] = ev
        buf.record_stream(side)
    main.wait_stream(side)                        # deviance partials written by the last splits


_SIDE = {}


def _side_stream(dev):
    k = str(dev)
    if k not in _SIDE:
        _SIDE[k] = torch.cuda.Stream(device=dev)
    return _SIDE[k]


def _wide_mode():
    return os.environ.get("H2O3_WIDE_GRAM", "bf3")


def gram_aug_bf3(X, W, z, P, step=1 << 19):
    """Augmented Gram of sqrt(W) [X[:, :P] | 1 | z] (z may be None) as
    [Pa, Pa] f64, Pa = round_up(P + 2, 64): per row chunk one HIP pass
    (gram_split_kernel) writes [hi | lo] bf16 halves and one bf16 GEMM with
    f32 output, C = hi^T [hi | lo], gives hi'hi + hi'lo + (hi'lo)^T."""
    lib = _lib()
    if lib is None:
        raise RuntimeError("gram extension not built (run __graft_entry__.build())")
    N, ldx = X.shape
    X = X.contiguous()
    Pa = -(-(P + 2) // 64) * 64
    W32, z32 = _f32(W), _f32(z)
    st = min(step, max(N, 1))
    nch = -(-N // st)
    grp = min(nch, _WIDE_GROUP)
    HL = torch.empty((grp * st, 2 * Pa), dtype=torch.bfloat16, device=X.device)
    G = torch.zeros((Pa, Pa), dtype=torch.float64, device=X.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    def split(i, a, r, buf, j, strm):
        rc = lib.h2o_gram_split(ctypes.c_void_p(X.data_ptr() + a * ldx * 4), ldx, P, Pa,
                                ctypes.c_void_p(0 if W32 is None else W32.data_ptr() + a * 4),
                                ctypes.c_void_p(0 if z32 is None else z32.data_ptr() + a * 4), r,
                                ctypes.c_void_p(buf.data_ptr() + j * st * 2 * Pa * 2), strm)
        if rc != 0:
            raise RuntimeError(f"h2o_gram_split failed: {rc}")

    if _overlap_ok(X, nch, grp):
        _pipelined_groups(split, HL, N, st, grp, Pa, G)
        return G
    for i, a in enumerate(range(0, N, st)):
        r = min(st, N - a)
        j = i % grp
        split(i, a, r, HL, j, stream)
        if r < st:
            HL[j * st + r:(j + 1) * st].zero_()
        if j == grp - 1 or i == nch - 1:
            _gram_group(HL[:(j + 1) * st], st, Pa, G)
    return G


def wide_fused_enabled():
    """The fused wide Gram (glm_wide_gram_kernel) is the default wide pass;
    H2O3_GLM_WIDE_FUSED=0 selects the split + library GEMM pass."""
    return os.environ.get("H2O3_GLM_WIDE_FUSED", "1") != "0"


def _wide_gram_assemble(part, S, NB, P, T=128):
    """Sum the slices' f64 tile partials and mirror the upper-triangle tiles
    into the (P + 2)^2 Gram (the z column left 0).  T = 256 tiles: the kernel
    skipped the lower-left quarter of diagonal tiles (taken here from the
    upper-right one).  Plain block copies (advanced-index assignment into a
    permuted view was ~10 ms at P = 1000)."""
    Tt = part.view(S, -1, T, T).sum(0)
    pairs = [(i, j) for i in range(NB) for j in range(i, NB)]
    assert len(pairs) == Tt.shape[0]
    n = NB * T
    G = torch.empty((n, n), dtype=torch.float64, device=part.device)
    for p, (i, j) in enumerate(pairs):
        blk = Tt[p]
        if i == j:
            if T == 256:
                blk[128:, :128] = blk[:128, 128:].T
            blk = 0.5 * (blk + blk.T)
        G[i * T:(i + 1) * T, j * T:(j + 1) * T] = blk
        if i != j:
            G[j * T:(j + 1) * T, i * T:(i + 1) * T] = blk.T
    m = P + 2
    if n >= m:
        G[:, P + 1:] = 0.0          # columns past the intercept: the z slot (and padding) stay 0
        G[P + 1:, :] = 0.0
        return G[:m, :m]
    out = torch.zeros((m, m), dtype=torch.float64, device=part.device)
    out[:P + 1, :P + 1] = G[:P + 1, :P + 1]
    return out


def wide_gram(X, P, wr, stream=None, bf3=True):
    """[X | 1]' diag(wr) [X | 1] (f64, (P + 2)^2 with a zero z column) by the
    hand-written MFMA kernel: 256 x 256 tiles (glm_wide_gram256_kernel,
    default) or 128 x 128 (H2O3_WIDE_TILE=128, glm_wide_gram_kernel).
    bf3=False (256 tiles): one bf16 MFMA per product instead of three."""
    lib = _lib()
    N, ldx = X.shape
    T = int(os.environ.get("H2O3_WIDE_TILE", 256))
    npad = -(-N // 64) * 64
    if wr.numel() < npad or wr.data_ptr() % 32:
        # the 256-tile kernel reads whole 64-row chunks of weights (zero past N)
        w2 = torch.zeros(npad, dtype=torch.float32, device=wr.device)
        w2[:N] = wr[:N]
        wr = w2
    NB = -(-(P + 1) // T)
    npairs = NB * (NB + 1) // 2
    from ..utils.timer import phase
    per_cu = 1 if T == 256 else 2
    S = int(os.environ.get("H2O3_WIDE_SLICES", 0)) or max(1, 256 * per_cu // npairs)
    # f32 runs between f64 folds: 32K rows for bf16x3 products; the plain bf16
    # Hessian (~2^-9 per product) folds once at the end (a 500K-row f32 run adds
    # ~1e-4 relative, far below its own rounding) -- 64K atomics per workgroup
    # instead of one per fold per 32K rows
    fold = 1024 if bf3 or T != 256 else 1 << 30
    with phase("glm.wide_gram.zero"):
        part = torch.zeros((npairs * S, T, T), dtype=torch.float64, device=X.device)
    stream = stream or ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    with phase("glm.wide_gram.kernel"):
        if T == 256:
            rc = lib.h2o_glm_wide_gram256(_ptr(X), ldx, P, N, _ptr(wr), S, fold, _ptr(part), 0, int(bool(bf3)),
                                          stream)
        else:
            rc = lib.h2o_glm_wide_gram(_ptr(X), ldx, P, N, _ptr(wr), S, fold, _ptr(part), 0, stream)
    if rc != 0:
        raise RuntimeError(f"h2o_glm_wide_gram failed: {rc}")
    with phase("glm.wide_gram.assemble"):
        return _wide_gram_assemble(part, S, NB, P, T)


_SPLIT_GRID = {}


def _wide_split_grid(lib, Pa):
    key = (torch.cuda.current_device(), Pa)
    if key not in _SPLIT_GRID:
        g = int(lib.h2o_glm_wide_split_grid(Pa))
        _SPLIT_GRID[key] = g if g > 0 else 2048
    return _SPLIT_GRID[key]


def glm_wide_irls(X, P, beta, b0, y, wprior=None, offset=None, codes=(1, 1), tvp=0.0, theta=1e-10, step=1 << 19,
                  fused=False, bf3=True, eta_only=False):
    """Fused IRLS pass for wide GLMs (P + 2 <= 1024).

    fused=True (needs the exact-gradient channel: the Gram carries no z
    column; bf3=False: a one-MFMA bf16 Hessian for the GLM's lowest
    precision tier): per row chunk glm_wide_split_kernel computes eta, the IRLS
    weight, deviance and X'r and writes only the row weights; then ONE
    glm_wide_gram_kernel launch builds [X | 1]' W [X | 1] straight from the
    f32 rows (bf16x3 MFMA, f64 folds) -- no bf16 planes, no library GEMM.
    fused=False: the kernel writes bf16 [hi | lo] planes of sqrt(W) [x | 1 |
    z] and one bf16 library GEMM per chunk group forms the Gram.

    Returns (G [Pa, Pa] f64 augmented Gram, deviance f64, g [Pa] f64
    exact-gradient channel X'r with g[P] = sum r, r = w (y - mu) dmu/deta /
    var: f32 VALU products over <= 64 rows per lane, f64 beyond).
    eta_only (fused): the eta / deviance / gradient pass alone, G is None --
    the deviance at a coefficient vector and X'r for lambda_max."""
    lib = _lib()
    if lib is None:
        raise RuntimeError("gram extension not built (run __graft_entry__.build())")
    N, ldx = X.shape
    X = X.contiguous()
    Pa = -(-(P + 2) // 64) * 64
    if Pa > 1024:
        raise ValueError("glm_wide_irls: P + 2 must be <= 1024")
    bt = _f32(beta)
    keep = [_f32(y), _f32(wprior), _f32(offset)]
    st = min(step, max(N, 1))
    nch = -(-N // st)
    if fused:
        from ..utils.timer import phase
        # one launch over every row (the kernel folds its f32 gradient
        # products into f64 every 64 rows), on a grid of whole resident
        # rounds: 24 launches of 2048 workgroups took 10.5 ms at 12.5M x 1000,
        # one launch of 768 takes 8.1 ms (scripts/wide_eta_mb.py)
        st, nch = max(N, 1), 1
        blocks = int(os.environ.get("H2O3_WIDE_ETA_BLOCKS", "0")) or _wide_split_grid(lib, Pa)
        dev = torch.zeros((nch, blocks), dtype=torch.float64, device=X.device)
        gbuf = torch.zeros((blocks, Pa), dtype=torch.float64, device=X.device)
        # row weights, zero-padded to whole 64-row chunks (the Gram kernel
        # reads each chunk's weights with scalar vector loads)
        wr = torch.empty(-(-N // 64) * 64, dtype=torch.float32, device=X.device)
        wr[N:].zero_()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        offp = lambda t, a: ctypes.c_void_p(0 if t is None else t.data_ptr() + a * 4)
        with phase("glm.wide_eta"):
            for i, a in enumerate(range(0, N, st)):
                r = min(st, N - a)
                rc = lib.h2o_glm_wide_split(ctypes.c_void_p(X.data_ptr() + a * ldx * 4), ldx, P, Pa, r, _ptr(bt),
                                            float(b0), offp(keep[0], a), offp(keep[1], a), offp(keep[2], a),
                                            int(codes[0]), int(codes[1]), float(tvp), float(theta), None,
                                            _ptr(dev[i]), blocks, _ptr(gbuf), offp(wr, a), stream)
                if rc != 0:
                    raise RuntimeError(f"h2o_glm_wide_split failed: {rc}")
        if eta_only:
            return None, dev.sum(), gbuf.sum(0)
        with phase("glm.wide_gram"):
            G = wide_gram(X, P, wr, stream, bf3=bf3)
        return G, dev.sum(), gbuf.sum(0)
    grp = min(nch, _WIDE_GROUP)
    HL = torch.empty((grp * st, 2 * Pa), dtype=torch.bfloat16, device=X.device)
    blocks = 2048
    dev = torch.zeros((nch, blocks), dtype=torch.float64, device=X.device)
    gbuf = torch.zeros((blocks, Pa), dtype=torch.float64, device=X.device)
    G = torch.zeros((Pa, Pa), dtype=torch.float64, device=X.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def off(t, a):
        return ctypes.c_void_p(0 if t is None else t.data_ptr() + a * 4)

    def split(i, a, r, buf, j, strm):
        rc = lib.h2o_glm_wide_split(ctypes.c_void_p(X.data_ptr() + a * ldx * 4), ldx, P, Pa, r, _ptr(bt),
                                    float(b0), off(keep[0], a), off(keep[1], a), off(keep[2], a), int(codes[0]),
                                    int(codes[1]), float(tvp), float(theta),
                                    ctypes.c_void_p(buf.data_ptr() + j * st * 2 * Pa * 2), _ptr(dev[i]), blocks,
                                    _ptr(gbuf), None, strm)
        if rc != 0:
            raise RuntimeError(f"h2o_glm_wide_split failed: {rc}")

    if _overlap_ok(X, nch, grp):
        _pipelined_groups(split, HL, N, st, grp, Pa, G)
        return G, dev.sum(), gbuf.sum(0)
    for i, a in enumerate(range(0, N, st)):
        r = min(st, N - a)
        j = i % grp
        split(i, a, r, HL, j, stream)
        if r < st:
            HL[j * st + r:(j + 1) * st].zero_()
        if j == grp - 1 or i == nch - 1:
            _gram_group(HL[:(j + 1) * st], st, Pa, G)
    return G, dev.sum(), gbuf.sum(0)


def weighted_gram_aug(X: torch.Tensor, W: torch.Tensor, z: torch.Tensor, P: int, step: int = 1 << 20):
    """Augmented weighted Gram of [X[:, :P] | 1 | z] for wide GLMs in ONE
    library GEMM per 1M-row chunk (rocBLAS/hipBLASLt fp32, f64 accumulation):
    returns (X'WX [P,P], X'W [P], X'Wz [P], sum W, sum Wz) as f64.  The
    transposed GEMVs X'W / X'Wz on a row-major X run at a fraction of the GEMM
    rate on ROCm (~475 ms vs the Gram's ~240 ms at N=12.5M, P=1000), riding
    them on the Gram as two extra columns costs ~0.2%."""
    N = X.shape[0]
    if X.device.type == "cuda" and _wide_mode() == "bf3":
        G = gram_aug_bf3(X, W, z, P)
        return G[:P, :P], G[:P, P], G[:P, P + 1], G[P, P], G[P, P + 1]
    G = torch.zeros((P + 2, P + 2), dtype=torch.float64, device=X.device)
    for a in range(0, N, step):
        s = W[a:a + step].to(torch.float32).clamp_min(0).sqrt()
        Xa = torch.cat([X[a:a + step, :P] * s.view(-1, 1), s.view(-1, 1),
                        (s * z[a:a + step].to(torch.float32)).view(-1, 1)], 1)
        G += (Xa.T @ Xa).to(torch.float64)
    return G[:P, :P], G[:P, P], G[:P, P + 1], G[P, P], G[P, P + 1]
