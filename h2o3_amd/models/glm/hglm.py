"""HGLM: GLM with random intercepts (gaussian fixed + gaussian random effects).

Reference: hex/glm/GLM.java fitHGLM / ComputeHGLMTask (h-likelihood of Lee &
Nelder; parameters HGLM=True, random_columns, rand_family=["gaussian"],
rand_link=["identity"]); outputs fixed coefficients, random effects `ubeta`,
dispersion of the residuals `varfix` and of the random effects `varranef`,
and the h-likelihood.

For the gaussian/gaussian case the h-likelihood estimates coincide with the
linear mixed model fitted by Henderson's mixed-model equations:

    [X'X    X'Z         ] [b]   [X'y]
    [Z'X    Z'Z + l I   ] [u] = [Z'y],   l = varfix / varranef,

with variance components updated by EM until they stop moving.  Z is the
one-hot design of each random (categorical) column, so Z'Z is diagonal and
X'Z / Z'y are per-level segment sums: all sufficient statistics come from one
GPU pass (Gram on the matrix cores + index_add per level) and an all-reduce,
the (p+q)^2 solve is tiny and runs on the host in float64.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ...parallel import collectives as coll
from ..datainfo import DataInfo
from ...core.groupsum import index_add as _ia
from ...ops import linalg_ops


def fit_hglm(est, spec):
    p = est._parms
    rc = p.get("random_columns") or []
    names = spec.frame.names
    rcols = [names[c] if isinstance(c, int) else c for c in rc]
    if not rcols:
        raise ValueError("HGLM needs random_columns")
    for c in rcols:
        if spec.frame.vec(c).type != "enum":
            raise ValueError(f"random column {c} must be categorical")
    fam = (p.get("family") or "gaussian").lower()
    if fam not in ("gaussian", "auto"):
        raise ValueError("HGLM supports family='gaussian' with rand_family='gaussian'")
    xfix = [c for c in spec.x if c not in rcols]
    di = DataInfo(spec.frame, xfix, standardize=False, missing_values_handling=p.get("missing_values_handling"),
                  plug_values=p.get("plug_values"))
    X, ok = di.expand(spec.frame, dtype=torch.float64, pad=False)
    y = spec.y_tensor().to(torch.float64)
    ok &= ~torch.isnan(y)
    w = spec.w_tensor()
    w = torch.ones_like(y) if w is None else w.to(torch.float64)
    w = torch.where(ok, w, torch.zeros_like(w))
    y = torch.where(ok, y, torch.zeros_like(y))
    n = X.shape[0]
    X1 = torch.cat([X, torch.ones((n, 1), dtype=torch.float64, device=X.device)], 1)   # intercept last
    P = X1.shape[1]
    # random-effect designs: one block per random column
    blocks, q_off, levels = [], [], []
    off = 0
    for c in rcols:
        v = spec.frame.vec(c)
        codes = v.data.long()
        L = len(v.domain)
        blocks.append((codes, L))
        q_off.append(off)
        levels.append(list(v.domain))
        off += L
    Q = off
    # sufficient statistics: X'WX, X'Wy, X'WZ, Z'WZ (diag + cross blocks), Z'Wy
    XtX = linalg_ops.tmm(X1, X1 * w.view(-1, 1))
    Xty = linalg_ops.tmm(X1, w * y)
    XtZ = torch.zeros((P, Q), dtype=torch.float64, device=X.device)
    ZtZ = torch.zeros((Q, Q), dtype=torch.float64, device=X.device)
    Zty = torch.zeros(Q, dtype=torch.float64, device=X.device)
    for bi, (codes, L) in enumerate(blocks):
        okc = (codes >= 0) & (w > 0)
        cc = codes.clamp(min=0)
        o = q_off[bi]
        wz = torch.where(okc, w, torch.zeros_like(w))
        XtZ[:, o:o + L] = _ia(torch.zeros((L, P), dtype=torch.float64, device=X.device),
                              cc, X1 * wz.view(-1, 1)).T
        Zty[o:o + L] = _ia(torch.zeros(L, dtype=torch.float64, device=X.device), cc, wz * y)
        for bj, (codes2, L2) in enumerate(blocks):
            o2 = q_off[bj]
            ok2 = okc & (codes2 >= 0)
            key = cc * L2 + codes2.clamp(min=0)
            cnt = _ia(torch.zeros(L * L2, dtype=torch.float64, device=X.device),
                      key, torch.where(ok2, w, torch.zeros_like(w)))
            ZtZ[o:o + L, o2:o2 + L2] = cnt.view(L, L2)
    yty = (w * y * y).sum().view(1)
    stats = torch.cat([XtX.reshape(-1), Xty, XtZ.reshape(-1), ZtZ.reshape(-1), Zty, yty, w.sum().view(1)])
    coll.allreduce_(stats)
    S = stats.cpu().numpy()
    o = 0
    XtX = S[o:o + P * P].reshape(P, P); o += P * P
    Xty = S[o:o + P]; o += P
    XtZ = S[o:o + P * Q].reshape(P, Q); o += P * Q
    ZtZ = S[o:o + Q * Q].reshape(Q, Q); o += Q * Q
    Zty = S[o:o + Q]; o += Q
    yty, nobs = float(S[o]), float(S[o + 1])
    # EM on the variance components (one varranef per random column)
    nb = len(blocks)
    sig_e = float(p.get("init_dispersion_parameter") or 1.0)
    sig_u = np.ones(nb)
    startval = p.get("startval")
    if startval is not None and len(startval) >= P + 1 + nb:
        sig_u = np.asarray(startval[P:P + nb], dtype=float)
        sig_e = float(startval[P + nb])
    max_it = int(p.get("max_iterations") or -1)
    max_it = 100 if max_it <= 0 else max_it
    eps = float(p.get("objective_epsilon") or -1)
    eps = 1e-6 if eps <= 0 else eps
    A = np.zeros((P + Q, P + Q))
    A[:P, :P], A[:P, P:], A[P:, :P], A[P:, P:] = XtX, XtZ, XtZ.T, ZtZ
    rhs = np.concatenate([Xty, Zty])
    sizes = [L for _, L in blocks]
    it = 0
    for it in range(1, max_it + 1):
        lam = np.concatenate([np.full(L, sig_e / max(sig_u[k], 1e-12)) for k, L in enumerate(sizes)])
        C = A.copy()
        C[P:, P:] += np.diag(lam)
        Ci = np.linalg.pinv(C)
        sol = Ci @ rhs
        b, u = sol[:P], sol[P:]
        # residual sum of squares from the sufficient statistics
        rss = yty - 2 * sol @ rhs + sol @ A @ sol
        new_u = np.empty(nb)
        edf = 0.0
        for k, L in enumerate(sizes):
            sl = slice(P + q_off[k], P + q_off[k] + L)
            uk = sol[sl]
            tr = float(np.trace(Ci[sl, sl]))
            new_u[k] = (uk @ uk + sig_e * tr) / L
            edf += L - tr * sig_e / max(sig_u[k], 1e-12)
        new_e = (rss + sig_e * (P + edf)) / nobs
        new_e = max(new_e, 1e-12)
        delta = abs(new_e - sig_e) / max(sig_e, 1e-12) + float(np.max(np.abs(new_u - sig_u) / np.maximum(sig_u, 1e-12)))
        sig_e, sig_u = new_e, np.maximum(new_u, 1e-12)
        if delta < eps:
            break
    lam = np.concatenate([np.full(L, sig_e / sig_u[k]) for k, L in enumerate(sizes)])
    C = A.copy()
    C[P:, P:] += np.diag(lam)
    sol = np.linalg.pinv(C) @ rhs
    b, u = sol[:P], sol[P:]
    rss = yty - 2 * sol @ rhs + sol @ A @ sol
    # h-likelihood: log f(y|u) + log f(u)
    hlik = -0.5 * (nobs * math.log(2 * math.pi * sig_e) + rss / sig_e)
    for k, L in enumerate(sizes):
        uk = u[q_off[k]:q_off[k] + L]
        hlik += -0.5 * (L * math.log(2 * math.pi * sig_u[k]) + float(uk @ uk) / sig_u[k])
    est._hglm = {"dinfo": di, "beta": b, "u": u, "q_off": q_off, "rcols": rcols, "levels": levels,
                 "varfix": sig_e, "varranef": sig_u.tolist(), "iterations": it, "hlik": hlik}
    names_f = di.coef_names + ["Intercept"]
    est._output["coefficients"] = {n: float(v) for n, v in zip(names_f, b)}
    est._output["ubeta"] = {c: dict(zip(levels[k], u[q_off[k]:q_off[k] + sizes[k]].tolist()))
                            for k, c in enumerate(rcols)}
    est._output["varfix"] = sig_e
    est._output["varranef"] = sig_u.tolist()
    est._output["hlik"] = hlik
    est._output["iterations"] = it
    est._output["model_summary"] = {"family": "gaussian", "link": "identity", "random_columns": rcols,
                                    "rand_family": "gaussian", "number_of_iterations": it}


def predict_hglm(est, frame):
    h = est._hglm
    X, _ = h["dinfo"].expand(frame, dtype=torch.float64, pad=False)
    eta = X @ torch.as_tensor(h["beta"][:-1], dtype=torch.float64, device=X.device) + float(h["beta"][-1])
    for k, c in enumerate(h["rcols"]):
        if c not in frame.names:
            continue
        v = frame.vec(c)
        idx = {d: i for i, d in enumerate(h["levels"][k])}
        remap = torch.tensor([idx.get(d, -1) for d in v.domain] or [-1], dtype=torch.long, device=X.device)
        codes = torch.where(v.data < 0, torch.full_like(v.data.long(), -1), remap[v.data.clamp(min=0).long()])
        uk = torch.as_tensor(h["u"][h["q_off"][k]:h["q_off"][k] + len(h["levels"][k])], dtype=torch.float64,
                             device=X.device)
        eta = eta + torch.where(codes >= 0, uk[codes.clamp(min=0)], torch.zeros_like(eta))
    return eta.view(-1, 1)
