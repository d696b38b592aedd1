"""Multinomial and ordinal GLM.

Reference: hex/glm/GLM.java fitIRLSM_multinomial / fitLBFGS and
hex/glm/GLMTask.GLMMultinomialGradientTask, ordinal via
GLMTask.GLMMultinomialGradientBaseTask (cumulative logit, "ologit").

Optimizer: smooth part by L-BFGS (torch, float64 parameters, f32 GEMMs on
the device), L1 by proximal-gradient (FISTA) iterations — both driven by the
same all-reduced gradient so the multi-GPU path is one all_reduce per
evaluation.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ...parallel import collectives as coll
from ..datainfo import DataInfo


def _loss_grad_multinomial(X, Y, w, B, b0, wsum):
    eta = X @ B.to(X.dtype) + b0.to(X.dtype)
    eta = eta.to(torch.float64)
    lse = torch.logsumexp(eta, 1)
    ll = (w * (lse - (eta * Y).sum(1))).sum()
    P = torch.softmax(eta, 1)
    R = (P - Y) * w.view(-1, 1)
    gB = (X.T @ R.to(X.dtype)).to(torch.float64)
    gb = R.sum(0)
    s = torch.cat([ll.view(1), gB.reshape(-1), gb])
    coll.allreduce_(s)
    K = B.shape[1]
    return float(s[0]) / wsum, s[1:1 + B.numel()].view_as(B) / wsum, s[1 + B.numel():] / wsum


def _loss_grad_ordinal(X, y, w, beta, theta, wsum, K):
    eta = (X @ beta.to(X.dtype)).to(torch.float64)
    th = torch.cumsum(torch.cat([theta[:1], torch.nn.functional.softplus(theta[1:])]), 0)
    # P(y<=k) = sigmoid(th_k - eta), k=0..K-2
    cdf = torch.sigmoid(th.view(1, -1) - eta.view(-1, 1))
    cdf = torch.cat([torch.zeros_like(eta).view(-1, 1), cdf, torch.ones_like(eta).view(-1, 1)], 1)
    pk = (cdf[:, 1:] - cdf[:, :-1]).clamp_min(1e-15)
    yi = y.long().clamp(min=0)
    ll = -(w * torch.log(pk[torch.arange(y.numel(), device=y.device), yi])).sum()
    return ll, pk


def fit_multinomial(est, spec, fam):
    p = est._parms
    from .interactions import interaction_pairs
    dinfo = DataInfo(spec.frame, spec.x, standardize=bool(p.get("standardize", True)),
                     missing_values_handling=p.get("missing_values_handling"), plug_values=p.get("plug_values"),
                     interactions=interaction_pairs(spec.x, p.get("interactions"), p.get("interaction_pairs")))
    X, ok = dinfo.expand(spec.frame)
    y = spec.y_tensor()
    ok &= y >= 0
    w = spec.w_tensor()
    w = torch.ones(y.numel(), dtype=torch.float64, device=X.device) if w is None else w.to(torch.float64)
    w = torch.where(ok, w, torch.zeros_like(w))
    K = spec.nclasses
    wsum = coll.allreduce_scalar(float(w.sum()))
    alpha = p.get("alpha")
    alpha = 0.0 if alpha is None and (p.get("solver") or "").upper() == "L_BFGS" else (0.5 if alpha is None else alpha)
    alpha = float(alpha[0] if isinstance(alpha, (list, tuple)) else alpha)
    lam = p.get("lambda_")
    Pp = dinfo.Pp
    dev = X.device
    est._dinfo = dinfo
    if fam == "multinomial":
        Y = torch.nn.functional.one_hot(y.clamp(min=0), K).to(torch.float64)
        B = torch.zeros((Pp, K), dtype=torch.float64, device=dev)
        cnt = (Y * w.view(-1, 1)).sum(0)
        coll.allreduce_(cnt)
        pri = (cnt / cnt.sum()).clamp_min(1e-10)
        b0 = torch.log(pri) - torch.log(pri).mean()
        if lam is None:
            _, gB, _ = _loss_grad_multinomial(X, Y, w, B, b0, wsum)
            lmax = float(gB.abs().max()) / max(alpha, 1e-2)
            lmr = 1e-4 if wsum / 16 > dinfo.P else 1e-2
            lam = 10 * lmr * lmax
        lam = float(lam[0] if isinstance(lam, (list, tuple)) else lam)
        l1, l2 = lam * alpha, lam * (1 - alpha)
        params = torch.cat([B.reshape(-1), b0]).clone()

        def f_g(th):
            Bm = th[: Pp * K].view(Pp, K)
            bb = th[Pp * K:]
            f, gB, gb = _loss_grad_multinomial(X, Y, w, Bm, bb, wsum)
            f += 0.5 * l2 * float((Bm ** 2).sum())
            gB = gB + l2 * Bm
            return f, torch.cat([gB.reshape(-1), gb])
        th = _optimize(f_g, params, l1, Pp * K, max_iter=int(p.get("max_iterations") or -1) if
                       int(p.get("max_iterations") or -1) > 0 else 200)
        B = th[: Pp * K].view(Pp, K)[: dinfo.P]
        b0 = th[Pp * K:]
        est._multi = {"kind": "multinomial", "B": B, "b0": b0}
        coefs = {}
        Bn = B.cpu().numpy()
        for k, cls in enumerate(spec.response_domain):
            bk, ik = dinfo.destandardize(Bn[:, k], float(b0[k]))
            coefs[cls] = {"Intercept": ik, **{n: float(v) for n, v in zip(dinfo.coef_names, bk)}}
        est._output["coefficients_table_multinomials"] = coefs
        est._output["coefficients"] = {f"{n}_{cls}": v for cls, d in coefs.items() for n, v in d.items()}
        est._output["variable_importances"] = {n: float(np.abs(Bn[i]).sum()) for i, n in enumerate(dinfo.coef_names)}
    else:  # ordinal
        beta = torch.zeros(Pp, dtype=torch.float64, device=dev)
        cnt = torch.bincount(y.clamp(min=0), weights=w, minlength=K).to(torch.float64)
        coll.allreduce_(cnt)
        cum = torch.cumsum(cnt / cnt.sum(), 0)[:-1].clamp(1e-6, 1 - 1e-6)
        t0 = torch.log(cum / (1 - cum))
        theta = torch.cat([t0[:1], torch.log(torch.expm1((t0[1:] - t0[:-1]).clamp_min(1e-6)))])
        lam = 0.0 if lam is None else float(lam[0] if isinstance(lam, (list, tuple)) else lam)
        l1, l2 = lam * alpha, lam * (1 - alpha)
        params = torch.cat([beta, theta]).clone()

        def f_g(th):
            t = th.detach().clone().requires_grad_(True)
            ll, _ = _loss_grad_ordinal(X, y, w, t[:Pp], t[Pp:], wsum, K)
            ll = ll / wsum
            ll.backward()
            g = t.grad.detach()
            s = torch.cat([ll.detach().view(1), g])
            coll.allreduce_(s)
            f = float(s[0]) + 0.5 * l2 * float((th[:Pp] ** 2).sum())
            g = s[1:].clone()
            g[:Pp] += l2 * th[:Pp]
            return f, g
        th = _optimize(f_g, params, l1, Pp, max_iter=200)
        est._multi = {"kind": "ordinal", "beta": th[:Pp][: dinfo.P], "theta": th[Pp:]}
        bn, _ = dinfo.destandardize(th[:Pp][: dinfo.P].cpu().numpy(), 0.0)
        est._output["coefficients"] = {n: float(v) for n, v in zip(dinfo.coef_names, bn)}
        est._output["variable_importances"] = {n: abs(float(v)) for n, v in zip(dinfo.coef_names, bn)}
    est._output["model_summary"] = {"family": fam, "lambda": lam, "alpha": alpha}


def _optimize(f_g, x0, l1, n_pen, max_iter=200, tol=1e-7):
    """L-BFGS (l1 == 0) or FISTA proximal gradient (l1 > 0)."""
    x = x0.clone()
    if l1 <= 0:
        m = 10
        S, Yh = [], []
        f, g = f_g(x)
        for it in range(max_iter):
            q = g.clone()
            al = []
            for s, yv in reversed(list(zip(S, Yh))):
                rho = 1.0 / float(yv @ s)
                a = rho * float(s @ q)
                al.append((a, rho, s, yv))
                q -= a * yv
            if S:
                gam = float(S[-1] @ Yh[-1]) / float(Yh[-1] @ Yh[-1])
                q *= gam
            for a, rho, s, yv in reversed(al):
                b = rho * float(yv @ q)
                q += (a - b) * s
            d = -q
            step = 1.0
            gd = float(g @ d)
            if gd >= 0:
                d = -g
                gd = float(g @ d)
                S, Yh = [], []
            while True:
                xn = x + step * d
                fn, gn = f_g(xn)
                if fn <= f + 1e-4 * step * gd or step < 1e-10:
                    break
                step *= 0.5
            s, yv = xn - x, gn - g
            if float(s @ yv) > 1e-12:
                S.append(s)
                Yh.append(yv)
                if len(S) > m:
                    S.pop(0)
                    Yh.pop(0)
            conv = abs(f - fn) < tol * max(1.0, abs(f))
            x, f, g = xn, fn, gn
            if conv or float(g.abs().max()) < 1e-8:
                break
        return x
    # FISTA with backtracking
    L = 1.0
    y = x.clone()
    t = 1.0
    f, g = f_g(y)
    for it in range(max_iter * 5):
        while True:
            z = y - g / L
            z[:n_pen] = torch.sign(z[:n_pen]) * torch.clamp(z[:n_pen].abs() - l1 / L, min=0)
            fz, gz = f_g(z)
            dz = z - y
            if fz <= f + float(g @ dz) + 0.5 * L * float(dz @ dz) + 1e-12:
                break
            L *= 2
        tn = (1 + math.sqrt(1 + 4 * t * t)) / 2
        yn = z + ((t - 1) / tn) * (z - x)
        if float((z - x).abs().max()) < 1e-7:
            x = z
            break
        x, t, y = z, tn, yn
        f, g = f_g(y)
        L = max(L * 0.9, 1e-6)
    return x


def predict_multi(est, frame):
    X, _ = est._dinfo.expand(frame)
    m = est._multi
    P = est._dinfo.P
    if m["kind"] == "multinomial":
        eta = (X[:, :P].to(torch.float64) @ m["B"]) + m["b0"].view(1, -1)
        return torch.softmax(eta, 1)
    eta = X[:, :P].to(torch.float64) @ m["beta"]
    th = m["theta"]
    thc = torch.cumsum(torch.cat([th[:1], torch.nn.functional.softplus(th[1:])]), 0)
    cdf = torch.sigmoid(thc.view(1, -1) - eta.view(-1, 1))
    cdf = torch.cat([torch.zeros_like(eta).view(-1, 1), cdf, torch.ones_like(eta).view(-1, 1)], 1)
    return (cdf[:, 1:] - cdf[:, :-1]).clamp_min(0)
