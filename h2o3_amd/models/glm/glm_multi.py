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
from ...core.groupsum import group_sum
from ...ops import linalg_ops


def _loss_grad_multinomial(X, Y, w, B, b0, wsum):
    eta = X @ B.to(X.dtype) + b0.to(X.dtype)
    eta = eta.to(torch.float64)
    lse = torch.logsumexp(eta, 1)
    ll = (w * (lse - (eta * Y).sum(1))).sum()
    P = torch.softmax(eta, 1)
    R = (P - Y) * w.view(-1, 1)
    gB = linalg_ops.tmm(X, R.to(X.dtype)).to(torch.float64)
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


def _loss_sqerr_ordinal(X, y, w, beta_ref, icpt):
    """GRADIENT_DESCENT_SQERR loss (GLMTask.computeGradientMultipliersSQERR):
    reference parameterisation eta_c = x.beta + icpt_c; for classes c < y an
    eta_c > 0 costs w eta_c^2 / 2, for y <= c < K-1 an eta_c <= 0 does."""
    eta = (X @ beta_ref.to(X.dtype)).to(torch.float64).view(-1, 1) + icpt.view(1, -1)
    c = torch.arange(icpt.numel(), device=eta.device).view(1, -1)
    yi = y.long().clamp(min=0).view(-1, 1)
    bad = torch.where(c < yi, eta > 0, eta <= 0)
    return (w.view(-1, 1) * 0.5 * torch.where(bad, eta * eta, torch.zeros_like(eta))).sum()


def _loss_lh_ordinal_ref(X, y, w, beta_ref, icpt):
    eta = (X @ beta_ref.to(X.dtype)).to(torch.float64).view(-1, 1) + icpt.view(1, -1)
    cdf = torch.sigmoid(eta)
    one = torch.ones_like(eta[:, :1])
    cdf = torch.cat([torch.zeros_like(one), cdf, one], 1)
    pk = (cdf[:, 1:] - cdf[:, :-1]).clamp_min(1e-15)
    yi = y.long().clamp(min=0)
    return -(w * torch.log(pk[torch.arange(y.numel(), device=y.device), yi])).sum()


def _fit_ordinal_gd(X, y, w, wsum, K, Pp, l1, l2, p, sqerr):
    """fitIRLSM_ordinal_default (GLM.java:1917): plain gradient descent with
    unit step on the obj_reg-scaled gradient, thresholds started from sorted
    seeded uniforms in [-K, K] (GLM.java:808), stopped when an update would
    un-order the thresholds, at max_iterations, or when the objective /
    coefficients stop moving.  Returns (beta_ref, icpt, iterations)."""
    seed = p.get("seed", -1)
    rs = np.random.RandomState((int(seed) if seed not in (None, -1) else 1234) & 0x7FFFFFFF)
    icpt = torch.as_tensor(np.sort((-1 + 2 * rs.random_sample(K - 1)) * K), dtype=torch.float64, device=X.device)
    beta = torch.zeros(Pp, dtype=torch.float64, device=X.device)
    loss_fn = _loss_sqerr_ordinal if sqerr else _loss_lh_ordinal_ref
    maxit = int(p.get("max_iterations") or -1)
    maxit = 50 if maxit <= 0 else maxit
    oe = float(p.get("objective_epsilon") or -1)
    oe = oe if oe > 0 else 1e-6
    be = float(p.get("beta_epsilon") or 1e-4)
    obj_reg = 1.0 / wsum

    def grad(b, t):
        bb = b.detach().clone().requires_grad_(True)
        tt = t.detach().clone().requires_grad_(True)
        f = loss_fn(X, y, w, bb, tt)
        f.backward()
        s = torch.cat([f.detach().view(1), bb.grad, tt.grad])
        coll.allreduce_(s)
        f = float(s[0]) * obj_reg + 0.5 * l2 * float((b ** 2).sum())
        return f, s[1:1 + Pp] * obj_reg + l2 * b, s[1 + Pp:] * obj_reg
    f, gb, gt = grad(beta, icpt)
    it = 0
    while it < maxit:
        nt = icpt - gt
        if bool((nt[1:] < nt[:-1]).any()):
            break           # thresholds would lose their order: stop with the last eligible ones
        nb = beta - (gb + l1 * torch.sign(beta))
        it += 1
        fn, gb, gt = grad(nb, nt)
        diff = max(float((nb - beta).abs().max()) if Pp else 0.0, float((nt - icpt).abs().max()))
        beta, icpt = nb, nt
        done = diff < be or abs(f - fn) < oe * max(abs(fn), 1e-12)
        f = fn
        if done:
            break
    return beta, icpt, it


def _ordinal_to_internal(beta_ref, icpt):
    """Reference (eta_c = x.b + t_c) -> the internal cumulative
    parameterisation (cdf_c = sigmoid(thc_c - x.beta), increments softplus)."""
    d = (icpt[1:] - icpt[:-1]).clamp_min(1e-12)
    return -beta_ref, torch.cat([icpt[:1], torch.log(torch.expm1(d))])


def _lambda_path(est, p, lmax, alpha, wsum, P):
    lam = p.get("lambda_")
    if lam is not None:
        lams = list(lam) if isinstance(lam, (list, tuple)) else [float(lam)]
        return sorted(lams, reverse=True) if p.get("lambda_search") else lams
    lmr = float(p.get("lambda_min_ratio") or -1)
    if lmr == -1:
        lmr = 1e-4 if wsum / 16 > P else 1e-2
        if alpha == 0:
            lmr *= 1e-2
    if p.get("lambda_search"):
        nl = int(p.get("nlambdas") or -1)
        nl = (30 if alpha == 0 else 100) if nl == -1 else nl
        dec = lmr ** (1.0 / max(nl - 1, 1))
        return [lmax * dec ** i for i in range(nl)]
    return [10 * lmr * lmax]


def fit_multinomial(est, spec, fam):
    """Multinomial / ordinal fit over the lambda path (warm started, GLM.java
    lambda-search early stopping), submodel picked by validation deviance
    when given.  Ordinal coefficients are reported in the reference's
    parameterisation (P(y <= c) = sigmoid(x.beta + intercept_c))."""
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
    solver = (p.get("solver") or "AUTO").upper()
    alpha = p.get("alpha")
    alpha = 0.0 if alpha is None and solver == "L_BFGS" else (0.5 if alpha is None else alpha)
    alpha = float(alpha[0] if isinstance(alpha, (list, tuple)) else alpha)
    Pp = dinfo.Pp
    dev = X.device
    est._dinfo = dinfo
    maxit = int(p.get("max_iterations") or -1)
    maxit = maxit if maxit > 0 else 200
    oe = float(p.get("objective_epsilon") or -1)
    ge = float(p.get("gradient_epsilon") or -1)
    # GLM.java:1176: objective_epsilon defaults to 1e-4 on a lambda search
    tol = oe if oe > 0 else (1e-4 if p.get("lambda_search") else 1e-7)
    gtol = ge if ge > 0 else 1e-8
    valid = None
    if spec.valid is not None:
        Xv, okv = dinfo.expand(spec.valid)
        yv = spec.y_tensor(spec.valid)
        valid = (Xv, yv, (okv & (yv >= 0)).to(torch.float64))
    path = []
    if fam == "multinomial":
        Y = torch.nn.functional.one_hot(y.clamp(min=0), K).to(torch.float64)
        B = torch.zeros((Pp, K), dtype=torch.float64, device=dev)
        cnt = (Y * w.view(-1, 1)).sum(0)
        coll.allreduce_(cnt)
        pri = (cnt / cnt.sum()).clamp_min(1e-10)
        b0 = torch.log(pri) - torch.log(pri).mean()
        _, gB, _ = _loss_grad_multinomial(X, Y, w, B, b0, wsum)
        lmax = float(gB.abs().max()) / max(alpha, 1e-2)
        params = torch.cat([B.reshape(-1), b0]).clone()
        null_dev = 2 * _loss_grad_multinomial(X, Y, w, B, b0, wsum)[0] * wsum

        def dev_of(th, Xm, ym, wm, wsm):
            Ym = torch.nn.functional.one_hot(ym.clamp(min=0), K).to(torch.float64)
            return 2 * _loss_grad_multinomial(Xm, Ym, wm, th[: Pp * K].view(Pp, K), th[Pp * K:], wsm)[0] * wsm

        for lam in _lambda_path(est, p, lmax, alpha, wsum, dinfo.P):
            l1, l2 = lam * alpha, lam * (1 - alpha)

            def f_g(th, l2=l2):
                Bm = th[: Pp * K].view(Pp, K)
                bb = th[Pp * K:]
                f, gB, gb = _loss_grad_multinomial(X, Y, w, Bm, bb, wsum)
                f += 0.5 * l2 * float((Bm ** 2).sum())
                gB = gB + l2 * Bm
                return f, torch.cat([gB.reshape(-1), gb])
            params = _optimize(f_g, params, l1, Pp * K, max_iter=maxit, tol=tol, gtol=gtol)
            path.append({"lambda": lam, "th": params.clone(), "dev": dev_of(params, X, y, w, wsum)})
            if _path_should_stop(est, path, null_dev, valid, dev_of, lmax):
                break
    else:  # ordinal
        cnt = group_sum(y.clamp(min=0), torch.ones_like(y, dtype=torch.float64) if w is None else w, K)
        coll.allreduce_(cnt)
        sqerr = solver == "GRADIENT_DESCENT_SQERR"
        null_beta = torch.zeros(Pp, dtype=torch.float64, device=dev)
        cum = torch.cumsum(cnt / cnt.sum(), 0)[:-1].clamp(1e-6, 1 - 1e-6)
        t0 = torch.log(cum / (1 - cum))
        theta0 = torch.cat([t0[:1], torch.log(torch.expm1((t0[1:] - t0[:-1]).clamp_min(1e-6)))])
        params = torch.cat([null_beta, theta0]).clone()

        def dev_of(th, Xm, ym, wm, wsm):
            return 2 * coll.allreduce_scalar(float(_loss_grad_ordinal(Xm, ym, wm, th[:Pp], th[Pp:], wsm, K)[0]))
        null_dev = dev_of(params, X, y, w, wsum)
        # lambda_max from the slope gradient at the intercept-only model
        t = params.detach().clone().requires_grad_(True)
        ll, _ = _loss_grad_ordinal(X, y, w, t[:Pp], t[Pp:], wsum, K)
        ll.backward()
        g = t.grad[:Pp].clone()
        coll.allreduce_(g)
        lams = _lambda_path(est, p, float((g / wsum).abs().max()) / max(alpha, 1e-2), alpha, wsum, dinfo.P)
        lmax = lams[0]
        for lam in lams:
            l1, l2 = lam * alpha, lam * (1 - alpha)
            if sqerr:
                b_ref, icpt, _ = _fit_ordinal_gd(X, y, w, wsum, K, Pp, l1, l2, p, sqerr=True)
                bi, thi = _ordinal_to_internal(b_ref, icpt)
                params = torch.cat([bi, thi])
            else:
                def f_g(th, l2=l2):
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
                params = _optimize(f_g, params, l1, Pp, max_iter=maxit, tol=tol, gtol=gtol)
            path.append({"lambda": lam, "th": params.clone(), "dev": dev_of(params, X, y, w, wsum)})
            if _path_should_stop(est, path, null_dev, valid, dev_of, lmax):
                break
    best = len(path) - 1
    if valid is not None and len(path) > 1:
        Xv, yv, wv = valid
        wsv = coll.allreduce_scalar(float(wv.sum()))
        best = int(np.argmin([dev_of(s["th"], Xv, yv, wv, wsv) for s in path]))
    th = path[best]["th"]
    lam = path[best]["lambda"]
    if fam == "multinomial":
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
        reg_coefs = [{f"{n}_{cls}": v for cls, d in _multi_coefs(s["th"], dinfo, Pp, K, spec).items()
                      for n, v in d.items()} for s in path]
    else:
        est._multi = {"kind": "ordinal", "beta": th[:Pp][: dinfo.P], "theta": th[Pp:]}
        coefs = _ordinal_coefs(th, dinfo, Pp, spec)
        est._output["coefficients_table_multinomials"] = coefs
        first = next(iter(coefs.values()))
        est._output["coefficients"] = {n: v for n, v in first.items() if n != "Intercept"}
        est._output["variable_importances"] = {n: abs(float(v)) for n, v in est._output["coefficients"].items()}
        reg_coefs = [{n: v for n, v in next(iter(_ordinal_coefs(s["th"], dinfo, Pp, spec).values())).items()}
                     for s in path]
    est._output["model_summary"] = {"family": fam, "lambda": lam, "alpha": alpha}
    est._output["lambda_best"] = lam
    est._output["alpha_best"] = alpha
    est._output["null_deviance"] = null_dev
    est._output["residual_deviance"] = path[best]["dev"]
    est._output["regularization_path"] = {
        "lambdas": [s["lambda"] for s in path], "alphas": [alpha] * len(path),
        "explained_deviance_train": [1 - s["dev"] / null_dev if null_dev > 0 else None for s in path],
        "explained_deviance_valid": None, "coefficients": reg_coefs}


def _multi_coefs(th, dinfo, Pp, K, spec):
    B = th[: Pp * K].view(Pp, K)[: dinfo.P].cpu().numpy()
    b0 = th[Pp * K:]
    out = {}
    for k, cls in enumerate(spec.response_domain):
        bk, ik = dinfo.destandardize(B[:, k], float(b0[k]))
        out[cls] = {"Intercept": ik, **{n: float(v) for n, v in zip(dinfo.coef_names, bk)}}
    return out


def _ordinal_coefs(th, dinfo, Pp, spec):
    """Per-class coefficients in the reference's ordinal layout: one shared
    slope vector (sign of x.beta in P(y <= c) = sigmoid(x.beta + t_c)) and a
    threshold per class; the last class has none (GLM.java:808)."""
    beta_int = th[:Pp][: dinfo.P].cpu().numpy()
    t = th[Pp:]
    thc = torch.cumsum(torch.cat([t[:1], torch.nn.functional.softplus(t[1:])]), 0).cpu().numpy()
    out = {}
    for c, cls in enumerate(spec.response_domain):
        ic = float(thc[c]) if c < thc.size else 0.0
        b, i = dinfo.destandardize(-beta_int, ic)
        out[cls] = {"Intercept": i, **{n: float(v) for n, v in zip(dinfo.coef_names, b)}}
    return out


def _path_should_stop(est, path, null_dev, valid, dev_of, lmax):
    """GLM.java:2976 lambda-search early stopping over the multinomial /
    ordinal path: the last 5 relative training-deviance improvements all
    under 1e-4, or (validation, no CV) all negative."""
    p = est._parms
    if not p.get("lambda_search") or not p.get("early_stopping", True) or len(path) < 5:
        return False
    devs = [null_dev] + [s["dev"] for s in path]
    rel = [(devs[i] - devs[i + 1]) / devs[i] if devs[i] else 0.0 for i in range(len(devs) - 1)][-5:]
    if path[-1]["lambda"] < lmax and max(rel) < 1e-4:
        return True
    if valid is not None and int(p.get("nfolds") or 0) <= 1:
        Xv, yv, wv = valid
        wsv = coll.allreduce_scalar(float(wv.sum()))
        if "vdev" not in path[-1]:
            for s in path:
                if "vdev" not in s:
                    s["vdev"] = dev_of(s["th"], Xv, yv, wv, wsv)
        vd = [s["vdev"] for s in path]
        relv = [(vd[i] - vd[i + 1]) / vd[i] if vd[i] else 0.0 for i in range(len(vd) - 1)][-5:]
        if len(relv) == 5 and max(relv) < 0:
            return True
    return False


def _optimize(f_g, x0, l1, n_pen, max_iter=200, tol=1e-7, gtol=1e-8):
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
            if conv or float(g.abs().max()) < gtol:
                break
        return x
    # FISTA with backtracking
    L = 1.0
    y = x.clone()
    t = 1.0
    f, g = f_g(y)
    f_prev = None
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
        if float((z - x).abs().max()) < 1e-7 or (f_prev is not None and abs(f_prev - fz) < tol * max(1.0, abs(fz))):
            x = z
            break
        f_prev = fz
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
