"""Generalized Linear Models.

Reference: hex/glm/GLM.java (GLMDriver: fitIRLSM / fitLBFGS / fitCOD,
lambda search, `lmax` at GLM.java:1409, default lambda = 10*lambda_min_ratio
*lambda_max at GLM.java:1164), hex/glm/GLMTask.java (GLMIterationTask:
Gram + X'Wz per iteration), hex/gram/Gram.java (Cholesky),
hex/optimization/ADMM.java / L_BFGS.java, hex/glm/GLMModel.java
(coefficients, p-values, deviance/AIC output).

Objective (reference convention): mean weighted negative log-likelihood +
lambda*(alpha*|b|_1 + (1-alpha)/2*|b|_2^2), intercept unpenalized.

MI355X design: the expanded design matrix lives in HBM (DataInfo); one
IRLS iteration is a fused elementwise pass (eta, mu, working weights and
response), ONE weighted-Gram launch on the f32 matrix cores
(ops/csrc/gram.hip, f64 fold-in), one GEMV for X'Wz, an all-reduce of the
(P+1)^2 sufficient statistics over RCCL, and a tiny f64 solve on the host
(Cholesky for ridge, covariance-update coordinate descent for L1 — the
same quadratic subproblem the reference hands to ADMM).
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from ...core.frame import H2OFrame
from ...core.vec import T_ENUM, T_REAL, Vec
from ...ops import linalg_ops
from ...parallel import cloud
from ...parallel import collectives as coll
from ..base import H2OEstimator, ScoreKeeper, ScoreSchedule, _LESS_IS_BETTER
from ..datainfo import DataInfo
from ...utils.timer import phase
from .. import metrics as mm

GLM_DEFAULTS = dict(family="AUTO", tweedie_variance_power=0.0,
                    tweedie_link_power=1.0, theta=1e-10, solver="AUTO", alpha=None, lambda_=None,
                    lambda_search=False, early_stopping=True, nlambdas=-1, standardize=True,
                    missing_values_handling="MeanImputation", plug_values=None, compute_p_values=False,
                    dispersion_parameter_method="pearson", init_dispersion_parameter=1.0,
                    remove_collinear_columns=False, intercept=True, non_negative=False, max_iterations=-1,
                    objective_epsilon=-1.0, beta_epsilon=1e-4, gradient_epsilon=-1.0, link="family_default",
                    startval=None, calc_like=False, prior=-1.0, cold_start=False, lambda_min_ratio=-1.0,
                    beta_constraints=None, max_active_predictors=-1, interactions=None, interaction_pairs=None,
                    obj_reg=-1.0, stopping_rounds=0, stopping_metric="auto", stopping_tolerance=0.001,
                    balance_classes=False, class_sampling_factors=None, max_after_balance_size=5.0,
                    max_confusion_matrix_size=20, max_runtime_secs=0.0, custom_metric_func=None,
                    generate_scoring_history=False, auc_type="auto", dispersion_epsilon=1e-4,
                    max_iterations_dispersion=3000, build_null_model=False,
                    fix_dispersion_parameter=False, HGLM=False, random_columns=None, rand_family=None,
                    rand_link=None, score_iteration_interval=-1, seed=-1, checkpoint=None)

_DEFAULT_LINK = {"gaussian": "identity", "binomial": "logit", "quasibinomial": "logit",
                 "fractionalbinomial": "logit", "poisson": "log", "gamma": "inverse", "tweedie": "tweedie",
                 "negativebinomial": "log", "multinomial": "multinomial", "ordinal": "ologit"}


class _Fam:
    """Variance / link / deviance for one family (GLMModel.GLMWeightsFun)."""

    def __init__(self, family, link, tvp=0.0, tlp=1.0, theta=1e-10):
        self.family, self.link, self.tvp, self.tlp, self.theta = family, link, tvp, tlp, theta

    def linkinv(self, eta):
        l = self.link
        if l == "identity":
            return eta
        if l == "logit":
            return torch.sigmoid(eta)
        if l == "log":
            return torch.exp(torch.clamp(eta, max=700))
        if l == "inverse":
            return 1.0 / torch.where(eta.abs() < 1e-10, torch.full_like(eta, 1e-10) * torch.sign(eta + 1e-300), eta)
        if l == "tweedie":
            return torch.exp(eta) if self.tlp == 0 else torch.pow(eta.clamp_min(1e-10), 1.0 / self.tlp)
        raise ValueError(l)

    def link_fn(self, mu):
        l = self.link
        if l == "identity":
            return mu
        if l == "logit":
            return math.log(mu / (1 - mu))
        if l == "log":
            return math.log(mu)
        if l == "inverse":
            return 1.0 / mu
        if l == "tweedie":
            return math.log(mu) if self.tlp == 0 else mu ** self.tlp
        raise ValueError(l)

    def dmu_deta(self, eta, mu):
        l = self.link
        if l == "identity":
            return torch.ones_like(eta)
        if l == "logit":
            return (mu * (1 - mu)).clamp_min(1e-10)
        if l == "log":
            return mu.clamp_min(1e-10)
        if l == "inverse":
            return -(mu * mu)
        if l == "tweedie":
            if self.tlp == 0:
                return mu.clamp_min(1e-10)
            return (1.0 / self.tlp) * torch.pow(eta.clamp_min(1e-10), 1.0 / self.tlp - 1)
        raise ValueError(l)

    def variance(self, mu):
        f = self.family
        if f == "gaussian":
            return torch.ones_like(mu)
        if f in ("binomial", "quasibinomial", "fractionalbinomial"):
            return (mu * (1 - mu)).clamp_min(1e-10)
        if f == "poisson":
            return mu.clamp_min(1e-10)
        if f == "gamma":
            return (mu * mu).clamp_min(1e-10)
        if f == "tweedie":
            return torch.pow(mu.clamp_min(1e-10), self.tvp)
        if f == "negativebinomial":
            return (mu + self.theta * mu * mu).clamp_min(1e-10)
        raise ValueError(f)

    def deviance(self, y, mu):
        f = self.family
        if f == "gaussian":
            return (y - mu) ** 2
        if f in ("binomial", "quasibinomial", "fractionalbinomial"):
            m = mu.clamp(1e-15, 1 - 1e-15)
            t1 = torch.where(y > 0, y * torch.log(y.clamp_min(1e-300) / m), torch.zeros_like(y))
            t2 = torch.where(y < 1, (1 - y) * torch.log((1 - y).clamp_min(1e-300) / (1 - m)), torch.zeros_like(y))
            return 2 * (t1 + t2)
        if f == "poisson":
            t = torch.where(y > 0, y * torch.log(y.clamp_min(1e-300) / mu.clamp_min(1e-300)), torch.zeros_like(y))
            return 2 * (t - (y - mu))
        if f == "gamma":
            return 2 * (-torch.log(y.clamp_min(1e-300) / mu) + (y - mu) / mu)
        if f == "tweedie":
            p = self.tvp
            if p == 0:
                return (y - mu) ** 2
            if p == 1:
                t = torch.where(y > 0, y * torch.log(y.clamp_min(1e-300) / mu), torch.zeros_like(y))
                return 2 * (t - (y - mu))
            if p == 2:
                return 2 * (-torch.log(y.clamp_min(1e-300) / mu) + (y - mu) / mu)
            a = torch.where(y > 0, torch.pow(y.clamp_min(0), 2 - p) / ((1 - p) * (2 - p)), torch.zeros_like(y))
            return 2 * (a - y * torch.pow(mu, 1 - p) / (1 - p) + torch.pow(mu, 2 - p) / (2 - p))
        if f == "negativebinomial":
            th = self.theta
            t1 = torch.where(y > 0, y * torch.log(y.clamp_min(1e-300) / mu), torch.zeros_like(y))
            t2 = (y + 1 / th) * torch.log((1 + th * y) / (1 + th * mu))
            return 2 * (t1 - t2)
        raise ValueError(f)


def _soft(x, t):
    return math.copysign(max(abs(x) - t, 0.0), x)


_CD = []


def _narrow_max():
    """Widest padded design on the narrow fused IRLS kernel (32-wide tile
    pairs, one pass); wider designs take the wide path (eta pass + 256-tile
    bf16 MFMA Gram).  128: at 10M x 200 (AutoML's GLM step without CV) the
    wide path trains in 2.1 s against 11.4 s on the 32-wide tile pairs, with
    the same tiers and fp64-level coefficients (profiles/glm_f64_r6/)."""
    return int(os.environ.get("H2O3_GLM_NARROW_MAX", "128"))


def _native_cd():
    """C++ coordinate descent (h2o3_amd/native/glm_solver.cpp), None if unbuilt."""
    if not _CD:
        fn = None
        try:
            import ctypes
            from ...ops import _native
            lib = _native.get_lib("glm_solver", required=False)
            if lib is not None:
                fn = lib.h2o_glm_cd
                vp, d, i = ctypes.c_void_p, ctypes.c_double, ctypes.c_int
                fn.argtypes = [i, vp, vp, vp, vp, vp, d, d, vp, i, d]
                fn.restype = i
        except Exception:  # noqa: BLE001
            fn = None
        _CD.append(fn)
    return _CD[0]


def _solve_quadratic(G, b, l1, l2, intercept, beta0=None, non_negative=False, max_iter=1000, tol=1e-10,
                     penalty_mask=None, lower=None, upper=None, active=None):
    """min 1/2 b'Gb - b'x + l1|b|_1 + l2/2|b|^2 (last coef = intercept, unpenalized),
    optionally with box constraints lower <= b <= upper (beta_constraints) and a
    subset of active coefficients (the others fixed at 0: collinear columns)."""
    P = G.shape[0]
    if active is not None and not bool(np.all(active)):
        idx = np.nonzero(active)[0]
        sub = _solve_quadratic(G[np.ix_(idx, idx)], b[idx], l1, l2, intercept and bool(active[-1]),
                               None if beta0 is None else beta0[idx],
                               non_negative if not np.ndim(non_negative) else np.asarray(non_negative)[idx],
                               max_iter, tol, None if penalty_mask is None else penalty_mask[idx],
                               None if lower is None else lower[idx], None if upper is None else upper[idx])
        out = np.zeros(P)
        out[idx] = sub
        return out
    pen = np.ones(P) if penalty_mask is None else penalty_mask.astype(float)
    if intercept:
        pen[-1] = 0.0
    nn = np.asarray(non_negative, dtype=bool) if np.ndim(non_negative) else np.full(P, bool(non_negative))
    if intercept:
        nn[-1] = False
    non_negative = bool(nn.any())
    lo = np.full(P, -np.inf) if lower is None else np.asarray(lower, dtype=np.float64)
    hi = np.full(P, np.inf) if upper is None else np.asarray(upper, dtype=np.float64)
    lo = np.where(nn, np.maximum(lo, 0.0), lo)
    boxed = bool(np.isfinite(lo).any() or np.isfinite(hi).any())
    if l1 == 0 and not boxed:
        import scipy.linalg as sla
        if l2 != 0:
            A = G.copy()
            A[np.diag_indices(P)] += l2 * pen
        else:
            A = G                                # cho_factor copies it (no extra diag matrix)
        # a ridge only when the plain factorization fails, and then relative to
        # each diagonal entry: an absolute ridge eps * max(diag) biases the
        # Newton fixed point (g = eps beta) of unstandardized designs by ~1e-5
        dA = np.diag(A)
        floor = 1e-12 * max(1.0, float(np.abs(dA).max()) if dA.size else 1.0)
        dead = dA <= 0
        for ridge in ((0.0, 1e-12, 1e-9) if not dead.any() else (1e-12, 1e-9)):
            try:
                Ar = A if ridge == 0.0 else A + np.diag(np.where(dead, floor, ridge * np.abs(dA)))
                cf = sla.cho_factor(Ar, lower=True, check_finite=False)
                return sla.cho_solve(cf, b, check_finite=False)
            except np.linalg.LinAlgError:
                continue
        return np.linalg.lstsq(A, b, rcond=None)[0]
    beta = np.zeros(P) if beta0 is None else np.clip(beta0.copy(), lo, hi)
    cd = _native_cd()
    if cd is not None:
        import ctypes
        Gc = np.ascontiguousarray(G, dtype=np.float64)
        arrs = [Gc, np.ascontiguousarray(b, dtype=np.float64), np.ascontiguousarray(pen, dtype=np.float64),
                np.ascontiguousarray(lo), np.ascontiguousarray(hi)]
        beta = np.ascontiguousarray(beta, dtype=np.float64)
        ptr = [a.ctypes.data_as(ctypes.c_void_p) for a in arrs]
        cd(P, *ptr, float(l1), float(l2), beta.ctypes.data_as(ctypes.c_void_p), int(max_iter), float(tol))
        return beta
    diag = np.diag(G) + l2 * pen
    grad = b - G @ beta
    for it in range(max_iter):
        maxd = 0.0
        for j in range(P):
            if diag[j] <= 0:
                continue
            old = beta[j]
            r = grad[j] + G[j, j] * old
            nb = min(max(_soft(r, l1 * pen[j]) / diag[j], lo[j]), hi[j])
            if nb != old:
                d = nb - old
                grad -= G[:, j] * d
                beta[j] = nb
                maxd = max(maxd, abs(d))
        if maxd < tol:
            break
    return beta


class GLMDriver:
    """IRLS state machine; `step()` = one IRLS iteration at the current lambda."""

    def __init__(self, est, spec):
        self.est = est
        p = est._parms
        self.spec = spec
        fam = (p.get("family") or "AUTO").lower()
        if fam == "auto":
            fam = "binomial" if spec.nclasses == 2 else ("multinomial" if spec.nclasses > 2 else "gaussian")
        self.family = fam
        link = p.get("link") or "family_default"
        if link == "family_default":
            link = _DEFAULT_LINK[fam]
        if fam == "tweedie" and link == "tweedie" and p.get("tweedie_link_power", 1.0) == 1.0:
            link_eff = "identity"
        else:
            link_eff = link
        self.fam = _Fam(fam, link_eff, float(p.get("tweedie_variance_power") or 0.0),
                        float(p.get("tweedie_link_power") or 1.0), float(p.get("theta") or 1e-10))
        from .interactions import interaction_pairs
        self.dinfo = DataInfo(spec.frame, spec.x, standardize=bool(p.get("standardize", True)),
                              missing_values_handling=p.get("missing_values_handling"),
                              plug_values=p.get("plug_values"), pad_extra=2,
                              interactions=interaction_pairs(spec.x, p.get("interactions"),
                                                             p.get("interaction_pairs")))
        # Pp = 128 runs the warp-specialised IRLS kernel, which reads rows of
        # round_up(P, 4) floats: at P = 100 the 28 padding columns (22 % of the
        # HBM stream) are never stored
        Pn = (self.dinfo.P + 3) // 4 * 4
        narrow = cloud.device().type == "cuda" and self.dinfo.Pp == 128 and Pn < 128
        self.X, ok = self.dinfo.expand(spec.frame, width=Pn if narrow else None)
        y = spec.y_tensor()
        if spec.is_classification:
            yy = (y == 1).to(torch.float64) if fam != "multinomial" else y.to(torch.float64)
            ok &= y >= 0
        else:
            yy = y.to(torch.float64)
            ok &= ~torch.isnan(yy)
            if fam == "binomial":
                # GLM.init (hex/glm/GLM.java:866): a numeric response must be 0/1
                nonbin = coll.allreduce_scalar(float((ok & (yy != 0) & (yy != 1)).sum()))
                if nonbin > 0:
                    raise ValueError("ERRR on field: _family: Binomial requires the response to be a 2-class "
                                     "categorical or a binary column (0/1)")
        w = spec.w_tensor()
        w = torch.ones_like(yy) if w is None else w.to(torch.float64)
        self.w = torch.where(ok, w, torch.zeros_like(w))
        self.y = torch.where(ok, yy, torch.zeros_like(yy))
        off = spec.offset_tensor()
        self.offset = off.to(torch.float64) if off is not None else None
        self.P = self.dinfo.P
        self.Pp = self.dinfo.Pp
        self.intercept = bool(p.get("intercept", True))
        self.wsum = coll.allreduce_scalar(float(self.w.sum()))
        self.nobs = coll.allreduce_scalar(float((self.w > 0).sum()))
        if self.wsum <= 0:
            raise ValueError("ERRR on field: _train: Training data has no rows with a valid response and "
                             "positive weight")
        self.ymu = coll.allreduce_scalar(float((self.w * self.y).sum())) / self.wsum
        # obj_reg: the objective is obj_reg * (-log-likelihood) + penalty
        # (GLM.java:1063, default 1 / sum of weights)
        orr = float(p.get("obj_reg") if p.get("obj_reg") is not None else -1.0)
        self.obj_reg = orr if orr > 0 else 1.0 / self.wsum
        alpha = p.get("alpha")
        solver = (p.get("solver") or "AUTO").upper()
        if alpha is None:
            alpha = 0.0 if solver == "L_BFGS" else 0.5
        self.alphas = [float(a) for a in alpha] if isinstance(alpha, (list, tuple)) else [float(alpha)]
        self.alpha = self.alphas[0]
        self.beta = np.zeros(self.P + 1)
        if self.intercept:
            mu0 = min(max(self.ymu, 1e-10), 1 - 1e-10) if self.fam.link == "logit" else self.ymu
            try:
                self.beta[-1] = self.fam.link_fn(mu0) if self.offset is None else 0.0
            except (ValueError, ZeroDivisionError):
                self.beta[-1] = 0.0
        self._init_beta = self.beta.copy()
        self._setup_constraints(p.get("beta_constraints"))
        sv = p.get("startval")
        ck = p.get("checkpoint")
        if ck is not None and sv is None:
            # checkpoint: continue from a previous model's coefficients (GLM.java
            # restarts the solver from the checkpointed model's beta)
            from ...core import dkv
            prev = dkv.get(ck) if isinstance(ck, str) else ck
            sv = prev.coef()
        if sv is not None:
            self._set_startval(sv)
        self.active = None     # collinear-column mask (remove_collinear_columns)
        self._hprec = None     # Hessian precision tier (None: not chosen yet), see _check_tier
        self.hessian_kappa = None
        self.iter = 0
        self.lambda_max = self._lambda_max()
        lam = p.get("lambda_")
        if lam is None:
            lam = p.get("Lambda")
        nl = int(p.get("nlambdas") or -1)
        self.nlambdas = (30 if self.alpha == 0 else 100) if nl == -1 else nl    # GLM.java:951
        lmr = float(p.get("lambda_min_ratio") or -1)
        if lmr == -1:
            lmr = 1e-4 if (self.nobs / 16) > self.P else 1e-2
            if self.alpha == 0:
                lmr *= 1e-2
        self.lambda_min_ratio = lmr
        if p.get("lambda_search"):
            nl = self.nlambdas
            if lam is None:
                dec = lmr ** (1.0 / max(nl - 1, 1))
                self.lambdas = [self.lambda_max * dec ** i for i in range(nl)]
            else:
                self.lambdas = sorted(list(lam) if isinstance(lam, (list, tuple)) else [lam], reverse=True)
        else:
            if lam is None:
                self.lambdas = [10 * lmr * self.lambda_max]
            else:
                self.lambdas = list(lam) if isinstance(lam, (list, tuple)) else [float(lam)]
        self.lam = self.lambdas[0]
        self.beta_eps = float(p.get("beta_epsilon") or 1e-4)
        oe = float(p.get("objective_epsilon") or -1)
        self.obj_eps = oe if oe > 0 else (1e-4 if p.get("lambda_search") else (1e-6 if self.lam == 0 else 1e-4))
        ge = float(p.get("gradient_epsilon") if p.get("gradient_epsilon") is not None else -1.0)
        if ge <= 0:                                                     # GLM.java:1182
            ge = (1e-6 if self.lambdas[0] == 0 else 1e-4) * (1e-2 if p.get("lambda_search") else 1.0)
        self.grad_eps = ge
        # stopping_rounds without lambda search switches GLM's own convergence
        # test off in favour of ScoreKeeper early stopping (GLM.java:946, :3137)
        self.early_stop_enabled = (not p.get("lambda_search")) and int(p.get("stopping_rounds") or 0) > 0
        self.converged = False
        self.last_obj = float("inf")

    # ---- constraints (GLM.java: beta_constraints frame names/lower_bounds/
    # upper_bounds/beta_given/rho; bounds are given on the original scale and
    # mapped to the standardized coefficients: b_std = b * sigma)
    def _setup_constraints(self, bc):
        P = self.P
        self.lower = self.upper = None
        self.rho = None
        if bc is None:
            return
        import pandas as pd
        df = bc.as_data_frame() if hasattr(bc, "as_data_frame") else pd.DataFrame(bc)
        lo = np.full(P + 1, -np.inf)
        hi = np.full(P + 1, np.inf)
        given = np.zeros(P + 1)
        rho = np.zeros(P + 1)
        pos = {n: i for i, n in enumerate(self.dinfo.coef_names)}
        scale = np.ones(P + 1)
        if self.dinfo.standardize:
            base = self.dinfo.n_cat_expanded
            for j in range(len(self.dinfo.num_cols)):
                scale[base + j] = self.dinfo.sigmas[j]
        for _, r in df.iterrows():
            name = str(r["names"])
            targets = [pos[name]] if name in pos else \
                [i for n, i in pos.items() if n.startswith(name + ".")]   # a categorical column: all its levels
            if not targets:
                raise ValueError(f"beta_constraints: unknown coefficient '{name}'")
            for i in targets:
                if "lower_bounds" in r and pd.notna(r["lower_bounds"]):
                    lo[i] = float(r["lower_bounds"]) * scale[i]
                if "upper_bounds" in r and pd.notna(r["upper_bounds"]):
                    hi[i] = float(r["upper_bounds"]) * scale[i]
                if "beta_given" in r and pd.notna(r["beta_given"]):
                    given[i] = float(r["beta_given"]) * scale[i]
                    rho[i] = float(r["rho"]) if "rho" in r and pd.notna(r["rho"]) else 1.0
        if np.any(lo > hi):
            raise ValueError("beta_constraints: lower bound above upper bound")
        self.lower, self.upper = lo, hi
        if rho.any():
            self.rho, self.beta_given = rho, given
        self.beta = np.clip(self.beta, lo, hi)

    def _set_startval(self, sv):
        """startval: initial coefficients on the original scale (names -> value,
        or a list in coef order with the intercept last)."""
        b = self.beta.copy()
        if isinstance(sv, dict):
            pos = {n: i for i, n in enumerate(self.dinfo.coef_names)}
            for n, v in sv.items():
                if n == "Intercept":
                    b[-1] = float(v)
                elif n in pos:
                    b[pos[n]] = float(v)
        else:
            sv = [float(v) for v in sv]
            if len(sv) != len(b):
                raise ValueError(f"Initial coefficient length ({len(sv)}) does not equal to actual GLM coefficient "
                                 f"length({len(b)}).  The order of coefficients should be the following:\n"
                                 + "\n".join(self.dinfo.coef_names) + "\n Intercept.")
            b[:] = sv
        if self.dinfo.standardize:
            base = self.dinfo.n_cat_expanded
            for j in range(len(self.dinfo.num_cols)):
                b[-1] += b[base + j] * self.dinfo.means[j]
                b[base + j] *= self.dinfo.sigmas[j]
        self.beta = b
        self._init_beta = b.copy()

    def _find_collinear(self, Gn):
        """Greedy Cholesky with a pivot tolerance over the standardized Gram
        (GLM.java removeCollinearColumns via Gram.qrCholesky): a column whose
        residual variance after the columns kept so far is < 1e-7 of its own
        variance is dropped (coefficient fixed at 0)."""
        n = Gn.shape[0]
        keep = np.ones(n, dtype=bool)
        L = np.zeros((n, n))
        kept = []
        order = ([n - 1] + list(range(n - 1))) if self.intercept else list(range(n))   # intercept first
        for j in order:
            v = Gn[j, j]
            if kept:
                lj = np.linalg.solve(L[np.ix_(kept, kept)], Gn[kept, j]) if kept else np.zeros(0)
                r = v - float(lj @ lj)
            else:
                lj, r = np.zeros(0), v
            if r <= 1e-7 * max(v, 1e-300) and kept:
                keep[j] = False
                continue
            L[j, kept] = lj
            L[j, j] = math.sqrt(max(r, 1e-300))
            kept.append(j)
        return keep

    # ---- device-side pieces
    def _eta(self, beta=None):
        b = self.beta if beta is None else beta
        if self.X.device.type == "cpu":
            # host path: f64 like the reference (f32 linear predictors move an
            # unstandardized design's solution by ~1e-4)
            bt = torch.as_tensor(b[: self.P], dtype=torch.float64)
            eta = self.X[:, : self.P].to(torch.float64) @ bt + b[-1]
            return eta + self.offset if self.offset is not None else eta
        bt = torch.zeros(self.X.shape[1], dtype=torch.float32, device=self.X.device)
        bt[: self.P] = torch.as_tensor(b[: self.P], dtype=torch.float32)
        eta = (self.X @ bt).to(torch.float64) + b[-1]
        if self.offset is not None:
            eta = eta + self.offset
        return eta

    def _wide_eta_codes(self):
        """Family codes when the wide fused eta kernel applies (the wide IRLS
        path of _irls_stats), else None."""
        codes = linalg_ops.glm_fused_codes(self.fam.family, self.fam.link, self.fam.tlp)
        if self.X.device.type == "cuda" and self.Pp > _narrow_max() and self.P + 2 <= 1024 and codes is not None and \
                linalg_ops._wide_mode() == "bf3" and linalg_ops.wide_fused_enabled():
            if not hasattr(self, "_y32"):
                self._y32 = self.y.to(torch.float32)
                self._w32 = self.w.to(torch.float32)
                self._off32 = None if self.offset is None else self.offset.to(torch.float32)
            return codes
        return None

    def _wide_eta_pass(self, codes, beta, b0):
        """(deviance, X'r) of the wide eta kernel at (beta[:P], b0): one pass
        over X instead of a GEMV plus torch elementwise passes."""
        bt = torch.as_tensor(np.asarray(beta[:self.P], dtype=np.float64), dtype=torch.float32, device=self.X.device)
        _, dev, gx = linalg_ops.glm_wide_irls(self.X, self.P, bt, float(b0), self._y32, self._w32, self._off32,
                                              codes, self.fam.tvp, self.fam.theta, fused=True, eta_only=True)
        return dev, gx

    def _lambda_max(self):
        # gradient of the mean log-likelihood at the intercept-only model
        e0 = self.fam.link_fn(min(max(self.ymu, 1e-10), 1 - 1e-10)) if self.fam.link == "logit" else \
            (self.fam.link_fn(max(self.ymu, 1e-10)) if self.fam.link in ("log", "inverse") else self.ymu)
        codes = self._wide_eta_codes()
        if codes is not None:
            # the wide eta kernel at beta = 0, intercept eta0: its gradient
            # channel is exactly X'r with r = w (y - mu) dmu/deta / var
            _, gx = self._wide_eta_pass(codes, np.zeros(self.P), float(e0))
            g = gx[:self.P].contiguous()
            coll.allreduce_(g)
            g = g * self.obj_reg
            amax = float(g.abs().max()) if g.numel() else 0.0
            return amax / max(1e-2, self.alpha)
        eta0 = torch.full_like(self.y, e0)
        if self.offset is not None:
            eta0 = eta0 + self.offset
        mu = self.fam.linkinv(eta0)
        d = self.fam.dmu_deta(eta0, mu)
        r = self.w * (self.y - mu) * d / self.fam.variance(mu)
        if self._native():
            # X'r rides the fused Gram pass (column P of the augmented Gram)
            g = linalg_ops.glm_irls(self.X, aug=self.P, W=r, width=self.Pp)[0][: self.P, self.P].contiguous()
        else:
            g = (self.X.to(torch.float64).T @ r)[: self.P]
        coll.allreduce_(g)
        g = g * self.obj_reg
        amax = float(g.abs().max()) if g.numel() else 0.0
        return amax / max(1e-2, self.alpha)

    def _native(self):
        return self.X.device.type == "cuda" and self.X.dtype == torch.float32 and self.Pp % 32 == 0 and \
            self.Pp <= _narrow_max() and self.Pp >= self.P + 2

    def _irls_stats_native(self):
        """One fused kernel pass: eta, IRLS weights, deviance, augmented Gram."""
        P = self.P
        codes = linalg_ops.glm_fused_codes(self.fam.family, self.fam.link, self.fam.tlp)
        if self.Pp & (self.Pp - 1):
            codes = None  # fused path needs a power-of-two padded width
        if not hasattr(self, "_y32"):
            self._y32 = self.y.to(torch.float32)
            self._w32 = None if bool((self.w == 1).all()) else self.w.to(torch.float32)
            self._off32 = None if self.offset is None else self.offset.to(torch.float32)
        self._gexact = None
        hp = self._hprec or ("bf16" if codes is not None and self._narrow_bf16_ok() else None)
        bf3 = None if hp is None else ("bf16" if hp == "bf16" else hp == "bf3")
        with phase("glm.irls_pass"):
            if codes is not None:
                bt = torch.zeros(self.Pp, dtype=torch.float32, device=self.X.device)
                bt[:P] = torch.as_tensor(self.beta[:P], dtype=torch.float32)
                if linalg_ops.glm_grad_supported(self.Pp):
                    # Hessian on the matrix cores + exact gradient channel (Newton on
                    # the exact gradient: see _finish_stats)
                    Gf, dev, gx = linalg_ops.glm_irls(self.X, aug=P, beta=bt, b0=float(self.beta[-1]),
                                                      y=self._y32, wprior=self._w32, offset=self._off32,
                                                      codes=codes, tvp=self.fam.tvp, theta=self.fam.theta,
                                                      width=self.Pp, grad=True, bf3=bf3,
                                                      grad_f64=self._hprec not in (None, "bf3", "bf16"))
                    self._gexact = torch.cat([gx[:P], gx[self.Pp:self.Pp + 1]])
                    self._gbeta = np.concatenate([self.beta[:P].astype(np.float32).astype(np.float64),
                                                  [float(np.float32(self.beta[-1]))]])
                else:
                    Gf, dev = linalg_ops.glm_irls(self.X, aug=P, beta=bt, b0=float(self.beta[-1]), y=self._y32,
                                                  wprior=self._w32, offset=self._off32, codes=codes,
                                                  tvp=self.fam.tvp, theta=self.fam.theta, width=self.Pp, bf3=bf3)
                dev = dev.view(1)
            else:
                eta = self._eta()
                mu = self.fam.linkinv(eta)
                d = self.fam.dmu_deta(eta, mu)
                W = self.w * d * d / self.fam.variance(mu)
                off = self.offset if self.offset is not None else 0.0
                z = (eta - off) + (self.y - mu) / d
                Gf, _ = linalg_ops.glm_irls(self.X, aug=P, W=W, z=z, width=self.Pp)
                dev = (self.w * self.fam.deviance(self.y, mu)).sum().view(1)
        return Gf[:P, :P], Gf[:P, P + 1].contiguous(), Gf[:P, P].contiguous(), Gf[P, P].view(1), \
            Gf[P, P + 1].view(1), dev

    # Hessian precision tiers of the Newton step beta + H^-1 g (g from the exact
    # gradient channel): the iteration contracts at rate ~ kappa * eps(H), so the
    # tier is picked from the Jacobi-scaled condition number kappa of the system
    # matrix.  Plain bf16 MFMA (eps ~ 4e-3; the fused wide Gram and the P + 2 <= 128
    # fused pass, both beside the exact gradient) while
    # kappa < 32, bf16x3 MFMA (eps ~ 2e-5) while kappa < 2e3, f32 MFMA
    # (eps ~ 1e-7) while kappa < 5e5, beyond that fp64 (the reference's Gram
    # precision, hex/gram/Gram.java:17) on the device's f64 GEMMs.
    _TIER_LIMITS = (("bf16", 32.0), ("bf3", 2e3), ("f32", 5e5), ("f64", float("inf")))

    def _narrow_bf16_ok(self):
        """The plain-bf16 Hessian tier of the P + 2 <= 128 fused kernel
        (glm_irls_ws_kernel LO = false): needs the exact-gradient channel and
        the bf16 MFMA path (H2O3_GLM_BF16=0 or H2O3_GLM_BF3=0 disable it)."""
        return self.Pp == 128 and linalg_ops.glm_grad_supported(self.Pp) and \
            os.environ.get("H2O3_GLM_BF16", "1") != "0" and os.environ.get("H2O3_GLM_BF3", "1") != "0"

    def _wide_bf16_ok(self):
        """The plain-bf16 Hessian tier exists for the fused wide Gram only
        (H2O3_GLM_WIDE_BF16=0 disables it)."""
        return linalg_ops.wide_fused_enabled() and os.environ.get("H2O3_GLM_WIDE_BF16", "1") != "0" and \
            os.environ.get("H2O3_WIDE_TILE", "256") == "256"

    def _tier_for(self, kappa):
        for name, lim in self._TIER_LIMITS:
            if kappa < lim:
                return name
        return "f64"

    @staticmethod
    def _scaled_cond(A, active=None):
        idx = np.arange(A.shape[0]) if active is None else np.flatnonzero(active[:A.shape[0]])
        d = np.diag(A)[idx]
        idx = idx[d > 0]
        if idx.size == 0:
            return 1.0
        d = 1.0 / np.sqrt(np.diag(A)[idx])
        # one copy (no fancy-index gather when every column takes part), scaled in place
        S = np.array(A, dtype=np.float64, order="F") if idx.size == A.shape[0] else \
            np.asfortranarray(A[np.ix_(idx, idx)])
        S *= d[:, None]
        S *= d[None, :]
        # LAPACK Cholesky + 1-norm condition estimate (dpotrf / dpocon: ~0.1 ms at
        # P = 100, where a threaded eigvalsh costs ~10 ms per IRLS iteration)
        from scipy.linalg import lapack
        anorm = float(np.abs(S).sum(0).max())
        c, info = lapack.dpotrf(S, lower=1, clean=0, overwrite_a=1)
        if info != 0:
            return float("inf")
        rc, info = lapack.dpocon(c, anorm, uplo="L")
        return float(1.0 / rc) if info == 0 and rc > 0 else float("inf")

    @staticmethod
    def _scaled_cond_dev(A):
        """_scaled_cond on a device system: Jacobi scaling, f64 Cholesky on
        the device and Hager's 1-norm estimate of ||S^-1|| (the estimator
        LAPACK dpocon runs), so the (P+1)^2 matrix never leaves the GPU.
        scripts/glm_devsolve_mb.py, P = 1001: 2.7 ms Cholesky + 1.7 ms
        estimate on the device vs 6.3 ms host dpotrf plus the copy."""
        d = A.diagonal()
        pos = d > 0
        if not bool(pos.all()):
            idx = torch.nonzero(pos).view(-1)
            if idx.numel() == 0:
                return 1.0
            A = A.index_select(0, idx).index_select(1, idx)
            d = A.diagonal()
        s = d.rsqrt()
        S = A * s.view(-1, 1) * s.view(1, -1)
        L, info = torch.linalg.cholesky_ex(S)
        return GLMDriver._hager_kappa(S, L, info)

    @staticmethod
    def _hager_kappa(S, L, info):
        """||S||_1 * est(||S^-1||_1) from the Cholesky factor L of S (Hager /
        Higham: at most 5 steps of two triangular solve pairs)."""
        anorm = S.abs().sum(0).max()
        n = S.shape[0]
        x = torch.full((n, 1), 1.0 / n, dtype=S.dtype, device=S.device)
        est = None
        for k in range(5):
            y = torch.cholesky_solve(x, L)
            z = torch.cholesky_solve(torch.sign(y), L)
            za = z.abs().view(-1)
            j = za.argmax()
            # one host read per estimator step: [info, ||y||_1, max|z|, z'x, j]
            h = torch.stack([info.to(S.dtype), y.abs().sum(), za[j], (z * x).sum(), j.to(S.dtype),
                             anorm]).cpu().numpy()
            if h[0] != 0:
                return float("inf")
            est = float(h[1])
            if k > 0 and h[2] <= h[3]:
                break
            x = torch.zeros_like(x)
            x[int(h[4])] = 1.0
        kappa = est * float(h[5])
        return kappa if np.isfinite(kappa) and kappa > 0 else float("inf")

    @staticmethod
    def _kappa_from_factor(A, L, info):
        """Scaled condition estimate of A reusing its Cholesky factor: the
        factor of S = D A D (D = diag(A)^-1/2) is D L, so the tier check costs
        no second factorization.  A failed factor (a zero-variance column,
        or indefinite) goes through _scaled_cond_dev's column filter."""
        if int(info) != 0:
            return GLMDriver._scaled_cond_dev(A)
        s = A.diagonal().rsqrt()
        return GLMDriver._hager_kappa(A * s.view(-1, 1) * s.view(1, -1), L * s.view(-1, 1), info)

    def _dev_system_ok(self):
        """The IRLS system of this step can be built, conditioned and solved
        on the device: wide designs (the host f64 Cholesky of a 1001^2
        system costs more than the device one) with a plain ridge-only
        quadratic (no l1, bounds, proximal terms, GAM penalties, collinear
        column removal or non-negativity -- those take the host solvers)."""
        p = self.est._parms
        return (self.X.device.type == "cuda" and self.P + 1 >= 256
                and os.environ.get("H2O3_GLM_DEV_SOLVE", "1") != "0"
                and self.lam * self.alpha == 0 and self.lower is None and self.upper is None
                and self.rho is None and self.active is None and self._penalty_matrix() is None
                and not p.get("remove_collinear_columns") and not p.get("non_negative")
                and not p.get("_nonneg_names"))

    def _dev_tier_ok(self):
        """Wide systems whose solve needs the host (l1 / bounds / non-negative
        coefficients) still get their condition estimate on the device: the
        (P+1)^2 statistics cross to the host once, after the tier check."""
        return (self.X.device.type == "cuda" and self.P + 1 >= 256
                and os.environ.get("H2O3_GLM_DEV_SOLVE", "1") != "0"
                and self.rho is None and self.active is None and self._penalty_matrix() is None
                and not self.est._parms.get("remove_collinear_columns"))

    def _check_tier_dev(self, Ga, b):
        """_check_tier on device statistics (scaled-condition estimate on a
        device Cholesky); recomputes the statistics on the device when the
        tier must rise."""
        while self._tiers_due():
            Gn, _, _, l2 = self._system(Ga, b)
            if l2 > 0:
                Gn = Gn.clone()
                Gn.diagonal()[:self.P] += l2
            want = self._tier_raise(self._scaled_cond_dev(Gn))
            if want is None:
                break
            self._sys_on_dev = True
            try:
                Ga, b, dev = self._irls_stats()
            finally:
                self._sys_on_dev = False
            self._stats_dev = dev
            if want == "f64":
                break
        return Ga, b

    def _step_solve_dev(self, Gn, bn, l2, L, info):
        """Ridge Newton step on the device from the factor L of Gn + ridge:
        (max |gradient|, new beta) with one host read; new is None when the
        Cholesky failed (the host solver's relative-ridge retries take over)."""
        bcur = self.beta if self.intercept else self.beta[:-1]
        bt = torch.as_tensor(bcur, dtype=torch.float64).to(Gn.device, non_blocking=True)
        gq = Gn @ bt - bn
        gq[:self.P] += l2 * bt[:self.P]
        new = torch.cholesky_solve(bn.view(-1, 1), L).view(-1)
        h = torch.cat([info.to(torch.float64).view(1), gq.abs().max().view(1), new]).cpu().numpy()
        if h[0] != 0 or not np.all(np.isfinite(h[2:])):
            return float(h[1]), None
        return float(h[1]), h[2:].copy()

    def _irls_stats(self):
        self._gexact = None
        if self._hprec == "f64" or self.X.device.type == "cpu":
            # fp64 tier on the device, and always on the host (the reference's
            # double Gram / gradient, hex/gram/Gram.java:17)
            return self._irls_stats_f64()
        if self._native():
            G, xz, xw, sw, swz, dev = self._irls_stats_native()
            return self._finish_stats(G, xz, xw, sw, swz, dev)
        codes = linalg_ops.glm_fused_codes(self.fam.family, self.fam.link, self.fam.tlp)
        if self.X.device.type == "cuda" and self.Pp > _narrow_max() and self.P + 2 <= 1024 and codes is not None and \
                linalg_ops._wide_mode() == "bf3":
            # one fused pass: eta + family + bf16 hi/lo split, then one bf16 GEMM
            with phase("glm.wide_pass"):
                if not hasattr(self, "_y32"):
                    self._y32 = self.y.to(torch.float32)
                    self._w32 = self.w.to(torch.float32)
                    self._off32 = None if self.offset is None else self.offset.to(torch.float32)
                P = self.P
                bt = torch.as_tensor(self.beta[:P], dtype=torch.float32, device=self.X.device)
                exact = os.environ.get("H2O3_GLM_EXACT_GRAD", "1") != "0"
                # fused: eta pass + one hand-written MFMA Gram kernel over the f32
                # rows (needs the exact gradient: its Gram has no z column)
                fused = exact and linalg_ops.wide_fused_enabled()
                # before the first condition estimate the fused path starts at the
                # plain bf16 Hessian tier when allowed (raised at iteration 1 if kappa says so)
                hp = self._hprec or ("bf16" if fused and self._wide_bf16_ok() else "bf3")
                Gf, dev, gx = linalg_ops.glm_wide_irls(self.X, P, bt, float(self.beta[-1]), self._y32,
                                                       self._w32, self._off32, codes, self.fam.tvp, self.fam.theta,
                                                       fused=fused, bf3=hp != "bf16")
                if exact:
                    self._gexact = gx[:P + 1]
                    self._gbeta = np.concatenate([self.beta[:P].astype(np.float32).astype(np.float64),
                                                  [float(np.float32(self.beta[-1]))]])
            with phase("glm.finish"):
                return self._finish_stats(Gf[:P, :P], Gf[:P, P + 1].contiguous(), Gf[:P, P].contiguous(),
                                          Gf[P, P].view(1), Gf[P, P + 1].view(1), dev.view(1))
        with phase("glm.eta"):
            eta = self._eta()
        with phase("glm.weights"):
            mu = self.fam.linkinv(eta)
            d = self.fam.dmu_deta(eta, mu)
            var = self.fam.variance(mu)
            W = (self.w * d * d / var)
            off = self.offset if self.offset is not None else 0.0
            z = (eta - off) + (self.y - mu) / d
            if self.fam.family == "gaussian" and self.fam.link == "identity":
                W = self.w
                z = self.y - off
            Wf = W.to(torch.float32)
        if self.X.device.type == "cuda" and self.Pp > _narrow_max() and bool((W >= 0).all()):
            with phase("glm.gram"):
                G, xw, xz, sw, swz = linalg_ops.weighted_gram_aug(self.X, W, z, self.P)
                dev = (self.w * self.fam.deviance(self.y, mu)).sum().view(1)
            return self._finish_stats(G, xz, xw, sw.view(1), swz.view(1), dev)
        with phase("glm.gram"):
            G = linalg_ops.weighted_gram(self.X, Wf)[: self.P, : self.P]
        with phase("glm.xtwz"):
            Wz = (W * z)
            xz = (self.X.T @ Wz.to(torch.float32)).to(torch.float64)[: self.P] if self.X.device.type == "cuda" else \
                (self.X.to(torch.float64).T @ Wz)[: self.P]
            # intercept row/col: X'W 1 and sum W, sum Wz
            xw = (self.X.T @ Wf).to(torch.float64)[: self.P]
            sw, swz = W.sum().view(1), Wz.sum().view(1)
            dev = (self.w * self.fam.deviance(self.y, mu)).sum().view(1)
        return self._finish_stats(G, xz, xw, sw, swz, dev)

    def _irls_stats_f64(self, step=1 << 21):
        """fp64 IRLS statistics on the device (chunked f64 GEMMs): Gram,
        exact gradient X'r (r = w (y - mu) dmu/deta / var) and deviance at the
        f64 coefficients.  The top precision tier for ill-conditioned designs."""
        P = self.P
        X = self.X
        dv = X.device
        bt = torch.as_tensor(self.beta[:P], dtype=torch.float64, device=dv)
        Ga = torch.zeros((P + 1, P + 1), dtype=torch.float64, device=dv)
        g = torch.zeros(P + 1, dtype=torch.float64, device=dv)
        dev = torch.zeros(1, dtype=torch.float64, device=dv)
        ident = self.fam.family == "gaussian" and self.fam.link == "identity"
        native = (X.is_cuda and X.dtype == torch.float32 and X.stride(1) == 1
                  and os.environ.get("H2O3_GLM_F64_MFMA", "1") == "1")
        with phase("glm.irls_f64"):
            for a in range(0, X.shape[0], step):
                if native:
                    Xc = None
                    eta = linalg_ops.xv_f64(X[a:a + step], P, bt, float(self.beta[-1]))
                else:
                    Xc = X[a:a + step, :P].to(torch.float64)
                    eta = Xc @ bt + float(self.beta[-1])
                if self.offset is not None:
                    eta = eta + self.offset[a:a + step]
                w, y = self.w[a:a + step], self.y[a:a + step]
                mu = self.fam.linkinv(eta)
                if ident:
                    W, r = w, w * (y - eta)
                else:
                    d = self.fam.dmu_deta(eta, mu)
                    wd = w * d / self.fam.variance(mu)
                    W, r = wd * d, wd * (y - mu)
                if native:
                    # exact f64 products on the f64 matrix cores, straight
                    # from the f32 rows (no f64 copy of X in the Gram)
                    Ga += linalg_ops.gram_f64_aug(X[a:a + step], P, W)
                    g[:P] += linalg_ops.xtr_f64(X[a:a + step], P, r)
                    g[P] += r.sum()
                else:
                    Xa = torch.cat([Xc, torch.ones((Xc.shape[0], 1), dtype=torch.float64, device=dv)], 1)
                    del Xc
                    Ga += (Xa * W.view(-1, 1)).T @ Xa
                    g += Xa.T @ r
                dev += (w * self.fam.deviance(y, mu)).sum()
        self._gexact = g
        self._gbeta = self.beta.copy()
        z = torch.zeros(P, dtype=torch.float64, device=dv)
        return self._finish_stats(Ga[:P, :P], z, Ga[:P, P].contiguous(), Ga[P, P].view(1),
                                  torch.zeros(1, dtype=torch.float64, device=dv), dev)

    def _finish_stats(self, G, xz, xw, sw, swz, dev):
        """All-reduce the IRLS sufficient statistics; returns (Gram [P+1, P+1]
        with the intercept last, right-hand side b, deviance).

        With the exact-gradient channel (self._gexact = X'r, r = w (y - mu)
        dmu/deta / var, at the f32 coefficients the kernel used) the
        right-hand side is G beta_f + g instead of the Gram's own X'Wz column:
        identical in exact arithmetic (X'Wz = X'W eta + X'r), but the solve is
        then a Newton step on an exact gradient, whose fixed point g = 0 does
        not depend on the precision of the bf16x3 Hessian."""
        gx = getattr(self, "_gexact", None)
        parts = [G.reshape(-1), xz, xw, sw, swz, dev] + ([gx] if gx is not None else [])
        stats = torch.cat([t.reshape(-1).to(torch.float64) for t in parts])
        coll.allreduce_(stats)
        P = self.P
        if stats.is_cuda:
            return self._finish_stats_dev(stats, gx is not None)
        host = stats.cpu().numpy()               # one device -> host copy
        o = 0
        G = host[o:o + P * P].reshape(P, P); o += P * P
        xz = host[o:o + P]; o += P
        xw = host[o:o + P]; o += P
        sw, swz, dev = float(host[o]), float(host[o + 1]), float(host[o + 2]); o += 3
        Ga = np.empty((P + 1, P + 1))
        Ga[:P, :P] = G
        Ga[:P, P] = Ga[P, :P] = xw
        Ga[P, P] = sw
        if gx is not None:
            g = host[o:o + P + 1]
            b = Ga @ self._gbeta + g
        else:
            b = np.concatenate([xz, [swz]])
        return Ga, b, dev

    def _finish_stats_dev(self, stats, exact):
        """_finish_stats for device statistics: the (P+1)^2 system and its
        right-hand side are assembled on the device and reach the host in ONE
        copy into a pinned buffer (two alternating buffers: a tier
        escalation recomputes the statistics while the first Ga is still
        referenced)."""
        P = self.P
        dev_ = stats.device
        o = 0
        G = stats[o:o + P * P].view(P, P); o += P * P
        xz = stats[o:o + P]; o += P
        xw = stats[o:o + P]; o += P
        sw, swz, devv = stats[o], stats[o + 1], stats[o + 2]; o += 3
        Ga = torch.empty((P + 1, P + 1), dtype=torch.float64, device=dev_)
        Ga[:P, :P] = G
        Ga[:P, P] = xw
        Ga[P, :P] = xw
        Ga[P, P] = sw
        if exact:
            gb = torch.as_tensor(self._gbeta, dtype=torch.float64).to(dev_, non_blocking=True)
            b = Ga @ gb + stats[o:o + P + 1]
        else:
            b = torch.cat([xz, swz.view(1)])
        if getattr(self, "_sys_on_dev", False):
            # the system stays on the device (step -> _step_solve_dev)
            return Ga, b, float(devv)
        out = torch.cat([Ga.reshape(-1), b, devv.view(1)])
        n = out.numel()
        bufs = getattr(self, "_pin_bufs", None)
        if bufs is None or bufs[0].numel() < n:
            bufs = self._pin_bufs = [torch.empty(n, dtype=torch.float64, pin_memory=True) for _ in range(2)]
            self._pin_i = 0
        self._pin_i = getattr(self, "_pin_i", 0) ^ 1
        host_t = bufs[self._pin_i][:n]
        host_t.copy_(out)                        # synchronous D2H into pinned memory
        host = host_t.numpy()
        m = (P + 1) * (P + 1)
        return host[:m].reshape(P + 1, P + 1), host[m:m + P + 1], float(host[m + P + 1])

    def _system(self, Ga, b):
        """The penalized quadratic the IRLS step solves: (Gn, bn, l1, l2)."""
        r = self.obj_reg
        Gn, bn = Ga * r, b * r
        if not self.intercept:
            Gn = Gn[:-1, :-1].contiguous() if torch.is_tensor(Gn) else Gn[:-1, :-1].copy()
            bn = bn[:-1].contiguous() if torch.is_tensor(bn) else bn[:-1].copy()
        l1 = self.lam * self.alpha
        l2 = self.lam * (1 - self.alpha)
        pen = self._penalty_matrix()
        if pen is not None:
            P = self.P
            Gn = Gn.copy()
            Gn[:P, :P] += pen
        if self.rho is not None:
            # proximal term rho/2 (b - beta_given)^2 of beta_constraints
            Gn = Gn.copy()
            bn = bn.copy()
            k = Gn.shape[0]
            Gn[np.diag_indices(k)] += self.rho[:k]
            bn += (self.rho * self.beta_given)[:k]
        return Gn, bn, l1, l2

    def _tiers_due(self):
        """The tier is (re)checked at iterations 1, 2, 4, 8, ... on the GPU."""
        if self.X.device.type != "cuda" or os.environ.get("H2O3_GLM_TIERS", "1") == "0":
            return False
        it = self.iter + 1
        return not (it & (it - 1))

    def _tier_raise(self, kappa):
        """Records kappa; returns the tier the statistics must be recomputed
        at when this one is too low for kappa (and switches to it), else
        None."""
        self.hessian_kappa = kappa
        order = [t for t, _ in self._TIER_LIMITS]
        wide = not self._native()
        cur = self._hprec
        bf16_ok = self._gexact is not None and (self._wide_bf16_ok() if wide else self._narrow_bf16_ok())
        if cur is None:
            ws_bf3 = self.Pp == 128 and os.environ.get("H2O3_GLM_BF3", "1") != "0"
            cur = ("bf16" if bf16_ok else "bf3") if (ws_bf3 if not wide else self._gexact is not None) else "f32"
        want = self._tier_for(kappa)
        if want == "bf16" and not bf16_ok:
            want = "bf3"
        if want == "f32" and (wide or self._gexact is None):
            # no f32 path with the gradient channel here: straight to fp64
            want = "f64"
        if order.index(want) > order.index(cur):
            self._hprec = want
            return want
        if self._hprec is None:
            self._hprec = cur
        return None

    def _check_tier(self, Ga, b):
        """Hessian precision tier from the scaled condition number of this
        iteration's system (checked at iterations 1, 2, 4, 8, ...); when the
        tier must rise, the statistics are recomputed at the new tier."""
        if not self._tiers_due():
            return Ga, b
        Gn, _, _, l2 = self._system(Ga, b)
        if l2 > 0:
            Gn = Gn.copy()
            Gn[np.arange(self.P), np.arange(self.P)] += l2
        want = self._tier_raise(self._scaled_cond(Gn, self.active))
        if want is not None:
            Ga, b, dev = self._irls_stats()
            self._stats_dev = dev
            return self._check_tier(Ga, b) if want != "f64" else (Ga, b)
        return Ga, b

    def _ridge_system_dev(self, Ga, b):
        """Device system (Gn, bn, l1, l2), A = Gn + the ridge on the
        penalized diagonal, and A's Cholesky factor."""
        Gn, bn, l1, l2 = self._system(Ga, b)
        A = Gn
        if l2 != 0:
            A = Gn.clone()
            pen = torch.full((A.shape[0],), l2, dtype=A.dtype, device=A.device)
            if self.intercept:
                pen[-1] = 0.0
            A.diagonal().add_(pen)
        L, info = torch.linalg.cholesky_ex(A)
        return Gn, bn, l1, l2, A, L, info

    def _step_dev(self, Ga, b):
        """Device-resident step: ONE f64 Cholesky per system serves both the
        tier check (scaled-condition estimate from the same factor) and the
        Newton solve; the statistics are recomputed only when the tier rises."""
        check = True
        while True:
            with phase("glm.system"):
                Gn, bn, l1, l2, A, L, info = self._ridge_system_dev(Ga, b)
            if not (check and self._tiers_due()):
                break
            with phase("glm.tier"):
                want = self._tier_raise(self._kappa_from_factor(A, L, info))
            if want is None:
                break
            self._sys_on_dev = True
            try:
                Ga, b, dev = self._irls_stats()
            finally:
                self._sys_on_dev = False
            self._stats_dev = dev
            check = want != "f64"
        with phase("glm.solve"):
            gmax, new = self._step_solve_dev(Gn, bn, l2, L, info)
        return Gn, bn, l1, l2, gmax, new

    def step(self):
        """One IRLS iteration (Gram on the matrix cores + host solve; wide
        ridge-only systems are conditioned and solved on the device)."""
        dev_solve = self._dev_system_ok()
        self._sys_on_dev = dev_solve or self._dev_tier_ok()
        try:
            Ga, b, dev = self._irls_stats()
        finally:
            self._sys_on_dev = False
        self._stats_dev = dev
        if torch.is_tensor(Ga) and dev_solve:
            Gn, bn, l1, l2, gmax, new = self._step_dev(Ga, b)
            if new is not None:
                return self._finish_step(new, gmax, self._stats_dev, l1, l2)
            Gn, bn = Gn.cpu().numpy(), bn.cpu().numpy()
            dev = self._stats_dev
        elif torch.is_tensor(Ga):
            # l1 / bounds: condition estimate on the device, solve on the host
            with phase("glm.tier"):
                Ga, b = self._check_tier_dev(Ga, b)
            Ga, b = Ga.cpu().numpy(), b.cpu().numpy()
            dev = self._stats_dev
            with phase("glm.system"):
                Gn, bn, l1, l2 = self._system(Ga, b)
        else:
            with phase("glm.tier"):
                Ga, b = self._check_tier(Ga, b)
            dev = self._stats_dev
            with phase("glm.system"):
                Gn, bn, l1, l2 = self._system(Ga, b)
        if self.est._parms.get("remove_collinear_columns") and self.active is None:
            self.active = self._find_collinear(Gn)
            self.removed_cols = [self.dinfo.coef_names[i] for i in range(self.P) if not self.active[i]]
        nonneg = bool(self.est._parms.get("non_negative"))
        nn_names = self.est._parms.get("_nonneg_names")
        if nn_names:
            s_ = set(nn_names)
            mask = np.array([nonneg or (c in s_) for c in self.dinfo.coef_names] + [False])
            nonneg = mask if self.intercept else mask[:-1]
        k = Gn.shape[0]
        # gradient of the penalized objective at the current beta (the IRLS
        # quadratic is exact to first order there): ComputationState.converged
        # stops when its max |.| (l1 subgradient) is under gradient_epsilon
        bcur = self.beta if self.intercept else self.beta[:-1]
        gq = Gn @ bcur - bn
        pen_idx = slice(0, self.P)
        gq[pen_idx] += l2 * bcur[pen_idx]
        gl1 = np.where(bcur[pen_idx] != 0, gq[pen_idx] + l1 * np.sign(bcur[pen_idx]),
                       np.sign(gq[pen_idx]) * np.maximum(np.abs(gq[pen_idx]) - l1, 0.0))
        gv = np.abs(np.concatenate([gl1, gq[self.P:]]))
        if self.active is not None:
            gv = np.where(self.active[:k], gv, 0.0)
        gmax = float(gv.max()) if gv.size else 0.0
        with phase("glm.solve"):
            new = _solve_quadratic(Gn, bn, l1, l2, self.intercept,
                                   beta0=self.beta if self.intercept else self.beta[:-1],
                                   non_negative=nonneg, lower=None if self.lower is None else self.lower[:k],
                                   upper=None if self.upper is None else self.upper[:k],
                                   active=None if self.active is None else self.active[:k])
        return self._finish_step(new, gmax, dev, l1, l2)

    def _finish_step(self, new, gmax, dev, l1, l2):
        r = self.obj_reg
        if not self.intercept:
            new = np.concatenate([new, [0.0]])
        diff = float(np.max(np.abs(new - self.beta))) if new.size else 0.0
        self.beta = new
        self.iter += 1
        obj = dev * r / 2 + l1 * np.abs(new[:-1]).sum() + l2 / 2 * (new[:-1] ** 2).sum()
        self.last_grad = gmax
        # gaussian/identity is solved exactly by one Newton step only when the
        # Hessian is exact (fp64 tier / host path); on a reduced-precision tier
        # the step carries ~kappa * eps(tier) relative error, removed by further
        # steps on the exact-gradient channel (iterative refinement)
        one_step = self.fam.family == "gaussian" and self.fam.link == "identity" and self._hprec in (None, "f64")
        self.converged = diff < self.beta_eps or abs(self.last_obj - obj) < self.obj_eps * max(abs(obj), 1e-12) or \
            one_step or (self.iter > 1 and gmax < self.grad_eps)
        if self.early_stop_enabled and not (self.fam.family == "gaussian" and self.fam.link == "identity"):
            self.converged = False
        self.last_obj = obj
        self.last_dev = dev
        return diff

    def _penalty_matrix(self):
        """Quadratic smoothing penalty (GAM): est._gam_penalty = (list of
        (coef names, S matrix)) mapped onto this driver's coefficient order."""
        if getattr(self, "_pen_cache", None) is not None:
            return self._pen_cache[0]
        spec = getattr(self.est, "_gam_penalty", None)
        pen = None
        if spec:
            pos = {n: i for i, n in enumerate(self.dinfo.coef_names)}
            pen = np.zeros((self.P, self.P))
            for names, S in spec:
                idx = [pos[n] for n in names]
                pen[np.ix_(idx, idx)] += S
        self._pen_cache = (pen,)
        return pen

    def deviance(self, beta=None):
        codes = self._wide_eta_codes()
        if codes is not None:
            b = self.beta if beta is None else beta
            dev, _ = self._wide_eta_pass(codes, b, float(b[-1]))
            return coll.allreduce_scalar(float(dev))
        eta = self._eta(beta)
        mu = self.fam.linkinv(eta)
        return coll.allreduce_scalar(float((self.w * self.fam.deviance(self.y, mu)).sum()))


class H2OGeneralizedLinearEstimator(H2OEstimator):
    algo = "glm"
    _defaults = GLM_DEFAULTS
    _balance_hidden = True

    def __init__(self, **kw):
        if "lambda" in kw:
            kw["lambda_"] = kw.pop("lambda")
        if "Lambda" in kw:
            kw["lambda_"] = kw.pop("Lambda")
        super().__init__(**kw)

    def _fit(self, spec):
        p = self._parms
        fam = (p.get("family") or "AUTO").lower()
        if fam == "auto":
            fam = "binomial" if spec.nclasses == 2 else ("multinomial" if spec.nclasses > 2 else "gaussian")
        if fam in ("gaussian", "poisson", "gamma", "tweedie", "negativebinomial") and spec.nclasses >= 2:
            # GLM.init (hex/glm/GLM.java:847)
            raise ValueError("ERRR on field: _response: Regression requires numeric response, got categorical.")
        if fam == "multinomial" and spec.nclasses <= 2:
            raise ValueError("ERRR on field: _family: Multinomial requires a categorical response with at least 3 "
                             "levels (for 2 class problem use family=binomial.")
        self._validate_glm(spec, fam)
        if fam == "multinomial" and spec.offset_column:
            # GLM.java:978: offset has no effect on multinomial and is ignored
            import warnings
            warnings.warn("offset_column has no effect on multinomial and will be ignored.")
        if fam in ("multinomial", "ordinal"):
            from .glm_multi import fit_multinomial
            return fit_multinomial(self, spec, fam)
        if p.get("HGLM"):
            from .hglm import fit_hglm
            return fit_hglm(self, spec)
        solver = (p.get("solver") or "AUTO").upper()
        if p.get("build_null_model"):
            # GLM.java:933 removePredictors: an intercept-only model
            spec.x = []
        drv = GLMDriver(self, spec)
        self._drv_family = drv.family
        maxit = int(p.get("max_iterations") or -1)
        if maxit == -1:
            # GLM.java:1035 (iterations accumulate over the lambda path)
            if solver == "L_BFGS":
                maxit = 10 * max(20, drv.P >> 2) * (10 if drv.alpha > 0 else 1)
            else:
                maxit = 10 * drv.nlambdas if p.get("lambda_search") else 50
        t0 = time.time()
        max_rt = float(p.get("max_runtime_secs") or 0)
        path = []
        self._scoring_history = []
        max_active = int(p.get("max_active_predictors") or -1)
        user_lams = p.get("lambda_")
        stop_rounds = int(p.get("stopping_rounds") or 0)
        sched = ScoreSchedule({"score_each_iteration": p.get("score_each_iteration"),
                               "score_tree_interval": p.get("score_iteration_interval")
                               if int(p.get("score_iteration_interval") or -1) > 0 else 0})
        metric_name = self._stopping_metric_name(spec)
        history = []
        scoring = bool(p.get("generate_scoring_history")) or drv.early_stop_enabled
        early_stop = False
        null_train = self._null_deviance(drv)
        null_valid = self._null_deviance_on(spec.valid, drv) if spec.valid is not None else None
        for ai, alpha in enumerate(drv.alphas):
            # one regularization path per alpha (GLM.java: alpha x lambda grid)
            if alpha != drv.alpha or len(drv.alphas) > 1:
                drv.alpha = alpha
                drv.beta = drv._init_beta.copy()
                if p.get("lambda_search") or user_lams is None:
                    drv.lambda_max = drv._lambda_max()
                    lmr = drv.lambda_min_ratio
                    if p.get("lambda_search") and user_lams is None:
                        nl = drv.nlambdas
                        dec = lmr ** (1.0 / max(nl - 1, 1))
                        drv.lambdas = [drv.lambda_max * dec ** i for i in range(nl)]
                    elif user_lams is None:
                        drv.lambdas = [10 * lmr * drv.lambda_max]
            # lambda-search early stopping (GLM.java:2923-2993): relative
            # deviance improvements of the last 5 submodels
            hist_tr, hist_te = [0.0] * 5, [0.0] * 5
            old_tr, old_te = null_train, null_valid
            nsub = 0
            for li, lam in enumerate(drv.lambdas):
                if drv.iter >= maxit or early_stop:
                    break
                drv.lam = lam
                drv.converged = False
                drv.last_obj = float("inf")
                if p.get("cold_start") and li > 0:
                    drv.beta = drv._init_beta.copy()
                while drv.iter < maxit and not drv.converged:
                    drv.step()
                    score, timed_out = self._tick(drv.iter, maxit, sched if scoring else None, False, t0, max_rt)
                    entry = {"iteration": drv.iter, "timestamp": time.time(), "duration": time.time() - t0,
                             "alpha": alpha, "lambda": lam, "negative_log_likelihood": drv.last_dev / 2,
                             "objective": drv.last_obj, "deviance_train": drv.last_dev / drv.wsum,
                             "gradient": drv.last_grad}
                    if score:
                        sched.started()
                        self._iter_score(drv, spec, entry)
                        sched.ended()
                    self._scoring_history.append(entry)
                    if score and drv.early_stop_enabled:
                        key = ("validation_" if spec.valid is not None else "training_") + metric_name
                        history.append(entry.get(key))
                        if ScoreKeeper.stop_early(history, stop_rounds, float(p.get("stopping_tolerance", 1e-3)),
                                                  metric_name in _LESS_IS_BETTER, metric=metric_name):
                            early_stop = True
                            break
                    if timed_out:
                        break
                dev = drv.deviance()
                beta, icpt = drv.dinfo.destandardize(drv.beta[:-1], drv.beta[-1])
                sm = {"lambda": lam, "alpha": alpha, "beta_std": drv.beta.copy(), "beta": beta,
                      "icpt": icpt, "deviance": dev, "explained_deviance_train": None, "iteration": drv.iter}
                path.append(sm)
                if max_active > 0 and int(np.sum(np.abs(drv.beta[:-1]) > 0)) + (1 if drv.intercept else 0) \
                        > max_active:
                    # GLM.java: the path stops once too many predictors are
                    # active; the submodel returned is the last one within it
                    if len(path) > 1:
                        path.pop()
                    break
                if p.get("lambda_search"):
                    dev_te = self._dev_on(spec.valid, sm, drv) if spec.valid is not None else None
                    hist_tr[nsub % 5] = (old_tr - dev) / old_tr if old_tr else 0.0
                    old_tr = dev
                    if dev_te is not None:
                        hist_te[nsub % 5] = (old_te - dev_te) / old_te if old_te else 0.0
                        old_te = dev_te
                    nsub += 1
                    if lam < drv.lambda_max and p.get("early_stopping", True) and drv.iter >= 5:
                        if max(hist_tr) < 1e-4:
                            break
                        if dev_te is not None and int(p.get("nfolds") or 0) <= 1 and max(hist_te) < 0:
                            break
                if self._tick(drv.iter, maxit, None, False, t0, max_rt)[1]:
                    break
        # pick submodel: best by validation deviance if given, else (several
        # alphas) by training deviance of each alpha's last lambda, else last
        best = len(path) - 1
        if spec.valid is not None and len(path) > 1 and (p.get("lambda_search") or len(drv.alphas) > 1):
            vdrv_devs = [self._dev_on(spec.valid, sm, drv) for sm in path]
            best = int(np.argmin(vdrv_devs))
        elif len(drv.alphas) > 1:
            ends = [i for i in range(len(path)) if i == len(path) - 1 or path[i + 1]["alpha"] != path[i]["alpha"]]
            best = min(ends, key=lambda i: path[i]["deviance"])
        sm = path[best]
        drv.alpha = sm["alpha"]
        pr = float(p.get("prior") or -1)
        if pr > 0 and drv.family == "binomial" and drv.intercept:
            # prior correction of the intercept for over/under-sampled data (GLMModel)
            ym = min(max(drv.ymu, 1e-10), 1 - 1e-10)
            corr = math.log(pr / (1 - pr)) - math.log(ym / (1 - ym))
            sm = dict(sm)
            sm["beta_std"] = sm["beta_std"].copy()
            sm["beta_std"][-1] += corr
            sm["icpt"] += corr
        self._drv = drv
        self._beta_std = sm["beta_std"]
        self._beta = sm["beta"]
        self._icpt = sm["icpt"]
        self._lambda_best = sm["lambda"]
        self._path = path
        self._dinfo = drv.dinfo
        self._fam = drv.fam
        self._finalize_outputs(drv, sm)
        self._dev_x_cache = {}
        drv.X = None

    def _dev_on(self, frame, sm, drv):
        # the frame's model matrix, response and row mask are built once per
        # fit (a lambda search evaluates every submodel on the validation
        # frame: re-expanding it per lambda was most of an AutoML GLM step)
        cache = self.__dict__.setdefault("_dev_x_cache", {})
        ent = cache.get(id(frame))
        if ent is None or ent[0] is not frame or ent[1] is not drv:
            cache.clear()
            X, ok = drv.dinfo.expand(frame)
            y = self._spec.y_tensor(frame)
            yy = (y == 1).to(torch.float64) if self._spec.is_classification else y.to(torch.float64)
            m = ok & (~torch.isnan(yy) if not self._spec.is_classification else (y >= 0))
            ent = cache[id(frame)] = (frame, drv, X, yy[m], m)
        _, _, X, ym, m = ent
        bt = torch.zeros(drv.Pp, dtype=torch.float32, device=X.device)
        bt[: drv.P] = torch.as_tensor(sm["beta_std"][: drv.P], dtype=torch.float32)
        eta = (X @ bt).to(torch.float64) + sm["beta_std"][-1]
        mu = drv.fam.linkinv(eta)
        return coll.allreduce_scalar(float(drv.fam.deviance(ym, mu[m]).sum()))

    def _null_deviance_on(self, frame, drv):
        """Deviance of the intercept-only (training mean) model on `frame`."""
        y = self._spec.y_tensor(frame)
        yy = (y == 1).to(torch.float64) if self._spec.is_classification else y.to(torch.float64)
        m = ~torch.isnan(yy) if not self._spec.is_classification else (y >= 0)
        mu = torch.full_like(yy[m], min(max(drv.ymu, 1e-10), 1 - 1e-10) if drv.fam.link == "logit" else drv.ymu)
        return coll.allreduce_scalar(float(drv.fam.deviance(yy[m], mu).sum()))

    def _stopping_metric_name(self, spec):
        m = (self._parms.get("stopping_metric") or "auto").lower()
        if m == "auto":
            return "logloss" if spec.is_classification else "deviance"
        return m

    def _iter_score(self, drv, spec, entry):
        """Training (and validation) metrics of the current coefficients
        (GLM.java scoreAndUpdateModel; generate_scoring_history and
        stopping_rounds read them)."""
        from ..tree.gbm import H2OGradientBoostingEstimator as _G
        self._beta_std, self._dinfo, self._fam = drv.beta.copy(), drv.dinfo, drv.fam
        mu = drv.fam.linkinv(drv._eta())
        raw = torch.stack([1 - mu, mu], 1) if spec.nclasses == 2 else mu.view(-1, 1)
        _G._add_metrics(entry, "training", self._metrics_from_raw(spec, spec.frame, raw))
        if spec.valid is not None:
            _G._add_metrics(entry, "validation", self._metrics_from_raw(spec, spec.valid,
                                                                        self._predict_raw(spec.valid)))

    def _validate_glm(self, spec, fam):
        """GLM.init (hex/glm/GLM.java:846-1017) parameter checks."""
        p = self._parms
        solver = (p.get("solver") or "AUTO").upper()
        link = (p.get("link") or "family_default").lower()
        if solver in ("GRADIENT_DESCENT_LH", "GRADIENT_DESCENT_SQERR") and fam != "ordinal":
            raise ValueError("ERRR on field: _solver: Solvers GRADIENT_DESCENT_LH and GRADIENT_DESCENT_SQERR are "
                             "only supported for ordinal regression.  Do not choose them unless you specify your "
                             "family to be ordinal")
        if (p.get("family") or "AUTO").lower() == "auto" and link != "family_default":
            nc = spec.nclasses
            ok = ("identity", "log", "inverse") if nc <= 1 else (("logit",) if nc == 2 else ("multinomial",))
            if link not in ok:
                raise ValueError(f"ERRR on field: _family: AUTO for underlying response requires the link to be "
                                 f"family_default or {', '.join(ok)}.")
        if fam == "binomial" and spec.nclasses > 2:
            raise ValueError("ERRR on field: _family: Binomial requires the response to be a 2-class categorical "
                             "or a binary column (0/1)")
        if fam in ("poisson", "negativebinomial", "gamma"):
            y = spec.y_tensor().to(torch.float64)
            ymin = coll.allreduce_scalar(float(torch.nan_to_num(y, nan=float("inf")).min()) if y.numel()
                                         else float("inf"), op="min")
            if fam == "gamma" and ymin <= 0:
                raise ValueError("ERRR on field: _family: Response value for gamma distribution must be greater "
                                 "than 0.")
            if fam != "gamma" and ymin < 0:
                raise ValueError("ERRR on field: _family: Poisson and Negative Binomial require response >= 0")
            if fam == "negativebinomial":
                th = float(p.get("theta") or 1e-10)
                if th <= 0 or th > 1:
                    raise ValueError("ERRR on field: _family: Illegal Negative Binomial theta value.  Valid theta "
                                     "values be > 0 and <= 1.")
        if fam == "ordinal":
            if spec.nclasses <= 2:
                raise ValueError("ERRR on field: _family: Ordinal requires a categorical response with at least 3 "
                                 "levels (for 2 class problem use family=binomial.")
            if link in ("oprobit", "ologlog"):
                raise ValueError("ERRR on field: _link: Ordinal regression only supports ologit as link.")
            if spec.offset_column:
                raise ValueError("ERRR on field: offset_column: does not work with ordinal family right now.  Will "
                                 "be fixed in the future.")
        if fam == "fractionalbinomial":
            y = spec.y_tensor().to(torch.float64)
            y = y[~torch.isnan(y)]
            lo = coll.allreduce_scalar(float(y.min()) if y.numel() else 0.0, op="min")
            hi = coll.allreduce_scalar(float(y.max()) if y.numel() else 0.0, op="max")
            if lo < 0 or hi > 1:
                raise ValueError(f"ERRR on field: response: Response '{spec.y}' must be between 0 and 1 for "
                                 f"fractional_binomial family. Min: {lo:f}, Max: {hi:f}")
        mvh = (p.get("missing_values_handling") or "MeanImputation").lower()
        if p.get("plug_values") is not None and mvh != "plugvalues":
            raise ValueError("ERRR on field: _missing_values_handling: When plug values are provided - Missing "
                             "Values Handling needs to be explicitly set to PlugValues.")
        if p.get("plug_values") is None and mvh == "plugvalues":
            raise ValueError("ERRR on field: _missing_values_handling: No plug values frame provided for Missing "
                             "Values Handling = PlugValues.")
        disp_fams = ("tweedie", "gamma", "negativebinomial")
        if p.get("build_null_model") and fam not in disp_fams:
            raise ValueError("ERRR on field: build_null_model: is only supported for tweedie, gamma and "
                             "negativebinomial familes")
        if p.get("max_iterations") is not None and int(p.get("max_iterations")) == 0:
            raise ValueError("ERRR on field: _max_iterations: if specified, must be >= 1.")
        if p.get("lambda_search") and int(p.get("stopping_rounds") or 0) > 0:
            raise ValueError("ERRR on field: early stop: cannot run when lambda_search=True.  Lambda_search has its "
                             "own early-stopping mechanism")
        if fam in ("multinomial", "ordinal") and (p.get("beta_constraints") is not None or p.get("non_negative")):
            what = "non_negative" if p.get("non_negative") else "beta_constraints"
            raise ValueError(f"ERRR on field: {what}: does not work with {fam} family.")
        method = (p.get("dispersion_parameter_method") or "pearson").lower()
        if method not in ("pearson", "deviance", "ml"):
            raise ValueError(f"dispersion_parameter_method must be one of pearson, deviance, ml; got {method}")
        if method == "ml":
            if fam != "gamma":
                raise ValueError("ERRR on field: dispersion_parameter_mode: ml can only be used for family gamma.")
            if int(p.get("max_iterations_dispersion") or 0) <= 0:
                raise ValueError("ERRR on field: max_iterations_dispersion: must > 0.")
            if float(p.get("dispersion_epsilon") if p.get("dispersion_epsilon") is not None else 1e-4) < 0:
                raise ValueError("ERRR on field: dispersion_epsilon: must >= 0.")
        if p.get("fix_dispersion_parameter") and fam not in disp_fams:
            raise ValueError("ERRR on field: fix_dispersion_parameter: is only supported for gamma, tweedie, "
                             "negativebinomial families.")
        if float(p.get("init_dispersion_parameter") if p.get("init_dispersion_parameter") is not None else 1) <= 0:
            raise ValueError("ERRR on field: init_dispersion_parameter: must exceed 0.0.")
        if p.get("compute_p_values") and p.get("beta_constraints") is not None:
            raise ValueError("ERRR on field: _compute_p_values: P-values can not be computed for constrained "
                             "problems")

    def _estimate_dispersion(self, drv):
        """Dispersion parameter for the p-values (GLM.java:2320-2344):
        1 for binomial / poisson, init_dispersion_parameter when fixed,
        else Pearson (sum w (y - mu)^2 / V(mu)) or deviance sum over
        nobs - 1 - #active predictors, or the maximum-likelihood estimate
        for gamma (GLM.java:2375 estimateMLSE: Newton on 1/phi with the
        di/trigamma sums as one fused device pass per iteration).
        Returns (dispersion, estimated)."""
        p = self._parms
        fam = drv.family
        init = float(p.get("init_dispersion_parameter") or 1.0)
        if fam in ("binomial", "poisson") or p.get("fix_dispersion_parameter"):
            return (1.0 if fam in ("binomial", "poisson") and not p.get("fix_dispersion_parameter") else init), False
        method = (p.get("dispersion_parameter_method") or "pearson").lower()
        mu = drv.fam.linkinv(drv._eta())
        w, y = drv.w, drv.y
        nact = drv.P - (int((~drv.active[: drv.P]).sum()) if drv.active is not None else 0)
        if method in ("pearson", "deviance"):
            if method == "deviance":
                s = (w * drv.fam.deviance(y, mu)).nan_to_num(0.0).sum()
            elif fam == "tweedie":
                s = (w * (y - mu) ** 2 / mu.abs().pow(drv.fam.tvp)).nan_to_num(0.0).sum()
            else:
                s = (w * (y - mu) ** 2 / drv.fam.variance(mu)).nan_to_num(0.0).sum()
            return coll.allreduce_scalar(float(s)) / max(drv.nobs - 1 - nact, 1), True
        # ml (gamma)
        pos = (y > 0) & (w > 0)
        wp, yp, mp = w[pos], y[pos], mu[pos]
        tmp = wp * yp / mp
        st = torch.stack([wp.sum(), (wp * torch.log(tmp)).sum(), tmp.sum()])
        coll.allreduce_(st)
        wsum, sum_ln, sum_yu = (float(v) for v in st)
        const = wsum + sum_ln - sum_yu
        alpha = 1.0 / init
        eps = float(p.get("dispersion_epsilon") if p.get("dispersion_epsilon") is not None else 1e-4)
        for _ in range(int(p.get("max_iterations_dispersion") or 3000)):
            dt = torch.stack([(wp * torch.special.digamma(wp * alpha)).sum(),
                              (wp * wp * torch.special.polygamma(1, wp * alpha)).sum()])
            coll.allreduce_(dt)
            num = wsum * math.log(alpha) - float(dt[0]) + const
            den = wsum / alpha - float(dt[1])
            if den == 0 or not math.isfinite(num / den):
                break
            change = num / den
            if abs(change) < eps:
                alpha -= change
                break
            alpha = alpha - change if alpha - change >= 0 else alpha * 0.5
        return 1.0 / alpha, True

    def _finalize_outputs(self, drv, sm):
        names = drv.dinfo.coef_names
        coefs = {"Intercept": float(self._icpt)}
        coefs.update({n: float(b) for n, b in zip(names, self._beta)})
        std = {"Intercept": float(self._beta_std[-1])}
        std.update({n: float(b) for n, b in zip(names, self._beta_std[:-1])})
        self._output["coefficients"] = coefs
        self._output["standardized_coefficients"] = std
        null_dev = self._null_deviance(drv)
        res_dev = sm["deviance"]
        nz = int(np.sum(np.abs(self._beta) > 0)) + (1 if drv.intercept else 0)
        self._output["null_deviance"] = null_dev
        self._output["residual_deviance"] = res_dev
        self._output["null_degrees_of_freedom"] = int(drv.nobs - (1 if drv.intercept else 0))
        self._output["residual_degrees_of_freedom"] = int(drv.nobs - nz)
        self._output["lambda_best"] = sm["lambda"]
        self._output["lambda_max"] = drv.lambda_max
        self._output["alpha_best"] = drv.alpha
        self._output["variable_importances"] = {n: abs(b) for n, b in zip(names, self._beta_std[:-1])}
        self._output["model_summary"] = {"family": drv.family, "link": drv.fam.link,
                                         "regularization": f"Elastic Net (alpha = {drv.alpha}, lambda = {sm['lambda']:.4g} )",
                                         "number_of_predictors_total": drv.P,
                                         "number_of_active_predictors": int(np.sum(np.abs(self._beta) > 0)),
                                         "number_of_iterations": drv.iter}
        self._output["aic"] = self._aic(drv, res_dev, nz)
        if self._parms.get("calc_like"):
            self._output["loglikelihood"] = self._loglik(drv)
        if getattr(drv, "removed_cols", None):
            self._output["removed_collinear_columns"] = list(drv.removed_cols)
        if self._parms.get("compute_p_values"):
            self._p_values(drv)
        # hex/glm/GLMModel.getRegularizationPath (GetGLMRegPathHandler): per
        # submodel lambda, alpha, explained training deviance 1 - dev / null dev,
        # and the coefficients (original and standardized scale)
        nd = float(self._output.get("null_deviance") or 0.0)
        self._output["regularization_path"] = {
            "lambdas": [s["lambda"] for s in self._path],
            "alphas": [s.get("alpha") for s in self._path],
            "explained_deviance_train": [(1.0 - float(s["deviance"]) / nd) if nd > 0 else None for s in self._path],
            "explained_deviance_valid": None,
            "coefficients": [dict(zip(names + ["Intercept"], list(s["beta"]) + [s["icpt"]])) for s in self._path],
            "coefficients_std": [dict(zip(names + ["Intercept"], [float(b) for b in s["beta_std"]]))
                                 for s in self._path]}

    def _null_deviance(self, drv):
        mu = torch.full_like(drv.y, drv.ymu)
        if drv.offset is not None and drv.intercept:
            # intercept-only fit with offset: a few Newton steps
            b0 = 0.0
            for _ in range(25):
                eta = drv.offset + b0
                m = drv.fam.linkinv(eta)
                d = drv.fam.dmu_deta(eta, m)
                W = drv.w * d * d / drv.fam.variance(m)
                g = coll.allreduce_scalar(float((drv.w * (drv.y - m) * d / drv.fam.variance(m)).sum()))
                h = coll.allreduce_scalar(float(W.sum()))
                if h <= 0:
                    break
                b0 += g / h
                if abs(g / h) < 1e-10:
                    break
            mu = drv.fam.linkinv(drv.offset + b0)
        return coll.allreduce_scalar(float((drv.w * drv.fam.deviance(drv.y, mu)).sum()))

    def _aic(self, drv, res_dev, k):
        f = drv.family
        n = drv.wsum
        if f == "gaussian":
            return n * (math.log(2 * math.pi * res_dev / n) + 1) + 2 + 2 * k
        if f in ("binomial", "quasibinomial", "fractionalbinomial"):
            return res_dev + 2 * k
        if f == "poisson":
            eta = drv._eta()
            mu = drv.fam.linkinv(eta)
            ll = float((drv.w * (drv.y * torch.log(mu.clamp_min(1e-300)) - mu - torch.lgamma(drv.y + 1))).sum())
            return -2 * coll.allreduce_scalar(ll) + 2 * k
        return float("nan")

    def _loglik(self, drv):
        """Log-likelihood of the fitted model (calc_like; GLMModel likelihood)."""
        eta = drv._eta()
        mu = drv.fam.linkinv(eta)
        y, w, f = drv.y, drv.w, drv.family
        if f in ("binomial", "quasibinomial", "fractionalbinomial"):
            m = mu.clamp(1e-15, 1 - 1e-15)
            ll = (w * (y * torch.log(m) + (1 - y) * torch.log(1 - m))).sum()
        elif f == "poisson":
            ll = (w * (y * torch.log(mu.clamp_min(1e-300)) - mu - torch.lgamma(y + 1))).sum()
        elif f == "gaussian":
            rss = coll.allreduce_scalar(float((w * (y - mu) ** 2).sum()))
            n = drv.wsum
            return -0.5 * n * (math.log(2 * math.pi * rss / n) + 1)
        else:
            return float("nan")
        return coll.allreduce_scalar(float(ll))

    def _p_values(self, drv):
        # the covariance comes from an fp64 Hessian at the final coefficients
        # (the reference's double Gram), not from the Newton step's bf16x3 / bf16
        # tier: the step only needed its precision for the convergence rate
        prev = drv._hprec
        drv._hprec = "f64"
        try:
            Ga, b, dev = drv._irls_stats()
        finally:
            drv._hprec = prev
        P = drv.P
        if not drv.intercept:
            Ga = Ga[:P, :P]
        try:
            inv = np.linalg.inv(Ga)
        except np.linalg.LinAlgError:
            inv = np.linalg.pinv(Ga)
        nz = P + (1 if drv.intercept else 0)
        disp, estimated = self._estimate_dispersion(drv)
        se_std = np.sqrt(np.maximum(np.diag(inv), 0) * disp)
        from scipy import stats
        beta = drv.beta if drv.intercept else drv.beta[:-1]
        z = beta / np.where(se_std > 0, se_std, np.nan)
        if estimated:
            # GLMModel.setZValues: Student t with nobs - rank degrees of freedom
            pv = 2 * stats.t.sf(np.abs(z), max(drv.nobs - nz, 1))
        else:
            pv = 2 * stats.norm.sf(np.abs(z))
        names = drv.dinfo.coef_names + (["Intercept"] if drv.intercept else [])
        # destandardized std errors for numeric columns
        se = se_std.copy()
        if drv.dinfo.standardize:
            base = drv.dinfo.n_cat_expanded
            for j in range(len(drv.dinfo.num_cols)):
                se[base + j] = se_std[base + j] / drv.dinfo.sigmas[j]
        self._output["std_errs"] = dict(zip(names, se.tolist()))
        self._output["z_values"] = dict(zip(names, z.tolist()))
        self._output["p_values"] = dict(zip(names, pv.tolist()))
        self._output["dispersion"] = disp
        self._output["dispersion_estimated"] = estimated

    # ---- accessors (h2o-py GLM API)
    def coef(self):
        return dict(self._output["coefficients"])

    def coef_norm(self):
        return dict(self._output["standardized_coefficients"])

    def coef_with_p_values(self):
        import pandas as pd
        c = self._output["coefficients"]
        rows = []
        for n in ["Intercept"] + [k for k in c if k != "Intercept"]:
            rows.append({"names": n, "coefficients": c[n], "std_error": self._output.get("std_errs", {}).get(n),
                         "z_value": self._output.get("z_values", {}).get(n),
                         "p_value": self._output.get("p_values", {}).get(n),
                         "standardized_coefficients": self._output["standardized_coefficients"].get(n)})
        return pd.DataFrame(rows)

    def null_deviance(self, train=False, valid=False, xval=False):
        return self._output.get("null_deviance")

    def residual_deviance(self, train=False, valid=False, xval=False):
        return self._output.get("residual_deviance")

    def aic(self, train=False, valid=False, xval=False):
        return self._output.get("aic")

    def null_degrees_of_freedom(self, **kw):
        return self._output.get("null_degrees_of_freedom")

    def residual_degrees_of_freedom(self, **kw):
        return self._output.get("residual_degrees_of_freedom")

    @staticmethod
    def makeGLMModel(model, coefs, threshold=0.5):
        """A copy of a trained binomial / regression GLM with user-given
        coefficients (h2o-py glm.py makeGLMModel -> hex/glm/
        MakeGLMModelHandler.java): coefs maps coefficient names (incl.
        "Intercept") to original-scale values; coefficients not named keep
        their values; the binomial decision threshold is set."""
        import copy
        if getattr(model, "_multi", None) is not None or getattr(model, "_hglm", None) is not None:
            raise ValueError("makeGLMModel supports binomial and regression GLMs")
        names = list(model._dinfo.coef_names)
        unknown = [k for k in coefs if k != "Intercept" and k not in names]
        if unknown:
            raise ValueError(f"unknown coefficient names: {unknown}")
        beta = np.array(model._beta, dtype=np.float64).copy()
        for j, n in enumerate(names):
            if n in coefs:
                beta[j] = float(coefs[n])
        icpt = float(coefs.get("Intercept", model._icpt))
        # original scale -> the standardized space the scorer uses (inverse of DataInfo.destandardize)
        bstd = beta.copy()
        istd = icpt
        di = model._dinfo
        if di.standardize:
            base = di.n_cat_expanded
            for j in range(len(di.num_cols)):
                bstd[base + j] = beta[base + j] * di.sigmas[j]
                istd += beta[base + j] * di.means[j]
        m = copy.copy(model)
        m._output = copy.deepcopy(model._output)
        m._beta, m._icpt = beta, icpt
        m._beta_std = np.concatenate([bstd, [istd]])
        m._output["coefficients"] = {"Intercept": icpt, **{n: float(b) for n, b in zip(names, beta)}}
        m._output["standardized_coefficients"] = {"Intercept": istd,
                                                  **{n: float(b) for n, b in zip(names, bstd)}}
        m._output["default_threshold"] = float(threshold)
        m._training_metrics = m._validation_metrics = m._cross_validation_metrics = None
        m._id = f"{model.model_id}_makeGLMModel"
        return m

    @staticmethod
    def getGLMRegularizationPath(model):
        return model._output["regularization_path"]

    def _predict_link(self, frame):
        X, _ = self._dinfo.expand(frame)
        bt = torch.zeros(self._dinfo.Pp, dtype=torch.float32, device=X.device)
        bt[: self._dinfo.P] = torch.as_tensor(self._beta_std[:-1], dtype=torch.float32)
        eta = (X @ bt).to(torch.float64) + float(self._beta_std[-1])
        off = self._spec.offset_column
        if off and off in frame.names:
            eta = eta + torch.nan_to_num(frame.vec(off).as_float(torch.float64))
        return eta

    def coefs_random(self):
        """Random effects per random column and level (HGLM)."""
        return dict(self._output.get("ubeta", {}))

    def _predict_raw(self, frame):
        if getattr(self, "_hglm", None) is not None:
            from .hglm import predict_hglm
            return predict_hglm(self, frame)
        if getattr(self, "_multi", None) is not None:
            from .glm_multi import predict_multi
            return predict_multi(self, frame)
        eta = self._predict_link(frame)
        mu = self._fam.linkinv(eta)
        if self._spec.nclasses == 2:
            return torch.stack([1 - mu, mu], 1)
        return mu.view(-1, 1)

    def _metrics_from_raw(self, spec, frame, raw, w=None, auc_type=None):
        m = super()._metrics_from_raw(spec, frame, raw, w, auc_type=auc_type)
        multi = getattr(self, "_multi", None)
        if m is not None and multi is not None and multi.get("kind") == "ordinal":
            # ordinal family -> ModelMetricsOrdinal (hex/ModelMetricsOrdinal.java): same hit ratios,
            # logloss and confusion matrix as multinomial, own category
            m.__class__ = mm.ModelMetricsOrdinal
            m.kind = "ordinal"
        if m is not None and multi is None and getattr(self, "_hglm", None) is None \
                and frame is spec.frame:
            m._m["null_deviance"] = self._output.get("null_deviance")
            m._m["residual_deviance"] = self._output.get("residual_deviance")
            m._m["AIC"] = self._output.get("aic")
        return m
