"""Generalized Additive Models.

Reference: hex/gam/GAM.java, GAMModel.java, hex/gam/GamSplines/
(CubicRegressionSplines.java: natural cubic regression spline with knot
values as coefficients, penalty D' B^-1 D; ThinPlateRegressionUtils /
ThinPlateDistanceWithKnots: eta(r) = |r|^3 in 1-D with the polynomial
null space; ISplines.java / MSplines.java: monotone I-splines and
M-splines of a given spline order), identifiability via a sum-to-zero
(centering) constraint Z from a QR of the column sums, penalties scaled by
`scale`, smoothers fed to GLM as extra columns named
<col>_cr_i / _tp_i / _is_i / _ms_i.

MI355X design: every basis is evaluated on the device in one vectorised
pass (searchsorted for the knot interval + gathers of the per-interval
cubic coefficients, Cox-de Boor recursion for B-splines over all rows at
once); the penalty enters the IRLS normal equations of the fused GLM
kernel's Gram on the host (P x P), so a GAM iteration costs exactly one
GLM iteration.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from ...core.frame import H2OFrame
from ...core.vec import T_REAL, Vec
from ...parallel import cloud
from ...parallel import collectives as coll
from .glm import GLM_DEFAULTS, H2OGeneralizedLinearEstimator

GAM_DEFAULTS = dict(GLM_DEFAULTS)
GAM_DEFAULTS.update(gam_columns=None, num_knots=None, knot_ids=None, bs=None, scale=None, keep_gam_cols=False,
                    spline_orders=None, splines_non_negative=None, standardize=False, lambda_=0.0,
                    standardize_tp_gam_cols=False, scale_tp_penalty_mat=False, store_knot_locations=False)

_SUFFIX = {0: "cr", 1: "tp", 2: "is", 3: "ms"}


# ---------------------------------------------------------------- bases
def _cr_matrices(knots):
    k = len(knots)
    h = np.diff(knots)
    D = np.zeros((k - 2, k))
    B = np.zeros((k - 2, k - 2))
    for i in range(k - 2):
        D[i, i], D[i, i + 1], D[i, i + 2] = 1 / h[i], -1 / h[i] - 1 / h[i + 1], 1 / h[i + 1]
        B[i, i] = (h[i] + h[i + 1]) / 3
        if i < k - 3:
            B[i, i + 1] = B[i + 1, i] = h[i + 1] / 6
    F = np.linalg.solve(B, D)
    Fp = np.vstack([np.zeros(k), F, np.zeros(k)])
    return Fp, D.T @ F


def cr_basis(x: torch.Tensor, knots: np.ndarray):
    """Natural cubic regression spline basis [n, k] (coefficients = f(knots)),
    as GamUtilsCubicRegression.expandOneGamCol: the knot interval by
    locateBin (x <= k_0 -> first, x >= k_last -> last interval) and the
    interval's cubic continued outside the knot range."""
    k = len(knots)
    Fp_np, S = _cr_matrices(knots)
    dev, dt = x.device, torch.float64
    kn = torch.as_tensor(knots, dtype=dt, device=dev)
    Fp = torch.as_tensor(Fp_np, dtype=dt, device=dev)
    h = kn[1:] - kn[:-1]
    xd = x.to(dt)
    j = (torch.searchsorted(kn, xd, right=True) - 1).clamp(0, k - 2)
    xl, xr, hj = kn[j], kn[j + 1], h[j]
    am, ap = (xr - xd) / hj, (xd - xl) / hj
    cm = ((xr - xd) ** 3 / hj - hj * (xr - xd)) / 6
    cp = ((xd - xl) ** 3 / hj - hj * (xd - xl)) / 6
    n = x.shape[0]
    X = cm.view(-1, 1) * Fp[j] + cp.view(-1, 1) * Fp[j + 1]
    r = torch.arange(n, device=dev)
    X[r, j] += am
    X[r, j + 1] += ap
    return X, S


def tp_constant(m, d):
    """GamUtilsThinPlateRegression.calTPConstantTerm."""
    from math import factorial, pi
    if d % 2 == 0:
        return (-1) ** (m + 1 + d // 2) / (2 ** (2 * m - 1) * pi ** (d / 2.0) * factorial(m - 1) *
                                           factorial(m - d // 2))
    return (-1) ** m * m / (factorial(2 * m) * pi ** ((d - 1) / 2.0))


def tp_distance(X, knots, m, ostd=None):
    """c * r^(2m-d) (times log r^(2m-d) for even d) between rows and knots
    (GamUtilsThinPlateRegression.calculateDistance); numpy or torch."""
    d = knots.shape[1]
    c = tp_constant(m, d)
    if isinstance(X, torch.Tensor):
        kn = torch.as_tensor(knots, dtype=torch.float64, device=X.device)
        diff = X.to(torch.float64).unsqueeze(1) - kn.unsqueeze(0)
        if ostd is not None:
            diff = diff * torch.as_tensor(ostd, dtype=torch.float64, device=X.device)
        dist = torch.sqrt((diff * diff).sum(-1)) ** (2 * m - d)
        val = c * dist
        if d % 2 == 0:
            val = torch.where(dist != 0, val * torch.log(dist.clamp_min(1e-300)), val)
        return val
    diff = np.asarray(X, dtype=np.float64)[:, None, :] - knots[None, :, :]
    if ostd is not None:
        diff = diff * np.asarray(ostd)
    dist = np.sqrt((diff * diff).sum(-1)) ** (2 * m - d)
    val = c * dist
    if d % 2 == 0:
        val = np.where(dist != 0, val * np.log(np.where(dist != 0, dist, 1.0)), val)
    return val


def tp_poly(X, terms, means=None, ostd=None):
    """Polynomial null-space basis (GamUtilsThinPlateRegression.calculatePolynomialBasis;
    with standardisation each predictor enters as x - mean * (1/std), as the
    reference computes it)."""
    Xd = X.to(torch.float64)
    if means is not None:
        Xd = Xd - torch.as_tensor(np.asarray(means) * np.asarray(ostd), dtype=torch.float64, device=X.device)
    cols = [torch.prod(Xd ** torch.as_tensor(e, dtype=torch.float64, device=X.device), 1) for e in terms]
    return torch.stack(cols, 1)


def tp_setup(knots, means, ostd, standardize):
    """Per-smoother thin-plate constants (GAM.java ThinPlateRegressionSmootherWithKnots):
    polynomial terms (degree < m, constant included), zCS = orthonormal
    complement of the polynomial values at the (demeaned) knots, and the
    penalty zCS' E_kk zCS expanded with zero rows for the polynomial part."""
    kn = np.asarray(knots, dtype=np.float64)
    k, d = kn.shape
    m = _tp_m(d)
    terms = _poly_terms(d, m)
    M = len(terms)
    dm = (kn - np.asarray(means)) * (np.asarray(ostd) if standardize else 1.0)
    T = np.stack([np.prod(dm ** np.asarray(e), 1) for e in terms], 1)          # [k, M]
    Q, _ = np.linalg.qr(T, mode="complete")
    zCS = Q[:, M:]                                                            # [k, k - M]
    Ekk = tp_distance(kn, kn, m, ostd if standardize else None)
    S = np.zeros((k, k))
    S[: k - M, : k - M] = zCS.T @ Ekk @ zCS
    return {"m": m, "M": M, "terms": terms, "zCS": zCS, "S": S}


def tp_ref_basis(X: torch.Tensor, knots: np.ndarray, setup, means, ostd, standardize):
    """Thin-plate regression spline with knots [n, k]: distances projected on
    zCS (k - M columns) followed by the M polynomial terms."""
    kn = np.asarray(knots, dtype=np.float64)
    E = tp_distance(X, kn, setup["m"], ostd if standardize else None)
    Xcs = E @ torch.as_tensor(setup["zCS"], dtype=torch.float64, device=X.device)
    P = tp_poly(X, setup["terms"], means if standardize else None, ostd if standardize else None)
    return torch.cat([Xcs, P], 1), setup["S"]


def _tp_m(d):
    return (d + 1) // 2 + 1


def _poly_terms(d, m):
    """Exponent tuples of the monomials of total degree < m in d variables."""
    import itertools
    return [e for e in itertools.product(range(m), repeat=d) if sum(e) < m]


def _bspline(x: torch.Tensor, knots: np.ndarray, order: int):
    """B-spline basis of `order` (degree order-1) with clamped boundary knots."""
    t = np.concatenate([[knots[0]] * (order - 1), knots, [knots[-1]] * (order - 1)])
    tt = torch.as_tensor(t, dtype=torch.float64, device=x.device)
    xd = x.to(torch.float64).clamp(float(knots[0]), float(knots[-1]))
    nb = len(t) - 1
    B = ((xd.view(-1, 1) >= tt[:-1]) & (xd.view(-1, 1) < tt[1:])).to(torch.float64)
    # right end belongs to the last non-empty interval
    last = int(np.nonzero(t[:-1] < t[1:])[0][-1])
    B[:, last] = torch.where(xd == tt[-1], torch.ones_like(xd), B[:, last])
    for d in range(1, order):
        nbd = nb - d
        left = tt[:nbd]
        den1 = tt[d:d + nbd] - left
        den2 = tt[d + 1:d + 1 + nbd] - tt[1:1 + nbd]
        a = torch.where(den1 > 0, (xd.view(-1, 1) - left) / den1.clamp_min(1e-300), torch.zeros_like(B[:, :nbd]))
        b = torch.where(den2 > 0, (tt[d + 1:d + 1 + nbd] - xd.view(-1, 1)) / den2.clamp_min(1e-300),
                        torch.zeros_like(B[:, :nbd]))
        B = a * B[:, :nbd] + b * B[:, 1:nbd + 1]
    return B


def _diff_penalty(m):
    Dm = np.diff(np.eye(m), 2, axis=0) if m > 2 else np.zeros((0, m))
    return Dm.T @ Dm


def ms_basis(x, knots, order):
    B = _bspline(x, knots, order)
    return B, _diff_penalty(B.shape[1])


def is_basis(x, knots, order):
    """I-splines: I_j(x) = sum_{m >= j} B_m(x) (order+1 B-splines), j >= 1."""
    B = _bspline(x, knots, order + 1)
    I = torch.flip(torch.cumsum(torch.flip(B, [1]), 1), [1])[:, 1:]
    return I, _diff_penalty(I.shape[1])


def _gname(c):
    return "_".join(c) if isinstance(c, tuple) else c


# ---------------------------------------------------------------- estimator
class H2OGeneralizedAdditiveEstimator(H2OGeneralizedLinearEstimator):
    algo = "gam"
    _defaults = GAM_DEFAULTS

    def _smoothers(self):
        p = self._parms
        gc = p.get("gam_columns") or []
        gc = [c if isinstance(c, str) else (c[0] if len(c) == 1 else tuple(c)) for c in gc]
        m = len(gc)

        def per(name, default):
            v = p.get(name)
            if v is None:
                return [default] * m
            return list(v) if isinstance(v, (list, tuple)) else [v] * m
        return gc, per("bs", 0), per("num_knots", None), per("scale", 1.0), per("spline_orders", 2), \
            per("splines_non_negative", True)

    def _basis(self, frame, c, bs, knots, order, gi=None):
        if bs == 1:
            cc_ = c if isinstance(c, tuple) else (c,)
            cols = [torch.where(torch.isnan(v), torch.full_like(v, self._col_means[cc]), v)
                    for cc, v in ((cc, frame.vec(cc).as_float(torch.float64)) for cc in cc_)]
            t = self._tp[gi]
            return tp_ref_basis(torch.stack(cols, 1), knots, t, t["means"], t["ostd"], t["standardize"])
        x = frame.vec(c).as_float(torch.float64)
        x = torch.where(torch.isnan(x), torch.full_like(x, self._col_means[c]), x)
        if bs == 0:
            return cr_basis(x, knots)
        if bs == 2:
            return is_basis(x, knots, order)
        if bs == 3:
            return ms_basis(x, knots, order)
        raise ValueError(f"unknown bs={bs}")

    def _gam_frame(self, frame, fit=False):
        vecs, names = [], []
        flat = {cc for c in self._gam_cols for cc in (c if isinstance(c, tuple) else (c,))}
        for c in frame.names:
            if c in flat and not self._parms.get("keep_gam_cols"):
                continue
            vecs.append(frame.vec(c))
            names.append(c)
        for gi, c in enumerate(self._gam_cols):
            bs, knots, order = self._bs[gi], self._knots[gi], self._orders[gi]
            X, S = self._basis(frame, c, bs, knots, order, gi)
            if fit:
                w = torch.ones(X.shape[0], dtype=X.dtype, device=X.device)
                cs = (X * w.view(-1, 1)).sum(0)
                coll.allreduce_(cs)
                if bs in (2,):   # I-splines keep monotone coefficients: no centering (reference)
                    Z = np.eye(X.shape[1])
                else:
                    Q, _ = np.linalg.qr(cs.cpu().numpy().reshape(-1, 1), mode="complete")
                    Z = Q[:, 1:]
                # penalty normalisation of the reference (GenCSSplineGamOneColumn.postGlobal):
                # S *= max_row(sum|basis|)^2 / ||S||_inf, then centred, x scale, x2 in the Gram
                rs = X.abs().sum(1).max()
                rs = float(coll.allreduce_(rs.view(1).clone(), "max")[0])
                inf = float(np.abs(S).sum(1).max()) if S.size else 0.0
                if inf > 0 and (bs != 1 or self._parms.get("scale_tp_penalty_mat")):
                    S = S * (rs * rs / inf)   # thin plate: only with scale_tp_penalty_mat (GAM.java:560)
                self._Z.append(Z)
                self._S.append(2.0 * (Z.T @ S @ Z))
            Xc = X @ torch.as_tensor(self._Z[gi], dtype=X.dtype, device=X.device)
            suf = _SUFFIX[bs]
            for i in range(Xc.shape[1]):
                vecs.append(Vec(Xc[:, i].to(torch.float32).contiguous(), T_REAL))
                names.append(f"{_gname(c)}_{suf}_{i}")
        return H2OFrame.from_vecs(vecs, names)

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, **kw):
        p = self._parms
        gc, bs, nk, scale, orders, nonneg = self._smoothers()
        bs = [1 if isinstance(c, tuple) else b for c, b in zip(gc, bs)]   # several columns: thin plate only
        self._gam_cols, self._bs, self._orders = list(gc), [int(b) for b in bs], [int(o) for o in orders]
        self._knots, self._Z, self._S = [], [], []
        self._col_means = {}
        self._tp = {}
        kids = p.get("knot_ids")
        for gi, c in enumerate(gc):
            if isinstance(c, tuple):
                self._knots.append(self._tp_knots(training_frame, c, nk[gi]))
                self._tp[gi] = self._tp_setup(training_frame, c, self._knots[gi])
                continue
            v = training_frame.vec(c)
            xs = v.as_float(torch.float64)
            xs = xs[~torch.isnan(xs)]
            xs = coll.all_gather_var(xs)
            self._col_means[c] = float(xs.mean())
            if kids and kids[gi] is not None:
                kf = kids[gi] if not isinstance(kids[gi], str) else __import__("h2o3_amd").get_frame(kids[gi])
                knots = np.sort(kf.as_data_frame().iloc[:, 0].values.astype(float))
            else:
                k = nk[gi] if nk[gi] is not None else (10 if self._bs[gi] in (0, 1) else 6)
                qs = np.linspace(0, 1, int(k))
                knots = np.unique(np.quantile(xs.cpu().numpy(), qs))
            if self._bs[gi] == 1:
                knots = knots.reshape(-1, 1)
                self._knots.append(knots)
                self._tp[gi] = self._tp_setup(training_frame, (c,), knots)
                continue
            self._knots.append(knots)
        gfr = self._gam_frame(training_frame, fit=True)
        vfr = self._gam_frame(validation_frame) if validation_frame is not None else None
        flat = {cc for c in gc for cc in (c if isinstance(c, tuple) else (c,))}
        xs_ = [c for c in (x or [n for n in training_frame.names if n != y]) if c not in flat]
        gam_names = [n for n in gfr.names if any(n.startswith(f"{_gname(c)}_{_SUFFIX[b]}_")
                                                 for c, b in zip(gc, self._bs))]
        self._gam_penalty = []
        for gi, c in enumerate(gc):
            nm = [n for n in gam_names if n.startswith(f"{_gname(c)}_{_SUFFIX[self._bs[gi]]}_")]
            self._gam_penalty.append((nm, float(scale[gi]) * self._S[gi]))
        if any(nonneg[gi] for gi in range(len(gc)) if self._bs[gi] == 2):
            self._parms.setdefault("_nonneg_names", [n for gi, c in enumerate(gc) if self._bs[gi] == 2
                                                     for n in gam_names if n.startswith(f"{c}_is_")])
        keep = xs_ + (sorted(flat) if p.get("keep_gam_cols") else [])
        super().train(x=[c for c in keep if c in gfr.names] + gam_names, y=y, training_frame=gfr,
                      validation_frame=vfr, **kw)
        self._output["knots"] = [k.tolist() for k in self._knots]
        self._output["gam_columns"] = self._gam_cols
        return self

    def _tp_setup(self, frame, cols, knots):
        """Raw means / inverse standard deviations of the smoother's columns
        (GAM.java:519-526) and the thin-plate constants (tp_setup)."""
        means, ostd = [], []
        for cc in cols:
            v = frame.vec(cc).as_float(torch.float64)
            ok = ~torch.isnan(v)
            st = torch.stack([v[ok].sum(), (v[ok] ** 2).sum(), ok.sum().to(torch.float64)])
            coll.allreduce_(st)
            s1, s2, cnt = (float(t) for t in st)
            mu = s1 / max(cnt, 1.0)
            var = max(s2 - cnt * mu * mu, 0.0) / max(cnt - 1.0, 1.0)
            means.append(mu)
            ostd.append(1.0 / np.sqrt(var) if var > 0 else 1.0)
        std = bool(self._parms.get("standardize_tp_gam_cols"))
        t = tp_setup(knots, means, ostd, std)
        t.update(means=np.asarray(means), ostd=np.asarray(ostd), standardize=std)
        return t

    def _tp_knots(self, frame, cols, k):
        """Knots of a multi-column thin plate smoother: num_knots distinct data
        rows drawn with the model seed (GAM.java picks knot rows from the data)."""
        xs = []
        for cc in cols:
            v = frame.vec(cc).as_float(torch.float64)
            self._col_means[cc] = float(coll.allreduce_scalar(float(torch.nansum(v)))) / max(
                coll.allreduce_scalar(float((~torch.isnan(v)).sum())), 1)
            xs.append(coll.all_gather_var(torch.where(torch.isnan(v), torch.full_like(v, self._col_means[cc]), v)))
        Xa = torch.stack(xs, 1).cpu().numpy()
        uniq = np.unique(Xa, axis=0)
        d = len(cols)
        M = len(_poly_terms(d, _tp_m(d)))
        k = int(k) if k is not None else max(10, M + 2)
        k = max(k, M + 1)
        seed = self._parms.get("seed", -1)
        rng = np.random.RandomState(1234 if seed in (None, -1) else int(seed) & 0x7FFFFFFF)
        idx = rng.choice(len(uniq), size=min(k, len(uniq)), replace=False)
        return uniq[np.sort(idx)]

    def _predict_raw(self, frame):
        if any(n.startswith(tuple(f"{_gname(c)}_{_SUFFIX[b]}_" for c, b in zip(self._gam_cols, self._bs)))
               for n in frame.names):
            return super()._predict_raw(frame)
        return super()._predict_raw(self._gam_frame(frame))

    def _metrics_from_raw(self, spec, frame, raw, w=None, auc_type=None):
        return super()._metrics_from_raw(spec, frame, raw, w, auc_type=auc_type)

    def model_performance(self, test_data=None, **kw):
        if test_data is not None and not any("_cr_" in n or "_tp_" in n or "_is_" in n or "_ms_" in n
                                             for n in test_data.names):
            test_data = self._gam_frame(test_data)
        return super().model_performance(test_data, **kw)
