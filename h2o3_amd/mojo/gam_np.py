"""numpy evaluation of the GAM smoother bases for the standalone scorer.

Mirror of models/glm/gam.py (cr_basis / tp_basis / is_basis / ms_basis),
written against numpy only so a GAM MOJO scores without torch (reference:
hex/genmodel/algos/gam/GamMojoModel.java evaluates the same splines)."""
from __future__ import annotations

import numpy as np


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
    return np.vstack([np.zeros(k), F, np.zeros(k)])


def cr_basis(x, knots):
    kn = np.asarray(knots, dtype=np.float64)
    k = len(kn)
    Fp = _cr_matrices(kn)
    h = np.diff(kn)
    j = np.clip(np.searchsorted(kn, x, side="right") - 1, 0, k - 2)
    xl, xr, hj = kn[j], kn[j + 1], h[j]
    xc = np.clip(x, kn[0], kn[-1])
    am, ap = (xr - xc) / hj, (xc - xl) / hj
    cm = ((xr - xc) ** 3 / hj - hj * (xr - xc)) / 6
    cp = ((xc - xl) ** 3 / hj - hj * (xc - xl)) / 6
    X = cm[:, None] * Fp[j] + cp[:, None] * Fp[j + 1]
    r = np.arange(len(x))
    X[r, j] += am
    X[r, j + 1] += ap
    e = np.eye(k)
    d0 = (e[1] - e[0]) / h[0] - h[0] / 6 * Fp[1]
    d1 = (e[-1] - e[-2]) / h[-1] + h[-1] / 6 * Fp[-2]
    lo, hi = x < kn[0], x > kn[-1]
    X = np.where(lo[:, None], e[0] + (x - kn[0])[:, None] * d0, X)
    X = np.where(hi[:, None], e[-1] + (x - kn[-1])[:, None] * d1, X)
    return X


def tp_basis(x, knots):
    kn = np.asarray(knots, dtype=np.float64)
    k = len(kn)
    E = np.abs(x[:, None] - kn[None, :]) ** 3 / 12.0
    T = np.stack([np.ones(k), kn], 1)
    Q, _ = np.linalg.qr(T, mode="complete")
    return np.concatenate([E @ Q[:, 2:], x[:, None]], 1)


def _bspline(x, knots, order):
    t = np.concatenate([[knots[0]] * (order - 1), knots, [knots[-1]] * (order - 1)])
    xd = np.clip(x, knots[0], knots[-1])
    nb = len(t) - 1
    B = ((xd[:, None] >= t[:-1]) & (xd[:, None] < t[1:])).astype(np.float64)
    last = int(np.nonzero(t[:-1] < t[1:])[0][-1])
    B[:, last] = np.where(xd == t[-1], 1.0, B[:, last])
    for d in range(1, order):
        nbd = nb - d
        left = t[:nbd]
        den1 = t[d:d + nbd] - left
        den2 = t[d + 1:d + 1 + nbd] - t[1:1 + nbd]
        with np.errstate(divide="ignore", invalid="ignore"):
            a = np.where(den1 > 0, (xd[:, None] - left) / np.where(den1 > 0, den1, 1), 0.0)
            b = np.where(den2 > 0, (t[d + 1:d + 1 + nbd] - xd[:, None]) / np.where(den2 > 0, den2, 1), 0.0)
        B = a * B[:, :nbd] + b * B[:, 1:nbd + 1]
    return B


def basis(x, bs, knots, order):
    knots = np.asarray(knots, dtype=np.float64)
    if bs == 0:
        return cr_basis(x, knots)
    if bs == 1:
        return tp_basis(x, knots)
    if bs == 2:
        B = _bspline(x, knots, order + 1)
        return np.flip(np.cumsum(np.flip(B, 1), 1), 1)[:, 1:]
    if bs == 3:
        return _bspline(x, knots, order)
    raise ValueError(bs)


def tp_multi_basis(X, knots):
    """numpy twin of models/glm/gam.py:tp_multi_basis."""
    import itertools
    n, d = X.shape
    m = (d + 1) // 2 + 1
    terms = [e for e in itertools.product(range(m), repeat=d) if sum(e) < m]
    kn = np.asarray(knots, dtype=np.float64)
    Tk = np.stack([np.prod(kn ** np.asarray(e), 1) for e in terms], 1)
    Q, _ = np.linalg.qr(Tk, mode="complete")
    ZT = Q[:, len(terms):]
    r = np.sqrt(((X[:, None, :] - kn[None, :, :]) ** 2).sum(-1))
    p = 2 * m - d
    E = np.where(r > 0, r ** p * np.log(np.maximum(r, 1e-300)), 0.0) if d % 2 == 0 else r ** p
    poly = [np.prod(X ** np.asarray(e, dtype=np.float64), 1)[:, None] for e in terms if sum(e) > 0]
    return np.concatenate([E @ ZT] + poly, 1)
