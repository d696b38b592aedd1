"""numpy evaluation of the GAM smoother bases for the standalone scorer.

Mirror of models/glm/gam.py (cr_basis / tp_ref_basis / is_basis / ms_basis),
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
    """GamUtilsCubicRegression.expandOneGamCol (cubic continued outside the knots)."""
    kn = np.asarray(knots, dtype=np.float64)
    k = len(kn)
    Fp = _cr_matrices(kn)
    h = np.diff(kn)
    j = np.clip(np.searchsorted(kn, x, side="right") - 1, 0, k - 2)
    xl, xr, hj = kn[j], kn[j + 1], h[j]
    am, ap = (xr - x) / hj, (x - xl) / hj
    cm = ((xr - x) ** 3 / hj - hj * (xr - x)) / 6
    cp = ((x - xl) ** 3 / hj - hj * (x - xl)) / 6
    X = cm[:, None] * Fp[j] + cp[:, None] * Fp[j + 1]
    r = np.arange(len(x))
    X[r, j] += am
    X[r, j + 1] += ap
    return X


def tp_constant(m, d):
    from math import factorial, pi
    if d % 2 == 0:
        return (-1) ** (m + 1 + d // 2) / (2 ** (2 * m - 1) * pi ** (d / 2.0) * factorial(m - 1) *
                                           factorial(m - d // 2))
    return (-1) ** m * m / (factorial(2 * m) * pi ** ((d - 1) / 2.0))


def tp_basis(X, knots, zcs, terms, means, ostd, standardize):
    """Thin plate with knots: c r^(2m-d) [log] distances on zCS, then the
    polynomial terms (numpy twin of models/glm/gam.py:tp_ref_basis)."""
    kn = np.asarray(knots, dtype=np.float64).reshape(len(knots), -1)
    X = np.asarray(X, dtype=np.float64).reshape(X.shape[0], -1)
    d = kn.shape[1]
    m = (d + 1) // 2 + 1
    diff = X[:, None, :] - kn[None, :, :]
    if standardize:
        diff = diff * np.asarray(ostd)
    dist = np.sqrt((diff * diff).sum(-1)) ** (2 * m - d)
    E = tp_constant(m, d) * dist
    if d % 2 == 0:
        E = np.where(dist != 0, E * np.log(np.where(dist != 0, dist, 1.0)), E)
    Xp = X - np.asarray(means) * np.asarray(ostd) if standardize else X
    poly = np.stack([np.prod(Xp ** np.asarray(e, dtype=np.float64), 1) for e in terms], 1)
    return np.concatenate([E @ np.asarray(zcs), poly], 1)


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
    if bs == 2:
        B = _bspline(x, knots, order + 1)
        return np.flip(np.cumsum(np.flip(B, 1), 1), 1)[:, 1:]
    if bs == 3:
        return _bspline(x, knots, order)
    raise ValueError(bs)


# ----------------------------------------------------------- reference I-splines
def _fill_knots(knots, m):
    """GamUtilsISplines.fillKnots: m-1 copies of each boundary knot added."""
    kn = list(np.asarray(knots, dtype=np.float64))
    up = max(m - 1, 0)
    return np.asarray([kn[0]] * up + kn + [kn[-1]] * up)


def _bspline_eval(x, t, i, order):
    """NBSplinesTypeII.BSplineBasis.evaluate of basis i of `order` over the
    filled knot sequence t (half-open support, 0 outside)."""
    kn = t[i:i + order + 1]
    inside = (x >= kn[0]) & (x < kn[-1])
    if order == 1:
        return inside.astype(np.float64)
    d0 = kn[order - 1] - kn[0]
    d1 = kn[order] - kn[1]
    a = (x - kn[0]) * (1.0 / d0 if d0 != 0 else 0.0) * _bspline_eval(x, t, i, order - 1)
    b = (kn[order] - x) * (1.0 / d1 if d1 != 0 else 0.0) * _bspline_eval(x, t, i + 1, order - 1)
    return np.where(inside, a + b, 0.0)


def ispline_basis(x, knots, order):
    """ISplines.gamifyVal for every value: basis j is 0 below its first knot,
    1 from its (order)-th knot on, else the sum of the order+1 B-splines from
    index j+1 (sumNBSpline)."""
    x = np.asarray(x, dtype=np.float64)
    kn = np.asarray(knots, dtype=np.float64)
    nI = len(kn) + order - 2
    tI = _fill_knots(kn, order)
    tB = _fill_knots(kn, order + 1)
    nB = len(kn) + order + 1 - 2
    Bv = [_bspline_eval(x, tB, b, order + 1) for b in range(nB)]
    out = np.zeros((x.shape[0], nI))
    for j in range(nI):
        ik = tI[j:j + order + 1]
        acc = np.zeros_like(x)
        live = np.ones(x.shape[0], dtype=bool)
        for b in range(j + 1, nB):
            bk = tB[b:b + order + 2]
            live &= ~(x < bk[0])
            acc += np.where(live, np.where(x >= bk[-1], 1.0, Bv[b]), 0.0)
        out[:, j] = np.where(x < ik[0], 0.0, np.where(x >= ik[order], 1.0, acc))
    return out
