"""Path-dependent TreeSHAP for the standalone MOJO scorers (numpy only).

Reference: h2o-genmodel hex/genmodel/algos/tree/TreeSHAP.java (EXTEND /
UNWIND / UNWOUND-SUM over the unique feature path, node weights as the
background distribution), TreeSHAPEnsemble.java, and the contribution
predictors of GbmMojoModel / DrfMojoModel (ContributionsPredictor*).

The recursion runs over the TREE NODES once for all rows: every element of
the feature path holds per-row vectors (one-fractions, path weights), the
hot / cold branches of the reference's per-row recursion become the 0/1
one-fraction of "this row goes this way", so one pass over a tree's nodes
scores the whole frame (models/tree/shap.py is the device version of the
same scheme for in-platform models).

A tree is given as flat node arrays: `left[j]`, `right[j]` (child node ids,
-1 for a leaf), `cover[j]` (training weight through node j), `value[j]`
(leaf value), `feat[j]` (split column) and a callable `go_left(j) -> bool
[n]` deciding the split for every row.
"""
from __future__ import annotations

import numpy as np


class _Path:
    __slots__ = ("d", "z", "o", "w")

    def __init__(self, d, z, o, w):
        self.d, self.z, self.o, self.w = d, z, o, w


def _extend(m, pz, po, pi, ones):
    depth = len(m)
    m.append(_Path(pi, pz, po, ones.copy() if depth == 0 else np.zeros_like(ones)))
    for i in range(depth - 1, -1, -1):
        m[i + 1].w = m[i + 1].w + po * m[i].w * ((i + 1) / (depth + 1))
        m[i].w = pz * m[i].w * ((depth - i) / (depth + 1))


def _nz(v):
    return np.where(v == 0, 1.0, v)


def _unwound_sum(m, k):
    depth = len(m) - 1
    one, zero = m[k].o, m[k].z
    nxt = m[depth].w
    total = np.zeros_like(nxt)
    nz = one != 0
    for i in range(depth - 1, -1, -1):
        tmp = nxt * (depth + 1) / ((i + 1) * _nz(one))
        t_zero = (m[i].w / zero) / ((depth - i) / (depth + 1)) if zero != 0 else np.zeros_like(tmp)
        total = total + np.where(nz, tmp, t_zero)
        nxt = np.where(nz, m[i].w - tmp * zero * ((depth - i) / (depth + 1)), nxt)
    return total


def _unwind(m, k):
    depth = len(m) - 1
    one, zero = m[k].o, m[k].z
    nxt = m[depth].w
    nz = one != 0
    for i in range(depth - 1, -1, -1):
        tmp = m[i].w
        w_one = nxt * (depth + 1) / ((i + 1) * _nz(one))
        w_zero = (tmp * (depth + 1) / (zero * (depth - i))) if zero != 0 else np.zeros_like(tmp)
        m[i].w = np.where(nz, w_one, w_zero)
        nxt = np.where(nz, tmp - m[i].w * zero * ((depth - i) / (depth + 1)), nxt)
    for i in range(k, depth):
        m[i].d, m[i].z, m[i].o = m[i + 1].d, m[i + 1].z, m[i + 1].o
    m.pop()


def tree_shap(left, right, cover, value, feat, go_left, n, phi, scale=1.0, root=0):
    """Adds one tree's contributions (times `scale`) into phi [n, F + 1]
    (last column = bias: the cover-weighted mean leaf value)."""
    ones = np.ones(n)
    cov = np.maximum(np.asarray(cover, dtype=np.float64), 0.0)
    rc = cov[root] if cov[root] > 0 else 1.0
    # bias: cover-weighted mean leaf value (iterative walk)
    bias = 0.0
    stack = [root]
    while stack:
        j = stack.pop()
        if left[j] < 0:
            bias += float(value[j]) * cov[j] / rc
        else:
            stack += [int(left[j]), int(right[j])]
    phi[:, -1] += scale * bias

    def rec(j, m, pz, po, pi):
        m = [_Path(e.d, e.z, e.o, e.w) for e in m]
        _extend(m, pz, po, pi, ones)
        if left[j] < 0:
            v = scale * float(value[j])
            for i in range(1, len(m)):
                phi[:, m[i].d] += _unwound_sum(m, i) * (m[i].o - m[i].z) * v
            return
        gl = go_left(j).astype(np.float64)
        cj = cov[j] if cov[j] > 0 else 1.0
        iz, io = 1.0, ones
        d = int(feat[j])
        for k in range(1, len(m)):
            if m[k].d == d:
                iz, io = m[k].z, m[k].o
                _unwind(m, k)
                break
        lj, rj = int(left[j]), int(right[j])
        rec(lj, m, cov[lj] / cj * iz, io * gl, d)
        rec(rj, m, cov[rj] / cj * iz, io * (1.0 - gl), d)

    rec(root, [], 1.0, ones, -1)


def contributions_frame(phi, names, top_n=None, bottom_n=None, compare_abs=False):
    """pandas frame of the reference's contribution output: one column per
    feature + BiasTerm, or the sorted top_feature_i / top_value_i (+ bottom)
    layout when top_n / bottom_n is given (-1 = all)."""
    import pandas as pd
    F = phi.shape[1] - 1
    if top_n is None and bottom_n is None:
        return pd.DataFrame({**{c: phi[:, j].astype(np.float32) for j, c in enumerate(names)},
                             "BiasTerm": phi[:, -1].astype(np.float32)})
    c = phi[:, :-1]
    key = np.abs(c) if compare_abs else c
    order = np.argsort(-key, axis=1, kind="stable")
    tn = F if (top_n is not None and top_n < 0) else (top_n or 0)
    bn = F if (bottom_n is not None and bottom_n < 0) else (bottom_n or 0)
    ar = np.arange(phi.shape[0])
    out = {}
    for i in range(min(tn, F)):
        j = order[:, i]
        out[f"top_feature_{i + 1}"] = [names[k] for k in j]
        out[f"top_value_{i + 1}"] = c[ar, j].astype(np.float32)
    for i in range(min(bn, F)):
        j = order[:, F - 1 - i]
        out[f"bottom_feature_{i + 1}"] = [names[k] for k in j]
        out[f"bottom_value_{i + 1}"] = c[ar, j].astype(np.float32)
    out["BiasTerm"] = phi[:, -1].astype(np.float32)
    return pd.DataFrame(out)
