"""TreeSHAP feature contributions (predict_contributions).

Reference: hex/tree/SharedTreeModelWithContributions.java and
hex/genmodel/algos/tree/TreeSHAP.java (path-dependent TreeSHAP of Lundberg
et al., "Consistent Individualized Feature Attribution for Tree
Ensembles", Algorithm 2: EXTEND / UNWIND / UNWOUND-SUM over the unique
feature path, node covers as the background distribution).

MI355X design: the recursion is over TREE NODES only (a few hundred per
tree); every path element carries per-ROW tensors (one-fractions and path
weights), so each EXTEND / UNWIND step is a handful of elementwise kernels
over all rows at once instead of a per-row recursion.  Both children are
visited with one-fraction = "row goes this way" (0/1 per row), which is
the vectorised form of the reference's hot/cold recursion.
"""
from __future__ import annotations

import torch

from .engine import Tree


def _go_left(tree: Tree, j: int, X: torch.Tensor) -> torch.Tensor:
    x = X[tree.feat[j]]
    isn = torch.isnan(x)
    if tree.is_cat[j] and tree.cat_left[j] is not None:
        mask = torch.as_tensor(tree.cat_left[j], dtype=torch.bool, device=X.device)
        code = torch.nan_to_num(x, nan=-1).long()
        inr = (code >= 0) & (code < mask.numel())
        bit = mask[code.clamp(0, max(mask.numel() - 1, 0))]
        return torch.where(isn | ~inr, torch.full_like(isn, bool(tree.na_left[j])), bit)
    # split points are stored / compared in f32 like the scoring kernel
    thr = torch.tensor(float(tree.thr[j]), dtype=torch.float32, device=X.device)
    return torch.where(isn, torch.full_like(isn, bool(tree.na_left[j])), x.to(torch.float32) < thr)


class _El:
    __slots__ = ("d", "z", "o", "w")

    def __init__(self, d, z, o, w):
        self.d, self.z, self.o, self.w = d, z, o, w

    def copy(self):
        return _El(self.d, self.z, self.o, self.w)


def _extend(m, pz, po, pi, ones):
    depth = len(m)
    m.append(_El(pi, pz, po, ones.clone() if depth == 0 else torch.zeros_like(ones)))
    for i in range(depth - 1, -1, -1):
        m[i + 1].w = m[i + 1].w + po * m[i].w * ((i + 1) / (depth + 1))
        m[i].w = pz * m[i].w * ((depth - i) / (depth + 1))


def _safe(v):
    return torch.where(v == 0, torch.ones_like(v), v)


def _unwound_sum(m, k):
    depth = len(m) - 1
    one, zero = m[k].o, m[k].z
    nxt = m[depth].w
    total = torch.zeros_like(nxt)
    nz = one != 0
    for i in range(depth - 1, -1, -1):
        tmp = nxt * (depth + 1) / ((i + 1) * _safe(one))
        t_zero = (m[i].w / zero) / ((depth - i) / (depth + 1)) if zero != 0 else torch.zeros_like(tmp)
        total = total + torch.where(nz, tmp, t_zero)
        nxt = torch.where(nz, m[i].w - tmp * zero * ((depth - i) / (depth + 1)), nxt)
    return total


def tree_shap(tree: Tree, X: torch.Tensor, phi: torch.Tensor, scale: float = 1.0):
    """Adds one tree's contributions into phi [N, F+1] (last column = bias)."""
    N = X.shape[1]
    ones = torch.ones(N, dtype=torch.float64, device=X.device)
    cover = [max(float(c), 0.0) for c in tree.weight]
    root = cover[0] if cover[0] > 0 else 1.0
    # bias: cover-weighted mean leaf value
    bias = 0.0
    for j in tree.leaves():
        bias += tree.value[j] * cover[j] / root
    phi[:, -1] += scale * bias

    def rec(j, m, pz, po, pi):
        m = [e.copy() for e in m]
        _extend(m, pz, po, pi, ones)
        if tree.left[j] < 0:
            v = scale * float(tree.value[j])
            for i in range(1, len(m)):
                w = _unwound_sum(m, i)
                phi[:, m[i].d] += w * (m[i].o - m[i].z) * v
            return
        gl = _go_left(tree, j, X).to(torch.float64)
        cj = cover[j] if cover[j] > 0 else 1.0
        iz, io = 1.0, ones
        d = tree.feat[j]
        for k in range(1, len(m)):
            if m[k].d == d:
                iz, io = m[k].z, m[k].o
                _unwind_full(m, k)
                break
        rec(tree.left[j], m, cover[tree.left[j]] / cj * iz, io * gl, d)
        rec(tree.right[j], m, cover[tree.right[j]] / cj * iz, io * (1 - gl), d)

    rec(0, [], 1.0, ones, -1)


def _unwind_full(m, k):
    """UNWIND exactly as the reference: recompute weights, shift d/z/o down."""
    depth = len(m) - 1
    one, zero = m[k].o, m[k].z
    nxt = m[depth].w
    nz = one != 0
    for i in range(depth - 1, -1, -1):
        tmp = m[i].w
        w_one = nxt * (depth + 1) / ((i + 1) * _safe(one))
        w_zero = (tmp * (depth + 1) / (zero * (depth - i))) if zero != 0 else torch.zeros_like(tmp)
        m[i].w = torch.where(nz, w_one, w_zero)
        nxt = torch.where(nz, tmp - m[i].w * zero * ((depth - i) / (depth + 1)), nxt)
    for i in range(k, depth):
        m[i].d, m[i].z, m[i].o = m[i + 1].d, m[i + 1].z, m[i + 1].o
    m.pop()


def forest_contributions(trees, X: torch.Tensor, F: int, scale: float = 1.0) -> torch.Tensor:
    """Sum of TreeSHAP contributions over `trees`; returns [N, F+1] float64."""
    phi = torch.zeros((X.shape[1], F + 1), dtype=torch.float64, device=X.device)
    for t in trees:
        tree_shap(t, X, phi, scale)
    return phi


def tree_contributions(model, frame, top_n=None, bottom_n=None, compare_abs=False):
    """predict_contributions for GBM / XGBoost / DRF (regression + binomial),
    in link space like the reference: row sum == raw margin prediction."""
    from ...core.frame import H2OFrame
    from ...core.vec import Vec, T_REAL, make_enum_from_strings
    spec = model._spec
    if spec.nclasses > 2:
        raise ValueError("Calculating contributions is currently not supported for multinomial models.")
    X = model._score_matrix(frame)
    names = list(spec.x)
    trees = [t for t, k in zip(model._forest.trees, model._forest.tclass) if k == 0]
    if model.algo == "drf":
        phi = forest_contributions(trees, X, len(names), scale=1.0 / max(1, len(trees)))
        if spec.nclasses == 2:
            # the reference's binomial DRF form (ScoreContributionsTaskDRF,
            # DRFModel.java:97-106: its trees score P(class 0)): 1/(F+1) -
            # contribution to P0 per column, which still sums to P(class 1)
            r = 1.0 / (len(names) + 1)
            phi[:, :-1] += r
            phi[:, -1] += r - 1.0
    else:
        phi = forest_contributions(trees, X, len(names))
        phi[:, -1] += float(model._init_f[0])
    if top_n is None and bottom_n is None:
        vecs = [Vec(phi[:, j].to(torch.float32).contiguous(), T_REAL) for j in range(phi.shape[1])]
        return H2OFrame.from_vecs(vecs, names + ["BiasTerm"])
    # sorted output: top_feature_i / top_value_i (+ bottom_*), BiasTerm last
    c = phi[:, :-1]
    key = c.abs() if compare_abs else c
    order = torch.argsort(key, dim=1, descending=True).cpu().numpy()
    cn = c.cpu().numpy()
    cols, out_names = [], []
    F = c.shape[1]
    tn = F if top_n is not None and top_n < 0 else (top_n or 0)
    bn = F if bottom_n is not None and bottom_n < 0 else (bottom_n or 0)
    import numpy as np
    for i in range(min(tn, F)):
        j = order[:, i]
        cols.append(make_enum_from_strings([names[k] for k in j]))
        cols.append(Vec(torch.tensor(cn[np.arange(len(j)), j], dtype=torch.float32, device=X.device), T_REAL))
        out_names += [f"top_feature_{i + 1}", f"top_value_{i + 1}"]
    for i in range(min(bn, F)):
        j = order[:, F - 1 - i]
        cols.append(make_enum_from_strings([names[k] for k in j]))
        cols.append(Vec(torch.tensor(cn[np.arange(len(j)), j], dtype=torch.float32, device=X.device), T_REAL))
        out_names += [f"bottom_feature_{i + 1}", f"bottom_value_{i + 1}"]
    cols.append(Vec(phi[:, -1].to(torch.float32).contiguous(), T_REAL))
    out_names.append("BiasTerm")
    return H2OFrame.from_vecs(cols, out_names)
