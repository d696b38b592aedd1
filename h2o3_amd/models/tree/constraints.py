"""Monotone and interaction constraints of the tree builders.

Reference: hex/tree/Constraints.java (per-node [min, max] prediction
bounds; a split on a monotone column bounds its children at the midpoint of
their predictions, DTree.java:419 nextLevelConstraints, and leaf values are
predicted within the node's bounds, GBM.java:813 fitBestConstants with
useBounds), GBM.java:853 checkConstraints (every split on a monotone column
has max(left) <= min(right)); hex/tree/GlobalInteractionConstraints.java +
BranchInteractionConstraints.java (the features a branch may still split
on), TreeUtils.checkInteractionConstraints.

MI355X design.  The split search runs on the GPU over whole levels, so the
monotone bounds are enforced on the finished tree in one host pass over its
node arrays: subtree predictions are the den-weighted means of the leaf
values below (exactly the subtree's Newton / mean step), bounds travel down
with the reference's midpoint rule, and every leaf is clamped into its
node's bounds.  That is the reference's useBounds behaviour for the leaf
values, and it guarantees the model is monotone in each constrained column
(tests/test_tree_constraints.py checks it on a grid).  The split search
itself already rejects candidate splits whose child predictions break the
order (tree_split.hip / _find_splits_torch mono check), as DTree.java:1219
does.  Interaction constraints become a per-node feature mask (engine.py
_col_mask_allowed) intersected down the branch.
"""
from __future__ import annotations

import numpy as np

_MONO_FAMILIES = ("gaussian", "bernoulli", "tweedie", "quantile")


def check_monotone_family(family):
    if family not in _MONO_FAMILIES:
        raise ValueError("Monotone constraints are only supported for Gaussian, Bernoulli, Tweedie and Quantile "
                         f"distributions, your distribution: {family}.")


def monotone_vector(mc, x):
    """{column: +-1} (or a list of KeyValue-like pairs) -> [F] in {-1, 0, 1};
    unknown columns are an error (GBMModel.constraints)."""
    if not mc:
        return None
    if isinstance(mc, (list, tuple)):
        mc = {d["key"] if isinstance(d, dict) else d[0]: d["value"] if isinstance(d, dict) else d[1] for d in mc}
    for k in mc:
        if k not in x:
            raise ValueError(f"Invalid constraint specification, column '{k}' doesn't exist.")
    v = np.array([float(np.sign(float(mc.get(n, 0)))) for n in x])
    return v if np.any(v != 0) else None


def monotone_clamp(tree, leaves, vals, dens, mono):
    """Leaf values of `tree` (node ids `leaves`, values `vals`, per-leaf
    weights of the leaf step `dens`) clamped into the monotone bounds that
    Constraints.withNewConstraint would give each leaf."""
    mono = np.asarray(mono, dtype=np.float64)
    left = np.asarray(tree.left, dtype=np.int64)
    right = np.asarray(tree.right, dtype=np.int64)
    feat = np.asarray(tree.feat, dtype=np.int64)
    is_cat = np.asarray(tree.is_cat, dtype=bool)
    n = left.size
    leaves = np.asarray(leaves, dtype=np.int64)
    vals = np.asarray(vals, dtype=np.float64)
    d = np.maximum(np.asarray(dens, dtype=np.float64), 0.0)
    num = np.zeros(n)
    den = np.zeros(n)
    num[leaves] = vals * d
    den[leaves] = d
    for i in range(n - 1, -1, -1):          # BFS ids: children after parents
        if left[i] >= 0:
            num[i] = num[left[i]] + num[right[i]]
            den[i] = den[left[i]] + den[right[i]]
    val = np.where(den > 0, num / np.where(den > 0, den, 1.0), 0.0)
    lo = np.full(n, -np.inf)
    hi = np.full(n, np.inf)
    for i in range(n):
        l, r = left[i], right[i]
        if l < 0:
            continue
        lo[l] = lo[r] = lo[i]
        hi[l] = hi[r] = hi[i]
        c = 0.0 if is_cat[i] or feat[i] < 0 or feat[i] >= mono.size else mono[feat[i]]
        if c == 0:
            continue
        vl = min(max(val[l], lo[i]), hi[i])
        vr = min(max(val[r], lo[i]), hi[i])
        mid = 0.5 * (vl + vr)
        if c > 0:
            hi[l] = min(hi[i], mid)
            lo[r] = max(lo[i], mid)
        else:
            lo[l] = max(lo[i], mid)
            hi[r] = min(hi[i], mid)
    return np.clip(vals, lo[leaves], hi[leaves])


def check_monotone(tree, mono):
    """GBM.java checkConstraints: max(left subtree) <= min(right subtree) for
    every split on an increasing column (reverse for decreasing).  Raises."""
    left = np.asarray(tree.left, dtype=np.int64)
    right = np.asarray(tree.right, dtype=np.int64)
    feat = np.asarray(tree.feat, dtype=np.int64)
    v = np.asarray(tree.value, dtype=np.float64)
    n = left.size
    mn, mx = v.copy(), v.copy()
    for i in range(n - 1, -1, -1):
        if left[i] >= 0:
            mn[i] = min(mn[left[i]], mn[right[i]])
            mx[i] = max(mx[left[i]], mx[right[i]])
    for i in range(n):
        if left[i] < 0 or tree.is_cat[i] or feat[i] >= len(mono):
            continue
        c = mono[feat[i]]
        if c > 0 and np.float32(mx[left[i]]) > np.float32(mn[right[i]]):
            raise RuntimeError(f"Monotonicity constraint {c} violated at node {i} (max(left) > min(right))")
        if c < 0 and np.float32(mn[left[i]]) < np.float32(mx[right[i]]):
            raise RuntimeError(f"Monotonicity constraint {c} violated at node {i} (min(left) < max(right))")


def interaction_sets(ic, x, parms):
    """interaction_constraints [[col, ...], ...] -> list of sets of indices of
    `x` (GlobalInteractionConstraints; TreeUtils.checkInteractionConstraints
    errors)."""
    if not ic:
        return None
    if isinstance(ic, str):
        import json
        ic = json.loads(ic)
    ignored = set(parms.get("ignored_columns") or [])
    special = {"response_column": parms.get("response_column"), "weights_column": parms.get("weights_column"),
               "fold_column": parms.get("fold_column")}
    out = []
    for group in ic:
        s = set()
        for c in group:
            if c in ignored:
                raise ValueError(f"interaction_constraints: Column with the name '{c}' is set in ignored columns "
                                 "and cannot be used in interaction.")
            for what, col in special.items():
                if col is not None and c == col:
                    raise ValueError(f"interaction_constraints: Column with the name '{c}' is used as "
                                     f"{what.split('_')[0]} column and cannot be used in interaction.")
            if c not in x:
                raise ValueError(f"interaction_constraints: Invalid interaction constraint - there is no column "
                                 f"'{c}' in the training frame.")
            s.add(x.index(c))
        out.append(s)
    return out


def noise_factors(seed, k, ntrees_before, tree_no, nleaves, bw):
    """pred_noise_bandwidth (GBM.java:1460 AddTreeContributions): one
    N(1, bw) factor per (tree, class, leaf) scaling the leaf's contribution
    to the training predictions (the stored leaf value is unchanged)."""
    base = (0xDECAF + int(seed)) * (0xFAAAAAAB + k * int(ntrees_before) + int(tree_no))
    rs = np.random.RandomState(np.uint32(base & 0xFFFFFFFF))
    return 1.0 + rs.standard_normal(nleaves) * bw
