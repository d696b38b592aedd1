"""Per-node NA direction (DTree.java:1475-1478): when NO row reaching a node
has an NA in the split column (nasplit == None), NAs of later data follow the
heavier child -- decided per node, not by whether the column had NAs
anywhere in training."""
import numpy as np
import pandas as pd
import pytest

import h2o3_amd
from h2o3_amd.estimators import H2OGradientBoostingEstimator, H2ORandomForestEstimator


def _rows_at_nodes(tree, X):
    """Training rows reaching every node (host traversal, x < thr left)."""
    at = {0: np.arange(X.shape[0])}
    out = {}
    stack = [0]
    while stack:
        i = stack.pop()
        rows = at[i]
        out[i] = rows
        if tree.left[i] < 0:
            continue
        x = X[rows, tree.feat[i]]
        nan = np.isnan(x)
        go_l = np.where(nan, bool(tree.na_left[i]), x < tree.thr[i])
        at[tree.left[i]], at[tree.right[i]] = rows[go_l], rows[~go_l]
        stack += [tree.left[i], tree.right[i]]
    return out


@pytest.mark.parametrize("algo", ["gbm", "drf"])
def test_na_direction_decided_per_node(algo):
    h2o3_amd.init(verbose=False)
    rng = np.random.RandomState(11)
    n = 6000
    x1 = rng.randn(n)
    x0 = rng.randn(n)
    # x0 has NAs only where x1 > 0.5: nodes on the x1 <= 0.5 side see none
    x0[(x1 > 0.5) & (rng.rand(n) < 0.3)] = np.nan
    y = np.where(np.nan_to_num(x0) * 1.5 + (x1 > 0.5) * 2.0 + 0.3 * rng.randn(n) > 0.6, "a", "b")
    df = pd.DataFrame({"x0": x0, "x1": x1, "y": y})
    fr = h2o3_amd.H2OFrame(df)
    m = (H2OGradientBoostingEstimator(ntrees=5, max_depth=4, seed=1) if algo == "gbm" else
         H2ORandomForestEstimator(ntrees=5, max_depth=4, seed=1, mtries=2, sample_rate=1.0))
    m.train(x=["x0", "x1"], y="y", training_frame=fr)
    X = np.stack([x0, x1], 1)
    checked = 0
    for tree in m._forest.trees:
        rows = _rows_at_nodes(tree, X)
        for i in range(tree.n_nodes):
            if tree.left[i] < 0 or tree.feat[i] != 0 or tree.is_cat[i] or not np.isfinite(tree.thr[i]):
                continue
            if np.isnan(X[rows[i], 0]).any():
                continue
            wl, wr = float(tree.weight[tree.left[i]]), float(tree.weight[tree.right[i]])
            assert bool(tree.na_left[i]) == (wl > wr), (i, wl, wr, tree.na_left[i])
            checked += 1
    assert checked > 0


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["gbm", "drf"])
def test_na_direction_decided_per_node_gpu(algo):
    """Same rule on the GPU paths (device-resident GBM tree: the node's NA
    weight on the winning column comes back in its split record)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    test_na_direction_decided_per_node(algo)
