"""TreeSHAP contributions: additivity + exact Shapley values on small trees."""
import itertools
import math

import numpy as np
import pandas as pd
import torch

import h2o3_amd as h2o
from h2o3_amd.estimators import (H2OGradientBoostingEstimator, H2ORandomForestEstimator,
                                 H2OXGBoostEstimator)
from h2o3_amd.models.tree.shap import _go_left, forest_contributions


def _df(n=600, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4))
    X[rng.random(n) < 0.05, 2] = np.nan
    df = pd.DataFrame(X, columns=list("abcd"))
    df["k"] = rng.choice(["u", "v", "w"], n)
    df["y"] = 2 * X[:, 0] - X[:, 1] * (df["k"] == "u") + np.nan_to_num(X[:, 2]) + rng.normal(scale=0.2, size=n)
    df["yb"] = np.where(df["y"] > 0, "p", "n")
    return df


def _cond_exp(tree, X, j, S):
    if tree.left[j] < 0:
        return tree.value[j]
    if tree.feat[j] in S:
        gl = bool(_go_left(tree, j, X)[0])
        return _cond_exp(tree, X, tree.left[j] if gl else tree.right[j], S)
    cl, cr = tree.weight[tree.left[j]], tree.weight[tree.right[j]]
    return (cl * _cond_exp(tree, X, tree.left[j], S) + cr * _cond_exp(tree, X, tree.right[j], S)) / (cl + cr)


def _exact_shap(tree, X, F):
    phi = np.zeros(F)
    for i in range(F):
        others = [f for f in range(F) if f != i]
        for r in range(len(others) + 1):
            for S in itertools.combinations(others, r):
                wgt = math.factorial(len(S)) * math.factorial(F - len(S) - 1) / math.factorial(F)
                phi[i] += wgt * (_cond_exp(tree, X, 0, set(S) | {i}) - _cond_exp(tree, X, 0, set(S)))
    return phi


def test_tree_shap_matches_exact_shapley():
    h2o.init()
    fr = h2o.H2OFrame(_df())
    m = H2OGradientBoostingEstimator(ntrees=3, max_depth=4, seed=1, min_rows=5)
    m.train(x=list("abcd") + ["k"], y="y", training_frame=fr)
    X = m._score_matrix(fr)
    F = X.shape[0]
    for t in m._forest.trees[:2]:
        for r in (0, 5, 17):
            xr = X[:, r:r + 1]
            phi = forest_contributions([t], xr, F)[0].cpu().numpy()
            ex = _exact_shap(t, xr, F)
            np.testing.assert_allclose(phi[:-1], ex, atol=1e-6)


def test_contributions_sum_to_margin_gbm_regression_and_binomial():
    h2o.init()
    fr = h2o.H2OFrame(_df())
    x = list("abcd") + ["k"]
    m = H2OGradientBoostingEstimator(ntrees=10, max_depth=5, seed=1)
    m.train(x=x, y="y", training_frame=fr)
    c = m.predict_contributions(fr).as_data_frame()
    p = m.predict(fr).as_data_frame()["predict"].values
    np.testing.assert_allclose(c.sum(1).values, p, rtol=1e-4, atol=1e-4)
    assert list(c.columns) == x + ["BiasTerm"]
    mb = H2OGradientBoostingEstimator(ntrees=10, max_depth=4, seed=1)
    mb.train(x=x, y="yb", training_frame=fr)
    cb = mb.predict_contributions(fr).as_data_frame()
    pb = mb.predict(fr).as_data_frame()["p"].values
    margin = np.log(pb / (1 - pb))
    np.testing.assert_allclose(cb.sum(1).values, margin, rtol=1e-3, atol=1e-3)
    top = mb.predict_contributions(fr, top_n=2, bottom_n=1).as_data_frame()
    assert list(top.columns) == ["top_feature_1", "top_value_1", "top_feature_2", "top_value_2",
                                 "bottom_feature_1", "bottom_value_1", "BiasTerm"]


def test_contributions_drf_xgboost():
    h2o.init()
    fr = h2o.H2OFrame(_df())
    x = list("abcd") + ["k"]
    d = H2ORandomForestEstimator(ntrees=5, max_depth=5, seed=2)
    d.train(x=x, y="y", training_frame=fr)
    c = d.predict_contributions(fr).as_data_frame()
    p = d.predict(fr).as_data_frame()["predict"].values
    np.testing.assert_allclose(c.sum(1).values, p, rtol=1e-4, atol=1e-4)
    xg = H2OXGBoostEstimator(ntrees=5, max_depth=4, seed=2)
    xg.train(x=x, y="y", training_frame=fr)
    c = xg.predict_contributions(fr).as_data_frame()
    p = xg.predict(fr).as_data_frame()["predict"].values
    np.testing.assert_allclose(c.sum(1).values, p, rtol=1e-4, atol=1e-4)
