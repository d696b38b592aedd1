import numpy as np
import pandas as pd
import pytest

import h2o3_amd
from h2o3_amd.estimators import H2OGradientBoostingEstimator


def _binary_frame(n=4000, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, 5)
    cat = rng.choice(["a", "b", "c", "d"], n)
    logit = X[:, 0] * 1.5 - X[:, 1] + (cat == "b") * 2
    y = (rng.rand(n) < 1 / (1 + np.exp(-logit))).astype(int)
    X[rng.rand(n) < 0.1, 3] = np.nan
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(5)])
    df["cat"] = cat
    df["y"] = np.where(y == 1, "yes", "no")
    return h2o3_amd.H2OFrame(df)


def test_gbm_binomial_trains_and_predicts():
    fr = _binary_frame()
    m = H2OGradientBoostingEstimator(ntrees=20, max_depth=4, seed=1)
    m.train(y="y", training_frame=fr)
    assert m.auc() > 0.85
    p = m.predict(fr)
    assert p.names == ["predict", "no", "yes"]
    vi = dict((k, v) for k, v, _, _ in m.varimp())
    assert vi["x0"] > vi["x4"]
    assert vi["cat"] > vi["x4"]


def test_gbm_regression_and_training_scoring_consistent():
    rng = np.random.RandomState(2)
    X = rng.randn(3000, 3)
    df = pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2], "y": X[:, 0] * 2 + np.sin(X[:, 1])})
    fr = h2o3_amd.H2OFrame(df)
    m = H2OGradientBoostingEstimator(ntrees=40, max_depth=4)
    m.train(y="y", training_frame=fr)
    assert m.r2() > 0.9
    Xs = m._score_matrix(fr)
    f_score = m._forest.predict(Xs, 1)[:, 0] + m._init_f[0]
    np.testing.assert_allclose(m._train_f[:, 0].cpu().numpy(), f_score.cpu().numpy(), rtol=1e-4, atol=1e-4)


def test_gbm_multinomial():
    rng = np.random.RandomState(3)
    X = rng.randn(3000, 4)
    cls = np.argmax(X[:, :3] + 0.3 * rng.randn(3000, 3), 1)
    df = pd.DataFrame(X, columns=list("abcd"))
    df["y"] = np.array(["r", "g", "b"])[cls]
    fr = h2o3_amd.H2OFrame(df)
    m = H2OGradientBoostingEstimator(ntrees=15, max_depth=3)
    m.train(y="y", training_frame=fr)
    assert m.logloss() < 0.7
    p = m.predict(fr)
    assert p.ncols == 4


@pytest.mark.parametrize("dist", ["poisson", "gamma", "tweedie", "laplace", "quantile", "huber"])
def test_gbm_distributions(dist):
    rng = np.random.RandomState(4)
    X = rng.rand(2000, 3)
    mu = np.exp(X[:, 0] + 0.5 * X[:, 1])
    y = rng.poisson(mu) + (0.5 if dist == "gamma" else 0)
    fr = h2o3_amd.H2OFrame(pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2], "y": y.astype(float)}))
    m = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, distribution=dist)
    m.train(y="y", training_frame=fr)
    pred = m.predict(fr).as_data_frame()["predict"].values
    assert np.isfinite(pred).all()
    assert np.corrcoef(pred, mu)[0, 1] > 0.5


def test_gbm_cv_and_early_stopping():
    fr = _binary_frame(3000, seed=5)
    m = H2OGradientBoostingEstimator(ntrees=200, max_depth=3, nfolds=3, stopping_rounds=3, seed=7,
                                     score_tree_interval=5)
    m.train(y="y", training_frame=fr)
    assert m.auc(xval=True) > 0.8
    assert len(m.cross_validation_models()) == 3
    assert len(m._forest) < 200
