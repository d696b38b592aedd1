"""Every estimator end-to-end on the GPU (HIP path), checked for quality."""
import numpy as np
import pandas as pd
import pytest
import torch

import h2o3_amd
from h2o3_amd import estimators as E

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frame():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.RandomState(0)
    n = 20000
    X = rng.randn(n, 6)
    c = rng.choice(list("pqrs"), n)
    logit = 1.5 * X[:, 0] - X[:, 1] + (c == "q") * 1.0 + X[:, 2] * X[:, 3]
    y = (rng.rand(n) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(6)])
    df["cat"] = c
    df.loc[rng.rand(n) < 0.03, "x2"] = np.nan
    df["y"] = np.where(y == 1, "yes", "no")
    df["r"] = 2 * X[:, 0] + np.sin(X[:, 1]) + 0.1 * rng.randn(n)
    return h2o3_amd.H2OFrame(df)


X = [f"x{i}" for i in range(6)] + ["cat"]


@pytest.mark.parametrize("name,make,min_auc", [
    ("gbm", lambda: E.H2OGradientBoostingEstimator(ntrees=30, max_depth=5, seed=1), 0.85),
    ("drf", lambda: E.H2ORandomForestEstimator(ntrees=20, max_depth=12, seed=1), 0.8),
    ("xgb", lambda: E.H2OXGBoostEstimator(ntrees=30, max_depth=5, seed=1), 0.85),
    ("glm", lambda: E.H2OGeneralizedLinearEstimator(family="binomial"), 0.8),
    ("dl", lambda: E.H2ODeepLearningEstimator(hidden=[32, 32], epochs=5, seed=1), 0.8),
    ("nb", lambda: E.H2ONaiveBayesEstimator(), 0.75),
])
def test_binomial_gpu(frame, name, make, min_auc):
    m = make()
    m.train(x=X, y="y", training_frame=frame)
    assert m.auc() > min_auc, (name, m.auc())


def test_regression_gpu(frame):
    m = E.H2OGradientBoostingEstimator(ntrees=30, max_depth=5)
    m.train(x=X, y="r", training_frame=frame)
    assert m.r2() > 0.95
    g = E.H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0)
    g.train(x=X, y="r", training_frame=frame)
    assert g.r2() > 0.8


def test_unsupervised_gpu(frame):
    k = E.H2OKMeansEstimator(k=4, seed=1)
    k.train(x=X[:6], training_frame=frame)
    assert k.tot_withinss() < k.totss()
    p = E.H2OPrincipalComponentAnalysisEstimator(k=3, transform="STANDARDIZE")
    p.train(x=X[:6], training_frame=frame)
    assert p.predict(frame).ncols == 3
    i = E.H2OIsolationForestEstimator(ntrees=20, seed=1)
    i.train(x=X[:6], training_frame=frame)
    assert i.predict(frame).nrows == frame.nrows


def test_gram_kernel_matches_torch():
    from h2o3_amd.ops import linalg_ops
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn((100003, 96), generator=g, device="cuda")
    w = torch.rand(100003, generator=g, device="cuda")
    G = linalg_ops.weighted_gram(X, w)
    R = (X.double().T @ (X.double() * w.double().view(-1, 1)))
    torch.testing.assert_close(G, R, rtol=1e-5, atol=1e-3)


def test_native_libraries_loaded():
    from h2o3_amd.ops import _native
    names = " ".join(_native.loaded_libs())
    for lib in ("tree_hist", "tree_split", "tree_predict", "gram"):
        assert lib in names, (lib, names)


def test_multinomial_gbm_device_path_matches_host_path(frame, monkeypatch):
    """Multinomial GBM on the position-ordered path (device gamma, one host
    copy per iteration) grows the same trees as the per-row leaf-id path."""
    df = frame.as_data_frame()
    df["y3"] = np.where(df["x0"] > 0.5, "hi", np.where(df["x0"] < -0.5, "lo", "mid"))
    fr = h2o3_amd.H2OFrame(df)
    x = [f"x{i}" for i in range(6)] + ["cat"]
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("H2O3_POS_LEAF", flag)
        m = E.H2OGradientBoostingEstimator(ntrees=6, max_depth=4, seed=1)
        m.train(x=x, y="y3", training_frame=fr)
        out[flag] = (m, m.predict(fr).as_data_frame().iloc[:, 1:].values)
    (a, pa), (b, pb) = out["1"], out["0"]
    assert len(a._forest.trees) == len(b._forest.trees) == 18
    for t1, t2 in zip(a._forest.trees, b._forest.trees):
        assert list(np.asarray(t1.feat)) == list(np.asarray(t2.feat))
    np.testing.assert_allclose(pa, pb, atol=2e-4)
    assert abs(a.logloss() - b.logloss()) < 1e-4 and a.mean_per_class_error() < 0.01
