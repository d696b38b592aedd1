import numpy as np
import pandas as pd
import pytest

import h2o3_amd
from h2o3_amd.estimators import (H2OKMeansEstimator, H2ONaiveBayesEstimator, H2OPrincipalComponentAnalysisEstimator,
                                 H2OSingularValueDecompositionEstimator)


def test_kmeans_recovers_clusters():
    rng = np.random.RandomState(0)
    cs = np.array([[0, 0], [10, 10], [-10, 10]])
    X = np.concatenate([c + rng.randn(300, 2) for c in cs])
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=["a", "b"]))
    m = H2OKMeansEstimator(k=3, standardize=False, seed=1)
    m.train(training_frame=fr)
    got = np.array(sorted(map(tuple, np.round(m.centers()))))
    assert np.allclose(got, np.array(sorted(map(tuple, cs))), atol=0.5)
    assert m.tot_withinss() < m.totss() * 0.05
    assert m.predict(fr).nrows == 900


def test_pca_matches_numpy():
    rng = np.random.RandomState(1)
    X = rng.randn(500, 4) @ rng.randn(4, 4)
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=list("abcd")))
    m = H2OPrincipalComponentAnalysisEstimator(k=2, transform="DEMEAN")
    m.train(training_frame=fr)
    ev = np.linalg.eigvalsh(np.cov(X.T))[::-1]
    np.testing.assert_allclose(np.array(m._output["std_deviation"]) ** 2, ev[:2], rtol=1e-4)
    assert m.predict(fr).ncols == 2


def test_svd():
    rng = np.random.RandomState(2)
    X = rng.randn(300, 3)
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=list("abc")))
    m = H2OSingularValueDecompositionEstimator(nv=3)
    m.train(training_frame=fr)
    s = np.linalg.svd(X, compute_uv=False)
    np.testing.assert_allclose(m.d(), s, rtol=1e-4)


def test_naive_bayes():
    rng = np.random.RandomState(3)
    n = 2000
    y = rng.randint(0, 2, n)
    x1 = rng.randn(n) + 2 * y
    c = np.where(rng.rand(n) < 0.8, np.where(y == 1, "p", "q"), "r")
    df = pd.DataFrame({"x1": x1, "c": c, "y": np.where(y == 1, "yes", "no")})
    m = H2ONaiveBayesEstimator(laplace=1)
    m.train(y="y", training_frame=h2o3_amd.H2OFrame(df))
    assert m.auc() > 0.9
