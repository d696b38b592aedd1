import numpy as np
import pandas as pd
import pytest

import h2o3_amd
from h2o3_amd import estimators as E
from h2o3_amd.mojo import MojoModel


def _df(n=600, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, 3)
    c = rng.choice(list("pqr"), n)
    y = (X[:, 0] + (c == "q") + 0.3 * rng.randn(n) > 0.3).astype(int)
    df = pd.DataFrame(X, columns=list("abc"))
    df["cat"] = c
    df.loc[rng.rand(n) < 0.05, "a"] = np.nan
    df["y"] = np.where(y == 1, "Y", "N")
    df["r"] = X[:, 0] * 2 + X[:, 1]
    return df


@pytest.mark.parametrize("make", [
    lambda: E.H2OGradientBoostingEstimator(ntrees=5, max_depth=3),
    lambda: E.H2ORandomForestEstimator(ntrees=5, max_depth=5),
    lambda: E.H2OXGBoostEstimator(ntrees=5, max_depth=3),
    lambda: E.H2OGeneralizedLinearEstimator(family="binomial"),
    lambda: E.H2ODeepLearningEstimator(hidden=[8], epochs=2, seed=1),
    lambda: E.H2ONaiveBayesEstimator(),
])
def test_mojo_roundtrip_binomial(tmp_path, make):
    df = _df()
    fr = h2o3_amd.H2OFrame(df)
    m = make()
    m.train(x=["a", "b", "c", "cat"], y="y", training_frame=fr)
    path = m.download_mojo(str(tmp_path))
    mojo = MojoModel.load(path)
    p_mojo = mojo.predict(df)
    p_in = m.predict(fr).as_data_frame()
    np.testing.assert_allclose(p_mojo["Y"].values, p_in["Y"].values, rtol=1e-4, atol=1e-4)
    g = h2o3_amd.import_mojo(path)
    np.testing.assert_allclose(g.predict(fr).as_data_frame()["Y"].values, p_in["Y"].values, rtol=1e-4, atol=1e-4)


def test_mojo_regression_and_kmeans(tmp_path):
    df = _df(seed=2)
    fr = h2o3_amd.H2OFrame(df)
    m = E.H2OGradientBoostingEstimator(ntrees=5, max_depth=3)
    m.train(x=["a", "b", "cat"], y="r", training_frame=fr)
    mojo = MojoModel.load(m.download_mojo(str(tmp_path)))
    np.testing.assert_allclose(mojo.predict(df)["predict"].values, m.predict(fr).as_data_frame()["predict"].values,
                               rtol=1e-4, atol=1e-4)
    k = E.H2OKMeansEstimator(k=3, seed=1)
    k.train(x=["a", "b", "c"], training_frame=fr)
    mk = MojoModel.load(k.download_mojo(str(tmp_path)))
    assert (mk.predict(df)["predict"].values == k.predict(fr).as_data_frame()["predict"].values).mean() > 0.99


def test_save_load_model(tmp_path):
    df = _df(seed=3)
    fr = h2o3_amd.H2OFrame(df)
    m = E.H2OGradientBoostingEstimator(ntrees=5, max_depth=3)
    m.train(x=["a", "b", "c", "cat"], y="y", training_frame=fr)
    p = h2o3_amd.save_model(m, str(tmp_path))
    m2 = h2o3_amd.load_model(p)
    assert abs(m2.auc() - m.auc()) < 1e-12
    np.testing.assert_allclose(m2.predict(fr).as_data_frame()["Y"].values, m.predict(fr).as_data_frame()["Y"].values,
                               rtol=1e-4, atol=1e-4)
