"""MOJO-side TreeSHAP contributions, experimental/modelDetails.json and the
Generic model (an imported MOJO served like a native model).

References: h2o-genmodel TreeSHAP.java / EasyPredictModelWrapper.java:196
(setEnableContributions), GbmMojoModel / DrfMojoModel contribution
predictors, hex/ModelMojoWriter.java:96 (writeModelDetails),
ModelJsonReader.java:27, hex/generic/GenericModel.java:449-498.
"""
import os

import numpy as np
import pandas as pd
import pytest
import torch

import h2o3_amd
from h2o3_amd.estimators import H2OGradientBoostingEstimator, H2ORandomForestEstimator
from h2o3_amd.mojo.genmodel import EasyPredictModelWrapper, MojoModel
from h2o3_amd.models.generic import H2OGenericEstimator

FIX = "/root/reference/h2o-genmodel/src/test/resources/hex/genmodel/algos/gbm/gbm_variable_importance.zip"


@pytest.fixture(scope="module")
def frames():
    h2o3_amd.init(verbose=False)
    rng = np.random.RandomState(3)
    n = 1500
    # f32-representable values: the frame stores f32, the reference-layout
    # scorer compares doubles against the f32 split points (split points are
    # data values, so an f64 value next to one may fall on the other side)
    X = rng.randn(n, 4).astype(np.float32).astype(np.float64)
    X[rng.rand(n, 4) < 0.05] = np.nan
    df = pd.DataFrame(X, columns=["a", "b", "c", "d"])
    df["k"] = rng.choice(["u", "v", "w", "z"], n)
    eta = np.nan_to_num(df.a.values) - np.nan_to_num(df.b.values) + (df.k == "w") * 0.8
    df["y"] = np.where(eta + 0.5 * rng.randn(n) > 0, "yes", "no")
    df["r"] = (eta + 0.3 * rng.randn(n)).astype(np.float32).astype(np.float64)
    return df, h2o3_amd.H2OFrame(df)


def _contrib_np(fr):
    return fr.as_data_frame()


def _check(model, df, fr, tmp_path, margin):
    xcols = ["a", "b", "c", "d", "k"]
    ref = model.predict_contributions(fr).as_data_frame()
    assert list(ref.columns) == xcols + ["BiasTerm"]
    np.testing.assert_allclose(ref.sum(1).values, margin, rtol=1e-5, atol=1e-5)
    for fmt in ("native", "h2o"):
        p = model.download_mojo(str(tmp_path / fmt), format=fmt)
        mj = MojoModel.load(p)
        got = mj.predict_contributions(df[xcols])
        assert list(got.columns) == xcols + ["BiasTerm"]
        np.testing.assert_allclose(got.values, ref.values, rtol=1e-6, atol=2e-6, err_msg=fmt)
        # EasyPredictModelWrapper with contributions enabled: one row
        w = EasyPredictModelWrapper(mj, enable_contributions=True)
        row = {c: df[c].iloc[7] for c in xcols}
        out = w.predict(row)
        np.testing.assert_allclose([out["contributions"][c] for c in xcols + ["BiasTerm"]], ref.iloc[7].values,
                                   rtol=1e-6, atol=2e-6)
        # sorted layout
        top = mj.predict_contributions(df[xcols].head(20), top_n=2, bottom_n=1)
        assert list(top.columns) == ["top_feature_1", "top_value_1", "top_feature_2", "top_value_2",
                                     "bottom_feature_1", "bottom_value_1", "BiasTerm"]


def test_gbm_mojo_contributions_match_model(frames, tmp_path):
    df, fr = frames
    m = H2OGradientBoostingEstimator(ntrees=12, max_depth=4, seed=1)
    m.train(x=["a", "b", "c", "d", "k"], y="y", training_frame=fr)
    p1 = m.predict(fr).as_data_frame()["yes"].values.astype(np.float64)
    _check(m, df, fr, tmp_path, np.log(p1 / (1 - p1)))


def test_gbm_regression_mojo_contributions(frames, tmp_path):
    df, fr = frames
    m = H2OGradientBoostingEstimator(ntrees=8, max_depth=3, seed=1)
    m.train(x=["a", "b", "c", "d", "k"], y="r", training_frame=fr)
    _check(m, df, fr, tmp_path, m.predict(fr).as_data_frame()["predict"].values)


def test_drf_mojo_contributions_reference_form(frames, tmp_path):
    """Binomial DRF: the reference's 1/(F+1) - contribution(P0) form, summing
    to P(class 1)."""
    df, fr = frames
    m = H2ORandomForestEstimator(ntrees=6, max_depth=5, seed=1)
    m.train(x=["a", "b", "c", "d", "k"], y="y", training_frame=fr)
    _check(m, df, fr, tmp_path, m.predict(fr).as_data_frame()["yes"].values)


@pytest.mark.skipif(not os.path.exists(FIX), reason="reference genmodel fixtures not present")
def test_generic_reports_fixture_model_details():
    """The reference fixture's experimental/modelDetails.json: training AUC /
    logloss / varimp of the ORIGINAL model, exposed by the Generic model."""
    h2o3_amd.init(verbose=False)
    g = H2OGenericEstimator.from_file(FIX)
    assert g._forest is not None and len(g._forest) == 50
    assert g.auc() == pytest.approx(0.9801618150931445, abs=1e-12)
    assert g.logloss() == pytest.approx(0.2675723908575812, abs=1e-12)
    assert g.mse() == pytest.approx(0.07338612397264782, abs=1e-12)
    vi = g.varimp(use_pandas=True)
    assert list(vi.columns)[:3] == ["variable", "relative_importance", "scaled_importance"]
    assert vi["scaled_importance"].max() == pytest.approx(1.0)
    assert g.model_performance()._m["nobs"] == 380


@pytest.mark.skipif(not os.path.exists(FIX), reason="reference genmodel fixtures not present")
def test_generic_device_scoring_matches_mojo_scorer():
    """Predictions on the platform's forest kernel equal the standalone MOJO
    scorer; contributions sum to the raw margin; leaf paths equal the MOJO's
    decision paths."""
    h2o3_amd.init(verbose=False)
    g = H2OGenericEstimator.from_file(FIX)
    mj = g._mojo
    rng = np.random.RandomState(0)
    n = 300
    df = pd.DataFrame({c: rng.uniform(0, 80, n) if c not in ("RACE", "DPROS", "DCAPS") else
                       rng.choice([1.0, 2.0, 3.0], n) for c in mj.features})
    df.iloc[::17, 1] = np.nan
    fr = h2o3_amd.H2OFrame(df)
    raw = mj.predict_raw(df)
    got = g.predict(fr).as_data_frame()
    np.testing.assert_allclose(got.iloc[:, 2].values, raw[:, -1], rtol=1e-5, atol=1e-6)
    c = g.predict_contributions(fr).as_data_frame()
    p1 = raw[:, -1]
    np.testing.assert_allclose(c.sum(1).values, np.log(p1 / (1 - p1)), rtol=1e-4, atol=1e-4)
    cm = mj.predict_contributions(df)
    np.testing.assert_allclose(c.values, cm.values, rtol=1e-5, atol=1e-5)
    la = g.predict_leaf_node_assignment(fr).as_data_frame()
    paths = mj.decision_paths(df)
    assert [str(v) for v in la.iloc[5].values] == paths[5]


def test_generic_round_trip_metrics(frames, tmp_path):
    """A model exported as a reference-layout MOJO and imported as Generic
    reports the original's training metrics and varimp; scoring on the device
    equals the original model."""
    df, fr = frames
    m = H2OGradientBoostingEstimator(ntrees=10, max_depth=4, seed=2)
    m.train(x=["a", "b", "c", "d", "k"], y="y", training_frame=fr)
    p = m.download_mojo(str(tmp_path), format="h2o")
    import zipfile
    assert "experimental/modelDetails.json" in zipfile.ZipFile(p).namelist()
    g = H2OGenericEstimator.from_file(p)
    assert g.auc() == pytest.approx(m.auc(), abs=1e-12)
    assert g.logloss() == pytest.approx(m.logloss(), abs=1e-12)
    v0, v1 = m.varimp(use_pandas=True), g.varimp(use_pandas=True)
    assert list(v0["variable"]) == list(v1["variable"])
    a = m.predict(fr).as_data_frame()["yes"].values
    b = g.predict(fr).as_data_frame()["yes"].values
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    perf = g.model_performance(fr)
    assert perf.auc() == pytest.approx(m.model_performance(fr).auc(), abs=1e-6)
