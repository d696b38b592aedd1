"""Reference-layout MOJO export (mojo/h2o_writer.py) round-trips through the
reference-layout reader (mojo/h2o_mojo.py, pinned against the reference's own
genmodel fixtures in tests/test_mojo_reference.py): predictions of the
exported MOJO equal the in-platform predictions."""
import numpy as np
import pandas as pd
import pytest


@pytest.fixture(scope="module")
def data():
    import h2o3_amd as h2o
    h2o.init(verbose=False)
    rng = np.random.RandomState(3)
    n = 1500
    X = rng.randn(n, 4)
    X[rng.rand(n) < 0.08, 1] = np.nan
    cat = rng.choice(list("abcdefghij"), n)
    big = rng.choice([f"L{i}" for i in range(45)], n)       # > 32 levels: general bitset
    logit = X[:, 0] - 0.7 * np.nan_to_num(X[:, 1]) + (cat == "c") * 1.5 - (big == "L7") * 2
    df = pd.DataFrame(X, columns=list("pqrs"))
    df["cat"] = cat
    df["big"] = big
    df["yb"] = np.where(rng.rand(n) < 1 / (1 + np.exp(-logit)), "yes", "no")
    df["yr"] = logit + 0.1 * rng.randn(n)
    df["ym"] = np.where(logit > 1, "hi", np.where(logit < -1, "lo", "mid"))
    return df, h2o.H2OFrame(df)


def _roundtrip(model, df, tmp_path):
    """Score the exported MOJO on the float32 values the platform's frame
    holds (numeric Vecs are f32 in HBM): the reference scorer compares the
    row's double against float32 split values, so scoring the unrounded f64
    inputs can flip rows that sit exactly on a split point."""
    from h2o3_amd.mojo import h2o_mojo
    path = model.download_mojo(str(tmp_path), format="h2o")
    m = h2o_mojo.load(path)
    d32 = df.copy()
    for c in d32.columns:
        if d32[c].dtype.kind == "f":
            d32[c] = d32[c].astype(np.float32).astype(np.float64)
    return m, m.predict(d32)


X = ["p", "q", "r", "s", "cat", "big"]


@pytest.mark.parametrize("y", ["yb", "yr", "ym"])
def test_gbm_h2o_mojo_roundtrip(data, y, tmp_path):
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    df, fr = data
    g = H2OGradientBoostingEstimator(ntrees=8, max_depth=4, seed=1)
    g.train(x=X, y=y, training_frame=fr)
    ours = g.predict(fr).as_data_frame()
    m, theirs = _roundtrip(g, df, tmp_path)
    cols = [c for c in ours.columns if c != "predict"] or ["predict"]
    np.testing.assert_allclose(theirs[cols].values.astype(float), ours[cols].values.astype(float), atol=2e-5)
    if y != "yr":
        assert (theirs["predict"].astype(str).values == ours["predict"].astype(str).values).mean() > 0.999


@pytest.mark.parametrize("y", ["yb", "yr", "ym"])
def test_drf_h2o_mojo_roundtrip(data, y, tmp_path):
    from h2o3_amd.estimators import H2ORandomForestEstimator
    df, fr = data
    d = H2ORandomForestEstimator(ntrees=6, max_depth=6, seed=2)
    d.train(x=X, y=y, training_frame=fr)
    ours = d.predict(fr).as_data_frame()
    m, theirs = _roundtrip(d, df, tmp_path)
    cols = [c for c in ours.columns if c != "predict"] or ["predict"]
    np.testing.assert_allclose(theirs[cols].values.astype(float), ours[cols].values.astype(float), atol=2e-5)


@pytest.mark.parametrize("family,y", [("binomial", "yb"), ("gaussian", "yr"), ("multinomial", "ym"),
                                      ("poisson", "yr")])
def test_glm_h2o_mojo_roundtrip(data, family, y, tmp_path):
    from h2o3_amd.estimators import H2OGeneralizedLinearEstimator
    df, fr = data
    d2 = df.copy()
    if family == "poisson":
        d2["yr"] = np.round(np.exp(np.clip(df["yr"].values, -2, 2) * 0.5))
        import h2o3_amd as h2o
        fr2 = h2o.H2OFrame(d2)
    else:
        fr2 = fr
    g = H2OGeneralizedLinearEstimator(family=family, lambda_=0.0)
    g.train(x=X, y=y, training_frame=fr2)
    ours = g.predict(fr2).as_data_frame()
    m, theirs = _roundtrip(g, d2, tmp_path)
    cols = [c for c in ours.columns if c != "predict"] or ["predict"]
    np.testing.assert_allclose(theirs[cols].values.astype(float), ours[cols].values.astype(float), rtol=1e-4,
                               atol=1e-5)


def test_h2o_mojo_files_layout(data, tmp_path):
    import zipfile
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    df, fr = data
    g = H2OGradientBoostingEstimator(ntrees=3, max_depth=3, seed=1)
    g.train(x=X, y="yb", training_frame=fr)
    path = g.download_mojo(str(tmp_path), format="h2o")
    names = zipfile.ZipFile(path).namelist()
    assert "model.ini" in names and "model.json" not in names
    assert {"trees/t00_000.bin", "trees/t00_000_aux.bin", "trees/t00_002.bin"} <= set(names)
    ini = zipfile.ZipFile(path).read("model.ini").decode()
    for key in ("algorithm = Gradient Boosting Machine", "n_trees = 3", "distribution = bernoulli",
                "mojo_version = 1.40", "[columns]", "[domains]"):
        assert key in ini


def test_kmeans_h2o_mojo_roundtrip(data, tmp_path):
    from h2o3_amd.estimators import H2OKMeansEstimator
    df, fr = data
    km = H2OKMeansEstimator(k=4, seed=3, standardize=True)
    km.train(x=["p", "r", "s", "cat"], training_frame=fr)
    ours = km.predict(fr).as_data_frame()["predict"].values
    m, theirs = _roundtrip(km, df, tmp_path)
    assert m.algo == "kmeans" and not m.supervised
    assert (theirs["predict"].values == ours).mean() > 0.998


def test_isolationforest_h2o_mojo_roundtrip(data, tmp_path):
    from h2o3_amd.estimators import H2OIsolationForestEstimator
    df, fr = data
    iso = H2OIsolationForestEstimator(ntrees=20, seed=4, sample_size=128)
    iso.train(x=["p", "q", "r", "s"], training_frame=fr)
    ours = iso.predict(fr).as_data_frame()
    m, theirs = _roundtrip(iso, df, tmp_path)
    np.testing.assert_allclose(theirs["mean_length"].values, ours["mean_length"].values, atol=1e-4)
    # the reference stores the normalising min / max TOTAL path lengths as ints
    rng_ = (iso._max_len - iso._min_len) * 20
    np.testing.assert_allclose(theirs["predict"].values, ours["predict"].values, atol=1.0 / rng_ + 1e-6)


def test_extended_isolationforest_h2o_mojo_roundtrip(data, tmp_path):
    from h2o3_amd.estimators import H2OExtendedIsolationForestEstimator
    df, fr = data
    eif = H2OExtendedIsolationForestEstimator(ntrees=15, sample_size=64, extension_level=2, seed=5)
    eif.train(x=["p", "r", "s"], training_frame=fr)
    ours = eif.predict(fr).as_data_frame()
    m, theirs = _roundtrip(eif, df, tmp_path)
    np.testing.assert_allclose(theirs["mean_length"].values, ours["mean_length"].values, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(theirs["anomaly_score"].values, ours["anomaly_score"].values, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("y,act", [("yb", "Rectifier"), ("yr", "Tanh"), ("ym", "RectifierWithDropout"),
                                   ("yb", "Maxout")])
def test_deeplearning_h2o_mojo_roundtrip(data, y, act, tmp_path):
    from h2o3_amd.estimators import H2ODeepLearningEstimator
    df, fr = data
    dl = H2ODeepLearningEstimator(hidden=[12, 7], epochs=3, seed=6, activation=act, reproducible=True)
    dl.train(x=X, y=y, training_frame=fr)
    ours = dl.predict(fr).as_data_frame()
    m, theirs = _roundtrip(dl, df, tmp_path)
    cols = [c for c in ours.columns if c != "predict"] or ["predict"]
    np.testing.assert_allclose(theirs[cols].values.astype(float), ours[cols].values.astype(float), rtol=2e-4,
                               atol=2e-4)


def test_word2vec_h2o_mojo_roundtrip(tmp_path):
    import h2o3_amd as h2o
    from h2o3_amd.estimators import H2OWord2vecEstimator
    from h2o3_amd.mojo import h2o_mojo
    rng = np.random.RandomState(0)
    vocab = [f"w{i}" for i in range(30)]
    words = []
    for _ in range(300):
        words += list(rng.choice(vocab, 6)) + [None]
    fr = h2o.H2OFrame(pd.DataFrame({"w": words}), column_types=["string"])
    w2v = H2OWord2vecEstimator(vec_size=8, epochs=2, min_word_freq=1, seed=1)
    w2v.train(training_frame=fr)
    m = h2o_mojo.load(w2v.download_mojo(str(tmp_path), format="h2o"))
    assert m.vec_size == 8 and len(m.embeddings) == len(w2v._vocab)
    for i, w in enumerate(w2v._vocab[:10]):
        np.testing.assert_allclose(m.transform(w), w2v._vecs[i].cpu().numpy(), rtol=1e-6)


@pytest.mark.parametrize("y", ["yb", "yr", "ym"])
def test_stackedensemble_h2o_mojo_roundtrip(data, y, tmp_path):
    from h2o3_amd.estimators import (H2OGradientBoostingEstimator, H2OGeneralizedLinearEstimator,
                                     H2ORandomForestEstimator, H2OStackedEnsembleEstimator)
    df, fr = data
    kw = dict(nfolds=3, keep_cross_validation_predictions=True, fold_assignment="Modulo", seed=1)
    g = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, **kw)
    g.train(x=X, y=y, training_frame=fr)
    d = H2ORandomForestEstimator(ntrees=4, max_depth=5, **kw)
    d.train(x=X, y=y, training_frame=fr)
    fam = {"yb": "binomial", "yr": "gaussian", "ym": "multinomial"}[y]
    gl = H2OGeneralizedLinearEstimator(family=fam, **kw)
    gl.train(x=["p", "r", "s", "cat"], y=y, training_frame=fr)
    se = H2OStackedEnsembleEstimator(base_models=[g, d, gl])
    se.train(x=X, y=y, training_frame=fr)
    ours = se.predict(fr).as_data_frame()
    m, theirs = _roundtrip(se, df, tmp_path)
    assert m.algo == "stackedensemble" and len(m.base) == 3
    cols = [c for c in ours.columns if c != "predict"] or ["predict"]
    np.testing.assert_allclose(theirs[cols].values.astype(float), ours[cols].values.astype(float), rtol=1e-4,
                               atol=1e-4)


@pytest.mark.parametrize("transform,x", [("STANDARDIZE", ["p", "r", "s", "cat"]), ("NONE", ["p", "r", "s"]),
                                         ("NORMALIZE", ["p", "r", "cat", "big"])])
def test_pca_h2o_mojo_roundtrip(data, transform, x, tmp_path):
    from h2o3_amd.estimators import H2OPrincipalComponentAnalysisEstimator
    df, fr = data
    pca = H2OPrincipalComponentAnalysisEstimator(k=3, transform=transform)
    pca.train(x=x, training_frame=fr)
    ours = pca.predict(fr).as_data_frame()
    m, theirs = _roundtrip(pca, df, tmp_path)
    np.testing.assert_allclose(theirs.values, ours.values[:, :3].astype(float), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("y", ["yb", "yr", "ym"])
def test_xgboost_h2o_mojo_roundtrip(data, y, tmp_path):
    """XGBoost export in the reference's XGBoost MOJO layout (one-hot feature
    space + native booster blob): categorical bitset splits become chains of
    indicator tests, NA levels the extra indicator per column."""
    from h2o3_amd.estimators import H2OXGBoostEstimator
    df, fr = data
    g = H2OXGBoostEstimator(ntrees=6, max_depth=4, seed=1)
    g.train(x=X, y=y, training_frame=fr)
    ours = g.predict(fr).as_data_frame()
    m, theirs = _roundtrip(g, df, tmp_path)
    assert m.algo == "xgboost"
    cols = [c for c in ours.columns if c != "predict"] or ["predict"]
    np.testing.assert_allclose(theirs[cols].values.astype(float), ours[cols].values.astype(float), atol=2e-5)
    if y != "yr":
        assert (theirs["predict"].astype(str).values == ours["predict"].astype(str).values).mean() > 0.999


@pytest.mark.parametrize("y,blending", [("yb", False), ("yb", True), ("yr", True), ("ym", False)])
def test_targetencoder_h2o_mojo_roundtrip(data, y, blending, tmp_path):
    """Reference-layout TargetEncoder MOJO (encoding_map.ini + column maps):
    the reader's encodings equal the in-platform transform (NA levels, unseen
    levels -> NA / prior, blending, one column per non-first class)."""
    from h2o3_amd.estimators import H2OTargetEncoderEstimator
    from h2o3_amd.mojo import h2o_mojo
    import h2o3_amd as h2o
    df, fr = data
    df = df.copy()
    df.loc[df.index[:40], "cat"] = None                      # NA level present in training
    fr2 = h2o.H2OFrame(df)
    te = H2OTargetEncoderEstimator(blending=blending, inflection_point=5, smoothing=3)
    te.train(x=["cat", "big"], y=y, training_frame=fr2)
    ours = te.transform(fr2, as_training=False).as_data_frame()
    m = h2o_mojo.load(te.download_mojo(str(tmp_path), format="h2o"))
    assert m.algo == "targetencoder"
    theirs = m.predict(df)
    for c in theirs.columns:
        np.testing.assert_allclose(theirs[c].values, ours[c].values, rtol=1e-9, atol=1e-12)
    # unseen level: 'big' had no NAs in training -> prior mean
    row = df.iloc[:1].copy()
    row["big"] = "never_seen"
    enc = m.predict(row)
    big_cols = [c for c in enc.columns if c.startswith("big")]
    for c in big_cols:
        cls = c[len("big"):-len("_te")]
        k = 1 if not cls else list(te._spec.response_domain).index(cls.lstrip("_"))
        assert enc[c].iloc[0] == pytest.approx(te._prior[max(k - 1, 0)] if len(te._prior) > 1 else te._prior[0])
