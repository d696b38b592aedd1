"""MOJO round trips for EIF, isotonic, CoxPH, uplift DRF, Word2Vec, TargetEncoder."""
import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.estimators import (H2OCoxProportionalHazardsEstimator, H2OExtendedIsolationForestEstimator,
                                 H2OIsotonicRegressionEstimator, H2OTargetEncoderEstimator,
                                 H2OUpliftRandomForestEstimator, H2OWord2vecEstimator)
from h2o3_amd.mojo.genmodel import MojoModel
from h2o3_amd.mojo.writer import build_mojo


def _rt(model, df):
    mm = MojoModel(build_mojo(model))
    return mm.predict(df)


def test_mojo_eif_isotonic_coxph():
    h2o.init()
    rng = np.random.default_rng(0)
    df = pd.DataFrame(rng.normal(size=(400, 3)), columns=list("abc"))
    fr = h2o.H2OFrame(df)
    m = H2OExtendedIsolationForestEstimator(ntrees=10, sample_size=64, extension_level=1, seed=1)
    m.train(training_frame=fr)
    np.testing.assert_allclose(_rt(m, df)["anomaly_score"].values, m.predict(fr).as_data_frame()["anomaly_score"].values,
                               rtol=1e-5)
    df2 = pd.DataFrame({"x": rng.uniform(0, 5, 300)})
    df2["y"] = np.log1p(df2.x) + rng.normal(scale=0.2, size=300)
    fr2 = h2o.H2OFrame(df2)
    iso = H2OIsotonicRegressionEstimator()
    iso.train(x="x", y="y", training_frame=fr2)
    df2f = df2.assign(x=df2.x.astype(np.float32).astype(float))   # the frame stores f32 reals
    np.testing.assert_allclose(_rt(iso, df2f)["predict"].values, iso.predict(fr2).as_data_frame()["predict"].values,
                               atol=1e-5)
    df3 = pd.DataFrame({"x1": rng.normal(size=300), "g": rng.choice(["p", "q"], 300)})
    df3["stop"] = np.ceil(rng.exponential(1 / np.exp(0.5 * df3.x1)) * 10)
    df3["event"] = (rng.random(300) < 0.8).astype(int)
    fr3 = h2o.H2OFrame(df3)
    cox = H2OCoxProportionalHazardsEstimator(stop_column="stop")
    cox.train(x=["x1", "g"], y="event", training_frame=fr3)
    np.testing.assert_allclose(_rt(cox, df3)["lp"].values, cox.predict(fr3).as_data_frame()["lp"].values, atol=1e-4)


def test_mojo_uplift_w2v_te():
    h2o.init()
    rng = np.random.default_rng(1)
    n = 800
    df = pd.DataFrame(rng.normal(size=(n, 2)), columns=["a", "b"])
    df["treatment"] = rng.choice(["control", "treatment"], n)
    df["y"] = np.where(rng.random(n) < 0.3 + 0.3 * (df.treatment == "treatment") * (df.a > 0), "1", "0")
    fr = h2o.H2OFrame(df)
    up = H2OUpliftRandomForestEstimator(ntrees=5, max_depth=3, treatment_column="treatment", seed=1)
    up.train(x=["a", "b"], y="y", training_frame=fr)
    np.testing.assert_allclose(_rt(up, df)["uplift_predict"].values,
                               up.predict(fr).as_data_frame()["uplift_predict"].values, atol=1e-5)
    words = list(rng.choice(["a", "b", "c", "d"], 600))
    wf = h2o.H2OFrame(pd.DataFrame({"w": words}), column_types=["string"])
    w2v = H2OWord2vecEstimator(vec_size=4, min_word_freq=1, epochs=2, seed=1)
    w2v.train(training_frame=wf)
    q = pd.DataFrame({"w": ["a", "zz"]})
    r = _rt(w2v, q)
    np.testing.assert_allclose(r.iloc[0].values, w2v._vecs[w2v._index["a"]].cpu().numpy(), rtol=1e-6)
    assert np.isnan(r.iloc[1].values).all()
    te_df = pd.DataFrame({"k": rng.choice(["x", "y", "z"], 500), "t": rng.normal(size=500)})
    tfr = h2o.H2OFrame(te_df)
    te = H2OTargetEncoderEstimator(noise=0.0, blending=True)
    te.train(x=["k"], y="t", training_frame=tfr)
    np.testing.assert_allclose(_rt(te, te_df)["k_te"].values, te.transform(tfr).as_data_frame()["k_te"].values,
                               atol=1e-5)


def test_rulefit_mojo_matches_in_memory_scoring():
    import numpy as np
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.estimators import H2ORuleFitEstimator
    from h2o3_amd.mojo.genmodel import MojoModel
    from h2o3_amd.mojo.writer import build_mojo
    h2o.init(verbose=False)
    rng = np.random.RandomState(0)
    n = 1500
    df = pd.DataFrame({"a": rng.randn(n), "b": rng.randn(n), "c": rng.choice(["u", "v", "w"], n)})
    df["y"] = np.where((df.a > 0.3) & (df.c != "u"), "yes", "no")
    fr = h2o.H2OFrame(df)
    m = H2ORuleFitEstimator(max_rule_length=3, max_num_rules=20, seed=1)
    m.train(y="y", training_frame=fr)
    pm = np.asarray(MojoModel(build_mojo(m)).predict_raw(df.drop(columns=["y"])))
    ph = m.predict(fr).as_data_frame()
    np.testing.assert_allclose(pm[:, -1], ph.iloc[:, -1].values, atol=1e-6)
