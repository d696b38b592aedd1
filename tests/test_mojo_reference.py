"""Reference-layout MOJO import (h2o-genmodel zip / directory layout).

Every expected value below is pinned by the reference's own genmodel tests
on the fixtures shipped in the reference tree (loaded read-only, parsed by
mojo/h2o_mojo.py -- nothing from the fixtures is executed):
  h2o-genmodel/src/test/java/hex/genmodel/algos/ensemble/StackedEnsemble*MojoTest.java
  h2o-genmodel/src/test/java/hex/genmodel/MojoPipelineBuilderTest.java
  h2o-genmodel/src/test/java/hex/genmodel/algos/glm/Glm*MojoModelTest.java
  h2o-genmodel/src/test/java/hex/genmodel/algos/gbm/GbmMojoModelTest.java
  h2o-genmodel/src/test/java/hex/genmodel/algos/kmeans/KMeansMojoModelTest.java
  h2o-genmodel/src/test/java/hex/genmodel/algos/word2vec/Word2VecMojoModelTest.java
"""
import os

import numpy as np
import pytest

R = "/root/reference/h2o-genmodel/src/test/resources/hex/genmodel/"
pytestmark = pytest.mark.skipif(not os.path.isdir(R), reason="reference fixtures not present")


def _load(p):
    from h2o3_amd.mojo import h2o_mojo
    return h2o_mojo.load(R + p)


def test_stacked_ensemble_binomial():
    m = _load("algos/ensemble/binomial.zip")
    p = m.predict_row({"AGE": "65", "RACE": "1", "DPROS": "2", "DCAPS": "1", "PSA": "1.4", "VOL": "0",
                       "GLEASON": "6"})
    assert p["predict"] == "0"
    np.testing.assert_allclose([p["p0"], p["p1"]], [0.8222695, 0.1777305], atol=1e-5)
    assert [b[0].algo for b in m.base] == ["gbm", "drf", "drf"]


def test_stacked_ensemble_regression_and_multinomial():
    r = _load("algos/ensemble/regression.zip")
    p = r.predict_row({"CAPSULE": "0", "RACE": "1", "DPROS": "2", "DCAPS": "1", "PSA": "1.4", "VOL": "0",
                       "GLEASON": "6"})
    assert abs(p["predict"] - 66.29695) < 1e-5
    mm = _load("algos/ensemble/multinomial.zip")
    p = mm.predict_row({"CAPSULE": "0", "AGE": "65", "DPROS": "2", "DCAPS": "1", "PSA": "1.4", "VOL": "0",
                        "GLEASON": "6"})
    assert p["predict"] == "1"
    np.testing.assert_allclose([p["p0"], p["p1"], p["p2"]], [0.006592327, 0.901237, 0.09217069], atol=1e-5)


def test_stacked_ensemble_pruned_base_models():
    m = _load("algos/ensemble/binomial_without_useless_models.zip")
    assert [i for i, b in enumerate(m.base) if b is not None] == [6]
    # the metalearner keeps a (zero) slot per pruned model; mu == threshold ties go to class 1
    assert m.predict_row({"AGE": "65"})["predict"] == "1"


def test_stacked_ensemble_with_deep_learning_base():
    m = _load("algos/ensemble/binomial_titanic.zip")
    row = {"pclass": 1.0, "survived": 1.0, "name": "Allison, Master. Hudson Trevor", "sex": "male", "age": 0.9167,
           "sibsp": 1.0, "parch": 2.0, "ticket": 113781.0, "fare": 151.55, "cabin": "C22 C26", "embarked": "S",
           "boat": 11.0, "body": float("nan"), "home.dest": "Montreal, PQ / Chesterville, ON"}
    p = m.predict_row(row)
    assert p["predict"] in ("0", "1") and abs(p["p0"] + p["p1"] - 1) < 1e-9
    assert "deeplearning" in [b[0].algo for b in m.base if b]


def test_kmeans_to_glm_pipeline():
    km = _load("algos/pipeline/kmeans_model.zip")
    glm = _load("algos/pipeline/glm_model.zip")
    for (age, race, dpros, dcaps, psa, vol, gl), exp in [((71, 1, 3.0, 2.0, 3.3, 0.0, 8.0), 0.7812266),
                                                        ((76, 2, 2.0, 1.0, 51.2, 20.0, 7.0), 0.5690164)]:
        c = int(km.predict({"AGE": age, "RACE": str(race)})["predict"][0])
        v = glm.predict({"CLUSTER": str(c), "DPROS": dpros, "DCAPS": dcaps, "PSA": psa, "VOL": vol,
                         "GLEASON": gl})["predict"][0]
        assert abs(v - exp) < 1e-7


def test_glm_binomial_score0():
    m = _load("algos/glm/prostate")
    data = np.array([[2, 73, 2, 1, 7.9, 18, 6], [1, 51, 3, 1, 8.9, 0, 6], [2, 57, 3, 1, 3.4, 30.8, 6],
                     [1, 65, 4, 1, 6.3, 0, 6], [1, 61, 3, 1, 1.5, 0, 5], [1, 56, 2, 2, 58, 0, 6],
                     [1, 72, 2, 1, 1.4, 24.2, 6], [1, 54, 2, 1, 18, 43, 9], [1, 62, 2, 1, 7.3, 0, 7],
                     [2, 63, 3, 1, 14.3, 16, 7], [1, 68, 1, 1, 5.4, 34, 5], [1, np.nan, 1, 1, 5.4, 34, 5]])
    exp = np.array([[0.0, 0.883740206424754, 0.11625979357524593], [1.0, 0.5591006829867439, 0.44089931701325613],
                    [0.0, 0.8200793110208472, 0.1799206889791528], [1.0, 0.4855023555733662, 0.5144976444266338],
                    [0.0, 0.8260781970262484, 0.17392180297375157], [1.0, 0.2685796973779421, 0.7314203026220579],
                    [0.0, 0.8265057623033865, 0.1734942376966135], [1.0, 0.1332488800455477, 0.8667511199544523],
                    [1.0, 0.5038183003787983, 0.49618169962120173], [1.0, 0.5384202639029669, 0.46157973609703307],
                    [0.0, 0.9543248143434919, 0.04567518565650803], [0.0, 0.9531416700165544, 0.046858329983445586]])
    np.testing.assert_allclose(m.score0(data), exp, atol=1e-7)


def test_glm_multinomial_score0():
    m = _load("algos/glm/multinomial")
    src = open("/root/reference/h2o-genmodel/src/test/java/hex/genmodel/algos/glm/GlmMultinomialMojoModelTest.java").read()
    import re
    blocks = re.findall(r"new double\[\]\{([^}]*)\}", src)
    rows = [[float(t) for t in b.split(",")] for b in blocks]
    data = np.array([r for r in rows if len(r) == 54])
    exp = np.array([r for r in rows if len(r) == 8])
    assert data.shape[0] == exp.shape[0] == 16
    np.testing.assert_allclose(m.score0(data), exp, atol=1e-6)


def test_gbm_calibrated_and_leaf_paths():
    m = _load("algos/gbm/calibrated")
    row = {"SegSumT": 18.7, "SegTSeas": 1.51, "SegLowFlow": 1.003, "DSDist": 132.53, "DSMaxSlope": 1.15,
           "USAvgT": 0.2, "USRainDays": 1.153, "USSlope": 8.3, "USNative": 0.34, "DSDam": 0.0, "Method": "electric"}
    p = m.predict_row(row)
    assert p["predict"] == "1"
    np.testing.assert_allclose([p["p0"], p["p1"]], [0.5416688, 0.4583312], atol=1e-5)
    np.testing.assert_allclose([p["cal_0"], p["cal_1"]], [0.3920402, 0.6079598], atol=1e-5)
    assert m.decision_paths({})[0] == ["LRLR", "LRLR", "LRLR", "LRLR", "LRLR", "RLLRR", "RLLRL", "RLLLL",
                                       "LRLRL", "RRLRL"]


def test_kmeans_rows_map_to_their_clusters():
    m = _load("algos/kmeans")
    rows = np.array([[2.0, 1.0, 22.0, 1.0, 0.0], [2.0, 1.0, 2.0, 3.0, 1.0], [2.0, 0.0, 27.0, 0.0, 2.0]])
    assert m.score0(rows)[:, 0].tolist() == [0.0, 1.0, 2.0]


def test_word2vec_embeddings():
    m = _load("algos/word2vec")
    np.testing.assert_allclose(m.transform("a"), [0.0, 1.0, 0.2], atol=1e-4)
    np.testing.assert_allclose(m.transform("b"), [1.0, 0.0, 0.8], atol=1e-4)
    assert m.transform("c") is None


def test_gbm_regression_tree_decode():
    """mojo.zip (GBM regression, 262 features, 20 trees): every tree decodes to
    a full binary tree and scores finite values (parity unpinned: the fixture
    ships no expected predictions)."""
    m = _load("mojo.zip")
    assert m.algo == "gbm" and m.ntree_groups == 20 and len(m.features) == 262
    for t in m.trees[0]:
        assert t.leaf.size == t.col.size + 1
    X = np.random.RandomState(0).randn(50, len(m.columns)) * 10
    X[::7, 3] = np.nan
    v = m.score0(X)[:, 0]
    assert np.isfinite(v).all()


def test_isolation_forests():
    i = _load("algos/isofor")
    row = {c: v for c, v in zip(i.columns, range(1, 10))}
    p = i.predict(row)
    assert list(p.columns) == ["predict", "mean_length"]
    assert abs(p["mean_length"][0] - sum(len(s) for s in i.decision_paths(row)[0]) / 10) < 10
    e = _load("algos/isoforextended")
    q = e.predict({"x": [3.0, 0.0], "y": [3.0, 0.0]})
    assert list(q.columns) == ["anomaly_score", "mean_length"] and len(q) == 2
    assert ((q["anomaly_score"] > 0) & (q["anomaly_score"] < 1)).all()


def test_generic_estimator_imports_reference_mojo(tmp_path):
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.estimators import H2OGenericEstimator
    h2o.init(verbose=False)
    g = H2OGenericEstimator.from_file(R + "algos/ensemble/binomial.zip")
    fr = h2o.H2OFrame(pd.DataFrame({"AGE": [65.0], "RACE": ["1"], "DPROS": ["2"], "DCAPS": [1.0], "PSA": [1.4],
                                    "VOL": [0.0], "GLEASON": [6.0]}))
    out = g.predict(fr).as_data_frame()
    assert abs(float(out["p1"][0]) - 0.1777305) < 1e-5
    m = h2o.import_mojo(R + "algos/pipeline/glm_model.zip")
    assert m._mojo.algo == "glm"


# ------------------------------------------------------------------ XGBoost
XR = "/root/reference/h2o-genmodel-extensions/xgboost/src/test/resources/hex/genmodel/algos/xgboost/"
PROSTATE = "/root/reference/h2o-py/h2o/h2o_data/prostate.csv"


@pytest.mark.skipif(not os.path.isdir(XR) or not os.path.exists(PROSTATE), reason="xgboost fixtures not present")
def test_xgboost_java_mojo_training_mse():
    """xgboost_java.zip (50-tree reg:squarederror booster on prostate, AGE
    response): the MOJO's own modelDetails.json records training MSE
    3.3232581458216086 and MAE 1.229596690127724 over the 380 rows;
    XGBoostJavaMojoModelTest.testConvertWithWeights pins the root weight 380."""
    import pandas as pd
    from h2o3_amd.mojo import h2o_mojo
    m = h2o_mojo.load(XR + "xgboost_java.zip")
    assert m.algo == "xgboost" and m.booster.name_obj == "reg:squarederror" and len(m.booster.trees) == 50
    assert float(m.booster.trees[0][1]["sum_hess"][0]) == 380.0
    df = pd.read_csv(PROSTATE)
    p = m.predict(df)["predict"].values
    err = p - df["AGE"].values
    assert abs((err ** 2).mean() - 3.3232581458216086) < 1e-6
    assert abs(np.abs(err).mean() - 1.229596690127724) < 1e-6


@pytest.mark.skipif(not os.path.isdir(XR), reason="xgboost fixtures not present")
def test_xgboost_multinomial_sparse_mojo():
    """xgboost.zip: multi:softprob booster over a 246-wide one-hot feature
    space (31 categoricals, 14 numerics, sparse = true: 0 -> missing).  The
    booster re-serializes byte-for-byte in length and scores valid class
    probabilities for rows with unseen / missing levels."""
    import zipfile
    import pandas as pd
    from h2o3_amd.mojo import h2o_mojo
    from h2o3_amd.mojo.xgb_booster import Booster
    raw = zipfile.ZipFile(XR + "xgboost.zip").read("boosterBytes")
    b = Booster.parse(raw)
    assert (b.num_feature, b.num_class, b.name_obj, len(b.trees)) == (246, 3, "multi:softprob", 15)
    assert len(b.to_bytes()) == len(raw)
    m = h2o_mojo.load(XR + "xgboost.zip")
    assert m.xgb_sparse and m.xgb_cats == 31 and m.xgb_nums == 14
    p = m.predict(pd.DataFrame([{"race": "Caucasian", "age": "[70-80)", "time_in_hospital": 3,
                                 "num_medications": 12, "diabetesMed": "Yes"},
                                {"race": "NotALevel", "number_inpatient": 0}]))
    probs = p[["<30", ">30", "NO"]].values
    np.testing.assert_allclose(probs.sum(1), 1.0, atol=1e-9)
    assert set(p["predict"]) <= {"<30", ">30", "NO"}


def test_svm_mojo():
    """SvmMojoModelTest.testPredict: all-zero row -> label 1, all-one row ->
    label 0 (Sparkling Water linear SVM fixture, mean imputation on)."""
    from h2o3_amd.mojo import h2o_mojo
    m = h2o_mojo.load(R + "algos/svm")
    assert m.algo == "svm" and m.nclasses == 2
    X = np.array([[0.0] * 6 + [np.nan], [1.0] * 6 + [np.nan]])
    preds = m.score0(X)
    assert list(preds[:, 0]) == [1.0, 0.0]
    # NaN features are mean-imputed: equals scoring the means explicitly
    Xn = np.full((1, 7), np.nan)
    Xm = np.concatenate([np.asarray(m.svm_means[:6]), [np.nan]]).reshape(1, 7)
    np.testing.assert_allclose(m.score0(Xn), m.score0(Xm))
