"""TF-IDF, grep, segment models."""
import math

import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OGeneralizedLinearEstimator, H2OGrepModel
from h2o3_amd.information_retrieval import tf_idf


def test_tf_idf():
    h2o.init()
    fr = h2o.H2OFrame(pd.DataFrame({"id": [0, 1, 2], "text": ["A b b c", "b c", "a a"]}),
                      column_types=["int", "string"])
    out = tf_idf(fr, "id", "text", case_sensitive=False).as_data_frame()
    r = out[(out.DocID == 0) & (out.Word == "b")].iloc[0]
    assert r.TF == 2
    assert math.isclose(r.IDF, math.log(4 / 3), rel_tol=1e-6)
    assert math.isclose(r["TF-IDF"], 2 * math.log(4 / 3), rel_tol=1e-6)
    a = out[(out.DocID == 2) & (out.Word == "a")].iloc[0]
    assert a.TF == 2 and math.isclose(a.IDF, math.log(4 / 3), rel_tol=1e-6)  # "A" lower-cased joins "a"


def test_grep():
    h2o.init()
    fr = h2o.H2OFrame(pd.DataFrame({"t": ["foo123", "bar", "foo9"]}), column_types=["string"])
    g = H2OGrepModel(regex=r"foo\d+")
    g.train(training_frame=fr)
    assert g.matches() == ["foo123", "foo9"]


def test_segment_models():
    h2o.init()
    rng = np.random.default_rng(0)
    n = 600
    seg = rng.choice(["s1", "s2", "s3"], n)
    x = rng.normal(size=n)
    slope = {"s1": 1.0, "s2": -2.0, "s3": 3.0}
    y = np.array([slope[s] for s in seg]) * x + rng.normal(scale=0.05, size=n)
    fr = h2o.H2OFrame(pd.DataFrame({"seg": seg, "x": x, "y": y}))
    est = H2OGeneralizedLinearEstimator(lambda_=0.0)
    sm = est.train_segments(x=["x"], y="y", training_frame=fr, segments=["seg"])
    tab = sm.as_frame().as_data_frame()
    assert list(tab["status"]) == ["SUCCEEDED"] * 3
    for s, b in slope.items():
        m = sm.get_model(seg=s)
        assert abs(m.coef()["x"] - b) < 0.05


def test_h2otree_jobs_timeline():
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    from h2o3_amd.tree import H2OTree
    h2o.init()
    rng = np.random.default_rng(0)
    df = pd.DataFrame({"a": rng.normal(size=300), "k": rng.choice(["p", "q"], 300)})
    df["y"] = df.a * 2 + (df.k == "p")
    fr = h2o.H2OFrame(df)
    m = H2OGradientBoostingEstimator(ntrees=3, max_depth=3)
    m.train(x=["a", "k"], y="y", training_frame=fr)
    t = H2OTree(m, 0)
    assert len(t) == len(t.left_children) == len(t.predictions)
    assert t.root_node.split_feature in ("a", "k")
    assert m._job.status == "DONE"
    assert any(e["event"] == "model_build_done" and e["model_id"] == m.model_id for e in h2o.timeline())


def test_persist_compressed_and_mrtask(tmp_path):
    import gzip
    import torch
    from h2o3_amd.core.mrtask import map_reduce
    h2o.init()
    p = tmp_path / "d.csv.gz"
    with gzip.open(p, "wt") as f:
        f.write("a,b\n1,2\n3,4\n5,6\n")
    fr = h2o.import_file(str(p))
    assert fr.shape == (3, 2)
    s = map_reduce(fr, lambda a, b: torch.stack([a.double().sum(), (a * b).double().sum()]))
    assert s.tolist() == [9.0, 1 * 2 + 3 * 4 + 5 * 6]


def test_grid_recovery(tmp_path):
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    from h2o3_amd.grid import H2OGridSearch
    h2o.init()
    rng = np.random.default_rng(0)
    df = pd.DataFrame({"a": rng.normal(size=300)})
    df["y"] = df.a * 2 + rng.normal(scale=0.1, size=300)
    fr = h2o.H2OFrame(df)
    g = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=3), {"max_depth": [2, 3]}, grid_id="gr",
                      recovery_dir=str(tmp_path))
    g.train(x=["a"], y="y", training_frame=fr)
    assert len(g.models) == 2
    g2 = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=3), {"max_depth": [2, 3, 4]}, grid_id="gr",
                       recovery_dir=str(tmp_path))
    g2.train(x=["a"], y="y", training_frame=fr)
    assert len(g2.models) == 3   # two recovered, one new


def test_sklearn_wrappers_and_transforms():
    from h2o3_amd.sklearn import H2OGradientBoostingClassifier, H2OGeneralizedLinearRegressor
    from h2o3_amd.transforms import H2OScaler
    rng = np.random.default_rng(0)
    X = rng.normal(size=(300, 3))
    y = np.where(X[:, 0] + X[:, 1] > 0, "a", "b")
    clf = H2OGradientBoostingClassifier(ntrees=10, max_depth=3).fit(X, y)
    assert clf.score(X, y) > 0.9
    assert clf.predict_proba(X).shape == (300, 2)
    reg = H2OGeneralizedLinearRegressor(lambda_=0.0).fit(X, 2 * X[:, 0] + 1)
    assert reg.score(X, 2 * X[:, 0] + 1) > 0.999
    fr = h2o.H2OFrame(pd.DataFrame(X, columns=list("abc")))
    sc = H2OScaler().fit(fr)
    t = sc.transform(fr).as_data_frame()
    assert abs(t["a"].mean()) < 1e-5 and abs(t["a"].std() - 1) < 1e-3
