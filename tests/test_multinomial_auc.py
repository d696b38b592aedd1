"""Multinomial AUC / PR-AUC and auc_type (hex/MultinomialAUC.java,
MultinomialAucType.java, ModelMetricsMultinomial.java:22): OVR and OVO
aggregates against sklearn's exact values, the AUTO / NONE / >50-class
rules, the reference's table layout, and exposure over REST."""
import numpy as np
import pandas as pd
import pytest
import torch

import h2o3_amd as h2o
from h2o3_amd.models import metrics as mm


def _probs(n=3000, K=4, seed=0):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, K, n)
    logits = rng.normal(size=(n, K)) + 1.2 * np.eye(K)[y]
    P = np.exp(logits)
    P /= P.sum(1, keepdims=True)
    w = rng.uniform(0.5, 2.0, n)
    return y, P, w


@pytest.mark.parametrize("weighted", [False, True])
def test_ovr_ovo_match_sklearn(weighted):
    from sklearn.metrics import roc_auc_score
    h2o.init(device="cpu", verbose=False)
    y, P, w = _probs()
    wt = torch.as_tensor(w) if weighted else None
    dom = ["a", "b", "c", "d"]
    for t, mc, avg in (("MACRO_OVR", "ovr", "macro"), ("WEIGHTED_OVR", "ovr", "weighted"),
                       ("MACRO_OVO", "ovo", "macro"), ("WEIGHTED_OVO", "ovo", "weighted")):
        m = mm.multinomial_metrics(torch.as_tensor(y), torch.as_tensor(P), wt, dom, auc_type=t)
        if mc == "ovo" and weighted:
            continue   # sklearn's ovo has no sample weights
        ref = roc_auc_score(y, P, multi_class=mc, average=avg, sample_weight=w if weighted else None)
        assert abs(m.auc() - ref) < 2e-3, (t, m.auc(), ref)
    tab = m.multinomial_auc_table()
    assert [r["type"] for r in tab][:6] == ["a vs Rest", "b vs Rest", "c vs Rest", "d vs Rest", "Macro OVR",
                                            "Weighted OVR"]
    assert len(tab) == 4 + 2 + 6 + 2 and tab[-2]["type"] == "Macro OVO"
    assert m.multinomial_aucpr_table()[0]["value"] > 0


def test_auto_none_and_class_cap():
    h2o.init(device="cpu", verbose=False)
    y, P, w = _probs()
    for t in ("AUTO", "NONE"):
        m = mm.multinomial_metrics(torch.as_tensor(y), torch.as_tensor(P), None, None, auc_type=t)
        assert np.isnan(m.auc()) and m.multinomial_auc_table() is None
    y2, P2, _ = _probs(n=2000, K=51)
    m = mm.multinomial_metrics(torch.as_tensor(y2), torch.as_tensor(P2), None, None, auc_type="MACRO_OVR")
    assert np.isnan(m.auc())                  # MAX_AUC_CLASSES = 50
    with pytest.raises(ValueError):
        mm.multinomial_metrics(torch.as_tensor(y), torch.as_tensor(P), None, None, auc_type="MICRO")


def test_model_auc_type_and_performance_override():
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    h2o.init(device="cpu", verbose=False)
    rng = np.random.default_rng(3)
    n = 2000
    X = rng.normal(size=(n, 3))
    y = np.where(X[:, 0] > 0.5, "hi", np.where(X[:, 0] < -0.5, "lo", "mid"))
    df = pd.DataFrame(X, columns=list("abc"))
    df["y"] = y
    fr = h2o.H2OFrame(df)
    g = H2OGradientBoostingEstimator(ntrees=5, seed=1, auc_type="WEIGHTED_OVO")
    g.train(x=list("abc"), y="y", training_frame=fr)
    assert 0.9 < g.auc() <= 1.0 and g.aucpr() > 0.8
    assert g.multinomial_auc_table()[-1]["type"] == "Weighted OVO"
    plain = H2OGradientBoostingEstimator(ntrees=5, seed=1)
    plain.train(x=list("abc"), y="y", training_frame=fr)
    assert np.isnan(plain.auc())
    assert plain.model_performance(fr, auc_type="MACRO_OVR").auc() > 0.9
    # max_confusion_matrix_size: no CM table past that many classes
    s = H2OGradientBoostingEstimator(ntrees=2, seed=1, max_confusion_matrix_size=2)
    s.train(x=list("abc"), y="y", training_frame=fr)
    assert s._training_metrics["cm"] is None


def test_gainslift_bins():
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    h2o.init(device="cpu", verbose=False)
    rng = np.random.default_rng(4)
    X = rng.normal(size=(3000, 3))
    df = pd.DataFrame(X, columns=list("abc"))
    df["y"] = np.where(X[:, 0] + 0.5 * rng.normal(size=3000) > 0, "p", "n")
    fr = h2o.H2OFrame(df)
    for bins, expect in ((-1, 16), (5, 5), (0, None)):
        g = H2OGradientBoostingEstimator(ntrees=5, seed=1, gainslift_bins=bins)
        g.train(x=list("abc"), y="y", training_frame=fr)
        gl = g._training_metrics.get("gains_lift_table")
        if expect is None:
            assert gl is None
        else:
            assert 0 < len(gl) <= expect and abs(gl[-1]["cumulative_capture_rate"] - 1) < 1e-9


def test_multinomial_auc_over_rest():
    import time
    from fastapi.testclient import TestClient
    from h2o3_amd.server import create_app
    h2o.init(device="cpu", verbose=False)
    c = TestClient(create_app())
    rng = np.random.default_rng(5)
    X = rng.normal(size=(600, 2))
    df = pd.DataFrame(X, columns=["a", "b"])
    df["y"] = np.where(X[:, 0] > 0.5, "hi", np.where(X[:, 0] < -0.5, "lo", "mid"))
    c.post("/3/PostFile", json={"data": df.to_dict(orient="list"), "destination_frame": "mauc.hex"})
    job = c.post("/3/ModelBuilders/gbm", json={"training_frame": "mauc.hex", "response_column": "y", "ntrees": 3,
                                                "auc_type": "MACRO_OVO", "model_id": "gbm_mauc"}).json()["job"]
    t0 = time.time()
    while job["status"] == "RUNNING" and time.time() - t0 < 60:
        time.sleep(0.05)
        job = c.get(f"/3/Jobs/{job['key']['name']}").json()["jobs"][0]
    tm = c.get("/3/Models/gbm_mauc").json()["models"][0]["output"]["training_metrics"]
    assert tm["AUC"] > 0.9 and tm["multinomial_auc_table"]["name"] == "Multinomial AUC values"
    assert tm["multinomial_aucpr_table"]["columns"][-1]["name"] == "auc_pr"
