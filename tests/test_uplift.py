"""Uplift DRF: recovers heterogeneous treatment effects; AUUC vs random."""
import numpy as np
import pandas as pd
import pytest
import torch

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OUpliftRandomForestEstimator
from h2o3_amd.models.tree.uplift import auuc_metrics


def _data(n=4000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 3))
    t = rng.integers(0, 2, n)
    base = 0.3
    effect = np.where(X[:, 0] > 0, 0.4, -0.1)
    p = np.clip(base + t * effect, 0.01, 0.99)
    y = (rng.random(n) < p).astype(int)
    df = pd.DataFrame(X, columns=["a", "b", "c"])
    df["treatment"] = np.where(t == 1, "treatment", "control")
    df["y"] = np.where(y == 1, "1", "0")
    return df, effect


@pytest.mark.parametrize("metric", ["KL", "Euclidean", "ChiSquared"])
def test_uplift_drf_recovers_effect(metric):
    h2o.init()
    df, effect = _data()
    fr = h2o.H2OFrame(df)
    m = H2OUpliftRandomForestEstimator(ntrees=10, max_depth=4, treatment_column="treatment", uplift_metric=metric,
                                       seed=1, min_rows=20)
    m.train(x=["a", "b", "c"], y="y", training_frame=fr)
    pr = m.predict(fr).as_data_frame()
    assert list(pr.columns) == ["uplift_predict", "p_y1_with_treatment", "p_y1_without_treatment"]
    u = pr["uplift_predict"].values
    assert u[df.a.values > 0.3].mean() > 0.25
    assert u[df.a.values < -0.3].mean() < 0.05
    perf = m.model_performance(fr)
    assert perf.auuc() > 0 and perf.qini() > 0
    assert abs(perf.ate() - u.mean()) < 1e-6
    vi = m.varimp(use_pandas=True)
    if metric == "KL":
        assert vi.iloc[0]["variable"] == "a"


def test_auuc_perfect_vs_random():
    rng = np.random.default_rng(3)
    n = 5000
    t = torch.tensor(rng.integers(0, 2, n), dtype=torch.float64)
    eff = torch.tensor(rng.uniform(-0.5, 0.5, n))
    y = (torch.rand(n, dtype=torch.float64) < (0.5 + t * eff).clamp(0, 1)).double()
    good = auuc_metrics(eff, y, t, nbins=100)["qini"]
    rand = auuc_metrics(torch.rand(n, dtype=torch.float64), y, t, nbins=100)["qini"]
    assert good["aecu"] > 5 * abs(rand["aecu"])
