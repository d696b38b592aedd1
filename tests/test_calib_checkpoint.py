"""Calibration (Platt / isotonic) and GBM checkpoint continuation."""
import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OGradientBoostingEstimator, H2ORandomForestEstimator


def _fr(seed=0, n=3000):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 3))
    p = 1 / (1 + np.exp(-(2 * X[:, 0] - X[:, 1])))
    df = pd.DataFrame(X, columns=list("abc"))
    df["y"] = np.where(rng.random(n) < p, "yes", "no")
    return h2o.H2OFrame(df)


def test_calibration_columns_and_quality():
    h2o.init()
    tr, cal = _fr(0), _fr(1)
    for cls, kw in ((H2OGradientBoostingEstimator, dict(ntrees=30, max_depth=5, learn_rate=0.3)),
                    (H2ORandomForestEstimator, dict(ntrees=10, max_depth=8))):
        for meth in ("PlattScaling", "IsotonicRegression"):
            m = cls(seed=1, calibrate_model=True, calibration_frame=cal, calibration_method=meth, **kw)
            m.train(x=list("abc"), y="y", training_frame=tr)
            pr = m.predict(cal).as_data_frame()
            assert {"cal_p0", "cal_p1"} <= set(pr.columns)
            np.testing.assert_allclose(pr.cal_p0 + pr.cal_p1, 1.0, atol=1e-5)
            y = (cal.as_data_frame()["y"].astype(str) == "yes").values
            ll = lambda q: -np.mean(y * np.log(np.clip(q, 1e-6, 1)) + (1 - y) * np.log(np.clip(1 - q, 1e-6, 1)))
            assert ll(pr.cal_p1.values) <= ll(pr["yes"].values) + 1e-2   # Platt: sigmoid of p, not of logit(p)


def test_gbm_checkpoint_continues_training():
    h2o.init()
    tr = _fr(2)
    full = H2OGradientBoostingEstimator(ntrees=20, max_depth=3, seed=5)
    full.train(x=list("abc"), y="y", training_frame=tr)
    half = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=5)
    half.train(x=list("abc"), y="y", training_frame=tr)
    cont = H2OGradientBoostingEstimator(ntrees=20, max_depth=3, seed=5, checkpoint=half.model_id)
    cont.train(x=list("abc"), y="y", training_frame=tr)
    assert cont.ntrees_built == 20
    a = full.predict(tr).as_data_frame()["yes"].values
    b = cont.predict(tr).as_data_frame()["yes"].values
    np.testing.assert_allclose(a, b, atol=1e-5)
