"""RuleFit recovers a rule-shaped signal."""
import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.estimators import H2ORuleFitEstimator


def test_rulefit_regression_and_binomial():
    h2o.init()
    rng = np.random.default_rng(0)
    n = 1500
    X = rng.uniform(0, 1, size=(n, 4))
    y = 3.0 * ((X[:, 0] > 0.5) & (X[:, 1] < 0.3)) + 0.5 * X[:, 2] + rng.normal(scale=0.1, size=n)
    df = pd.DataFrame(X, columns=list("abcd"))
    df["y"] = y
    fr = h2o.H2OFrame(df)
    m = H2ORuleFitEstimator(min_rule_length=2, max_rule_length=3, rule_generation_ntrees=20, seed=1)
    m.train(x=list("abcd"), y="y", training_frame=fr)
    ri = m.rule_importance()
    assert len(ri) > 0
    top = ri.iloc[0]["rule"]
    assert "a" in top and "b" in top, ri.head()
    pred = m.predict(fr).as_data_frame()["predict"].values
    assert np.corrcoef(pred, y)[0, 1] > 0.95
    df["yb"] = np.where(y > 1.5, "hi", "lo")
    fr2 = h2o.H2OFrame(df)
    mb = H2ORuleFitEstimator(min_rule_length=1, max_rule_length=2, rule_generation_ntrees=10, seed=1,
                             model_type="RULES")
    mb.train(x=list("abcd"), y="yb", training_frame=fr2)
    assert mb.auc() > 0.95
    assert mb.predict_rules(fr2, ["rule_0"]).ncol == 1
