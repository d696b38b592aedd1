"""Infogram: a redundant copy of a strong feature is relevant but carries no
net information; fair infogram flags proxies of the protected column."""
import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OInfogram


def test_core_and_fair_infogram():
    h2o.init()
    rng = np.random.default_rng(0)
    n = 3000
    a = rng.normal(size=n)
    b = rng.normal(size=n)
    noise = rng.normal(size=n)
    prot = rng.integers(0, 2, n)
    proxy = prot + 0.1 * rng.normal(size=n)
    logit = 2 * a + 1.5 * b + 1.0 * prot
    y = np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "1", "0")
    df = pd.DataFrame({"a": a, "b": b, "noise": noise, "proxy": proxy, "prot": prot.astype(str), "y": y})
    fr = h2o.H2OFrame(df)
    ig = H2OInfogram(algorithm_params={"ntrees": 20, "max_depth": 3}, seed=1)
    ig.train(x=["a", "b", "noise"], y="y", training_frame=fr)
    t = ig.get_admissible_score_frame().as_data_frame().set_index("column")
    assert t.loc["a", "admissible"] == 1
    assert t.loc["noise", "admissible"] == 0
    fair = H2OInfogram(algorithm_params={"ntrees": 20, "max_depth": 3}, seed=1, protected_columns=["prot"])
    fair.train(x=["a", "b", "noise", "proxy", "prot"], y="y", training_frame=fr)
    tf = fair.get_admissible_score_frame().as_data_frame().set_index("column")
    assert tf.loc["a", "safety_index"] > tf.loc["proxy", "safety_index"]
    assert "a" in fair.get_admissible_features()
