"""Parameters forwarded by the GLM wrappers and the GLM checkpoint restart."""
import numpy as np
import pandas as pd

import h2o3_amd
from h2o3_amd.estimators import (H2OANOVAGLMEstimator, H2OGeneralizedLinearEstimator, H2OModelSelectionEstimator,
                                 H2OUpliftRandomForestEstimator)


def _fr(seed=0, n=600):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, 3)
    df = pd.DataFrame(X, columns=list("abc"))
    df["g"] = rng.choice(["u", "v"], n)
    df["y"] = 2 * X[:, 0] - X[:, 1] + 0.1 * rng.randn(n)
    return h2o3_amd.H2OFrame(df)


def test_glm_checkpoint_restarts_from_coefficients():
    fr = _fr()
    m = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0)
    m.train(x=["a", "b", "c"], y="y", training_frame=fr)
    m2 = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0, checkpoint=m, max_iterations=1)
    m2.train(x=["a", "b", "c"], y="y", training_frame=fr)
    for k, v in m.coef().items():
        assert abs(m2.coef()[k] - v) < 1e-6


def test_wrappers_forward_glm_parameters():
    fr = _fr(1)
    a = H2OANOVAGLMEstimator(family="gaussian", lambda_search=False, non_negative=True, solver="IRLSM")
    a.train(x=["a", "b"], y="y", training_frame=fr)
    assert a._full._parms["non_negative"] is True and a._full._parms["solver"] == "IRLSM"
    ms = H2OModelSelectionEstimator(mode="maxr", max_predictor_number=2, beta_epsilon=1e-6, nlambdas=3)
    ms.train(x=["a", "b", "c"], y="y", training_frame=fr)
    assert len(ms.coef()) >= 1
