import numpy as np
import pandas as pd

import h2o3_amd
from h2o3_amd.estimators import H2ODeepLearningEstimator


def test_dl_binomial_and_regression():
    rng = np.random.RandomState(0)
    X = rng.randn(3000, 5)
    logit = 2 * X[:, 0] - X[:, 1] ** 2 + X[:, 2]
    y = (rng.rand(3000) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame(X, columns=list("abcde"))
    df["y"] = np.where(y == 1, "t", "f")
    df["r"] = X[:, 0] * 3 + np.sin(X[:, 1])
    fr = h2o3_amd.H2OFrame(df)
    m = H2ODeepLearningEstimator(hidden=[32, 32], epochs=20, seed=1)
    m.train(x=list("abcde"), y="y", training_frame=fr)
    assert m.auc() > 0.85
    assert m.varimp() is not None
    m2 = H2ODeepLearningEstimator(hidden=[32], epochs=30, seed=1, activation="Tanh")
    m2.train(x=list("abcde"), y="r", training_frame=fr)
    assert m2.r2() > 0.9


def test_autoencoder_anomaly():
    rng = np.random.RandomState(1)
    X = rng.randn(2000, 4)
    X[:, 3] = X[:, 0] + X[:, 1]
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=list("abcd")))
    m = H2ODeepLearningEstimator(autoencoder=True, hidden=[3], epochs=20, seed=2)
    m.train(training_frame=fr)
    a = m.anomaly(fr)
    assert a.nrows == 2000
    assert m.deepfeatures(fr, 0).ncols == 3
