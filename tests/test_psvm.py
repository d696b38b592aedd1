"""PSVM vs sklearn SVC (RBF) on a non-linear problem."""
import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OSupportVectorMachineEstimator


def test_psvm_matches_svc_accuracy():
    from sklearn.svm import SVC
    h2o.init()
    rng = np.random.default_rng(0)
    n = 600
    X = rng.normal(size=(n, 2))
    y = np.where((X ** 2).sum(1) < 1.2, "in", "out")
    df = pd.DataFrame(X, columns=["a", "b"])
    df["y"] = y
    fr = h2o.H2OFrame(df)
    m = H2OSupportVectorMachineEstimator(hyper_param=1.0, gamma=0.5, rank_ratio=0.3, seed=1)
    m.train(x=["a", "b"], y="y", training_frame=fr)
    pred = m.predict(fr).as_data_frame()["predict"].values
    acc = (pred == y).mean()
    svc = SVC(C=1.0, gamma=0.5).fit(X, y)
    acc_ref = (svc.predict(X) == y).mean()
    assert acc > acc_ref - 0.03, (acc, acc_ref)
    assert m._output["svs_count"] > 0
    agree = (pred == svc.predict(X)).mean()
    assert agree > 0.95
