import numpy as np
import pandas as pd

import h2o3_amd
from h2o3_amd.automl import H2OAutoML
from h2o3_amd.estimators import (H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                                 H2ORandomForestEstimator, H2OStackedEnsembleEstimator)
from h2o3_amd.grid import H2OGridSearch


def _frame(n=1500, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, 4)
    logit = 1.5 * X[:, 0] - X[:, 1] + X[:, 2] * X[:, 3]
    y = (rng.rand(n) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame(X, columns=list("abcd"))
    df["y"] = np.where(y == 1, "1", "0")
    fr = h2o3_amd.H2OFrame(df)
    fr["y"] = fr["y"].asfactor()
    return fr


def test_grid_cartesian_and_random():
    fr = _frame()
    g = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=10, seed=1),
                      hyper_params={"max_depth": [2, 4], "learn_rate": [0.05, 0.2]})
    g.train(y="y", training_frame=fr)
    assert len(g.models) == 4
    sg = g.get_grid(sort_by="auc", decreasing=True)
    aucs = [m.auc() for m in sg.models]
    assert aucs == sorted(aucs, reverse=True)
    g2 = H2OGridSearch(H2OGradientBoostingEstimator, hyper_params={"max_depth": [2, 3, 4, 5], "ntrees": [5, 10]},
                       search_criteria={"strategy": "RandomDiscrete", "max_models": 3, "seed": 1})
    g2.train(y="y", training_frame=fr)
    assert len(g2.models) == 3


def test_stacked_ensemble():
    fr = _frame(seed=1)
    common = dict(nfolds=3, fold_assignment="Modulo", keep_cross_validation_predictions=True, seed=1)
    m1 = H2OGradientBoostingEstimator(ntrees=20, max_depth=3, **common)
    m1.train(y="y", training_frame=fr)
    m2 = H2ORandomForestEstimator(ntrees=20, **common)
    m2.train(y="y", training_frame=fr)
    m3 = H2OGeneralizedLinearEstimator(family="binomial", **common)
    m3.train(y="y", training_frame=fr)
    se = H2OStackedEnsembleEstimator(base_models=[m1, m2, m3])
    se.train(y="y", training_frame=fr)
    assert se.auc() > 0.8
    assert se.predict(fr).ncols == 3


def test_automl_small():
    fr = _frame(800, seed=2)
    aml = H2OAutoML(max_models=4, seed=1, nfolds=3, exclude_algos=["DeepLearning"])
    aml.train(y="y", training_frame=fr)
    lb = aml.leaderboard.as_data_frame()
    assert len(lb) >= 4
    assert aml.leader is not None
    assert "auc" in lb.columns
    assert aml.leader.predict(fr).nrows == fr.nrows
