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


def test_automl_stacked_ensemble_metrics_are_cross_validated():
    """StackedEnsembleModel.java:371 / StackedEnsembleStepsProvider.java:146:
    in AutoML the metalearner is cross-validated with the AutoML nfolds and the
    ensemble's leaderboard metrics are those CV metrics.  On a pure-noise
    response no model -- ensembles included -- may look better than chance
    (training metrics of base models refit on all rows would)."""
    import numpy as np
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.automl import H2OAutoML
    h2o.init(verbose=False)
    rng = np.random.RandomState(0)
    n = 3000
    df = pd.DataFrame(rng.randn(n, 6), columns=list("abcdef"))
    df["y"] = np.where(rng.rand(n) < 0.5, "yes", "no")
    aml = H2OAutoML(max_models=3, nfolds=3, seed=1, verbosity=None, include_algos=["GLM", "XGBoost",
                                                                                   "StackedEnsemble"])
    aml.train(y="y", training_frame=h2o.H2OFrame(df))
    lb = aml.leaderboard.as_data_frame()
    se = lb[lb["model_id"].str.startswith("StackedEnsemble")]
    assert len(se) >= 1
    assert (se["auc"] < 0.56).all()
    for m in aml.models:
        if m.algo == "stackedensemble":
            assert m._cross_validation_metrics is not None


def test_automl_time_allocation_by_work_weight():
    """ModelingStep.java:550: a step gets remaining budget x weight / remaining
    weight of its priority group + the Stacked Ensembles."""
    from h2o3_amd.automl import H2OAutoML
    aml = H2OAutoML(max_runtime_secs=100, seed=1)
    import time
    aml._t0 = time.time()
    pending = [("DRF", "def_1"), ("GBM", "def_1"), ("XGBoost", "grid_1"), ("StackedEnsemble", "all")]
    aml._assign_step_time(pending[0], pending)
    share = aml._step_deadline - time.time()
    assert 30 < share < 34          # 100 s x 10 / (10 + 10 + 10 SE)
    aml._assign_step_time(pending[2], pending[2:])
    assert 70 < aml._step_deadline - time.time() < 76   # grid: 30 / (30 + 10)


import pytest  # noqa: E402


def test_automl_adaptive_stopping_tolerance():
    """AutoML.java:357: unset stopping_tolerance = min(0.05, max(0.001,
    1/sqrt((1 - NA fraction) * nrows)))."""
    import numpy as np
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.automl import H2OAutoML
    h2o.init(verbose=False)
    df = pd.DataFrame({"a": np.arange(4000, dtype=float), "b": np.ones(4000)})
    df.loc[:999, "a"] = np.nan                      # NA fraction 1000 / 8000
    fr = h2o.H2OFrame(df)
    aml = H2OAutoML(max_models=1)
    aml._set_stopping_tolerance(fr)
    assert aml.stopping_tolerance == pytest.approx(1 / np.sqrt(0.875 * 4000))
    big = H2OAutoML(max_models=1, stopping_tolerance=0.0001)
    big._set_stopping_tolerance(fr)
    assert big.stopping_tolerance == 0.0001


def test_automl_exploitation_steps_rebuild_every_family():
    """The lr_annealing / lr_search steps refit the family leader from its own
    parameters: those must be ones its estimator accepts (an XGBoost leader
    once failed on the shared-default names it carries)."""
    from h2o3_amd.estimators import H2OXGBoostEstimator
    fr = _frame(600, seed=3)
    aml = H2OAutoML(max_models=2, seed=1, nfolds=0, include_algos=["XGBoost", "GBM"], verbosity=None)
    aml.train(y="y", training_frame=fr)
    data = {"train": fr, "valid": None, "x": list("abcd"), "y": "y", "blending": None, "leaderboard": None,
            "weights": None, "fold": None}
    aml.max_models = 10          # room for the refits
    aml._step_deadline = None
    n_models = len(aml.models)
    for algo, step in (("XGBoost", "lr_search"), ("GBM", "lr_annealing")):
        cls = H2OXGBoostEstimator if algo == "XGBoost" else H2OGradientBoostingEstimator
        aml._exploit(algo, cls, step, data)
    msgs = " ".join(r["message"] for r in aml.event_log_rows)
    assert "failed" not in msgs, msgs
    assert "lr_search_selection" in msgs, msgs
    assert len(aml.models) >= n_models
