"""ANOVA GLM type-III tests and ModelSelection subset search."""
import itertools

import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OANOVAGLMEstimator, H2OModelSelectionEstimator


def test_anovaglm_detects_main_effect_and_interaction():
    h2o.init()
    rng = np.random.default_rng(0)
    n = 1200
    a = rng.normal(size=n)
    b = rng.normal(size=n)
    g = rng.choice(["u", "v", "w"], n)
    y = 2 * a + 1.5 * a * b + (g == "u") * 1.0 + rng.normal(size=n)
    fr = h2o.H2OFrame(pd.DataFrame({"a": a, "b": b, "g": g, "y": y}))
    m = H2OANOVAGLMEstimator(family="gaussian", highest_interaction_term=2)
    m.train(x=["a", "b", "g"], y="y", training_frame=fr)
    r = m.summary().set_index("predictors_interactions")
    assert r.loc["a", "p_values"] < 1e-10
    assert r.loc["a:b", "p_values"] < 1e-10
    assert r.loc["g", "p_values"] < 1e-6
    assert r.loc["b:g", "p_values"] > 1e-3
    assert r.loc["g", "df"] == 2


def _ms_frame(seed=1):
    rng = np.random.default_rng(seed)
    n = 800
    X = rng.normal(size=(n, 6))
    y = 3 * X[:, 1] - 2 * X[:, 4] + 0.5 * X[:, 0] + rng.normal(size=n)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(6)])
    df["y"] = y
    return df


def _r2(df, cols):
    X = np.column_stack([np.ones(len(df))] + [df[c].values for c in cols])
    beta = np.linalg.lstsq(X, df["y"].values, rcond=None)[0]
    r = df["y"].values - X @ beta
    return 1 - (r @ r) / ((df["y"] - df["y"].mean()) ** 2).sum()


def test_modelselection_allsubsets_maxr_backward():
    h2o.init()
    df = _ms_frame()
    fr = h2o.H2OFrame(df)
    xs = [f"x{i}" for i in range(6)]
    m = H2OModelSelectionEstimator(mode="allsubsets", max_predictor_number=3)
    m.train(x=xs, y="y", training_frame=fr)
    preds = m.get_best_model_predictors()
    assert set(preds[1]) == {"x1", "x4"}
    for k in (1, 2, 3):
        best = max(_r2(df, list(s)) for s in itertools.combinations(xs, k))
        assert abs(m.get_best_R2_values()[k - 1] - best) < 1e-4
    mr = H2OModelSelectionEstimator(mode="maxr", max_predictor_number=3)
    mr.train(x=xs, y="y", training_frame=fr)
    assert set(mr.get_best_model_predictors()[2]) == {"x0", "x1", "x4"}
    assert set(mr.coef(2)) == {"Intercept", "x1", "x4"}
    mb = H2OModelSelectionEstimator(mode="backward", min_predictor_number=2)
    mb.train(x=xs, y="y", training_frame=fr)
    last = mb.get_best_model_predictors()[-1]
    assert set(last) == {"x1", "x4"}
