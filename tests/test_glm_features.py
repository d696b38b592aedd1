"""GLM feature parity: beta_constraints, interactions (+ MOJO replay),
remove_collinear_columns, alpha grid, startval, prior, calc_like, HGLM."""
import numpy as np
import pandas as pd
import pytest

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OGeneralizedLinearEstimator as GLM


@pytest.fixture(scope="module")
def data():
    h2o.init(verbose=False)
    rng = np.random.RandomState(0)
    n = 3000
    df = pd.DataFrame({"a": rng.randn(n), "b": rng.randn(n), "c": rng.choice(["u", "v", "w"], n),
                       "d": rng.choice(["p", "q"], n)})
    df["c2"] = df["a"] * 2.0
    df["y"] = 1 + 2 * df.a - 3 * df.b + 1.5 * df.a * df.b + (df.c == "v") * df.a * 2 + rng.randn(n) * 0.1
    return df


def test_interactions_and_collinear(data):
    fr = h2o.H2OFrame(data)
    m = GLM(family="gaussian", lambda_=0, interactions=["a", "b", "c"], remove_collinear_columns=True)
    m.train(y="y", training_frame=fr)
    c = m.coef()
    assert c["a_b"] == pytest.approx(1.5, abs=0.02)
    assert c["a_c.v"] == pytest.approx(2.0, abs=0.02)
    assert m._output["removed_collinear_columns"] == ["c2"] and c["c2"] == 0.0
    from h2o3_amd.mojo.genmodel import MojoModel
    from h2o3_amd.mojo.writer import build_mojo
    pm = np.asarray(MojoModel(build_mojo(m)).predict(data.drop(columns=["y"]))).reshape(-1)
    ph = m.predict(fr).as_data_frame().iloc[:, 0].values
    np.testing.assert_allclose(pm, ph, rtol=1e-4, atol=1e-4)


def test_beta_constraints_and_startval(data):
    fr = h2o.H2OFrame(data)
    bc = h2o.H2OFrame(pd.DataFrame({"names": ["a", "b"], "lower_bounds": [0.0, -1.0], "upper_bounds": [1.0, 10.0]}))
    m = GLM(family="gaussian", lambda_=0, beta_constraints=bc)
    m.train(y="y", x=["a", "b", "c", "d"], training_frame=fr)
    c = m.coef()
    assert c["a"] == pytest.approx(1.0, abs=1e-6) and c["b"] == pytest.approx(-1.0, abs=1e-6)
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.models.glm.glm import GLMDriver
    est = GLM(family="gaussian", lambda_=0, startval={"a": 2.0, "b": -3.0, "Intercept": 1.0})
    drv = GLMDriver(est, TrainSpec(fr, ["a", "b"], "y"))
    beta, icpt = drv.dinfo.destandardize(drv.beta[:-1], drv.beta[-1])
    np.testing.assert_allclose(beta, [2.0, -3.0], atol=1e-9)
    assert icpt == pytest.approx(1.0, abs=1e-9)


def test_alpha_grid_prior_calc_like(data):
    fr = h2o.H2OFrame(data)
    tr, va = fr.split_frame([0.8], seed=1)
    m = GLM(family="gaussian", alpha=[0.0, 0.5, 1.0], lambda_search=True, nlambdas=8)
    m.train(y="y", x=["a", "b", "c", "d"], training_frame=tr, validation_frame=va)
    assert m._output["alpha_best"] in (0.0, 0.5, 1.0)
    assert len({h["alpha"] for h in m._scoring_history}) == 3
    df = data.copy()
    df["yb"] = (df.y > 1).astype(int)
    fb = h2o.H2OFrame(df)
    base = GLM(family="binomial", lambda_=0, calc_like=True)
    base.train(y="yb", x=["a", "b"], training_frame=fb)
    pri = GLM(family="binomial", lambda_=0, prior=0.1)
    pri.train(y="yb", x=["a", "b"], training_frame=fb)
    ym = df.yb.mean()
    shift = np.log(0.1 / 0.9) - np.log(ym / (1 - ym))
    assert pri.coef()["Intercept"] == pytest.approx(base.coef()["Intercept"] + shift, abs=1e-6)
    assert base._output["loglikelihood"] < 0


def test_hglm_random_intercepts():
    rng = np.random.RandomState(0)
    n, G = 5000, 40
    g = rng.randint(0, G, n)
    u = rng.randn(G) * 2.0
    x = rng.randn(n)
    y = 1.0 + 0.5 * x + u[g] + rng.randn(n)
    fr = h2o.H2OFrame(pd.DataFrame({"x": x, "g": [f"G{i}" for i in g], "y": y}))
    m = GLM(family="gaussian", HGLM=True, random_columns=["g"], rand_family=["gaussian"])
    m.train(y="y", x=["x", "g"], training_frame=fr)
    assert m.coef()["x"] == pytest.approx(0.5, abs=0.05)
    assert m._output["varfix"] == pytest.approx(1.0, abs=0.1)
    ue = np.array([m.coefs_random()["g"][f"G{i}"] for i in range(G)])
    assert np.corrcoef(u, ue)[0, 1] > 0.99


def test_native_cd_matches_python_cd():
    """C++ coordinate descent (native/glm_solver.cpp) == the reference-style
    Python CD on a penalised, boxed quadratic."""
    import numpy as np
    from h2o3_amd.models.glm import glm as glm_mod
    rng = np.random.default_rng(0)
    P = 40
    A = rng.standard_normal((400, P))
    G = A.T @ A / 400
    b = rng.standard_normal(P)
    lo = np.full(P, -0.3)
    hi = np.full(P, 0.5)
    nat = glm_mod._solve_quadratic(G, b, 0.05, 0.01, True, lower=lo, upper=hi)
    cd = glm_mod._CD[:]
    try:
        glm_mod._CD[:] = [None]
        py = glm_mod._solve_quadratic(G, b, 0.05, 0.01, True, lower=lo, upper=hi)
    finally:
        glm_mod._CD[:] = cd
    assert np.abs(nat - py).max() < 1e-7
    assert (nat == 0).sum() > 0 and nat.min() >= -0.3 - 1e-12 and nat[:-1].max() <= 0.5 + 1e-12
