"""GLM parameter semantics (hex/glm/GLM.java init + fit): dispersion
estimation (pearson / deviance / ml, fix_dispersion_parameter,
GLM.java:2320-2420), build_null_model (:933), obj_reg (:1063), lambda-search
early stopping (:2977), stopping_rounds / generate_scoring_history
(:946, :3186), gradient_epsilon (:1182), ordinal GRADIENT_DESCENT_SQERR
(:1917, GLMTask.computeGradientMultipliersSQERR) and the GLM.init errors."""
import numpy as np
import pandas as pd
import pytest
from scipy import optimize, special

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OGeneralizedLinearEstimator as GLM


@pytest.fixture(scope="module")
def gamma_data():
    h2o.init(device="cpu", verbose=False)
    rng = np.random.default_rng(7)
    n = 3000
    X = rng.normal(size=(n, 3))
    mu = np.exp(0.5 + 0.3 * X[:, 0] - 0.2 * X[:, 1])
    shape = 2.5
    y = rng.gamma(shape, mu / shape)
    df = pd.DataFrame(X, columns=["a", "b", "c"])
    df["y"] = y
    return df, h2o.H2OFrame(df)


def _mu(m, fr):
    return m.predict(fr).as_data_frame().iloc[:, 0].values


def test_dispersion_pearson_and_deviance(gamma_data):
    df, fr = gamma_data
    y = df["y"].values
    for method in ("pearson", "deviance"):
        m = GLM(family="gamma", link="log", lambda_=0, compute_p_values=True, dispersion_parameter_method=method)
        m.train(x=["a", "b", "c"], y="y", training_frame=fr)
        mu = _mu(m, fr)
        if method == "pearson":
            s = np.sum((y - mu) ** 2 / mu ** 2)
        else:
            s = np.sum(2 * (-np.log(y / mu) + (y - mu) / mu))
        want = s / (len(y) - 1 - 3)
        assert m._output["dispersion"] == pytest.approx(want, rel=1e-4)
        assert m._output["dispersion_estimated"]
    # the true dispersion is 1 / shape = 0.4
    assert 0.3 < m._output["dispersion"] < 0.5


def test_dispersion_ml_gamma(gamma_data):
    df, fr = gamma_data
    y = df["y"].values
    m = GLM(family="gamma", link="log", lambda_=0, compute_p_values=True, dispersion_parameter_method="ml",
            dispersion_epsilon=1e-10)
    m.train(x=["a", "b", "c"], y="y", training_frame=fr)
    mu = _mu(m, fr)
    # independent MLE of the gamma shape a = 1 / phi at the fitted means
    score = lambda a: np.sum(np.log(a) + 1 + np.log(y / mu) - y / mu - special.digamma(a))
    a = optimize.brentq(score, 1e-3, 1e3, xtol=1e-12)
    assert m._output["dispersion"] == pytest.approx(1.0 / a, rel=1e-5)
    # a looser epsilon / fewer iterations give a different (less converged) value
    m2 = GLM(family="gamma", link="log", lambda_=0, compute_p_values=True, dispersion_parameter_method="ml",
             max_iterations_dispersion=1)
    m2.train(x=["a", "b", "c"], y="y", training_frame=fr)
    assert m2._output["dispersion"] != pytest.approx(m._output["dispersion"], rel=1e-6)


def test_fix_dispersion_and_pvalues(gamma_data):
    _, fr = gamma_data
    a = GLM(family="gamma", link="log", lambda_=0, compute_p_values=True)
    a.train(x=["a", "b", "c"], y="y", training_frame=fr)
    b = GLM(family="gamma", link="log", lambda_=0, compute_p_values=True, fix_dispersion_parameter=True,
            init_dispersion_parameter=2.0)
    b.train(x=["a", "b", "c"], y="y", training_frame=fr)
    assert b._output["dispersion"] == 2.0 and not b._output["dispersion_estimated"]
    se_a, se_b = a._output["std_errs"]["a"], b._output["std_errs"]["a"]
    assert se_b / se_a == pytest.approx(np.sqrt(2.0 / a._output["dispersion"]), rel=1e-6)
    with pytest.raises(ValueError, match="fix_dispersion_parameter"):
        GLM(family="gaussian", fix_dispersion_parameter=True).train(x=["a"], y="y", training_frame=fr)
    with pytest.raises(ValueError, match="ml can only be used for family gamma"):
        GLM(family="gaussian", dispersion_parameter_method="ml").train(x=["a"], y="y", training_frame=fr)
    with pytest.raises(ValueError, match="init_dispersion_parameter"):
        GLM(family="gamma", init_dispersion_parameter=0).train(x=["a"], y="y", training_frame=fr)


def test_build_null_model(gamma_data):
    df, fr = gamma_data
    m = GLM(family="gamma", link="log", build_null_model=True)
    m.train(x=["a", "b", "c"], y="y", training_frame=fr)
    assert list(m.coef()) == ["Intercept"]
    assert m.coef()["Intercept"] == pytest.approx(np.log(df["y"].mean()), rel=1e-6)
    with pytest.raises(ValueError, match="build_null_model"):
        GLM(family="gaussian", build_null_model=True).train(x=["a"], y="y", training_frame=fr)


def test_obj_reg_scales_lambda(gamma_data):
    df, fr = gamma_data
    n = len(df)
    a = GLM(family="gaussian", alpha=0.5, lambda_=0.02, obj_reg=0.5 / n, standardize=True)
    a.train(x=["a", "b", "c"], y="y", training_frame=fr)
    b = GLM(family="gaussian", alpha=0.5, lambda_=0.04, standardize=True)
    b.train(x=["a", "b", "c"], y="y", training_frame=fr)
    for k in "abc":
        assert a.coef()[k] == pytest.approx(b.coef()[k], rel=1e-6, abs=1e-9)
    c = GLM(family="gaussian", alpha=0.5, lambda_=0.02, standardize=True)
    c.train(x=["a", "b", "c"], y="y", training_frame=fr)
    assert abs(c.coef()["a"] - a.coef()["a"]) > 1e-4


@pytest.fixture(scope="module")
def bin_data():
    h2o.init(device="cpu", verbose=False)
    rng = np.random.default_rng(3)
    n = 4000
    X = rng.normal(size=(n, 5))
    p = 1 / (1 + np.exp(-(X @ np.array([1.0, -0.5, 0.25, 0.0, 0.0]))))
    df = pd.DataFrame(X, columns=list("abcde"))
    df["y"] = np.where(rng.random(n) < p, "yes", "no")
    return df, h2o.H2OFrame(df)


def test_stopping_rounds_and_scoring_history(bin_data):
    _, fr = bin_data
    with pytest.raises(ValueError, match="lambda_search"):
        GLM(family="binomial", lambda_search=True, stopping_rounds=2).train(x=list("abcde"), y="y",
                                                                            training_frame=fr)
    m = GLM(family="binomial", lambda_=0, stopping_rounds=2, stopping_tolerance=1e-3, score_each_iteration=True)
    m.train(x=list("abcde"), y="y", training_frame=fr)
    sh = m._scoring_history
    assert all("training_logloss" in e for e in sh)
    # GLM's own convergence is off: it stops by ScoreKeeper (2 * k scored
    # iterations at least), before max_iterations
    assert 4 <= len(sh) < 50
    g = GLM(family="binomial", lambda_=0, generate_scoring_history=True, score_iteration_interval=2)
    g.train(x=list("abcde"), y="y", training_frame=fr)
    scored = [e["iteration"] for e in g._scoring_history if "training_logloss" in e]
    assert scored and all(i % 2 == 0 for i in scored)
    plain = GLM(family="binomial", lambda_=0)
    plain.train(x=list("abcde"), y="y", training_frame=fr)
    assert not any("training_logloss" in e for e in plain._scoring_history)


def test_gradient_epsilon_and_max_iterations(bin_data):
    _, fr = bin_data
    tight = GLM(family="binomial", lambda_=0, beta_epsilon=1e-12, objective_epsilon=1e-14, gradient_epsilon=1e-14)
    tight.train(x=list("abcde"), y="y", training_frame=fr)
    loose = GLM(family="binomial", lambda_=0, beta_epsilon=1e-12, objective_epsilon=1e-14, gradient_epsilon=0.05)
    loose.train(x=list("abcde"), y="y", training_frame=fr)
    assert len(loose._scoring_history) < len(tight._scoring_history)
    one = GLM(family="binomial", lambda_=0, max_iterations=1)
    one.train(x=list("abcde"), y="y", training_frame=fr)
    assert len(one._scoring_history) == 1
    with pytest.raises(ValueError, match="max_iterations"):
        GLM(family="binomial", max_iterations=0).train(x=list("abcde"), y="y", training_frame=fr)


def test_lambda_search_defaults(bin_data):
    _, fr = bin_data
    m = GLM(family="binomial", lambda_search=True, alpha=0, early_stopping=False)
    m.train(x=list("abcde"), y="y", training_frame=fr)
    assert len(m._output["regularization_path"]["lambdas"]) == 30      # ridge: 30 lambdas
    m = GLM(family="binomial", lambda_search=True, alpha=0.5, early_stopping=False)
    m.train(x=list("abcde"), y="y", training_frame=fr)
    assert len(m._output["regularization_path"]["lambdas"]) == 100


@pytest.fixture(scope="module")
def ord_data():
    h2o.init(device="cpu", verbose=False)
    rng = np.random.default_rng(11)
    n = 3000
    X = rng.normal(size=(n, 2))
    lat = 1.5 * X[:, 0] - 0.7 * X[:, 1] + rng.logistic(size=n)
    y = np.digitize(lat, [-1.0, 0.5, 2.0])
    df = pd.DataFrame(X, columns=["a", "b"])
    df["y"] = pd.Categorical([f"c{v}" for v in y])
    return df, h2o.H2OFrame(df)


def test_ordinal_reference_sign_and_sqerr(ord_data):
    df, fr = ord_data
    lh = GLM(family="ordinal", lambda_=0)
    lh.train(x=["a", "b"], y="y", training_frame=fr)
    # reference parameterisation P(y <= c) = sigmoid(x.beta + t_c): a larger
    # latent makes the low classes less likely -> negative slope on 'a'
    assert lh.coef()["a"] < -1.0 and lh.coef()["b"] > 0.4
    tab = lh._output["coefficients_table_multinomials"]
    icpts = [tab[c]["Intercept"] for c in ["c0", "c1", "c2"]]
    assert icpts == sorted(icpts)
    sq = GLM(family="ordinal", lambda_=0, solver="GRADIENT_DESCENT_SQERR", seed=5, max_iterations=200)
    sq.train(x=["a", "b"], y="y", training_frame=fr)
    pred = sq.predict(fr).as_data_frame()["predict"].astype(str).values
    acc = float(np.mean(pred == df["y"].astype(str).values))
    assert acc > 0.45                  # well above the 4-class chance level
    assert sq.coef()["a"] < 0
    assert sq.coef() != lh.coef()
    with pytest.raises(ValueError, match="GRADIENT_DESCENT"):
        GLM(family="binomial", solver="GRADIENT_DESCENT_LH").train(x=["a"], y="y", training_frame=fr)


def test_multinomial_lambda_search_path(ord_data):
    _, fr = ord_data
    m = GLM(family="multinomial", lambda_search=True, nlambdas=10, early_stopping=False)
    m.train(x=["a", "b"], y="y", training_frame=fr)
    rp = m._output["regularization_path"]
    assert len(rp["lambdas"]) == 10 and rp["lambdas"] == sorted(rp["lambdas"], reverse=True)
    ex = rp["explained_deviance_train"]
    assert ex[-1] > ex[0]
    with pytest.raises(ValueError, match="non_negative"):
        GLM(family="multinomial", non_negative=True).train(x=["a", "b"], y="y", training_frame=fr)


def test_glm_init_errors(gamma_data):
    df, fr = gamma_data
    neg = df.copy()
    neg["y"] = neg["y"] - 10
    nfr = h2o.H2OFrame(neg)
    with pytest.raises(ValueError, match="greater than 0"):
        GLM(family="gamma").train(x=["a"], y="y", training_frame=nfr)
    with pytest.raises(ValueError, match="response >= 0"):
        GLM(family="poisson").train(x=["a"], y="y", training_frame=nfr)
    with pytest.raises(ValueError, match="theta"):
        GLM(family="negativebinomial", theta=2.0).train(x=["a"], y="y", training_frame=fr)
    with pytest.raises(ValueError, match="between 0 and 1"):
        GLM(family="fractionalbinomial").train(x=["a"], y="y", training_frame=fr)
    with pytest.raises(TypeError):
        GLM(generate_variable_inflation_factors=True)      # not a parameter of the reference GLM
