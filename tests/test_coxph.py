"""CoxPH vs an independent numpy/scipy maximisation of the Efron/Breslow
partial likelihood (parity unpinned against R survival: not installed)."""
import numpy as np
import pandas as pd
import pytest
from scipy.optimize import minimize

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OCoxProportionalHazardsEstimator


def _negll(beta, X, start, stop, ev, efron):
    eta = X @ beta
    r = np.exp(eta)
    ll = 0.0
    for t in np.unique(stop[ev == 1]):
        at = (stop == t) & (ev == 1)
        risk = (stop >= t) & (start < t)
        d = at.sum()
        R0 = r[risk].sum()
        D0 = r[at].sum()
        ll += eta[at].sum()
        for l in range(d):
            f = l / d if efron else 0.0
            ll -= np.log(R0 - f * D0)
    return -ll


def _data(n=400, seed=0, start=False):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 2))
    T = rng.exponential(1 / np.exp(0.7 * X[:, 0] - 0.5 * X[:, 1]))
    T = np.ceil(T * 10)  # integer times: exact ties in f32 and f64
    C = np.ceil(rng.exponential(20.0, n))
    stop = np.minimum(T, C)
    ev = (T <= C).astype(int)
    st = np.where(rng.random(n) < 0.3, np.floor(stop * 0.3), 0.0) if start else np.zeros(n)
    return pd.DataFrame({"x1": X[:, 0], "x2": X[:, 1], "start": st, "stop": stop, "event": ev})


@pytest.mark.parametrize("ties", ["efron", "breslow"])
@pytest.mark.parametrize("use_start", [False, True])
def test_coxph_matches_direct_maximisation(ties, use_start):
    h2o.init()
    df = _data(start=use_start)
    fr = h2o.H2OFrame(df)
    m = H2OCoxProportionalHazardsEstimator(stop_column="stop", start_column="start" if use_start else None, ties=ties)
    m.train(x=["x1", "x2"], y="event", training_frame=fr)
    X = df[["x1", "x2"]].values
    ref = minimize(_negll, np.zeros(2), args=(X, df.start.values if use_start else np.full(len(df), -np.inf),
                                              df.stop.values, df.event.values, ties == "efron"), method="BFGS",
                   options={"gtol": 1e-9})
    c = m.coef()
    np.testing.assert_allclose([c["x1"], c["x2"]], ref.x, atol=1e-4)
    assert m._output["loglik"] == pytest.approx(-ref.fun, rel=1e-6)
    assert 0.6 < m.concordance() < 0.9
    lp = m.predict(fr).as_data_frame()["lp"].values
    xb = X @ ref.x
    np.testing.assert_allclose(lp, xb - xb.mean(), atol=1e-3)


def test_coxph_stratified_and_categorical():
    h2o.init()
    df = _data(600, seed=3)
    rng = np.random.default_rng(3)
    df["g"] = rng.choice(["p", "q"], len(df))
    df["s"] = rng.choice(["s1", "s2"], len(df))
    fr = h2o.H2OFrame(df)
    m = H2OCoxProportionalHazardsEstimator(stop_column="stop", stratify_by=["s"])
    m.train(x=["x1", "x2", "g"], y="event", training_frame=fr)
    t = m._output["coefficients_table"]
    assert list(t["names"]) == ["g.q", "x1", "x2"]
    assert abs(m.coef()["x1"] - 0.7) < 0.25


@pytest.mark.parametrize("use_all", [False, True])
def test_coxph_h2o_mojo_roundtrip(use_all, tmp_path):
    """Reference-layout CoxPH MOJO (CoxPHMojoWriter layout: coef, x_mean_cat /
    x_mean_num blobs, strata_i keys) scored by the reference-layout reader
    equals the in-platform centred linear predictor."""
    from h2o3_amd.mojo import h2o_mojo
    h2o.init()
    df = _data(500, seed=5)
    rng = np.random.default_rng(5)
    df["g"] = rng.choice(["p", "q", "r"], len(df))
    df["s"] = rng.choice(["s1", "s2", "s3"], len(df))
    fr = h2o.H2OFrame(df)
    m = H2OCoxProportionalHazardsEstimator(stop_column="stop", stratify_by=["s"], use_all_factor_levels=use_all)
    m.train(x=["x1", "x2", "g"], y="event", training_frame=fr)
    ours = m.predict(fr).as_data_frame()["lp"].values
    mj = h2o_mojo.load(m.download_mojo(str(tmp_path), format="h2o"))
    assert mj.algo == "coxph" and mj.cox_strata_len == 1 and len(mj.cox_strata) == 3
    d32 = df.copy()
    for c in ("x1", "x2"):
        d32[c] = d32[c].astype(np.float32).astype(np.float64)
    theirs = mj.predict(d32)["lp"].values
    np.testing.assert_allclose(theirs, ours, atol=2e-5)


def test_segmented_sums_match_index_add():
    """_Seg (sort once, cumsum differences) == index_add_ into few bins."""
    import torch
    from h2o3_amd.models.coxph import _Seg
    g = torch.Generator().manual_seed(0)
    key = torch.randint(0, 7, (5000,), generator=g)
    key[:100] = 0
    v = torch.randn(5000, 3, generator=g, dtype=torch.float64)
    ref = torch.zeros(9, 3, dtype=torch.float64).index_add_(0, key, v)
    torch.testing.assert_close(_Seg(key, 9)(v), ref)
    torch.testing.assert_close(_Seg(key, 9)(v[:, 0]), ref[:, 0])


def test_coxph_baseline_hazard_breslow():
    """calc_cumhaz (CoxPH.java:503): Breslow baseline hazard at each distinct
    stop time = weighted events / risk still at stake, risks exp((x - mean).b)."""
    h2o.init()
    df = _data(300, seed=5)
    fr = h2o.H2OFrame(df)
    m = H2OCoxProportionalHazardsEstimator(stop_column="stop", ties="breslow")
    m.train(x=["x1", "x2"], y="event", training_frame=fr)
    b = np.array([m.coef()["x1"], m.coef()["x2"]])
    X = df[["x1", "x2"]].values
    r = np.exp((X - X.mean(0)) @ b)
    times = np.unique(df.stop.values)
    want_h = np.array([df.event.values[df.stop.values == t].sum() / r[df.stop.values >= t].sum() for t in times])
    bh = m.baseline_hazard_frame.as_data_frame()
    bs = m.baseline_survival_frame.as_data_frame()
    assert list(bh.columns) == ["t", "baseline hazard"]
    np.testing.assert_allclose(bh["t"].values, times)
    np.testing.assert_allclose(bh["baseline hazard"].values, want_h, rtol=1e-6, atol=1e-12)
    np.testing.assert_allclose(bs["baseline survival"].values, np.exp(-np.cumsum(want_h)), rtol=1e-6)
    ch = m._output["cumhaz_0"]
    assert np.all(np.diff(ch) >= 0) and ch[-1] == pytest.approx(np.cumsum(want_h)[-1], rel=1e-6)


def test_coxph_interactions_and_interactions_only():
    h2o.init()
    df = _data(500, seed=6)
    df["x3"] = np.random.default_rng(6).normal(size=len(df))
    fr = h2o.H2OFrame(df)
    m = H2OCoxProportionalHazardsEstimator(stop_column="stop", interaction_pairs=[("x1", "x3")],
                                           interactions_only=["x3"])
    m.train(x=["x1", "x2", "x3"], y="event", training_frame=fr)
    names = list(m._output["coefficients_table"]["names"])
    assert "x3" not in names and "x1_x3" in names and "x1" in names
    # the interaction column is the product of its parents
    X = np.c_[df.x1, df.x2, df.x1 * df.x3]
    ref = minimize(_negll, np.zeros(3), args=(X, np.full(len(df), -np.inf), df.stop.values, df.event.values, True),
                   method="BFGS", options={"gtol": 1e-9})
    c = m.coef()
    np.testing.assert_allclose([c["x1"], c["x2"], c["x1_x3"]], ref.x, atol=1e-4)
    with pytest.raises(ValueError, match="interactions_only"):
        H2OCoxProportionalHazardsEstimator(stop_column="stop", interactions_only=["zz"]).train(
            x=["x1", "x2"], y="event", training_frame=fr)
