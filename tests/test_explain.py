"""Partial dependence, permutation importance, H statistic, explain()."""
import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator


def _fr(n=800, seed=1):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4))
    df = pd.DataFrame(X, columns=list("abcd"))
    df["k"] = rng.choice(["u", "v"], n)
    df["y"] = 3 * X[:, 0] + X[:, 1] * X[:, 2] * 2 + (df["k"] == "u") + rng.normal(scale=0.1, size=n)
    return h2o.H2OFrame(df)


def test_pdp_linear_model_is_linear():
    h2o.init()
    fr = _fr()
    m = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0.0)
    m.train(x=list("abcd") + ["k"], y="y", training_frame=fr)
    pdp = m.partial_plot(fr, cols=["a", "k"], nbins=10, plot=False)
    a = pdp[0]
    assert list(a.columns) == ["a", "mean_response", "stddev_response", "std_error_mean_response"]
    slope = np.diff(a["mean_response"]) / np.diff(a["a"])
    np.testing.assert_allclose(slope, m.coef()["a"], rtol=1e-3)
    assert len(pdp[1]) == 2 and set(pdp[1]["k"]) == {"u", "v"}


def test_permutation_importance_ranks_signal_first():
    h2o.init()
    fr = _fr()
    m = H2OGradientBoostingEstimator(ntrees=20, max_depth=4, seed=1)
    m.train(x=list("abcd") + ["k"], y="y", training_frame=fr)
    pi = m.permutation_importance(fr, n_samples=-1, seed=3)
    assert pi["Variable"].iloc[0] == "a"
    assert pi.set_index("Variable").loc["d", "Scaled Importance"] < 0.05
    pr = m.permutation_importance(fr, n_repeats=2, seed=3)
    assert list(pr.columns) == ["Variable", "Run 1", "Run 2"]


def test_h_statistic_detects_interaction():
    h2o.init()
    fr = _fr()
    m = H2OGradientBoostingEstimator(ntrees=30, max_depth=4, seed=1)
    m.train(x=list("abcd") + ["k"], y="y", training_frame=fr)
    h_bc = m.h(fr, ["b", "c"])
    h_ad = m.h(fr, ["a", "d"])
    assert h_bc > 0.3 and h_ad < h_bc


def test_explain_tables():
    h2o.init()
    fr = _fr()
    m = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1)
    m.train(x=list("abcd") + ["k"], y="y", training_frame=fr)
    ex = h2o.explain(m, fr, top_n_features=2)
    assert {"varimp", "pdp", "shap_summary", "residual_analysis"} <= set(ex)
    assert len(ex["pdp"]) == 2
    er = h2o.explain_row(m, fr, 3)
    assert "shap_explain_row" in er


def test_explain_plots_and_heatmaps(tmp_path):
    """explain(plot=True) draws every section (matplotlib Agg); heatmap data
    follows the reference's varimp / model_correlation definitions."""
    import matplotlib
    matplotlib.use("Agg")
    from h2o3_amd.models import explain_plots as xp
    h2o.init()
    fr = _fr()
    x = list("abcd") + ["k"]
    m1 = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1)
    m1.train(x=x, y="y", training_frame=fr)
    m2 = H2OGradientBoostingEstimator(ntrees=5, max_depth=2, seed=2)
    m2.train(x=x, y="y", training_frame=fr)
    m3 = H2OGradientBoostingEstimator(ntrees=8, max_depth=4, seed=3)
    m3.train(x=x, y="y", training_frame=fr)
    ex = h2o.explain(m1, fr, top_n_features=2, plot=True)
    figs = ex["plots"]
    assert {"pdp", "ice", "shap_summary", "learning_curve"} <= set(figs)
    for f in list(figs["pdp"].values()) + [figs["shap_summary"], figs["learning_curve"]]:
        assert hasattr(f, "savefig")
    figs["shap_summary"].savefig(tmp_path / "shap.png")
    assert (tmp_path / "shap.png").stat().st_size > 1000
    vi = xp.varimp([m1, m2, m3])
    assert set(vi.columns) == {m1.model_id, m2.model_id, m3.model_id}
    assert np.allclose(vi.max(0).values, 1.0)      # each model scaled to its top variable
    mc = xp.model_correlation([m1, m2, m3], fr)
    assert np.allclose(np.diag(mc.values), 1.0) and (mc.values <= 1 + 1e-9).all()
    exm = h2o.explain([m1, m2, m3], fr, top_n_features=1, plot=True)
    assert "varimp_heatmap" in exm["plots"] and "model_correlation_heatmap" in exm["plots"]
    er = m1.explain_row(fr, 2, plot=True)
    assert hasattr(er["plots"]["shap_explain_row"], "savefig")
    import matplotlib.pyplot as plt
    plt.close("all")
