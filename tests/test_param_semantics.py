"""Parameter semantics pinned to the reference's rules (not only "the model
changes"): early stopping (hex/ScoreKeeper.java:278 stopEarly), GBM
learn_rate_annealing (GBM.java:726 effective_learning_rate and the 1e-6
stop at :586), class_sampling_factors with balance_classes (the training
class distribution and the probability correction back to the priors,
GenModel.correctProbabilities).  Exact numbers follow from the rules on
crafted data; where the reference ships no fixture the expected values are
derived in the test ("parity unpinned" against reference outputs)."""
import math

import numpy as np
import pandas as pd
import pytest

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OGradientBoostingEstimator
from h2o3_amd.models.base import ScoreKeeper


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2o.init(verbose=False)


def _ref_stop(h, k, tol, less, lb0=False):
    """Independent transcription of ScoreKeeper.stopEarly over a history
    that excludes the initial (0-iteration) scoring event."""
    n = len(h)
    if k == 0 or n < 2 * k:
        return False
    avg = [sum(h[n - 2 * k + i + j] for j in range(k)) / k for i in range(k + 1)]
    if any(math.isnan(a) for a in avg):
        return False
    last, new = avg[0], avg[1:]
    if lb0 and last == 0.0:
        return True
    ext = min(new) if less else max(new)
    sg = lambda v: (v > 0) - (v < 0)  # noqa: E731
    if sg(max(avg)) != sg(min(avg)) or sg(ext) != sg(last):
        return False
    if last == 0:
        return False
    r = ext / last
    return r >= 1 - tol if less else r <= 1 + tol


@pytest.mark.parametrize("hist,k,tol,less,metric,expect", [
    ([1.0, 0.9, 0.8, 0.79, 0.789], 2, 0.01, True, "mse", False),      # 0.7895 / 0.85 = 0.929 < 0.99
    ([1.0, 0.9, 0.8, 0.79, 0.789], 2, 0.1, True, "mse", True),
    ([0.7, 0.8, 0.85, 0.851, 0.851], 2, 0.01, False, "auc", False),   # 0.851 / 0.825 = 1.03 > 1.01
    ([0.7, 0.8, 0.85, 0.851, 0.851], 2, 0.05, False, "auc", True),
    ([0.2, 0.1, 0.0, 0.0, 0.0], 1, 0.0, True, "misclassification", True),   # lower bound 0 reached
    ([0.2, 0.1, 0.0, 0.0, 0.0], 1, 0.0, True, "deviance", False),           # not bounded: 0 / 0
    ([0.3, 0.2, -0.1, 0.1], 1, 0.5, True, "deviance", False),                # mixed signs
    ([1.0, float("nan"), 0.5, 0.5], 1, 0.5, True, "mse", True),              # NaN outside the windows
    ([1.0, 0.5, float("nan"), 0.5], 1, 0.5, True, "mse", False),
    ([1.0, 1.0, 1.0], 2, 0.0, True, "mse", False),                           # fewer than 2k events
])
def test_stop_early_is_the_reference_rule(hist, k, tol, less, metric, expect):
    lb0 = metric in ("mse", "auc", "misclassification")
    assert _ref_stop(hist, k, tol, less, lb0) == expect
    assert ScoreKeeper.stop_early(hist, k, tol, less, metric=metric) == expect


@pytest.mark.parametrize("metric,key,less", [("MSE", "training_rmse", True), ("logloss", "training_logloss", True),
                                             ("AUC", "training_auc", False),
                                             ("misclassification", "training_classification_error", True)])
def test_gbm_stops_exactly_where_the_rule_fires(metric, key, less):
    """score_each_iteration + stopping_rounds: the model keeps exactly the
    trees up to the first scoring event where stopEarly fires on the
    history of `metric` (MSE replayed from the RMSE column squared)."""
    rng = np.random.default_rng(4)
    n = 600
    X = rng.normal(size=(n, 3))
    yb = np.where(rng.random(n) < 1 / (1 + np.exp(-(X[:, 0] + 0.3 * rng.normal(size=n)))), "a", "b")
    df = pd.DataFrame(X, columns=["x0", "x1", "x2"])
    df["y"] = yb
    fr = h2o.H2OFrame(df)
    k, tol = 2, 0.02
    m = H2OGradientBoostingEstimator(ntrees=60, max_depth=3, learn_rate=0.3, seed=1, score_each_iteration=True,
                                     stopping_rounds=k, stopping_metric=metric, stopping_tolerance=tol)
    m.train(x=["x0", "x1", "x2"], y="y", training_frame=fr)
    sh = m.scoring_history()
    vals = [float(v) for v in sh[key].values if v == v]
    if metric == "MSE":
        vals = [v * v for v in vals]
    lb0 = metric != "deviance"
    stop_at = next((i + 1 for i in range(len(vals)) if _ref_stop(vals[:i + 1], k, tol, less, lb0)), None)
    ntrees = m.ntrees_built
    if stop_at is None:
        assert ntrees == 60
    else:
        assert ntrees == stop_at < 60, (ntrees, stop_at)


def test_learn_rate_annealing_effective_rate_per_tree():
    """Gaussian stumps on a two-level step: tree t's leaves are the mean
    residuals times learn_rate * annealing^(t - 1) (the first tree uses
    learn_rate / annealing, GBM.java:726 with _ntrees = trees already built)."""
    x = np.linspace(0, 1, 400)
    y = np.where(x < 0.5, 0.0, 10.0)
    fr = h2o.H2OFrame(pd.DataFrame({"x": x, "y": y}))
    lr, a = 0.2, 0.5
    m = H2OGradientBoostingEstimator(ntrees=3, max_depth=1, learn_rate=lr, learn_rate_annealing=a, seed=1,
                                     min_rows=1, distribution="gaussian")
    m.train(x=["x"], y="y", training_frame=fr)
    f, want = 5.0, []
    for t in range(3):
        f = f + lr * a ** (t - 1) * (10.0 - f)          # right leaf (left is symmetric)
        want.append(f)
    p = m.predict(fr).as_data_frame()["predict"].values
    assert p[-1] == pytest.approx(want[-1], rel=1e-5)
    assert p[0] == pytest.approx(10.0 - want[-1], rel=1e-5, abs=1e-4)


def test_learn_rate_annealing_stops_below_1e6():
    """GBMTest.java:2996-3016 shape: annealing 0.5 stops the model before
    ntrees once learn_rate * 0.5^(ntrees - 1) < 1e-6: 0.1 * 0.5^17 < 1e-6
    after the 18th tree."""
    rng = np.random.default_rng(2)
    df = pd.DataFrame({"x": rng.normal(size=300)})
    df["y"] = np.where(df.x + 0.5 * rng.normal(size=300) > 0, "p", "q")
    m = H2OGradientBoostingEstimator(ntrees=100, max_depth=3, learn_rate=0.1, learn_rate_annealing=0.5, seed=0,
                                     min_rows=10)
    m.train(x=["x"], y="y", training_frame=h2o.H2OFrame(df))
    assert m.ntrees_built == 18


def test_sampling_factors_rule():
    """MRUtils.sampleFrameStratified factors: default = every class up to the
    majority count; user factors taken as given; both scaled down so the
    balanced size stays <= max_after_balance_size x the original."""
    from h2o3_amd.models.balance import sampling_factors
    c = np.array([900.0, 100.0])
    assert sampling_factors(c, None, 5.0) == pytest.approx([1.0, 9.0])
    assert sampling_factors(c, None, 1.5) == pytest.approx(np.array([1.0, 9.0]) * 1500 / 1800)
    assert sampling_factors(c, [1, 4], 5.0) == pytest.approx([1.0, 4.0])
    assert sampling_factors(c, [2, 4], 1.0) == pytest.approx(np.array([2.0, 4.0]) * 1000 / 2200)
    with pytest.raises(ValueError):
        sampling_factors(c, [1, 2, 3], 5.0)


def test_balance_classes_distributions_and_correction():
    """balance_classes + class_sampling_factors=[1, 4] on a 9:1 frame: the
    balanced frame holds exactly n0 + 4 n1 rows (integer factors), the model
    records prior [0.9, 0.1] and model distribution [0.9, 0.4] / 1.3, and
    predictions are corrected back so the mean P(minority) tracks the prior
    (not the balanced 0.31)."""
    from h2o3_amd.models.balance import balance_frame, class_counts
    rng = np.random.default_rng(7)
    n = 2000
    x = rng.normal(size=n)
    y = np.where(np.arange(n) < n // 10, "min", "maj")
    x = x + np.where(y == "min", 0.8, 0.0)
    df = pd.DataFrame({"x": x, "y": y})
    fr = h2o.H2OFrame(df)
    fr["y"] = fr["y"].asfactor()
    dom = fr.vec("y").domain
    imin = dom.index("min")
    f = [1.0, 1.0]
    f[imin] = 4.0
    bal = balance_frame(fr, "y", f, seed=3)
    cb = class_counts(bal, "y")
    assert cb[imin] == 4 * (n // 10) and cb[1 - imin] == n - n // 10
    m = H2OGradientBoostingEstimator(ntrees=20, max_depth=3, seed=1, balance_classes=True,
                                     class_sampling_factors=f)
    m.train(x=["x"], y="y", training_frame=fr)
    prior = np.array(m._output["prior_class_distribution"])
    model = np.array(m._output["model_class_distribution"])
    assert prior[imin] == pytest.approx(0.1) and model[imin] == pytest.approx(0.4 / 1.3)
    p = m.predict(fr).as_data_frame()["min"].values
    assert abs(p.mean() - 0.1) < 0.03, p.mean()
    mu = H2OGradientBoostingEstimator(ntrees=20, max_depth=3, seed=1)
    mu.train(x=["x"], y="y", training_frame=fr)
    pu = mu.predict(fr).as_data_frame()["min"].values
    assert np.corrcoef(p, pu)[0, 1] > 0.9
