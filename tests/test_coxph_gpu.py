"""CoxPH risk-set terms on the GPU (grouped-sum kernel for the [n, P]
segment sums, row-contiguous scans, split-K small Grams) against the same
terms on the host, and a GPU fit against the host fit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _data(n, P, seed, start):
    g = np.random.default_rng(seed)
    X = g.normal(size=(n, P))
    T = np.ceil(g.exponential(1 / np.exp(0.5 * X[:, 0] - 0.3 * X[:, 1])) * 50)   # ties
    C = np.ceil(g.exponential(100.0, n))
    stop = np.minimum(T, C)
    ev = (T <= C).astype(float)
    st = np.where(g.random(n) < 0.3, np.floor(stop * 0.3), 0.0) if start else None
    w = g.uniform(0.5, 2.0, n)
    return X, st, stop, ev, w


@pytest.mark.parametrize("start,efron", [(False, True), (True, True), (False, False)])
def test_coxph_terms_gpu_match_host(start, efron):
    from h2o3_amd.models.coxph import _Stratum
    X, st, stop, ev, w = _data(120_000, 10, 3, start)
    beta = np.linspace(-0.2, 0.3, 10)
    out = []
    for dev in ("cpu", "cuda"):
        t = lambda a: None if a is None else torch.as_tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
        s = _Stratum(t(X), t(st), t(stop), t(ev), t(w), efron)
        ll, gr, H = s.terms(t(beta))
        out.append((ll, gr.cpu().numpy(), H.cpu().numpy()))
    (l0, g0, H0), (l1, g1, H1) = out
    assert abs(l0 - l1) <= 1e-9 * abs(l0)
    np.testing.assert_allclose(g1, g0, rtol=1e-8, atol=1e-8 * np.abs(g0).max())
    np.testing.assert_allclose(H1, H0, rtol=1e-8, atol=1e-8 * np.abs(H0).max())


def test_coxph_fit_gpu():
    assert torch.cuda.is_available()
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.estimators import H2OCoxProportionalHazardsEstimator
    h2o.init(verbose=False)
    X, _, stop, ev, _ = _data(200_000, 4, 5, False)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(4)])
    df["stop"], df["event"] = stop, ev.astype(int)
    m = H2OCoxProportionalHazardsEstimator(stop_column="stop")
    m.train(x=[f"x{i}" for i in range(4)], y="event", training_frame=h2o.H2OFrame(df))
    coef = m.coef()
    assert abs(coef["x0"] - 0.5) < 0.05 and abs(coef["x1"] + 0.3) < 0.05, coef
