"""Isotonic regression, target encoding, aggregator."""
import numpy as np
import pandas as pd
import pytest

import h2o3_amd as h2o
from h2o3_amd.estimators import (H2OAggregatorEstimator, H2OIsotonicRegressionEstimator,
                                 H2OTargetEncoderEstimator)
from h2o3_amd.models.isotonic import pava


def test_pava_matches_sklearn():
    from sklearn.isotonic import IsotonicRegression
    rng = np.random.default_rng(0)
    x = np.sort(rng.uniform(0, 10, 300))
    y = np.log1p(x) + rng.normal(scale=0.3, size=300)
    h2o.init()
    fr = h2o.H2OFrame(pd.DataFrame({"x": x, "y": y}))
    m = H2OIsotonicRegressionEstimator()
    m.train(x="x", y="y", training_frame=fr)
    p = m.predict(fr).as_data_frame()["predict"].values
    ref = IsotonicRegression().fit(x, y).predict(x)
    np.testing.assert_allclose(p, ref, atol=1e-4)
    # out of bounds
    t = h2o.H2OFrame(pd.DataFrame({"x": [-1.0, 5.0, 11.0]}))
    p2 = m.predict(t).as_data_frame()["predict"].values
    assert np.isnan(p2[0]) and np.isnan(p2[2]) and not np.isnan(p2[1])
    mc = H2OIsotonicRegressionEstimator(out_of_bounds="clip")
    mc.train(x="x", y="y", training_frame=fr)
    p3 = mc.predict(t).as_data_frame()["predict"].values
    assert p3[0] == pytest.approx(ref[0], abs=1e-4) and p3[2] == pytest.approx(ref[-1], abs=1e-4)


def _te_frame():
    rng = np.random.default_rng(1)
    n = 1000
    k = rng.choice(["a", "b", "c", "d"], n, p=[0.5, 0.3, 0.15, 0.05])
    rate = {"a": 0.2, "b": 0.5, "c": 0.8, "d": 0.9}
    y = np.array([rng.random() < rate[v] for v in k])
    df = pd.DataFrame({"k": k, "y": np.where(y, "yes", "no"), "num": rng.normal(size=n),
                       "fold": rng.integers(0, 3, n)})
    return df


def test_target_encoder_none_kfold_loo():
    h2o.init()
    df = _te_frame()
    fr = h2o.H2OFrame(df)
    fr["y"] = fr["y"].asfactor()
    te = H2OTargetEncoderEstimator(noise=0.0)
    te.train(x=["k"], y="y", training_frame=fr)
    out = te.transform(fr).as_data_frame()
    exp = df.groupby("k")["y"].apply(lambda s: (s == "yes").mean())
    np.testing.assert_allclose(out["k_te"].values, df["k"].map(exp).values, atol=1e-6)
    # leave-one-out on training
    te2 = H2OTargetEncoderEstimator(noise=0.0, data_leakage_handling="LeaveOneOut")
    te2.train(x=["k"], y="y", training_frame=fr)
    o2 = te2.transform(fr, as_training=True).as_data_frame()
    yy = (df["y"] == "yes").astype(float)
    g = df.assign(yy=yy).groupby("k")["yy"]
    loo = (df["k"].map(g.sum()) - yy) / (df["k"].map(g.count()) - 1)
    np.testing.assert_allclose(o2["k_te"].values, loo.values, atol=1e-6)
    # kfold: out-of-fold means
    te3 = H2OTargetEncoderEstimator(noise=0.0, data_leakage_handling="KFold", fold_column="fold")
    te3.train(x=["k"], y="y", training_frame=fr)
    o3 = te3.transform(fr, as_training=True).as_data_frame()
    for f in range(3):
        tr = df[df.fold != f]
        m = tr.groupby("k")["y"].apply(lambda s: (s == "yes").mean())
        sel = df.fold == f
        np.testing.assert_allclose(o3.loc[sel.values, "k_te"].values, df.loc[sel, "k"].map(m).values, atol=1e-6)
    # blending pulls small levels towards the prior
    te4 = H2OTargetEncoderEstimator(noise=0.0, blending=True, inflection_point=100, smoothing=10)
    te4.train(x=["k"], y="y", training_frame=fr)
    o4 = te4.transform(fr).as_data_frame()
    prior = (df.y == "yes").mean()
    d_raw = exp["d"]
    d_bl = o4.loc[(df.k == "d").values, "k_te"].iloc[0]
    assert abs(d_bl - prior) < abs(d_raw - prior)


def test_aggregator_reduces_rows():
    h2o.init()
    rng = np.random.default_rng(2)
    centers = rng.normal(scale=10, size=(20, 3))
    X = np.concatenate([c + rng.normal(scale=0.1, size=(300, 3)) for c in centers])
    fr = h2o.H2OFrame(pd.DataFrame(X, columns=["a", "b", "c"]))
    ag = H2OAggregatorEstimator(target_num_exemplars=100, rel_tol_num_exemplars=0.5, seed=1)
    ag.train(training_frame=fr)
    af = ag.aggregated_frame.as_data_frame()
    assert 50 <= len(af) <= 150
    assert int(af["counts"].sum()) == 6000


def test_aggregator_blocked_leader_matches_sequential():
    """_leader (blocked: GPU distances to earlier blocks' exemplars, pairwise
    closeness within a block) picks exactly the exemplars of the plain
    sequential leader pass."""
    import numpy as np
    import torch
    from h2o3_amd.models.aggregator import _leader
    g = torch.Generator().manual_seed(5)
    C = torch.rand((3000, 4), generator=g, dtype=torch.float64)
    r2 = 0.05
    ref = []
    Cn = C.numpy()
    for i in range(Cn.shape[0]):
        if ref and (((Cn[ref] - Cn[i]) ** 2).sum(1) <= r2).any():
            continue
        ref.append(i)
    assert _leader(C, r2, block=256) == ref
    assert _leader(C, r2, budget=10, block=64) == ref[:11]
