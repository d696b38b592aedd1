"""Shard-local munging prims (core/dist_ops.py) at one rank against numpy /
pandas references of the reference semantics (Quantile.java, AstTable,
AstPivot, AstMelt, AstRankWithinGroupBy, CreateInteractions,
AstDropDuplicates).  The 2-rank runs of the same prims are compared with
the one-rank results in tests/test_distributed.py (dist_worker.py)."""
import math

import numpy as np
import pandas as pd
import pytest
import torch

import h2o3_amd as h2o
from h2o3_amd.core import dist_ops
from h2o3_amd.core.vec import T_REAL, Vec


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2o.init(verbose=False)


def _df(n=3000, seed=3):
    rng = np.random.default_rng(seed)
    df = pd.DataFrame({"a": rng.integers(0, 5, n).astype(float), "b": rng.choice(["x", "y", "z"], n),
                       "v": rng.normal(size=n), "t": rng.integers(0, 50, n).astype(float)})
    df.loc[::17, "v"] = np.nan
    df.loc[::23, "a"] = np.nan
    return df


@pytest.mark.parametrize("method", ["interpolate", "low", "high", "average"])
def test_quantile_exact_vs_sorted(method):
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.normal(size=20000), np.full(3000, 0.25), rng.exponential(size=5000) * 1e6])
    probs = [0.0, 0.001, 0.1, 0.25, 0.333, 0.5, 0.75, 0.9, 0.999, 1.0]
    got = dist_ops.quantile_values(Vec(torch.tensor(x), T_REAL), probs, method)
    xs = np.sort(x)
    n = len(xs)
    for p, g in zip(probs, got):
        h = (n - 1) * p
        lo = int(math.floor(h))
        hi = min(lo + 1, n - 1)
        ref = {"low": xs[lo], "high": xs[hi], "average": (xs[lo] + xs[hi]) / 2 if h != lo else xs[lo],
               "interpolate": xs[lo] + (h - lo) * (xs[hi] - xs[lo])}[method]
        assert g == pytest.approx(ref, rel=1e-12, abs=1e-12), (p, g, ref)


def test_weighted_quantile():
    rng = np.random.default_rng(1)
    x = rng.normal(size=12000)
    w = rng.random(12000)
    probs = [0.1, 0.5, 0.9]
    got = dist_ops.quantile_values(Vec(torch.tensor(x), T_REAL), probs, weights=torch.tensor(w))
    o = np.argsort(x, kind="stable")
    cw = np.cumsum(w[o])
    for p, g in zip(probs, got):
        i = min(int(np.searchsorted(cw, p * cw[-1])), len(x) - 1)
        assert g == pytest.approx(x[o][i], rel=1e-12)


def test_table_unique_hist():
    df = _df()
    fr = h2o.H2OFrame(df)
    t1 = fr["t"].table().as_data_frame()
    assert list(t1.columns) == ["t", "Count"]                 # integer fast path (AstTable)
    ref = df.groupby("t").size()
    assert t1["Count"].tolist() == ref.tolist() and t1["t"].tolist() == ref.index.tolist()
    tv = fr["v"].table().as_data_frame()
    assert list(tv.columns) == ["v", "Counts"]
    t2 = fr[["b", "a"]].table().as_data_frame()
    ref2 = df.dropna(subset=["a"]).groupby(["b", "a"]).size().reset_index(name="Counts")
    assert t2["Counts"].tolist() == ref2["Counts"].tolist()
    assert t2["b"].tolist() == ref2["b"].tolist()
    sp = fr[["b", "a"]].table(dense=False).as_data_frame()
    piv = ref2.pivot(index="b", columns="a", values="Counts").fillna(0)
    assert list(sp.columns) == ["b"] + [repr(float(c)) for c in piv.columns]
    assert np.array_equal(sp.iloc[:, 1:].values, piv.values)
    u = fr["b"].unique().as_data_frame()
    assert sorted(u.iloc[:, 0].tolist()) == ["x", "y", "z"]
    h = fr["v"].hist(breaks=10)
    hd = h.as_data_frame()
    assert hd["counts"].sum() == df.v.notna().sum()


def test_cor_cov():
    df = _df()
    fr = h2o.H2OFrame(df[["v", "t"]])
    assert fr["t"].cor(fr["t"]) == pytest.approx(1.0)
    c = fr.cor(use="complete.obs").as_data_frame().values
    ref = df[["v", "t"]].dropna().corr().values
    assert np.allclose(c, ref, atol=1e-12)
    sp = fr.cor(use="complete.obs", method="Spearman").as_data_frame().values
    d2 = df[["v", "t"]].dropna()
    rk = np.argsort(np.argsort(d2.values, axis=0, kind="stable"), axis=0, kind="stable")
    assert np.allclose(sp, np.corrcoef(rk.T), atol=1e-12)
    cv = h2o.H2OFrame(df[["t"]].assign(u=df.t * 2 + 1)).var().as_data_frame().values
    assert np.allclose(cv, np.cov(np.stack([df.t.values, df.t.values * 2 + 1])), atol=1e-9)


def test_drop_duplicates_pivot_melt():
    df = _df(800)
    fr = h2o.H2OFrame(df)
    for keep in ("first", "last"):
        got = fr.drop_duplicates(["a", "b"], keep=keep).as_data_frame()
        ref = df.drop_duplicates(["a", "b"], keep=keep)
        assert got["t"].tolist() == ref["t"].tolist()
    dp = pd.DataFrame({"i": [3.0, 1.0, 1.0, 2.0, 3.0, 1.0], "c": ["p", "q", "p", "p", "q", "q"],
                       "v": [np.nan, 2.0, 3.0, 4.0, 5.0, 6.0]})
    pv = h2o.H2OFrame(dp).pivot("i", "c", "v").as_data_frame()
    assert list(pv.columns) == ["i", "p", "q"]
    assert pv["i"].tolist() == [1.0, 2.0, 3.0]
    assert pv["p"].tolist()[:2] == [3.0, 4.0] and math.isnan(pv["p"].tolist()[2])     # first non-NA
    q = pv["q"].tolist()
    assert q[0] == 2.0 and math.isnan(q[1]) and q[2] == 5.0
    dm = pd.DataFrame({"id": [1.0, 2.0], "x": [10.0, np.nan], "y": [30.0, 40.0]})
    m = h2o.H2OFrame(dm).melt(["id"], skipna=False).as_data_frame()
    assert m["id"].tolist() == [1.0, 1.0, 2.0, 2.0]                                   # row-major (AstMelt)
    assert m["variable"].tolist() == ["x", "y", "x", "y"]
    m2 = h2o.H2OFrame(dm).melt(["id"], skipna=True).as_data_frame()
    assert m2["value"].tolist() == [10.0, 30.0, 40.0]


def test_rank_within_group_by_and_interaction():
    df = _df(600)
    fr = h2o.H2OFrame(df)
    r = fr.rank_within_group_by(["b"], ["t"], [True], "rk").as_data_frame()
    for b, g in r.groupby("b"):
        assert g["t"].is_monotonic_increasing
        assert g["rk"].tolist() == list(range(1, len(g) + 1))
    r2 = fr.rank_within_group_by(["b"], ["v"], [False], "rk").as_data_frame()
    assert r2["rk"].isna().sum() == df.v.isna().sum()
    di = pd.DataFrame({"p": ["a", "a", "b", "b", "b", "c"], "q": ["u", "u", "v", "u", "v", "v"]})
    fi = h2o.H2OFrame(di)
    fi["p"] = fi["p"].asfactor()
    fi["q"] = fi["q"].asfactor()
    it = fi.interaction(["p", "q"], pairwise=False, max_factors=2, min_occurrence=1)
    dom = it._vecs[0].domain
    assert dom[:2] == ["a_u", "b_v"] and dom[-1] == "other"
    assert it.as_data_frame().iloc[:, 0].tolist() == ["a_u", "a_u", "b_v", "other", "b_v", "other"]
