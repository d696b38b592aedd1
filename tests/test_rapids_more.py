"""Rapids prims the reference client sends for model utilities
(PermutationVarImp, makeLeaderboard, model.reset.threshold, sumaxis,
h2o.mad, mode, rename, millis) -- checked against numpy / the in-process
API."""
import numpy as np
import pandas as pd

import h2o3_amd as h2o
from h2o3_amd.core import dkv
from h2o3_amd.core.frame import H2OFrame
from h2o3_amd.core.rapids import rapids
from h2o3_amd.estimators import H2OGradientBoostingEstimator


def test_model_and_reducer_prims():
    h2o.init()
    rng = np.random.default_rng(0)
    n = 300
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.choice(list("xyz"), n)})
    df["y"] = np.where(df.a + df.b > 0, "p", "n")
    fr = H2OFrame(df)
    fr["c"] = fr["c"].asfactor()
    fr["y"] = fr["y"].asfactor()
    dkv.put("rp.hex", fr)
    m = H2OGradientBoostingEstimator(ntrees=3, model_id="rp_gbm", seed=1)
    m.train(x=["a", "b", "c"], y="y", training_frame=fr)
    dkv.put("rp_gbm", m)
    pvi = rapids('(PermutationVarImp rp_gbm rp.hex "AUTO" 1000 1 [] 1)')
    assert pvi.nrow == 3
    rs = rapids("(sumaxis (cols rp.hex [0 1]) 1 1)").as_data_frame().iloc[:, 0].values
    np.testing.assert_allclose(rs, df.a + df.b, rtol=1e-5, atol=1e-5)
    cs = rapids("(sumaxis (cols rp.hex [0 1]) 1 0)").as_data_frame().values[0]
    np.testing.assert_allclose(cs, [df.a.sum(), df.b.sum()], rtol=1e-5)
    old = rapids("(model.reset.threshold rp_gbm 0.99)").as_data_frame().values[0, 0]
    assert 0 < old < 1
    p = m.predict(fr).as_data_frame()
    assert (p["predict"] == np.where(p["p"] >= 0.99, "p", "n")).all()
    x = df.a.values
    np.testing.assert_allclose(rapids('(h2o.mad (cols rp.hex [0]) "interpolate" 1.4826)'),
                               1.4826 * np.median(np.abs(x - np.median(x))), rtol=1e-4)
    assert rapids("(mode (cols rp.hex [2]))") == float(np.argmax(np.bincount(pd.Categorical(df.c).codes)))
    lb = rapids('(makeLeaderboard ["rp_gbm"] "rp.hex" "AUTO" [] "AUTO")')
    assert lb.nrow == 1
    rapids('(rename "rp.hex" "rp2.hex")')
    assert dkv.get("rp2.hex") is not None and dkv.get("rp.hex") is None
    assert rapids("(millis)") > 1.6e12


def test_perfect_auc_and_ddply():
    from sklearn.metrics import roc_auc_score
    h2o.init()
    rng = np.random.default_rng(1)
    n = 200
    df = pd.DataFrame({"p": rng.random(n), "y": rng.integers(0, 2, n), "g": rng.choice(list("ab"), n),
                       "v": rng.normal(size=n)})
    fr = H2OFrame(df)
    fr["g"] = fr["g"].asfactor()
    dkv.put("dd.hex", fr)
    np.testing.assert_allclose(rapids("(perfectAUC (cols dd.hex [0]) (cols dd.hex [1]))"),
                               roc_auc_score(df.y, df.p), rtol=1e-9)
    out = rapids("(ddply dd.hex [2] { x . (mean (cols x 3) 1 0) })").as_data_frame()
    np.testing.assert_allclose(out["ddply_C1"].values, df.groupby("g").v.mean().values, rtol=1e-5)


def test_isotonic_pav_and_grouped_permute():
    h2o.init()
    rng = np.random.default_rng(2)
    n = 100
    x = rng.random(n)
    dkv.put("pav.hex", H2OFrame(pd.DataFrame({"y": x + rng.normal(size=n) * 0.1, "x": x, "w": np.ones(n)})))
    out = rapids("(isotonic.pav pav.hex)").as_data_frame()
    assert (np.diff(out["y"].values) >= -1e-12).all() and (np.diff(out["x"].values) >= 0).all()
    df = pd.DataFrame({"g": [1, 1, 1, 2, 2], "side": [0, 1, 1, 0, 1], "amt": [5.0, 6, 7, 8, 9], "id": [10, 11, 12, 13, 14]})
    dkv.put("gp.hex", H2OFrame(df))
    gp = rapids("(grouped_permute gp.hex 2 [0] 1 3)").as_data_frame()
    assert len(gp) == 2 + 1 and list(gp.columns) == ["g", "In", "Out", "InAmnt", "OutAmnt"]


def test_rowwise_apply_prod_and_row_assign():
    """apply(margin=1) with a reducer runs as one device reduction (matches
    the per-row loop), prod is exact, := with a row list scatters once."""
    import numpy as np
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.core import dkv, rapids
    h2o.init(device="cpu", verbose=False)
    rng = np.random.default_rng(0)
    df = pd.DataFrame(rng.normal(size=(50, 3)), columns=list("abc"))
    df.loc[3, "a"] = np.nan
    fr = h2o.H2OFrame(df)
    fr.frame_id = "RW"
    dkv.put("RW", fr)
    fast = rapids.rapids("(apply RW 1 {x . (sum x)})").as_data_frame().iloc[:, 0].values
    loop = rapids.rapids("(apply RW 1 {x . (+ (sum x) 0)})").as_data_frame().iloc[:, 0].values
    np.testing.assert_allclose(fast, loop, equal_nan=True)
    np.testing.assert_allclose(fast, df.sum(1, skipna=False).values, rtol=1e-5, atol=1e-6, equal_nan=True)
    m = rapids.rapids("(apply RW 1 {x . (mean x 1)})").as_data_frame().iloc[:, 0].values
    np.testing.assert_allclose(m, df.mean(1).values, rtol=1e-5, atol=1e-6)
    sd = rapids.rapids("(apply RW 1 {x . (sd x 1)})").as_data_frame().iloc[:, 0].values
    np.testing.assert_allclose(sd, df.std(1).values, rtol=1e-5, atol=1e-6)
    small = h2o.H2OFrame(pd.DataFrame({"v": [1.5, 2.0, -3.0, 4.0]}))
    small.frame_id = "PR"
    dkv.put("PR", small)
    assert rapids.rapids("(prod PR)") == -36.0
    r = rapids.rapids("(:= RW 7 [1] [0 5 49])").as_data_frame()["b"]
    assert r[0] == 7 and r[5] == 7 and r[49] == 7 and r[1] != 7
