"""Worker for tests/test_distributed_gpu.py: one rank of a gloo cloud whose
ranks all share cuda:0 (RCCL refuses two ranks on one device, gloo moves the
GPU tensors through the host).  Every HIP kernel of the multi-rank tree path
runs: feature reduce-scatter of level histograms, and for DRF with mtries the
node-sharded pair path (pair histograms reduce-scattered by node, per-rank
pair scoring / selection, all-gather of the per-node records), which only
works when every rank draws the same column sample and pads the node count
the same way.

Dumps the grown trees (per node: split feature, threshold, NA direction,
child ids) and predictions on the full frame to JSON (rank 0).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_df(n=20000, F=40, seed=11):
    import numpy as np
    import pandas as pd
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, F))
    X[rng.random((n, F)) < 0.02] = np.nan
    logit = 1.5 * np.nan_to_num(X[:, 0]) - np.nan_to_num(X[:, 1]) + 0.7 * np.nan_to_num(X[:, 2] * X[:, 3])
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(F)])
    df["c0"] = np.array(list("abcdefghij"))[rng.integers(0, 10, n)]
    logit += np.where(df["c0"].isin(["a", "c", "f"]), 1.0, -0.5)
    df["y"] = np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "yes", "no")
    df["yr"] = logit + rng.normal(scale=0.3, size=n)
    # a 600-level categorical (histograms wider than 256 bins: the narrow /
    # wide pair scoring split) and 0/1 row weights (zero-weight rows skip
    # their code gathers)
    lv = rng.integers(0, 600, n)
    df["hc"] = np.array([f"h{v}" for v in range(600)])[lv]
    df["yr"] += rng.normal(size=600)[lv]
    df["w01"] = (rng.random(n) > 0.2).astype(float)
    return df


def _trees(m):
    out = []
    for t in m._forest.trees:
        out.append({"feat": [int(v) for v in t.feat], "left": [int(v) for v in t.left],
                    "thr": [float(v) for v in t.thr]})
    return out


def run(out_path):
    import h2o3_amd as h2o
    from h2o3_amd.estimators import H2OGradientBoostingEstimator, H2ORandomForestEstimator
    h2o.init(verbose=False)
    from h2o3_amd.parallel import cloud
    assert cloud.device().type == "cuda" or os.environ.get("H2O3_WORKER_CPU_OK") == "1"
    df = make_df()
    fr = h2o.H2OFrame(df)
    x = [c for c in df.columns if c not in ("y", "yr", "hc", "w01")]
    res = {"world": cloud.world(), "backend": cloud.info()["backend"]}
    # DRF, mtries = sqrt(41) -> 6 of 41 features per node: the row-direct pair path
    drf = H2ORandomForestEstimator(ntrees=3, max_depth=8, seed=3, sample_rate=1.0, mtries=6, min_rows=20)
    drf.train(x=x, y="yr", training_frame=fr)
    res["drf_trees"] = _trees(drf)
    res["drf_pred"] = drf.predict(fr).as_data_frame()["predict"].tolist()
    # DRF on the all-pair-path layout: position-ordered response payload,
    # 600-level categorical, zero-weight rows
    drf2 = H2ORandomForestEstimator(ntrees=2, max_depth=10, seed=5, sample_rate=1.0, mtries=6, min_rows=10,
                                    weights_column="w01")
    drf2.train(x=x + ["hc"], y="yr", training_frame=fr)
    res["drf2_trees"] = _trees(drf2)
    # GBM binomial: level histograms reduce-scattered by feature
    gbm = H2OGradientBoostingEstimator(ntrees=4, max_depth=6, seed=1, min_rows=20)
    gbm.train(x=x, y="y", training_frame=fr)
    res["gbm_trees"] = _trees(gbm)
    res["gbm_logloss"] = gbm.logloss()
    # numeric-only frame: the packed-record split path (per-rank split_select2,
    # record + mask all-gather, async partition, look-ahead histograms)
    xn = [c for c in x if c != "c0"]
    gbm2 = H2OGradientBoostingEstimator(ntrees=4, max_depth=7, seed=1, min_rows=20)
    gbm2.train(x=xn, y="y", training_frame=fr)
    res["gbm2_trees"] = _trees(gbm2)
    res["gbm2_logloss"] = gbm2.logloss()
    # numeric-only, 32 features: the device-resident tree (devtree.py) with
    # its stream-ordered collectives -- without sampling (gbm3), with row and
    # per-node column sampling (gbm4), and gbm4's configuration on the level
    # loop (gbm5)
    xd = [f"x{i}" for i in range(32)]
    qg = dict(ntrees=4, max_depth=6, seed=1, min_rows=20, histogram_type="QuantilesGlobal", nbins=255)
    smp = dict(sample_rate=0.8, col_sample_rate=0.7)
    for key, kw, lvl in (("gbm3", {}, False), ("gbm4", smp, False), ("gbm5", smp, True)):
        old_env = os.environ.get("H2O3_DEV_TREE")
        if lvl:
            os.environ["H2O3_DEV_TREE"] = "0"
        try:
            m = H2OGradientBoostingEstimator(**qg, **kw)
            m.train(x=xd, y="y", training_frame=fr)
        finally:
            if old_env is None:
                os.environ.pop("H2O3_DEV_TREE", None)
            else:
                os.environ["H2O3_DEV_TREE"] = old_env
        res[key + "_trees"] = _trees(m)
        res[key + "_logloss"] = m.logloss()
        res[key + "_devtree"] = bool(getattr(m, "_used_devtree", False))
    from h2o3_amd.ops import _native
    res["native"] = _native.loaded_libs()
    if cloud.rank() == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    cloud.barrier()
    cloud.shutdown()


if __name__ == "__main__":
    run(sys.argv[1])
