"""Worker for tests/test_distributed.py: one rank of a gloo (CPU) cloud.

Trains the same models on the same data as the single-process run and
dumps global results (metrics, coefficients, tree structure) to JSON.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_df(n=4000, seed=7):
    import numpy as np
    import pandas as pd
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 6))
    logit = 1.5 * X[:, 0] - X[:, 1] + 0.5 * X[:, 2] * X[:, 3]
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(6)])
    df["cat"] = np.where(X[:, 4] > 0, "a", "b")
    df["yr"] = 2.0 * X[:, 0] + X[:, 5] + rng.normal(scale=0.1, size=n)
    df["y"] = np.where(y == 1, "yes", "no")
    return df


def run(out_path):
    import h2o3_amd as h2o
    from h2o3_amd.estimators import (H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                                     H2OKMeansEstimator, H2ORandomForestEstimator)
    h2o.init(verbose=False)
    fr = h2o.H2OFrame(make_df())
    x = [f"x{i}" for i in range(6)] + ["cat"]
    res = {"nrow": fr.nrow}
    gbm = H2OGradientBoostingEstimator(ntrees=5, max_depth=4, seed=1, min_rows=5)
    gbm.train(x=x, y="y", training_frame=fr)
    res["gbm_auc"] = gbm.auc()
    res["gbm_logloss"] = gbm.logloss()
    # reference UniformAdaptive: per-node bins over the parent's range (feature slices per rank)
    gua = H2OGradientBoostingEstimator(ntrees=5, max_depth=5, seed=1, min_rows=5, histogram_type="UniformAdaptive",
                                       nbins_top_level=256)
    gua.train(x=x, y="y", training_frame=fr)
    res["gbm_ua_logloss"] = gua.logloss()
    glm = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0.0)
    glm.train(x=x, y="y", training_frame=fr)
    res["glm_coef"] = glm.coef()
    res["glm_auc"] = glm.auc()
    glmr = H2OGeneralizedLinearEstimator(family="gaussian", alpha=0.5, lambda_=0.01)
    glmr.train(x=x, y="yr", training_frame=fr)
    res["glmr_coef"] = glmr.coef()
    drf = H2ORandomForestEstimator(ntrees=3, max_depth=5, seed=3, sample_rate=1.0, mtries=7)
    drf.train(x=x, y="yr", training_frame=fr)
    res["drf_rmse"] = drf.rmse()
    km = H2OKMeansEstimator(k=3, seed=5, init="PlusPlus", standardize=True)
    km.train(x=[f"x{i}" for i in range(6)], training_frame=fr)
    res["km_tot_withinss"] = km.tot_withinss()
    # multinomial metrics + multinomial AUC: sums and merged sketches, no row gathers
    import numpy as np
    df3 = make_df()
    df3["y3"] = np.where(df3.x0 > 0.5, "hi", np.where(df3.x0 < -0.5, "lo", "mid"))
    fr3 = h2o.H2OFrame(df3)
    g3 = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1, auc_type="MACRO_OVO")
    g3.train(x=x, y="y3", training_frame=fr3)
    m3 = g3.model_performance(fr3)
    res["multi"] = {"logloss": m3.logloss(), "auc": m3.auc(), "aucpr": m3.aucpr(),
                    "cm": m3["cm"]["matrix"], "hr": [r["hit_ratio"] for r in m3["hit_ratio_table"]],
                    "wovr": g3.model_performance(fr3, auc_type="WEIGHTED_OVR").auc()}
    # Deep Learning: model averaging per iteration (default), elastic averaging,
    # sharded data (no replication) and single-node mode -- every rank must end
    # with the same model
    from h2o3_amd.estimators import H2ODeepLearningEstimator
    from h2o3_amd.parallel import collectives as coll
    dl_res = {}
    for tag, kw in (("avg", {}), ("elastic", dict(elastic_averaging=True)),
                    ("shard", dict(replicate_training_data=False, train_samples_per_iteration=1000)),
                    ("single", dict(single_node_mode=True))):
        dl = H2ODeepLearningEstimator(hidden=[16], epochs=4, seed=3, **kw)
        dl.train(x=x, y="y", training_frame=fr)
        sig = float(sum(float(L.W.double().sum()) + float(L.b.double().sum()) for L in dl._layers))
        sigs = coll.all_gather_object(sig)
        dl_res[tag] = {"auc": dl.auc(), "same": max(sigs) - min(sigs) < 1e-9 * max(1.0, abs(sig))}
    res["dl"] = dl_res
    # munging without frame gathers: sort / group-by / merge equal the one-rank results
    import pandas as pd
    rng = np.random.default_rng(11)
    nm = 600
    dm = pd.DataFrame({"k1": rng.integers(0, 7, nm).astype(float), "k2": rng.choice(["u", "v", "w"], nm),
                       "v": rng.normal(size=nm), "t": rng.integers(0, 1000, nm).astype(float)})
    dm.loc[::37, "v"] = np.nan
    dm.loc[::53, "k1"] = np.nan
    fm = h2o.H2OFrame(dm)
    srt = fm.sort(["k2", "k1", "t"], ascending=[True, False, True]).as_data_frame()
    res["mung_sort"] = srt.astype(str).values.tolist()
    gb = fm.group_by(["k2", "k1"]).count().sum("v", na="rm").mean("v", na="rm").min("v").max("v").sd("v", na="rm") \
        .median("t").get_frame().as_data_frame()
    res["mung_gb"] = gb.round(9).astype(str).values.tolist()
    dy = pd.DataFrame({"k1": np.arange(0, 9).astype(float), "w": np.arange(9) * 10.0})
    fy = h2o.H2OFrame(dy)
    for how, kw in (("inner", {}), ("left", {"all_x": True}), ("right", {"all_y": True})):
        mg = fm[["k1", "t"]].merge(fy, **kw).as_data_frame()
        res[f"mung_merge_{how}"] = mg.round(9).astype(str).values.tolist()
    mb = gbm.model_performance(fr)
    res["bin_tab_rows"] = len(mb["thresholds_and_metric_scores"]["threshold"])
    res["bin_prauc"] = mb.aucpr()
    res["persist"] = _persist_roundtrip(h2o, fr, x, os.path.dirname(out_path))
    res["dist_ops"] = _dist_ops(h2o)
    res["drf_pairs"] = _drf_pairs(h2o)
    from h2o3_amd.parallel import cloud
    if cloud.rank() == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    cloud.barrier()
    cloud.shutdown()


def _drf_pairs(h2o):
    """DRF with mtries << F (the row-direct pair-histogram path) on numeric
    and high-cardinality categorical features: the trees must not depend on
    the number of ranks (packed / sparse pair exchange)."""
    import numpy as np
    import pandas as pd
    from h2o3_amd.estimators import H2ORandomForestEstimator
    from h2o3_amd.parallel import collectives as coll
    rng = np.random.default_rng(5)
    n, F = 6000, 40
    X = rng.normal(size=(n, F))
    df = pd.DataFrame(X, columns=[f"f{i}" for i in range(F)])
    for c in range(4):
        df[f"c{c}"] = [f"L{v}" for v in rng.integers(0, 60, n)]
    df["y"] = X[:, 0] + 0.5 * X[:, 1] * X[:, 2] + (df["c0"].str[1:].astype(int) % 7) * 0.2 + 0.1 * rng.normal(size=n)
    fr = h2o.H2OFrame(df)
    for c in range(4):
        fr[f"c{c}"] = fr[f"c{c}"].asfactor()
    coll.reset_bytes()
    m = H2ORandomForestEstimator(ntrees=2, max_depth=10, mtries=6, seed=11, sample_rate=1.0, min_rows=2)
    m.train(y="y", training_frame=fr)
    trees = [[list(map(int, t.feat)), [round(float(v), 9) if np.isfinite(v) else str(v) for v in t.thr]]
             for t in m._forest.trees]
    by = coll.bytes_report()
    # classification: whole-number histograms (bootstrap counts, class counts)
    # take the lossless int32 transport
    fr["yc"] = (fr["y"] > 0.2).asfactor()
    mc = H2ORandomForestEstimator(ntrees=2, max_depth=10, mtries=6, seed=12, sample_rate=1.0, min_rows=2)
    mc.train(x=[c for c in fr.names if c not in ("y", "yc")], y="yc", training_frame=fr)
    trees_c = [[list(map(int, t.feat)), [round(float(v), 9) if np.isfinite(v) else str(v) for v in t.thr]]
               for t in mc._forest.trees]
    return {"trees": trees, "rmse": round(m.rmse(), 9), "trees_c": trees_c, "logloss_c": round(mc.logloss(), 9),
            "a2a_levels": sorted({k[0] for k, v in by.items() if k[1] == "all_to_all_single" and k[0].startswith("tree")})}


def _dist_ops(h2o):
    """Shard-local munging prims (core/dist_ops.py): the results must not
    depend on the number of ranks."""
    import numpy as np
    import pandas as pd
    rng = np.random.default_rng(21)
    n = 5000
    df = pd.DataFrame({"a": rng.integers(0, 6, n).astype(float), "b": rng.choice(["x", "y", "z", "w"], n),
                       "v": rng.normal(size=n), "t": rng.integers(0, 40, n).astype(float),
                       "c": rng.choice(["p", "q", "r"], n)})
    df.loc[::17, "v"] = np.nan
    df.loc[::29, "a"] = np.nan
    fr = h2o.H2OFrame(df)
    fr["c"] = fr["c"].asfactor()
    fr["b"] = fr["b"].asfactor()

    def rows(f):
        d = f.as_data_frame()
        return [[None if (isinstance(v, float) and v != v) else (round(v, 9) if isinstance(v, float) else str(v))
                 for v in r] for r in d.values.tolist()]
    out = {}
    out["quantile"] = rows(fr[["v", "t"]].quantile([0.01, 0.25, 0.5, 0.9]))
    out["quantile_w"] = rows(fr[["v", "t"]].quantile([0.2, 0.7], weights_column="t"))
    out["table1"] = rows(fr["t"].table())
    out["table2"] = rows(fr[["b", "a"]].table())
    out["table_sparse"] = rows(fr[["b", "c"]].table(dense=False))
    out["unique"] = rows(fr["a"].unique())
    out["hist"] = rows(fr["v"].hist(breaks=12))
    out["cor"] = rows(fr[["v", "t", "a"]].cor(use="complete.obs"))
    out["spearman"] = rows(fr[["v", "t"]].cor(use="complete.obs", method="Spearman"))
    out["dedup"] = rows(fr.drop_duplicates(["a", "b"], keep="last"))
    out["pivot"] = rows(fr[fr["a"] >= 0].pivot("a", "c", "v"))
    out["melt"] = rows(fr[["t", "v", "a"]].melt(["t"], skipna=True))
    out["rank"] = rows(fr.rank_within_group_by(["b"], ["t", "v"], [True, False], "rk"))
    out["inter"] = rows(fr.interaction(["b", "c"], pairwise=False, max_factors=7, min_occurrence=2))
    gb = fr.group_by(["b"]).median("v", na="rm").mode("t").get_frame()
    out["gb_med_mode"] = rows(gb)
    out["sort_dups"] = rows(fr.sort(["c", "t"], ascending=[False, True]))
    # AstTopN / AstImpute-by-group / AstApply / AstFillNA / AstDistance without frame gathers
    out["topn"] = rows(fr.topN("v", 3))
    out["bottomn"] = rows(fr.bottomN("t", 2))
    for meth in ("mean", "median", "mode"):
        f2 = h2o.H2OFrame(df)
        f2["b"] = f2["b"].asfactor()
        col = "b" if meth == "mode" else "v"
        if meth == "mode":
            f2[::11, "b"] = None
        keys = f2.impute(col, method=meth, by=["a"])
        out[f"impute_{meth}"] = rows(f2[[col, "a"]]) + [["keys"]] + rows(keys[0] if isinstance(keys, list) else keys)
    out["apply_num"] = rows(fr[["v", "t"]].apply(lambda r: (0.0 if r["v"] != r["v"] else r["v"]) + 2 * r["t"], axis=1))
    out["apply_str"] = rows(fr[["t"]].apply(lambda r: "hi" if r["t"] > 20 else "lo", axis=1))
    fz = h2o.H2OFrame(pd.DataFrame({"x": [np.nan if (i % 600) < 7 or 2490 <= i < 2510 else float(i)
                                          for i in range(n)]}))
    out["fill_fwd"] = rows(fz.fillna("forward", maxlen=5))
    out["fill_bwd"] = rows(fz.fillna("backward", maxlen=12))
    out["distance"] = rows(fr[["v", "t"]][:50, :].fillna("forward", maxlen=100).distance(
        h2o.H2OFrame(pd.DataFrame({"v": [0.5, -1.0, 2.0], "t": [3.0, 10.0, 30.0]}))))
    return out


def _persist_roundtrip(h2o, fr, x, out_dir):
    """Binary save / load of models with row-sharded state: a CV GBM with
    kept holdout predictions and a GLRM (per-row X).  The archive must hold
    every row and the loaded model must hold this rank's shard again."""
    import torch
    from h2o3_amd.estimators import H2OGeneralizedLowRankEstimator, H2OGradientBoostingEstimator
    from h2o3_amd.parallel import cloud
    from h2o3_amd.parallel import collectives as coll
    out = {}
    d = os.path.join(out_dir, f"models_w{cloud.world()}")
    cv = H2OGradientBoostingEstimator(ntrees=3, max_depth=3, seed=1, nfolds=2, fold_assignment="Modulo",
                                      keep_cross_validation_predictions=True)
    cv.train(x=x, y="y", training_frame=fr)
    p = h2o.save_model(cv, d, force=True)
    lm = h2o.load_model(p)
    hold0 = coll.all_gather_var(cv._cv_holdout.double())
    hold1 = coll.all_gather_var(lm._cv_holdout.double())
    out["cv_holdout_local_rows_ok"] = bool(coll.all_gather_object(lm._cv_holdout.shape[0] == fr.nlocal) ==
                                           [True] * cloud.world())
    out["cv_holdout_equal"] = bool(torch.equal(hold0, hold1))
    out["cv_holdout_sum"] = round(float(hold1.sum()), 9)
    cvp = lm.cross_validation_holdout_predictions()
    out["cv_pred_rows"] = cvp.nrow
    glrm = H2OGeneralizedLowRankEstimator(k=2, seed=3, max_iterations=20)
    glrm.train(x=[f"x{i}" for i in range(6)], training_frame=fr)
    p = h2o.save_model(glrm, d, force=True)
    lg = h2o.load_model(p)
    x0 = coll.all_gather_var(glrm._X.detach().double())
    x1 = coll.all_gather_var(lg._X.detach().double())
    out["glrm_x_equal"] = bool(torch.equal(x0, x1))
    out["glrm_x_rows"] = int(x1.shape[0])
    return out


if __name__ == "__main__":
    run(sys.argv[1])
