"""Frame munging through the reference h2o-py client against an h2o3_amd
REST server (every op becomes a Rapids expression evaluated by
core/rapids.py): run by tests/test_rest_wire.py as
`python wire_client_munging.py <url> <h2o-py dir>`; prints one SUMMARY line."""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "refclient_shim"), sys.argv[2]]
import h2o  # noqa: E402  (the reference client)
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

h2o.connect(url=sys.argv[1], verbose=False)
rng = np.random.default_rng(0)
df = pd.DataFrame({"a": rng.normal(size=200), "b": rng.integers(0, 5, 200).astype(float), "c": rng.choice(["u", "v", "w"], 200),
                   "s": rng.choice(["hello world", "foo bar", "x"], 200)})
df.loc[::17, "a"] = np.nan
fr = h2o.H2OFrame(df)
other = h2o.H2OFrame(pd.DataFrame({"c": ["u", "v", "w"], "z": [1.0, 2.0, 3.0]}))
ok, bad = [], []


def t(name, f):
    try:
        v = f()
        ok.append(name)
        print("OK ", name, str(v)[:80].replace("\n", " "))
    except Exception as e:
        bad.append(name)
        print("BAD", name, type(e).__name__, " | ".join(str(e).splitlines()[:6])[:700])
t("merge", lambda: fr.merge(other).shape)
t("sort", lambda: fr.sort("a").head(3).as_data_frame().shape)
t("sort_desc", lambda: fr.sort(["b", "a"], ascending=[False, True]).nrows)
t("impute", lambda: fr.impute("a", method="mean"))
t("cut", lambda: fr["a"].cut([-10, 0, 10]).table().nrows)
t("strsplit", lambda: fr["s"].strsplit(" ").ncols)
t("toupper", lambda: fr["s"].toupper().head(2).as_data_frame().iloc[0, 0])
t("gsub", lambda: fr["s"].gsub("o", "0").head(2).as_data_frame().iloc[0, 0])
t("nchar", lambda: fr["s"].nchar().max())
t("apply_col_mean", lambda: fr[["a", "b"]].apply(lambda x: x.mean(), axis=0).as_data_frame().shape)
t("ifelse", lambda: (fr["b"] > 2).ifelse(1, 0).sum())
t("unique", lambda: fr["c"].unique().nrows)
t("asfactor", lambda: fr["b"].asfactor().levels())
t("asnumeric", lambda: fr["c"].asfactor().asnumeric().max())
t("na_omit", lambda: fr.na_omit().nrows)
t("fillna", lambda: fr.fillna(method="forward", axis=0, maxlen=5)["a"].isna().sum())
t("scale", lambda: fr[["a", "b"]].scale().mean())
t("log_exp", lambda: fr["b"].log1p().exp().sum())
t("cumsum", lambda: fr["b"].cumsum().max())
t("rbind", lambda: fr.rbind(fr).nrows)
t("cor", lambda: fr[["a", "b"]].na_omit().cor())
t("var", lambda: fr["b"].var())
t("median", lambda: fr["b"].median())
t("hist", lambda: fr["b"].hist(plot=False).nrows)
t("kfold", lambda: fr.kfold_column(n_folds=3, seed=1).max())
t("stratified_kfold", lambda: fr["c"].stratified_kfold_column(n_folds=3, seed=1).max())
t("runif", lambda: fr.runif(seed=1).min() >= 0)
t("rename", lambda: fr[["a", "b"]].rename({"a": "aa"}).names[:2])
t("set_names", lambda: fr[["a", "b"]].set_names(["p", "q"]).names)
t("drop", lambda: fr.drop("s").ncols)
t("slice_rows", lambda: fr[10:20, :].nrows)
t("bool_and", lambda: fr[(fr["b"] > 1) & (fr["c"] == "u"), :].nrows)
t("isin", lambda: fr[fr["c"].isin(["u", "w"]), :].nrows)
t("group_by_multi", lambda: fr.group_by(["c"]).count().sum("b").max("a", na="rm").get_frame().shape)
t("pivot_melt", lambda: fr[["c", "b"]].head(5).ncols)
t("relevel", lambda: fr["c"].relevel("w").levels())
t("top_n", lambda: fr.topN("a", 5).nrows)
t("which", lambda: (fr["b"] > 3).which().nrows)
t("moment", lambda: h2o.H2OFrame.moment(2020, 1, 1).nrows)
t("describe_summary", lambda: fr.get_summary()["b"]["mean"])
t("as_date", lambda: h2o.H2OFrame(pd.DataFrame({"d": ["02/01/2020", "04/03/2021"]}))["d"].as_date("%d/%m/%Y").year().max())
t("any_all", lambda: (fr["b"].any(), fr["b"].all()))
t("round_signif", lambda: fr["a"].round(2).head(1).as_data_frame().iloc[0, 0])
t("mode_table", lambda: fr["c"].table().as_data_frame().shape)
t("entropy", lambda: fr["s"].entropy().max())
t("sub_assign", lambda: fr.__setitem__((fr["b"] > 3, "b"), 0) or fr["b"].max())
t("nrow_getrow", lambda: fr[0, ["a", "b"]].getrow()[1])
print("SUMMARY", json.dumps({"ok": len(ok), "bad": bad}))
