"""The reference's own Python client (h2o-py, loaded from the reference tree)
driving an h2o3_amd REST server: run by tests/test_rest_wire.py as
`python wire_client.py <url> <h2o-py dir>`; prints one RESULT json line."""
import json
import os
import sys
import tempfile

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "refclient_shim"), sys.argv[2]]
import h2o  # noqa: E402  (the reference client)
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
url = sys.argv[1]
h2o.connect(url=url, verbose=False)
rng = np.random.default_rng(0)
df = pd.DataFrame({"a": rng.normal(size=400), "b": rng.normal(size=400), "c": rng.choice(["u", "v", "w"], 400)})
df["y"] = np.where(df.a + df.b + (df.c == "u") > 0.3, "yes", "no")
df["r"] = 2 * df.a - df.b + rng.normal(size=400) * 0.1
fr = h2o.H2OFrame(df)
out = {}


def step(k, v):
    out[k] = v
    print(k, v, flush=True)


step("shape", list(fr.shape))
step("mean_a", fr["a"].mean()[0] if isinstance(fr["a"].mean(), list) else fr["a"].mean())
fr["a2"] = fr["a"] * 2
step("a2_sum", fr["a2"].sum())
sub = fr[fr["a"] > 0, :]
step("sub_rows", sub.nrows)
step("levels", fr["c"].levels())
tr, te = fr.split_frame(ratios=[0.75], seed=1)
step("split", [tr.nrows, te.nrows])
pdf = fr.as_data_frame()
step("as_df", list(pdf.shape))
fr.describe()
step("pandas_roundtrip", float(pdf["a"].sum()))
from h2o.estimators import H2OGradientBoostingEstimator, H2OGeneralizedLinearEstimator, H2OKMeansEstimator
m = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1)
m.train(x=["a", "b", "c"], y="y", training_frame=tr, validation_frame=te)
step("auc", [m.auc(), m.auc(valid=True)])
step("cm", m.confusion_matrix().to_list())
step("varimp", m.varimp()[:2])
step("sh", list(m.scoring_history().shape))
perf = m.model_performance(te)
step("perf_auc", perf.auc())
p = m.predict(te)
step("pred", list(p.shape))
g = H2OGeneralizedLinearEstimator(family="gaussian")
g.train(x=["a", "b"], y="r", training_frame=fr)
step("glm_coef", g.coef())
step("glm_r2", g.r2())
k = H2OKMeansEstimator(k=3, seed=1)
k.train(x=["a", "b"], training_frame=fr)
step("km", k.tot_withinss())
step("km_centers", len(k.centers()))
d = tempfile.mkdtemp()
step("mojo", os.path.basename(m.download_mojo(d)))
step("ls", len(h2o.ls()))
m2 = h2o.get_model(m.model_id)
step("get_model", m2.model_id)
h2o.remove(p)
from h2o.estimators import H2ORandomForestEstimator, H2ODeepLearningEstimator, H2OXGBoostEstimator
from h2o.grid.grid_search import H2OGridSearch
drf = H2ORandomForestEstimator(ntrees=5, seed=1); drf.train(x=["a", "b", "c"], y="y", training_frame=fr)
step("drf_auc", drf.auc())
dl = H2ODeepLearningEstimator(hidden=[8], epochs=2, seed=1); dl.train(x=["a", "b"], y="r", training_frame=fr)
step("dl_rmse", dl.rmse())
xg = H2OXGBoostEstimator(ntrees=5, seed=1); xg.train(x=["a", "b", "c"], y="y", training_frame=fr)
step("xgb_auc", xg.auc())
grid = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=3), hyper_params={"max_depth": [2, 3]}, grid_id="gw")
grid.train(x=["a", "b"], y="y", training_frame=fr)
step("grid", len(grid.model_ids))
step("grid_sorted", grid.get_grid(sort_by="auc", decreasing=True).model_ids)
step("table", list(fr["c"].table().as_data_frame().shape))
gb = fr.group_by("c").mean("a").get_frame()
step("group_by", list(gb.as_data_frame().shape))
step("quantile", list(fr["a"].quantile([0.5]).as_data_frame().shape))
fr2 = fr.cbind(fr["a"] + 1)
step("cbind", fr2.ncols)
step("nunique", fr["c"].nlevels())
step("isna", fr["a"].isna().sum())
fr["c2"] = fr["c"].ascharacter()
step("ascharacter", fr.types["c2"])
from h2o.automl import H2OAutoML
aml = H2OAutoML(max_models=2, seed=1, include_algos=["GLM", "GBM"], nfolds=2, project_name="aw")
aml.train(x=["a", "b"], y="y", training_frame=fr)
step("aml_leader", aml.leader.model_id)
step("aml_lb", list(aml.leaderboard.as_data_frame().shape))
d2 = tempfile.mkdtemp()
saved = h2o.save_model(m, path=d2, force=True)
step("saved", os.path.exists(saved))
m3 = h2o.load_model(saved)
step("loaded_auc", m3.model_performance(te).auc())
csv_path = os.path.join(d2, "fr.csv")
h2o.export_file(tr, csv_path, force=True)
step("exported_rows", sum(1 for _ in open(csv_path)) - 1)
pte = m.predict(te)
mm = h2o.make_metrics(pte["yes"], te["y"])
step("make_metrics_auc", mm.auc())
pd_tabs = m.partial_plot(te, cols=["a"], plot=False, nbins=5)
step("pdp_rows", pd_tabs[0].as_data_frame().shape[0] if hasattr(pd_tabs[0], "as_data_frame") else len(pd_tabs[0].cell_values))
fm = h2o.H2OFrame(pd.DataFrame({"u": rng.normal(size=50), "v": rng.normal(size=50)}))
fm.insert_missing_values(fraction=0.2, seed=1)
step("missing", int(fm.isna().sum()))
print("RESULT", json.dumps(out, default=str))
