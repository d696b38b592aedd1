"""Model-level calls of the reference h2o-py client against an h2o3_amd REST
server: cross-validation outputs, contributions / leaf assignment / staged
probabilities, metrics accessors, GLM regularization path, autoencoder
anomaly and deep features, PCA importance, Isolation Forest, Naive Bayes,
Stacked Ensemble over a CV'd base model, K-Means, CoxPH, Target Encoder.
Run by tests/test_rest_wire.py as `python wire_client_models.py <url> <h2o-py dir>`."""
import json
import os
import sys
import tempfile

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "refclient_shim"), sys.argv[2]]
import h2o  # noqa: E402  (the reference client)
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
from h2o.estimators import *  # noqa: E402,F401,F403

h2o.connect(url=sys.argv[1], verbose=False)
rng = np.random.default_rng(0)
df = pd.DataFrame({"a": rng.normal(size=500), "b": rng.normal(size=500), "c": rng.choice(["u", "v", "w"], 500)})
df["y"] = np.where(df.a + df.b > 0, "yes", "no"); df["r"] = df.a * 2 + rng.normal(size=500) * 0.1
fr = h2o.H2OFrame(df)
ok, bad = [], []


def t(name, f):
    try:
        v = f(); ok.append(name); print("OK ", name, str(v)[:100].replace("\n", " "))
    except Exception as e:
        bad.append(name); print("BAD", name, type(e).__name__, " | ".join(str(e).splitlines()[:5])[:600])
gbm = H2OGradientBoostingEstimator(ntrees=5, seed=1, nfolds=3, keep_cross_validation_predictions=True)
gbm.train(x=["a", "b", "c"], y="y", training_frame=fr)
t("xval_auc", lambda: gbm.auc(xval=True))
t("cv_summary", lambda: gbm.cross_validation_metrics_summary().as_data_frame().shape)
t("cv_models", lambda: len(gbm.cross_validation_models()))
t("cv_holdout", lambda: gbm.cross_validation_holdout_predictions().nrows)
t("contrib", lambda: gbm.predict_contributions(fr).ncols)
t("leaf_assign", lambda: gbm.predict_leaf_node_assignment(fr).ncols)
t("staged", lambda: gbm.staged_predict_proba(fr).ncols)
t("gains_lift", lambda: gbm.gains_lift().as_data_frame().shape)
t("roc", lambda: len(gbm.roc()[0]))
t("F1", lambda: gbm.F1())
t("logloss_xval", lambda: gbm.logloss(xval=True))
t("summary", lambda: gbm.summary().as_data_frame().shape)
t("params", lambda: gbm.actual_params["ntrees"])
t("model_perf_print", lambda: str(gbm.model_performance(fr))[:30])
t("varimp_pd", lambda: gbm.varimp(use_pandas=True).shape)
t("mojo_predict", lambda: gbm.download_mojo(tempfile.mkdtemp()))
glm = H2OGeneralizedLinearEstimator(family="binomial", lambda_search=True, nlambdas=5)
glm.train(x=["a", "b", "c"], y="y", training_frame=fr)
t("glm_coef_norm", lambda: len(glm.coef_norm()))
t("glm_std_coef_plot_data", lambda: glm._model_json["output"]["coefficients_table"].as_data_frame().shape)
t("glm_reg_path", lambda: len(H2OGeneralizedLinearEstimator.getGLMRegularizationPath(glm)["lambdas"]))
t("glm_null_dev", lambda: glm.null_deviance())
t("glm_aic", lambda: glm.aic())
dl = H2OAutoEncoderEstimator(hidden=[5], epochs=1, seed=1)
dl.train(x=["a", "b"], training_frame=fr)
t("ae_anomaly", lambda: dl.anomaly(fr).nrows)
t("deepfeatures", lambda: dl.deepfeatures(fr, 0).ncols)
pca = H2OPrincipalComponentAnalysisEstimator(k=2); pca.train(x=["a", "b"], training_frame=fr)
t("pca_predict", lambda: pca.predict(fr).ncols)
t("pca_varimp", lambda: pca.varimp(use_pandas=False)[:1])
iso = H2OIsolationForestEstimator(ntrees=5, seed=1); iso.train(x=["a", "b"], training_frame=fr)
t("iso_predict", lambda: iso.predict(fr).ncols)
nb = H2ONaiveBayesEstimator(); nb.train(x=["a", "c"], y="y", training_frame=fr)
t("nb_auc", lambda: nb.auc())
se = H2OStackedEnsembleEstimator(base_models=[gbm], metalearner_algorithm="glm")
t("se_train", lambda: se.train(x=["a", "b", "c"], y="y", training_frame=fr) or se.auc())
km = H2OKMeansEstimator(k=3, estimate_k=False); km.train(x=["a", "b"], training_frame=fr)
t("km_size", lambda: km.size())
t("km_betweenss", lambda: km.betweenss())
cox = H2OCoxProportionalHazardsEstimator(stop_column="tm")
fr2 = fr.cbind(h2o.H2OFrame(pd.DataFrame({"tm": rng.exponential(size=500) + 0.1, "ev": rng.integers(0, 2, 500)})))
t("coxph", lambda: cox.train(x=["a", "b"], y="ev", training_frame=fr2) or cox.model_id)
te = H2OTargetEncoderEstimator()
t("te", lambda: te.train(x=["c"], y="y", training_frame=fr) or te.transform(fr).ncols)
print("SUMMARY", json.dumps({"ok": len(ok), "bad": bad}))
