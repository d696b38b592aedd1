"""The reference client's module paths (h2o.estimators.gbm, h2o.frame,
h2o.transforms.preprocessing, h2o.assembly, h2o.cross_validation,
h2o.model.metrics.*, h2o.scoring, ...) resolve to the h2o3_amd
implementations (h2o/_modules.py), plus the pieces added for them:
H2OAssembly munging steps, fold iterators, makeGLMModel, make_leaderboard,
regression metric functions, session S3 credentials."""
import importlib

import numpy as np
import pandas as pd
import pytest


def test_every_reference_module_path_imports():
    from h2o._modules import MODULES
    bad = []
    for m, names in MODULES.items():
        mod = importlib.import_module(m)
        bad += [f"{m}.{n}" for n in names if not hasattr(mod, n)]
    assert len(MODULES) > 100 and not bad, bad
    from h2o.estimators.gbm import H2OGradientBoostingEstimator  # noqa: F401
    from h2o.sklearn import H2OGradientBoostingClassifier  # noqa: F401
    from h2o.tree import H2OTree  # noqa: F401
    from h2o.estimators.deeplearning import H2OAutoEncoderEstimator
    assert H2OAutoEncoderEstimator()._parms["autoencoder"] is True


def _frame(n=400, seed=0):
    from h2o3_amd.core.frame import H2OFrame
    rng = np.random.default_rng(seed)
    df = pd.DataFrame({"a": rng.normal(size=n) * 2 + 1, "b": rng.normal(size=n), "c": rng.choice(list("xyz"), n)})
    df["y"] = (df.a * 0.7 - df.b + rng.normal(size=n) > 0.5).astype(int)
    fr = H2OFrame(df)
    fr["c"] = fr["c"].asfactor()
    fr["y"] = fr["y"].asfactor()
    return fr, df


def test_assembly_steps():
    from h2o.assembly import H2OAssembly
    from h2o.frame import H2OFrame
    from h2o.transforms.preprocessing import H2OBinaryOp, H2OCol, H2OColOp, H2OColSelect
    fr, df = _frame()
    asm = H2OAssembly(steps=[("select", H2OColSelect(["a", "b", "c"])),
                             ("cos_a", H2OColOp(op=H2OFrame.cos, col="a", inplace=True)),
                             ("a_plus_b", H2OBinaryOp(op=H2OFrame.__add__, col="a", right=H2OCol("b"),
                                                      inplace=False, new_col_name="ab")),
                             ("b_times_2", H2OBinaryOp(op=H2OFrame.__mul__, col="b", right=2, inplace=True))])
    out = asm.fit(fr).as_data_frame()
    assert asm.names == ["select", "cos_a", "a_plus_b", "b_times_2"]
    assert list(out.columns) == ["a", "b", "c", "ab"]
    np.testing.assert_allclose(out["a"], np.cos(df.a), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out["ab"], np.cos(df.a) + df.b, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out["b"], 2 * df.b, rtol=1e-5, atol=1e-6)


def test_kfold_iterators():
    from h2o.cross_validation import H2OKFold, H2OStratifiedKFold
    fr, _ = _frame()
    folds = list(H2OKFold(fr, n_folds=4, seed=1))
    assert len(folds) == 4
    tests = np.stack([t.as_data_frame().iloc[:, 0].values for _, t in folds])
    assert (tests.sum(0) == 1).all()                   # each row in exactly one test fold
    tr, te = folds[0]
    assert (tr.as_data_frame().iloc[:, 0].values + te.as_data_frame().iloc[:, 0].values == 1).all()
    sf = list(H2OStratifiedKFold(fr["y"], n_folds=3, seed=2))
    assert len(sf) == 3


def test_make_glm_model_and_leaderboard_and_metric_fns():
    from h2o.estimators.glm import H2OGeneralizedLinearEstimator
    from h2o.estimators.gbm import H2OGradientBoostingEstimator
    from h2o.model.models.regression import h2o_mean_squared_error, h2o_r2_score, h2o_mean_absolute_error
    from h2o.scoring import make_leaderboard
    fr, df = _frame()
    glm = H2OGeneralizedLinearEstimator(family="binomial")
    glm.train(x=["a", "b", "c"], y="y", training_frame=fr)
    same = H2OGeneralizedLinearEstimator.makeGLMModel(glm, glm.coef())
    p1 = glm.predict(fr).as_data_frame()["p1"].values
    np.testing.assert_allclose(same.predict(fr).as_data_frame()["p1"].values, p1, atol=1e-6)
    c = dict(glm.coef(), a=0.0, Intercept=0.25)
    m = H2OGeneralizedLinearEstimator.makeGLMModel(glm, c, threshold=0.3)
    eta = 0.25 + c["b"] * df.b + df.c.map({k: c.get(f"c.{k}", 0.0) for k in "xyz"})
    np.testing.assert_allclose(m.predict(fr).as_data_frame()["p1"].values, 1 / (1 + np.exp(-eta)), atol=1e-5)
    with pytest.raises(ValueError):
        H2OGeneralizedLinearEstimator.makeGLMModel(glm, {"nope": 1.0})
    gbm = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1)
    gbm.train(x=["a", "b", "c"], y="y", training_frame=fr)
    lb = make_leaderboard([glm, gbm], fr).as_data_frame()
    assert set(lb["model_id"]) == {glm.model_id, gbm.model_id} and "auc" in lb.columns
    a, p = fr["a"], fr["a"] * 0.9
    mse = h2o_mean_squared_error(a, p)
    np.testing.assert_allclose(mse, np.mean((0.1 * df.a) ** 2), rtol=1e-5)
    np.testing.assert_allclose(h2o_mean_absolute_error(a, p), np.mean(np.abs(0.1 * df.a)), rtol=1e-5)
    np.testing.assert_allclose(h2o_r2_score(a, p), 1 - np.sum((0.1 * df.a) ** 2) / np.sum((df.a - df.a.mean()) ** 2),
                               rtol=1e-5)


def test_tables_and_s3_credentials():
    from h2o.model.confusion_matrix import ConfusionMatrix
    from h2o.persist import remove_s3_credentials, set_s3_credentials
    from h2o.two_dim_table import H2OTwoDimTable
    t = H2OTwoDimTable("T", col_header=["x", "y"], cell_values=[[1, 2], [3, 4]])
    assert t["y"] == [2, 4] and list(t.as_data_frame().columns) == ["x", "y"]
    cm = ConfusionMatrix([[5, 1], [2, 7]], domains=["a", "b"])
    assert cm.to_list() == [[5, 1], [2, 7]]
    from h2o3_amd.core import persist
    set_s3_credentials("AKID", "SECRET", "TOK")
    assert persist._s3_cfg()[2:] == ("AKID", "SECRET", "TOK")
    remove_s3_credentials()
    assert persist._S3_CREDS == {}
