"""h2o-py API surface parity: frame prims, top-level helpers, UDF metrics and
distributions, grid save/load/resume, AutoML plans / preprocessing / recovery,
early stopping for DRF and XGBoost (CPU)."""
import math
import os

import numpy as np
import pandas as pd
import pytest

import h2o
import h2o3_amd
from h2o3_amd.estimators import (H2OGradientBoostingEstimator, H2ORandomForestEstimator,
                                 H2OXGBoostEstimator)


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2o3_amd.init(verbose=False)


def _fr():
    return h2o.H2OFrame({"a": [1.0, 2, 3, None, 5], "b": ["x", "y", "x", "z", "x"], "c": [0, 0, 1, 1, 0]})


def test_frame_reducers_and_levels():
    fr = _fr()
    assert fr.anyfactor() and fr.any_na_rm()
    assert fr["b"].categories() == ["x", "y", "z"]
    assert fr["b"].append_levels(["q"]).levels()[0] == ["x", "y", "z", "q"]
    assert fr["b"].set_level("y").as_data_frame()["b"].tolist() == ["y"] * 5
    assert fr["b"].relevel_by_frequency().levels()[0][0] == "x"
    assert fr.filter_na_cols(0.1) == [1, 2]
    assert fr[0, :].getrow() == [1.0, "x", 0.0]
    assert fr["a"].idxmax().as_data_frame().iloc[0, 0] == 4
    assert fr["c"].which().as_data_frame()["which"].tolist() == [2, 3]
    assert fr["b"].isin(["x", "z"]).as_data_frame()["b"].tolist() == [1, 0, 1, 1, 1]
    assert fr["b"].match(["z", "x"]).as_data_frame()["b"].tolist() == [2, 0, 2, 1, 2]
    assert fr["a"].rep_len(7).nrows == 7
    x = np.array([1.0, 2, 3, 5])
    m2 = ((x - x.mean()) ** 2).mean()
    assert fr["a"].skewness(na_rm=True)[0] == pytest.approx(((x - x.mean()) ** 3).sum() / 5 / (
        ((x - x.mean()) ** 2).sum() / 5) ** 1.5)
    assert fr["a"].kurtosis(na_rm=True)[0] > 0 and m2 > 0


def test_mktime_isax_and_missing_values():
    t = h2o.H2OFrame.mktime(2020, 0, 14).as_data_frame().iloc[0, 0]
    assert str(t).startswith("2020-01-15")
    ts = h2o.H2OFrame(np.random.RandomState(0).randn(6, 12))
    r = ts.isax(3, 4)
    assert r.names == ["iSax_index", "c0", "c1", "c2"]
    idx = r.as_data_frame()["iSax_index"].tolist()
    assert all(len(s.split("_")) == 3 and s.count("^4") == 3 for s in idx)
    fr = h2o.H2OFrame(np.ones((400, 3)))
    fr.insert_missing_values(0.25, seed=3)
    na = sum(fr.nacnt())
    assert 200 < na < 400


def test_frame_save_load(tmp_path):
    fr = _fr()
    p = fr.save(str(tmp_path / "f1"))
    g = h2o.load_frame("copy", p)
    a, b = fr.as_data_frame(), g.as_data_frame()
    assert g.types == fr.types
    pd.testing.assert_frame_equal(a, b)


def test_top_level_helpers(tmp_path):
    assert h2o.estimate_cluster_mem(10, 1_000_000) >= 1
    with pytest.raises(ValueError):
        h2o.estimate_cluster_mem(2, 10, num_cols=3)
    iris = h2o.load_dataset("iris")
    assert iris.shape == (150, 5) and iris["class"].nlevels()[0] == 3
    assert h2o.as_list(_fr()).shape == (5, 3)
    path = h2o.download_csv(_fr(), str(tmp_path / "x.csv"))
    assert os.path.exists(path)
    import sqlite3
    db = str(tmp_path / "t.db")
    con = sqlite3.connect(db)
    con.execute("create table t(a real, b text)")
    con.executemany("insert into t values (?, ?)", [(1.0, "u"), (2.0, "v")])
    con.commit()
    con.close()
    s = h2o.import_sql_select(f"jdbc:sqlite:{db}", "select * from t where a > 1", "", "")
    assert s.nrows == 1
    t = h2o.import_sql_table(f"jdbc:sqlite:{db}", "t", "", "", columns=["b"], fetch_mode="SINGLE")
    assert t.shape == (2, 1) and t.names == ["b"]
    assert h2o.import_sql_table(f"jdbc:sqlite:{db}", "t", "", "").shape == (2, 2)
    with pytest.raises(ValueError):
        h2o.import_sql_table(f"jdbc:sqlite:{db}", "t; drop table t", "", "")


def test_frame_moment():
    import datetime
    one = h2o.H2OFrame.moment(2020, 2, 30)          # invalid date -> NA (AstMoment)
    assert one.shape == (1, 1) and one.types == {"time": "time"} and one.isna().sum() == 1
    fr = h2o.H2OFrame(pd.DataFrame({"y": [2020, 2021], "m": [1, 12]}))
    t = h2o.H2OFrame.moment(year=fr["y"], month=fr["m"], day=15, hour=3)
    assert t.nrows == 2 and t.year().as_data_frame()["time"].tolist() == [2020, 2021]
    assert t.month().as_data_frame()["time"].tolist() == [1, 12]
    d = h2o.H2OFrame.moment(date=datetime.date(2021, 5, 6), time=datetime.time(1, 2, 3))
    assert d.hour().as_data_frame()["time"].tolist() == [1]


class _MaeMetric:
    def map(self, pred, act, w, o, model):
        return [w * abs(act[0] - pred[0]), w]

    def reduce(self, l, r):
        return [l[0] + r[0], l[1] + r[1]]

    def metric(self, l):
        return l[0] / l[1]


_GAUSS_SRC = '''
class MyGauss:
    def link(self):
        return "identity"
    def init(self, w, o, y):
        return [w * (y - o), w]
    def gradient(self, y, f):
        return y - f
    def gamma(self, w, y, z, f):
        return [w * z, w]
'''


def test_custom_metric_and_distribution():
    rng = np.random.RandomState(0)
    X = rng.randn(400, 3)
    y = X[:, 0] * 2 + rng.randn(400) * 0.1
    fr = h2o.H2OFrame(pd.DataFrame({"x0": X[:, 0], "x1": X[:, 1], "x2": X[:, 2], "y": y}))
    ref = h2o.upload_custom_metric(_MaeMetric, func_name="mae_udf")
    assert ref.startswith("python:mae_udf=")
    m = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1, custom_metric_func=ref)
    m.train(y="y", training_frame=fr)
    tm = m._training_metrics
    assert tm["custom_metric_name"] == "mae_udf"
    assert tm["custom_metric_value"] == pytest.approx(tm["mae"], rel=1e-4)
    dref = h2o.upload_custom_distribution(_GAUSS_SRC, class_name="MyGauss", func_name="g_udf")
    mc = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1, distribution="custom",
                                      custom_distribution_func=dref)
    mc.train(y="y", training_frame=fr)
    mg = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1, distribution="gaussian")
    mg.train(y="y", training_frame=fr)
    assert mc.rmse() == pytest.approx(mg.rmse(), rel=1e-4)


def test_drf_xgb_early_stopping():
    rng = np.random.RandomState(1)
    X = rng.randn(600, 4)
    y = (X[:, 0] + rng.randn(600) > 0).astype(int)
    fr = h2o.H2OFrame(pd.DataFrame({**{f"x{i}": X[:, i] for i in range(4)}, "y": y}))
    fr["y"] = fr["y"].asfactor()
    tr, va = fr.split_frame([0.7], seed=1)
    d = H2ORandomForestEstimator(ntrees=500, max_depth=6, seed=1, stopping_rounds=2, score_tree_interval=2,
                                 stopping_tolerance=0.01)
    d.train(y="y", training_frame=tr, validation_frame=va)
    assert len(d._forest) < 500
    x = H2OXGBoostEstimator(ntrees=500, max_depth=4, seed=1, stopping_rounds=2, score_tree_interval=2,
                            stopping_tolerance=0.01)
    x.train(y="y", training_frame=tr, validation_frame=va)
    assert len(x._forest) < 500
    assert "validation_logloss" in x._scoring_history[-1]


def test_grid_save_load_and_resume(tmp_path):
    from h2o3_amd.grid import H2OGridSearch
    rng = np.random.RandomState(2)
    X = rng.randn(300, 3)
    fr = h2o.H2OFrame(pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "y": X[:, 0] - X[:, 1]}))
    g = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=5, seed=1), {"max_depth": [2, 3]}, grid_id="gsl")
    g.train(y="y", training_frame=fr)
    p = h2o.save_grid(str(tmp_path / "grid"), "gsl")
    g2 = h2o.load_grid(p)
    assert sorted(g2.model_ids) == sorted(g.model_ids)
    pr = g2.models[0].predict(fr)
    assert pr.nrows == 300
    # interrupted grid: only the first combination finished
    rec = str(tmp_path / "rec")
    g3 = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=5, seed=1), {"max_depth": [2, 3, 4]}, grid_id="grec",
                       recovery_dir=rec, search_criteria={"strategy": "Cartesian", "max_models": 1})
    g3.train(y="y", training_frame=fr)
    assert len(g3.models) == 1
    import json
    st = json.load(open(os.path.join(rec, "grec.grid.json")))
    st["search_criteria"] = {"strategy": "Cartesian"}
    json.dump(st, open(os.path.join(rec, "grec.grid.json"), "w"))
    res = h2o.resume(rec)
    assert len(res) == 1 and len(res[0].models) == 3


def test_automl_plan_preprocessing_recovery(tmp_path):
    from h2o3_amd.automl import H2OAutoML, _expand_plan
    assert _expand_plan(["GBM"])[:2] == [("GBM", "def_5"), ("GBM", "def_2")]
    assert _expand_plan([("XGBoost", "grids")]) == [("XGBoost", "grid_1")]
    rng = np.random.RandomState(3)
    n = 400
    cat = rng.randint(0, 40, n)
    eff = rng.randn(40)
    yv = (eff[cat] + rng.randn(n) * 0.5 > 0).astype(int)
    df = pd.DataFrame({"hc": [f"L{c}" for c in cat], "x": rng.randn(n), "y": yv})
    fr = h2o.H2OFrame(df)
    fr["y"] = fr["y"].asfactor()
    rec = str(tmp_path / "aml")
    aml = H2OAutoML(max_models=2, nfolds=3, seed=1, project_name="aml_plan",
                    modeling_plan=[("GBM", ["def_1"]), ("GLM", "defaults"), "StackedEnsemble"],
                    preprocessing=["target_encoding"], recovery_dir=rec)
    aml.train(y="y", training_frame=fr)
    lb = aml.leaderboard.as_data_frame()
    ids = lb["model_id"].tolist()
    assert any(i.startswith("GBM_1_AutoML") for i in ids) and any(i.startswith("GLM_1") for i in ids)
    assert any(i.startswith("StackedEnsemble_") for i in ids)
    assert any(r["stage"] == "Preprocessing" for r in aml.event_log_rows)
    assert aml.predict(fr).nrows == n
    assert os.path.exists(os.path.join(rec, "aml_plan.automl.json"))
