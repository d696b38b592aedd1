"""The reference client's object API resolves on live objects.

Every public name of the reference h2o-py classes (parsed with `ast` from
/root/reference/h2o-py/h2o) must exist on the corresponding trained object:
H2OGridSearch (grid/grid_search.py), H2OAutoML and its base mixin
(automl/_base.py, automl/_estimator.py), the model classes (model/model_base.py
and the category mixins model/models/*.py) and the `h2o.explanation` module
(explanation/_explain.py + explanation/__init__.py).  Exclusions are listed
with their reason.
"""
import ast
import os

import numpy as np
import pandas as pd
import pytest

REF = "/root/reference/h2o-py/h2o"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference h2o-py client not present")



def _public(relpath, cls):
    src = open(os.path.join(REF, relpath)).read()
    for n in ast.walk(ast.parse(src)):
        if isinstance(n, ast.ClassDef) and n.name == cls:
            return sorted({m.name for m in n.body if isinstance(m, ast.FunctionDef) and not m.name.startswith("_")})
    raise AssertionError(f"{cls} not in {relpath}")


def _module_functions(relpath):
    src = open(os.path.join(REF, relpath)).read()
    return sorted({n.name for n in ast.parse(src).body if isinstance(n, ast.FunctionDef) and not n.name.startswith("_")})


def _all_list(relpath):
    src = open(os.path.join(REF, relpath)).read()
    out = set()
    for n in ast.walk(ast.parse(src)):
        if isinstance(n, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in n.targets):
            out |= {e.value for e in n.value.elts}
    return out


@pytest.fixture(scope="module")
def data():
    import h2o3_amd
    h2o3_amd.init(verbose=False)
    rng = np.random.RandomState(0)
    df = pd.DataFrame(rng.randn(400, 4), columns=list("abcd"))
    df["y"] = np.where(df.a - df.b + 0.5 * rng.randn(400) > 0, "p", "q")
    df["r"] = df.a * 2 + rng.randn(400)
    return h2o3_amd.H2OFrame(df)


def _missing(obj, names):
    return [n for n in names if not hasattr(obj, n)]


def test_grid_object_api(data):
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    from h2o3_amd.grid import H2OGridSearch
    g = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=3, seed=1), {"max_depth": [2, 3]})
    g.train(x=["a", "b", "c", "d"], y="y", training_frame=data)
    names = _public("grid/grid_search.py", "H2OGridSearch")
    assert not _missing(g, names), _missing(g, names)
    assert g.hyper_names == ["max_depth"]
    assert set(g.model_performance().keys()) == set(g.model_ids)
    assert all(v is not None for v in g.gini().values())
    assert all(v is None for v in g.coef().values())
    assert set(g.varimp(use_pandas=True)) == set(g.model_ids)
    assert len(g.get_summary()) == 2
    st = g.sort_by("auc", increasing=False)
    assert list(st["model_ids"]) == g.get_grid("auc", decreasing=True).model_ids
    pf = g.pareto_front(data)
    assert pf.nrows >= 1 and pf.figure() is not None
    # start / join / resume: an asynchronous build of a wider space continues the grid
    g2 = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=2, seed=1), {"max_depth": [2, 3, 4]},
                       search_criteria={"strategy": "Cartesian", "max_models": 2})
    g2.start(x=["a", "b"], y="y", training_frame=data)
    g2.join()
    assert len(g2.models) == 2
    g2.resume(max_models=3)
    assert len(g2.models) == 3 and len(set(map(repr, (m._grid_params for m in g2.models)))) == 3


def test_automl_object_api(data, tmp_path):
    from h2o3_amd.automl import H2OAutoML
    aml = H2OAutoML(max_models=2, seed=1, nfolds=0, include_algos=["GLM", "GBM"])
    aml.train(x=["a", "b", "c", "d"], y="y", training_frame=data)
    names = set(_public("automl/_base.py", "H2OAutoMLBaseMixin")) | set(_public("automl/_estimator.py", "H2OAutoML"))
    # the reference attaches these to the mixin in explanation.register_explain_methods
    names |= {"pd_multi_plot", "varimp_heatmap", "model_correlation_heatmap", "explain", "explain_row",
              "model_correlation", "varimp"}
    assert not _missing(aml, names), _missing(aml, names)
    p = aml.download_mojo(str(tmp_path))
    assert os.path.exists(p)
    pf = aml.pareto_front()
    assert pf.nrows >= 1 and pf.figure() is not None
    lb = aml.get_leaderboard("ALL").as_data_frame()
    assert {"training_time_ms", "predict_time_per_row_ms", "algo"} <= set(lb.columns)


def test_model_object_api(data):
    from h2o3_amd.estimators import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator,
                                     H2OGradientBoostingEstimator, H2OKMeansEstimator)
    x = ["a", "b", "c", "d"]
    base = _public("model/model_base.py", "ModelBase")
    binom = _public("model/models/binomial.py", "H2OBinomialModel")
    reg = _public("model/models/regression.py", "H2ORegressionModel")
    clus = _public("model/models/clustering.py", "H2OClusteringModel")
    for m in (H2OGradientBoostingEstimator(ntrees=3), H2OGeneralizedLinearEstimator(family="binomial"),
              H2ODeepLearningEstimator(epochs=1, hidden=[5], seed=1)):
        m.train(x=x, y="y", training_frame=data)
        assert not _missing(m, base + binom), (type(m).__name__, _missing(m, base + binom))
    r = H2OGradientBoostingEstimator(ntrees=3)
    r.train(x=x, y="r", training_frame=data)
    assert not _missing(r, base + reg), _missing(r, base + reg)
    km = H2OKMeansEstimator(k=3, seed=1)
    km.train(x=x, training_frame=data)
    assert not _missing(km, base + clus), _missing(km, base + clus)
    # answers of the algorithms a method does not apply to follow the reference client
    g = H2OGradientBoostingEstimator(ntrees=2)
    g.train(x=x, y="y", training_frame=data)
    assert g.coef() is None and g.coef_norm() is None
    with pytest.raises(ValueError):
        g.coef_with_p_values()
    with pytest.raises(ValueError):
        g.rotation()


def test_explanation_module_exports():
    import h2o.explanation as ex
    names = set(_module_functions("explanation/_explain.py")) | _all_list("explanation/__init__.py") | \
        set(_module_functions("explanation/__init__.py"))
    assert not [n for n in names if not hasattr(ex, n)], [n for n in names if not hasattr(ex, n)]
    from h2o3_amd.explanation import pareto_front_indices
    x = np.array([1.0, 2.0, 3.0, 1.5, 4.0])
    y = np.array([0.5, 0.7, 0.9, 0.4, 0.8])
    # top left: maximise y, minimise x
    assert pareto_front_indices(x, y, top=True, left=True).tolist() == [0, 1, 2]
    # bottom left: minimise both
    assert pareto_front_indices(x, y, top=False, left=True).tolist() == [0, 3]
