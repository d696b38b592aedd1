"""scikit-learn compatible wrappers (reference: h2o-py h2o/sklearn/wrapper.py,
which generates H2O<Algo>Classifier / Regressor / Estimator classes around
every H2O estimator).  fit/predict/predict_proba/score accept numpy arrays
or pandas frames; get_params/set_params make them usable in sklearn
pipelines and grid searches."""
from __future__ import annotations

import numpy as np
import pandas as pd

from .. import estimators as _E


def _to_frame(X, y=None, names=None):
    from ..core.frame import H2OFrame
    df = X.copy() if isinstance(X, pd.DataFrame) else pd.DataFrame(np.asarray(X),
                                                                   columns=names or [f"C{i + 1}" for i in range(np.asarray(X).shape[1])])
    if y is not None:
        df["__target__"] = np.asarray(y)
    return H2OFrame(df), [c for c in df.columns if c != "__target__"]


class _Base:
    _est_cls = None
    _kind = "estimator"

    def __init__(self, **params):
        self._params = params
        self.estimator_ = None

    def get_params(self, deep=True):
        return dict(self._params)

    def set_params(self, **p):
        self._params.update(p)
        return self

    def fit(self, X, y=None, **kw):
        import h2o3_amd as h2o
        h2o.init()
        est = self._est_cls(**self._params)
        if y is not None and self._kind == "classifier":
            y = np.asarray(y).astype(str)
        fr, xs = _to_frame(X, y)
        self._names = xs
        if y is not None:
            if self._kind == "classifier":
                fr["__target__"] = fr["__target__"].asfactor()
            est.train(x=xs, y="__target__", training_frame=fr)
            if self._kind == "classifier":
                self.classes_ = np.asarray(est._spec.response_domain)
        else:
            est.train(x=xs, training_frame=fr)
        self.estimator_ = est
        return self

    def _frame(self, X):
        fr, _ = _to_frame(X, names=self._names)
        return fr

    def predict(self, X):
        out = self.estimator_.predict(self._frame(X)).as_data_frame()
        p = out.iloc[:, 0].values
        if self._kind == "classifier":
            return p.astype(str)
        return p

    def predict_proba(self, X):
        out = self.estimator_.predict(self._frame(X)).as_data_frame()
        return out[[c for c in self.classes_]].values

    def score(self, X, y):
        p = self.predict(X)
        if self._kind == "classifier":
            return float((p == np.asarray(y).astype(str)).mean())
        y = np.asarray(y, dtype=float)
        return float(1 - ((y - p) ** 2).sum() / ((y - y.mean()) ** 2).sum())


def _make(name, cls, kind):
    return type(name, (_Base,), {"_est_cls": cls, "_kind": kind})


_ALGOS = {"GradientBoosting": _E.H2OGradientBoostingEstimator, "RandomForest": _E.H2ORandomForestEstimator,
          "XGBoost": _E.H2OXGBoostEstimator, "GeneralizedLinear": _E.H2OGeneralizedLinearEstimator,
          "DeepLearning": _E.H2ODeepLearningEstimator, "NaiveBayes": _E.H2ONaiveBayesEstimator,
          "StackedEnsemble": _E.H2OStackedEnsembleEstimator, "RuleFit": _E.H2ORuleFitEstimator}
for _n, _c in _ALGOS.items():
    globals()[f"H2O{_n}Classifier"] = _make(f"H2O{_n}Classifier", _c, "classifier")
    globals()[f"H2O{_n}Regressor"] = _make(f"H2O{_n}Regressor", _c, "regressor")
for _n, _c in {"KMeans": _E.H2OKMeansEstimator, "PrincipalComponentAnalysis": _E.H2OPrincipalComponentAnalysisEstimator,
               "IsolationForest": _E.H2OIsolationForestEstimator,
               "ExtendedIsolationForest": _E.H2OExtendedIsolationForestEstimator}.items():
    globals()[f"H2O{_n}Estimator"] = _make(f"H2O{_n}Estimator", _c, "estimator")
