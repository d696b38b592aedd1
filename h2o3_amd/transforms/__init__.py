"""Frame transformers (reference: h2o-py h2o/transforms/preprocessing.py
H2OScaler / H2OColSelect, decomposition.py H2OPCA / H2OSVD) with the
fit / transform / fit_transform protocol."""
from __future__ import annotations

import torch

from ..core.frame import H2OFrame
from ..core.vec import T_REAL, Vec


class H2OScaler:
    def __init__(self, center=True, scale=True):
        self.center, self.scale = center, scale
        self.means = self.stds = None

    def fit(self, X, y=None, **params):
        cols = [c for c in X.names if X.vec(c).is_numeric]
        self.means = {c: (X.vec(c).rollups()["mean"] if self.center else 0.0) for c in cols}
        self.stds = {c: (X.vec(c).rollups()["sigma"] if self.scale else 1.0) or 1.0 for c in cols}
        return self

    def transform(self, X, y=None, **params):
        vecs = []
        for c in X.names:
            v = X.vec(c)
            if c in self.means:
                vecs.append(Vec(((v.as_float(torch.float32) - self.means[c]) / self.stds[c]).contiguous(), T_REAL))
            else:
                vecs.append(v)
        return H2OFrame.from_vecs(vecs, list(X.names))

    def fit_transform(self, X, y=None, **params):
        return self.fit(X).transform(X)

    def inverse_transform(self, X, y=None, **params):
        vecs = []
        for c in X.names:
            v = X.vec(c)
            if c in self.means:
                vecs.append(Vec((v.as_float(torch.float32) * self.stds[c] + self.means[c]).contiguous(), T_REAL))
            else:
                vecs.append(v)
        return H2OFrame.from_vecs(vecs, list(X.names))


class H2OColSelect:
    def __init__(self, cols):
        self.cols = list(cols)

    def fit(self, X, y=None, **p):
        return self

    def transform(self, X, y=None, **p):
        return X[:, self.cols]

    def fit_transform(self, X, y=None, **p):
        return self.transform(X)


class _Decomp:
    _cls = None

    def __init__(self, **params):
        self.params = params
        self.model = None

    def fit(self, X, y=None, **p):
        self.model = self._cls(**self.params)
        self.model.train(training_frame=X)
        return self

    def transform(self, X, y=None, **p):
        return self.model.predict(X)

    def fit_transform(self, X, y=None, **p):
        return self.fit(X).transform(X)


def _pca():
    from ..estimators import H2OPrincipalComponentAnalysisEstimator
    return H2OPrincipalComponentAnalysisEstimator


def _svd():
    from ..estimators import H2OSingularValueDecompositionEstimator
    return H2OSingularValueDecompositionEstimator


class H2OPCA(_Decomp):
    @property
    def _cls(self):
        return _pca()


class H2OSVD(_Decomp):
    @property
    def _cls(self):
        return _svd()
