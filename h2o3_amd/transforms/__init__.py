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


# ---------------------------------------------------------------- munging steps
class TransformAttributeError(AttributeError):
    pass


class H2OTransformer:
    """fit / transform protocol of the frame transformers
    (h2o-py h2o/transforms/transform_base.py)."""

    def fit(self, X, y=None, **params):
        return self

    def transform(self, X, y=None, **params):
        raise NotImplementedError

    def fit_transform(self, X, y=None, **params):
        return self.fit(X, y, **params).transform(X, y, **params)

    def inverse_transform(self, X, y=None, **params):
        raise NotImplementedError


class H2OColOp(H2OTransformer):
    """A column operation: op (an H2OFrame method, e.g. H2OFrame.cos) on column
    col; inplace replaces the column, else the result is cbind-ed as
    new_col_name (h2o-py preprocessing.H2OColOp)."""

    def __init__(self, op, col=None, inplace=True, new_col_name=None, **params):
        if isinstance(col, (list, tuple)):
            raise ValueError("col must be None or a single column.")
        self.fun, self.col, self.inplace, self.new_col_name, self.params = op, col, inplace, new_col_name, params

    def _apply(self, X):
        src = X[self.col] if self.col is not None else X
        return self.fun(src, **self.params) if self.params else self.fun(src)

    def transform(self, X, y=None, **params):
        res = self._apply(X)
        if self.inplace:
            X[self.col] = res
            return X
        if self.new_col_name is not None:
            res.names = [self.new_col_name]
        return X.cbind(res)


class H2OCol:
    """A column reference used as an operand of H2OBinaryOp."""

    def __init__(self, column):
        self.col = column


class H2OBinaryOp(H2OColOp):
    """col <op> operand, the operand a constant or H2OCol (left= or right=)."""

    def __init__(self, op, col, inplace=True, new_col_name=None, left=None, right=None, **params):
        super().__init__(op, col, inplace, new_col_name, **params)
        self.left, self.right = left, right

    def _apply(self, X):
        def val(o):
            return X[o.col] if isinstance(o, H2OCol) else o
        if self.left is not None:
            return self.fun(val(self.left), X[self.col])
        return self.fun(X[self.col], val(self.right))
