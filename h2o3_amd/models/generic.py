"""Generic model: score an imported MOJO inside the platform.

Reference: hex/generic/Generic.java / GenericModel.java (wraps a MOJO read
by h2o-genmodel so it can be scored and evaluated like a native model).
"""
from __future__ import annotations

import numpy as np
import torch

from ..core.frame import H2OFrame
from ..parallel import cloud
from .base import H2OEstimator, TrainSpec


class H2OGenericEstimator(H2OEstimator):
    algo = "generic"
    _defaults = dict(model_key=None, path=None)

    @classmethod
    def from_file(cls, file=None, model_id=None):
        est = cls(path=file, model_id=model_id)
        est._load(file)
        return est

    def _load(self, path):
        from ..mojo.genmodel import MojoModel
        self._mojo = MojoModel.load(path)
        m = self._mojo.meta
        self._x = m["x"]
        self._y = m.get("response")
        self._ncls = self._mojo.nclasses
        self.supervised_learning = self._y is not None

    def train(self, x=None, y=None, training_frame=None, **kw):
        self._load(self._parms.get("path") or self._parms.get("model_key"))
        return self

    def _predict_raw(self, frame):
        df = frame.as_data_frame(local=True)          # each rank scores its own row shard
        raw = self._mojo.predict_raw(df)
        return torch.as_tensor(np.asarray(raw, dtype=np.float64), device=cloud.device())

    def predict(self, test_data, **kw):
        import pandas as pd
        return H2OFrame(self._mojo.predict(test_data.as_data_frame(local=True)), _local=True)

    def model_performance(self, test_data=None, **kw):
        spec = TrainSpec(test_data, self._x, self._y)
        if self._mojo.response_domain and test_data.vec(self._y).type == "enum":
            spec.response_domain = self._mojo.response_domain
            spec.nclasses = len(spec.response_domain)
        self._spec = spec
        return self._metrics_from_raw(spec, test_data, self._predict_raw(test_data))
