"""Segment models: one model per segment of the data.

Reference: hex/segments/SegmentModelsBuilder.java, SegmentModels.java,
h2o-py h2o/model/segment_models.py (train_segments(segment_columns=...,
segment_models_id, parallelism): the segment frame lists every segment,
its model id, status and errors; as_frame() returns that table).

MI355X design: segments are row masks over the resident frame (no copy
to other nodes); each segment's model trains on the same device in turn
(a model per segment is usually small, so the device is shared serially;
the reference's `parallelism` maps to sequential execution here).
"""
from __future__ import annotations

import itertools
import traceback

import pandas as pd
import torch

from ..core import dkv
from ..core.frame import H2OFrame


class H2OSegmentModels:
    def __init__(self, segment_models_id=None):
        self.segment_models_id = segment_models_id or dkv.make_key("segment_models")
        self._rows = []
        self._models = {}

    def as_frame(self):
        return H2OFrame(pd.DataFrame(self._rows))

    def get_model(self, **segment):
        key = tuple(sorted(segment.items()))
        return self._models.get(key)


def train_segments(estimator, x=None, y=None, training_frame=None, segment_columns=None, segments=None,
                   segment_models_id=None, parallelism=1, verbose=False, **train_kw):
    segment_columns = [segment_columns] if isinstance(segment_columns, str) else list(segment_columns)
    df = training_frame[:, segment_columns].as_data_frame()
    if segments is not None:
        sdf = segments.as_data_frame() if isinstance(segments, H2OFrame) else pd.DataFrame(segments)
        combos = [tuple(r) for r in sdf[segment_columns].itertuples(index=False)]
    else:
        combos = sorted(set(tuple(r) for r in df.itertuples(index=False)), key=lambda t: tuple(map(str, t)))
    out = H2OSegmentModels(segment_models_id)
    cls = type(estimator)
    parms = {k: v for k, v in estimator._user_parms().items() if k != "model_id"}
    for combo in combos:
        mask = torch.ones(training_frame.nlocal, dtype=torch.bool)
        for c, v in zip(segment_columns, combo):
            col = df[c]
            mask &= torch.as_tensor((col == v).values if not (isinstance(v, float) and v != v) else col.isna().values)
        idx = torch.nonzero(mask).view(-1).tolist()
        row = {c: v for c, v in zip(segment_columns, combo)}
        try:
            sub = training_frame[idx, :]
            m = cls(**parms)
            xs = [c for c in (x or sub.names) if c not in segment_columns and c != y]
            m.train(x=xs, y=y, training_frame=sub, **train_kw)
            out._models[tuple(sorted(row.items()))] = m
            row.update(model=m.model_id, status="SUCCEEDED", errors=None, warnings=None)
        except Exception as e:  # noqa: BLE001 - a failing segment is reported, not raised (reference)
            row.update(model=None, status="FAILED", errors=str(e), warnings=None)
            if verbose:
                traceback.print_exc()
        out._rows.append(row)
    dkv.put(out.segment_models_id, out)
    return out
