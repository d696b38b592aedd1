"""Leaderboard (reference: hex/leaderboard/Leaderboard.java).

Rows sorted by the problem's default metric (AUC for binomial,
mean_per_class_error for multinomial, mean_residual_deviance for
regression), computed on the leaderboard frame when given, else on the
cross-validation metrics, else validation, else training.
"""
from __future__ import annotations

import math
import time

_DEFAULT = {2: "auc", 1: "mean_residual_deviance"}
_COLS = {"binomial": ["auc", "logloss", "aucpr", "mean_per_class_error", "rmse", "mse"],
         "multinomial": ["mean_per_class_error", "logloss", "rmse", "mse"],
         "regression": ["rmse", "mse", "mae", "rmsle", "mean_residual_deviance"]}
_KEY = {"auc": "AUC", "logloss": "logloss", "aucpr": "pr_auc", "mean_per_class_error": "mean_per_class_error",
        "rmse": "RMSE", "mse": "MSE", "mae": "mae", "rmsle": "rmsle", "mean_residual_deviance": "mean_residual_deviance",
        "deviance": "mean_residual_deviance"}


class Leaderboard:
    def __init__(self, models, sort_metric="AUTO", frame=None):
        self.frame = frame
        models = [m for m in models if m is not None]
        self.kind = "regression"
        if models and models[0]._spec is not None and models[0]._spec.nclasses == 2:
            self.kind = "binomial"
        elif models and models[0]._spec is not None and models[0]._spec.nclasses > 2:
            self.kind = "multinomial"
        sm = (sort_metric or "AUTO").lower()
        if sm == "auto":
            sm = {"binomial": "auc", "multinomial": "mean_per_class_error", "regression": "mean_residual_deviance"}[self.kind]
        self.sort_metric = sm
        self._cache = {}
        self._ptime = {}
        dec = sm in ("auc", "aucpr")
        self.models = sorted(models, key=lambda m: self._score(m, sm), reverse=dec)

    def _metrics(self, m):
        if m.model_id in self._cache:
            return self._cache[m.model_id]
        if self.frame is not None:
            t0 = time.perf_counter()
            mt = m.model_performance(self.frame)
            self._ptime[m.model_id] = 1000.0 * (time.perf_counter() - t0) / max(int(self.frame.nrows), 1)
        else:
            mt = m._cross_validation_metrics or m._validation_metrics or m._training_metrics
        self._cache[m.model_id] = mt
        return mt

    def _score(self, m, metric):
        mt = self._metrics(m)
        v = None if mt is None else mt.get(_KEY.get(metric, metric))
        if v is None or (isinstance(v, float) and math.isnan(v)):
            return -math.inf if metric in ("auc", "aucpr") else math.inf
        return v

    def _predict_time(self, m):
        """Per-row scoring time in ms (LeaderboardExtensionsProvider's
        predict_time_per_row_ms): timed on the leaderboard frame when the board
        was scored on one, else on up to 10k rows of the model's training frame."""
        if m.model_id not in self._ptime:
            fr = getattr(getattr(m, "_spec", None), "frame", None)
            if fr is None:
                return float("nan")
            n = min(int(fr.nrows), 10000)
            sub = fr[:n, :] if n < int(fr.nrows) else fr
            t0 = time.perf_counter()
            m.predict(sub)
            self._ptime[m.model_id] = 1000.0 * (time.perf_counter() - t0) / max(n, 1)
        return self._ptime[m.model_id]

    def as_frame(self, extra_columns=None):
        from ..core.frame import H2OFrame
        return H2OFrame(self.as_pandas(extra_columns), column_types={"model_id": "string"})

    def as_pandas(self, extra_columns=None):
        """The leaderboard rows as a host table (replicated on every rank; no
        frame, so REST reads need no collectives)."""
        import pandas as pd
        rows = []
        for m in self.models:
            r = {"model_id": m.model_id}
            for c in _COLS[self.kind]:
                v = self._score(m, c)
                r[c] = v if math.isfinite(v) else float("nan")
            if extra_columns in ("ALL", "training_time_ms") or (isinstance(extra_columns, list) and "training_time_ms" in extra_columns):
                r["training_time_ms"] = int(m._run_time * 1000)
            if extra_columns == "ALL" or (isinstance(extra_columns, list) and "predict_time_per_row_ms" in extra_columns):
                r["predict_time_per_row_ms"] = self._predict_time(m)
            if extra_columns == "ALL" or (isinstance(extra_columns, list) and "algo" in extra_columns):
                r["algo"] = m.algo
            rows.append(r)
        return pd.DataFrame(rows, columns=["model_id"] + list(_COLS[self.kind]) if not rows else None)


def make_leaderboard(object, leaderboard_frame=None, sort_metric="AUTO", extra_columns=(), scoring_data="AUTO"):
    """Leaderboard frame over models, grids and AutoML runs (reference h2o-py
    h2o/scoring.py make_leaderboard -> hex/leaderboard/Leaderboard.java):
    scored on leaderboard_frame when given, else on the xval / valid / train
    metrics (scoring_data narrows that choice)."""
    def models_of(o):
        if isinstance(o, (list, tuple)):
            return [m for x in o for m in models_of(x)]
        if hasattr(o, "models") and not hasattr(o, "model_id"):
            return list(o.models)
        if isinstance(o, str):
            from ..core import dkv
            return models_of(dkv.get(o))
        return [o]
    models = models_of(object)
    sd = str(scoring_data).lower()
    if leaderboard_frame is None and sd in ("train", "valid", "xval"):
        attr = {"train": "_training_metrics", "valid": "_validation_metrics", "xval": "_cross_validation_metrics"}[sd]
        lb = Leaderboard(models, sort_metric)
        lb._cache = {m.model_id: getattr(m, attr) for m in models}
        lb.models = sorted(models, key=lambda m: lb._score(m, lb.sort_metric),
                           reverse=lb.sort_metric in ("auc", "aucpr"))
    else:
        lb = Leaderboard(models, sort_metric, leaderboard_frame)
    ec = extra_columns if isinstance(extra_columns, str) else (list(extra_columns) if extra_columns else None)
    return lb.as_frame(ec)
