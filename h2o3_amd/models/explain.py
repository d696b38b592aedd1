"""Model explainability: partial dependence, permutation importance,
Friedman-Popescu H statistic, and the data behind h2o.explain().

Reference: hex/PartialDependence.java (grid over a column, mean / stddev /
std-error of the response with the column forced to each grid value),
water/rapids/PermutationVarImp.java (metric drop when one column is
permuted, n_repeats, n_samples), hex/tree/FriedmanPopescusH.java
(H^2 from centred partial dependences), h2o-py/h2o/explanation/_explain.py
(explain() / explain_row() assemble varimp, SHAP summary, PDP/ICE,
residual analysis, leaderboard).

Everything here is built from the model's batched device predict(): one
scoring pass per grid point / permutation, no per-row host work.  explain()
returns the tables the reference plots and, with plot=True, the matplotlib
figures too (models/explain_plots.py).
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_ENUM, T_REAL, Vec
from ..parallel import cloud
from ..parallel import collectives as coll


def _replace(frame: H2OFrame, col: str, vec: Vec) -> H2OFrame:
    vecs = [vec if n == col else frame.vec(n) for n in frame.names]
    return H2OFrame.from_vecs(vecs, list(frame.names))


def _response(model, frame, target=None) -> torch.Tensor:
    """Per-row response used by PDP: p(class) for classifiers, predict otherwise."""
    raw = model._predict_raw(frame)
    spec = model._spec
    if spec is not None and spec.nclasses >= 2:
        dom = spec.response_domain
        k = dom.index(target) if target is not None else (1 if spec.nclasses == 2 else 0)
        return raw[:, k].to(torch.float64)
    return raw[:, 0].to(torch.float64)


def _wstats(v: torch.Tensor, w: torch.Tensor | None):
    if w is None:
        w = torch.ones_like(v)
    ok = ~torch.isnan(v)
    v, w = v[ok], w[ok]
    s = torch.stack([w.sum(), (w * v).sum(), (w * v * v).sum(), torch.tensor(float(v.numel()),
                                                                             dtype=v.dtype, device=v.device)])
    coll.allreduce_(s)
    sw, sv, svv, n = (float(x) for x in s)
    mean = sv / sw if sw > 0 else float("nan")
    var = max(svv / sw - mean * mean, 0.0) * (n / (n - 1) if n > 1 else 1.0) if sw > 0 else float("nan")
    sd = math.sqrt(var) if var == var else float("nan")
    return mean, sd, (sd / math.sqrt(n) if n > 0 else float("nan"))


def _grid(vec: Vec, nbins, user_split=None, include_na=False):
    if vec.type == T_ENUM:
        levels = list(range(len(vec.domain)))
        vals = [float(i) for i in levels]
        labels = list(vec.domain)
    elif user_split is not None:
        vals = [float(v) for v in user_split]
        labels = vals
    else:
        r = vec.rollups()
        lo, hi = float(r["min"]), float(r["max"])
        if vec.type != T_REAL and hi - lo + 1 <= nbins:   # integer columns: every value
            vals = [float(v) for v in np.arange(lo, hi + 1)]
        else:
            vals = list(np.linspace(lo, hi, nbins)) if hi > lo else [lo]
        labels = vals
    if include_na:
        vals = vals + [float("nan")]
        labels = list(labels) + [float("nan")]
    return vals, labels


def partial_dependence(model, frame: H2OFrame, cols, nbins=20, weight_column=None, include_na=False,
                       user_splits=None, targets=None, row_index=None):
    """Returns one pandas DataFrame per column: [col, mean_response,
    stddev_response, std_error_mean_response] (PartialDependence.java)."""
    if isinstance(cols, str):
        cols = [cols]
    w = frame.vec(weight_column).as_float(torch.float64) if weight_column else None
    if row_index is not None:
        frame = frame[int(row_index), :]
        w = None
    out = []
    tg = targets if targets else [None]
    for c in cols:
        vec = frame.vec(c)
        vals, labels = _grid(vec, nbins, (user_splits or {}).get(c), include_na)
        for t in tg:
            rows = []
            for v, lab in zip(vals, labels):
                if vec.type == T_ENUM:
                    code = -1 if v != v else int(v)
                    nv = Vec(torch.full((frame.nlocal,), code, dtype=torch.int32, device=vec.data.device),
                             T_ENUM, vec.domain)
                else:
                    nv = Vec(torch.full((frame.nlocal,), v, dtype=torch.float32, device=vec.data.device), T_REAL)
                resp = _response(model, _replace(frame, c, nv), t)
                m, sd, se = _wstats(resp, w)
                rows.append((lab, m, sd, se))
            df = pd.DataFrame(rows, columns=[c, "mean_response", "stddev_response", "std_error_mean_response"])
            if t is not None:
                df.attrs["target"] = t
            out.append(df)
    return out


def ice(model, frame: H2OFrame, col, nbins=20, max_rows=50, seed=0):
    """Individual conditional expectation curves for up to max_rows rows:
    DataFrame [row, col value, response]."""
    n = frame.nrow
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(n, size=min(n, max_rows), replace=False))
    sub = frame[list(map(int, idx)), :]
    vec = sub.vec(col)
    vals, labels = _grid(vec, nbins)
    recs = []
    for v, lab in zip(vals, labels):
        if vec.type == T_ENUM:
            nv = Vec(torch.full((sub.nlocal,), int(v), dtype=torch.int32, device=vec.data.device), T_ENUM, vec.domain)
        else:
            nv = Vec(torch.full((sub.nlocal,), v, dtype=torch.float32, device=vec.data.device), T_REAL)
        r = _response(model, _replace(sub, col, nv)).cpu().numpy()
        for i, rv in zip(idx, r):
            recs.append((int(i), lab, float(rv)))
    return pd.DataFrame(recs, columns=["row", col, "response"])


# ------------------------------------------------------------------ permutation varimp
_LOWER_BETTER = {"mse", "rmse", "mae", "rmsle", "logloss", "mean_per_class_error", "mean_residual_deviance"}
_METRIC_KEY = {"auc": "AUC", "aucpr": "pr_auc", "mse": "MSE", "rmse": "RMSE", "logloss": "logloss", "mae": "mae",
               "rmsle": "rmsle", "mean_per_class_error": "mean_per_class_error",
               "mean_residual_deviance": "mean_residual_deviance", "r2": "r2"}


def _perm_metric(model, frame, metric):
    mt = model.model_performance(frame)
    return float(mt.get(_METRIC_KEY.get(metric, metric)))


def permutation_importance(model, frame: H2OFrame, metric="AUTO", n_samples=10000, n_repeats=1, features=None,
                           seed=-1):
    """Metric degradation when a column is randomly permuted
    (PermutationVarImp.java).  Returns a pandas DataFrame: Variable,
    Relative Importance, Scaled Importance, Percentage (n_repeats == 1) or
    Variable, Run 1..Run n (n_repeats > 1)."""
    spec = model._spec
    metric = (metric or "AUTO").lower()
    if metric == "auto":
        metric = "logloss" if spec.nclasses >= 2 else "rmse"
    rng = np.random.default_rng(None if seed in (-1, None) else seed)
    if n_samples is not None and 0 < n_samples < frame.nrow:
        idx = np.sort(rng.choice(frame.nrow, size=n_samples, replace=False))
        frame = frame[list(map(int, idx)), :]
    base = _perm_metric(model, frame, metric)
    feats = list(features) if features else list(spec.x)
    runs = np.zeros((len(feats), n_repeats))
    for r in range(n_repeats):
        for i, c in enumerate(feats):
            vec = frame.vec(c)
            perm = torch.as_tensor(rng.permutation(frame.nlocal), device=vec.data.device)
            data = vec.data[perm] if isinstance(vec.data, torch.Tensor) else vec.data[perm.cpu().numpy()]
            nv = Vec(data, vec.type, vec.domain)
            val = _perm_metric(model, _replace(frame, c, nv), metric)
            runs[i, r] = (val - base) if metric in _LOWER_BETTER else (base - val)
    if n_repeats > 1:
        df = pd.DataFrame(runs, columns=[f"Run {i + 1}" for i in range(n_repeats)])
        df.insert(0, "Variable", feats)
        return df
    rel = runs[:, 0]
    order = np.argsort(-rel)
    mx = rel.max() if rel.size and rel.max() > 0 else 1.0
    tot = rel[rel > 0].sum() if (rel > 0).any() else 1.0
    return pd.DataFrame({"Variable": [feats[i] for i in order], "Relative Importance": rel[order],
                         "Scaled Importance": rel[order] / mx, "Percentage": rel[order] / tot})


# ------------------------------------------------------------------ Friedman-Popescu H
def h_statistic(model, frame: H2OFrame, variables, max_rows=200, seed=0):
    """Friedman & Popescu H statistic for the joint effect of `variables`
    (FriedmanPopescusH.java): H^2 = sum (F_S - sum_j F_j)^2 / sum F_S^2 over
    data points, with centred partial dependences evaluated AT the data."""
    variables = list(variables)
    n = frame.nrow
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(n, size=min(n, max_rows), replace=False))
    sub = frame[list(map(int, idx)), :]
    pts = {v: sub.vec(v).data.clone() for v in variables}
    m = sub.nlocal

    def pd_at(vs):
        out = np.zeros(m)
        for i in range(m):
            f = sub
            for v in vs:
                vec = sub.vec(v)
                val = pts[v][i]
                f = _replace(f, v, Vec(torch.full((m,), val.item(), dtype=vec.data.dtype, device=vec.data.device),
                                        vec.type, vec.domain))
            out[i] = float(_response(model, f).mean())
        return out - out.mean()

    joint = pd_at(variables)
    singles = [pd_at([v]) for v in variables]
    num = ((joint - sum(singles)) ** 2).sum()
    den = (joint ** 2).sum()
    return float(math.sqrt(num / den)) if den > 0 else 0.0


# ------------------------------------------------------------------ explain()
def explain(models, frame: H2OFrame, columns=None, top_n_features=5, include_explanations="ALL",
            exclude_explanations=(), plot=False, **kw):
    """h2o.explain(): dict of tables keyed like the reference's explanation
    sections; plot=True adds out["plots"][section] figures (varimp heatmap,
    model correlation, SHAP summary, PD / PD-multi, ICE, residual analysis,
    learning curve)."""
    if not isinstance(models, (list, tuple)):
        models = [models]
    ex = set(exclude_explanations or ())
    if include_explanations not in (None, "ALL"):
        inc = {include_explanations} if isinstance(include_explanations, str) else set(include_explanations)
        ex |= {"leaderboard", "varimp", "pdp", "shap_summary", "residual_analysis", "confusion_matrix", "ice",
               "varimp_heatmap", "model_correlation_heatmap", "learning_curve"} - inc
    out = {}
    m0 = models[0]
    if len(models) > 1 and "leaderboard" not in ex:
        from ..automl.leaderboard import Leaderboard
        out["leaderboard"] = Leaderboard(models, frame=frame).as_frame().as_data_frame()
    if "varimp" not in ex:
        vi = {}
        for m in models:
            try:
                vi[m.model_id] = m.varimp(use_pandas=True)
            except Exception:  # noqa: BLE001 - some algos have no varimp
                pass
        out["varimp"] = vi
    cols = columns
    if cols is None:
        cols = list(m0._spec.x)
        try:
            v = m0.varimp(use_pandas=True)
            if v is not None and len(v):
                cols = list(v["variable"])[:top_n_features]
        except Exception:  # noqa: BLE001
            cols = cols[:top_n_features]
    if "pdp" not in ex:
        out["pdp"] = {c: partial_dependence(m0, frame, c)[0] for c in cols}
    if "shap_summary" not in ex and m0.algo in ("gbm", "drf", "xgboost") and m0._spec.nclasses <= 2:
        out["shap_summary"] = m0.predict_contributions(frame).as_data_frame()
    if "residual_analysis" not in ex and m0._spec.nclasses < 2:
        p = m0.predict(frame).as_data_frame()["predict"].values
        y = frame[m0._spec.y].as_data_frame().iloc[:, 0].values
        out["residual_analysis"] = pd.DataFrame({"fitted": p, "residual": y - p})
    if "confusion_matrix" not in ex and m0._spec.nclasses >= 2:
        out["confusion_matrix"] = m0.model_performance(frame).confusion_matrix()
    if plot:
        from . import explain_plots as xp
        figs = {}
        if len(models) > 1:
            if "varimp_heatmap" not in ex:
                try:
                    figs["varimp_heatmap"] = xp.varimp_heatmap(models)
                except RuntimeError:
                    pass
            if "model_correlation_heatmap" not in ex:
                figs["model_correlation_heatmap"] = xp.model_correlation_heatmap(models, frame)
            if "pdp" not in ex:
                figs["pdp"] = {c: xp.pd_multi_plot(models, frame, c) for c in cols}
        else:
            if "varimp" not in ex and out.get("varimp"):
                figs["varimp"] = m0.varimp_plot(server=True)
            if "pdp" not in ex:
                figs["pdp"] = {c: xp.pd_plot(m0, frame, c) for c in cols}
            if "ice" not in ex:
                figs["ice"] = {c: xp.ice_plot(m0, frame, c) for c in cols}
        if "shap_summary" in out:
            figs["shap_summary"] = xp.shap_summary_plot(m0, frame)
        if "residual_analysis" in out:
            figs["residual_analysis"] = xp.residual_analysis_plot(m0, frame)
        if "learning_curve" not in ex:
            figs["learning_curve"] = xp.learning_curve_plot(m0)
        out["plots"] = figs
    return out


def explain_row(models, frame: H2OFrame, row_index, columns=None, top_n_features=5, plot=False, **kw):
    if not isinstance(models, (list, tuple)):
        models = [models]
    m0 = models[0]
    row = frame[int(row_index), :]
    out = {}
    shap = m0.algo in ("gbm", "drf", "xgboost") and m0._spec.nclasses <= 2
    if shap:
        out["shap_explain_row"] = m0.predict_contributions(row).as_data_frame()
    cols = columns or list(m0._spec.x)[:top_n_features]
    out["ice"] = {c: partial_dependence(m0, frame, c, row_index=row_index)[0] for c in cols}
    if plot:
        from . import explain_plots as xp
        figs = {"ice": {c: xp.pd_plot(m0, frame, c, row_index=row_index) for c in cols}}
        if shap:
            figs["shap_explain_row"] = xp.shap_explain_row_plot(m0, frame, row_index)
        out["plots"] = figs
    return out
