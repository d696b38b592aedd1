"""h2o.explain() plots: variable-importance heatmap, model correlation
heatmap, SHAP summary / explain-row, partial dependence (single / multi
model), ICE, residual analysis, learning curves.

Reference: h2o-py/h2o/explanation/_explain.py (varimp / varimp_heatmap,
model_correlation / model_correlation_heatmap with single-linkage leaf
ordering `_calculate_clustering_indices`, shap_summary_plot,
shap_explain_row_plot, pd_plot, pd_multi_plot, ice_plot,
residual_analysis_plot, learning_curve_plot, explain / explain_row).

The data comes from the device-side explainability code (models/explain.py,
TreeSHAP, batched predict); matplotlib (Agg) only draws.  Every plot
function returns a matplotlib Figure; the `*_data` helpers and `varimp()` /
`model_correlation()` return the tables the plots are drawn from.
"""
from __future__ import annotations

import re

import numpy as np
import pandas as pd


def _plt():
    import matplotlib
    if matplotlib.get_backend().lower() not in ("agg", "module://matplotlib_inline.backend_inline"):
        try:
            matplotlib.use("Agg")
        except Exception:  # noqa: BLE001 - a backend is already active
            pass
    import matplotlib.pyplot as plt
    return plt


def _shorten_model_ids(ids):
    rx = re.compile(r"(.*)_AutoML_[\d_]+((?:_.*)?)$")
    short = [rx.sub(r"\1\2", i) for i in ids]
    return short if len(set(short)) == len(set(ids)) else list(ids)


def _clustering_order(matrix):
    """Leaf order of a single-linkage clustering of the matrix's columns."""
    cols = matrix.shape[1]
    dist = np.full((cols, cols), np.inf)
    for a in range(cols):
        for b in range(a + 1, cols):
            dist[a, b] = dist[b, a] = float(np.sum((matrix[:, a] - matrix[:, b]) ** 2))
    groups = [[i] for i in range(cols)]
    for _ in range(cols - 1):
        idx = int(np.argmin(dist))
        x, y = idx % cols, idx // cols
        groups[x].append(groups[y])
        groups[y] = []
        dist[x, :] = np.min(dist[[x, y], :], axis=0)
        dist[y, :] = np.inf
        dist[:, y] = np.inf
        dist[x, x] = np.inf

    def flat(g):
        for e in g:
            if isinstance(e, list):
                yield from flat(e)
            else:
                yield e
    return list(flat(groups))


def _models(models):
    if hasattr(models, "leader") and hasattr(models, "leaderboard"):
        from ..core import dkv
        return [dkv.get(mid) for mid in models._leaderboard_ids()] if hasattr(models, "_leaderboard_ids") else \
            list(models._models)
    return list(models) if isinstance(models, (list, tuple)) else [models]


def _consolidated_varimp(model):
    """Variable importance per ORIGINAL column (one-hot levels summed)."""
    vi = model.varimp(use_pandas=True)
    x = list(model._spec.x)
    out = {c: 0.0 for c in x}
    if vi is None:
        return out
    for name, val in zip(vi["variable"], vi["relative_importance"] if "relative_importance" in vi else vi.iloc[:, 1]):
        base = name if name in out else name.split(".")[0]
        if base in out:
            out[base] += float(val)
    tot = max(out.values()) or 1.0
    return {k: v / tot for k, v in out.items()}


def varimp(models, num_of_features=20, cluster=True, use_pandas=True):
    ms = []
    for m in _models(models):
        try:
            if m.varimp(use_pandas=True) is not None:
                ms.append(m)
        except Exception:  # noqa: BLE001 - algos without varimp are skipped like the reference
            pass
    if not ms:
        raise RuntimeError("No model with variable importance")
    x = list(ms[0]._spec.x)
    V = np.array([[_consolidated_varimp(m).get(c, 0.0) for c in x] for m in ms])
    if num_of_features is not None:
        ranks = np.amax(V, axis=0).argsort()
        mask = (ranks.max() - ranks) < num_of_features
        V = V[:, mask]
        x = [c for i, c in enumerate(x) if mask[i]]
    if cluster and len(ms) > 2:
        o = _clustering_order(V)
        x = [x[i] for i in o]
        V = V[:, o].T
        o = _clustering_order(V)
        ms = [ms[i] for i in o]
        V = V[:, o]
    else:
        V = V.T
    ids = _shorten_model_ids([m.model_id for m in ms])
    if use_pandas:
        return pd.DataFrame(V, columns=ids, index=x)
    return V, ids, x


def _heatmap(M, xlabels, ylabels, title, vmin=None, vmax=None, figsize=(8, 6)):
    plt = _plt()
    fig, ax = plt.subplots(figsize=figsize)
    im = ax.imshow(M, cmap="RdYlBu_r", vmin=vmin, vmax=vmax, aspect="auto")
    ax.set_xticks(range(len(xlabels)))
    ax.set_xticklabels(xlabels, rotation=45, ha="right")
    ax.set_yticks(range(len(ylabels)))
    ax.set_yticklabels(ylabels)
    fig.colorbar(im, ax=ax)
    ax.set_title(title)
    fig.tight_layout()
    return fig


def varimp_heatmap(models, top_n=None, num_of_features=20, figsize=(16, 9), cluster=True, colormap="RdYlBu_r",
                   save_plot_path=None):
    df = varimp(models[:top_n] if top_n and isinstance(models, list) else models, num_of_features, cluster)
    fig = _heatmap(df.values, list(df.columns), list(df.index), "Variable Importance Heatmap", 0, 1, figsize)
    if save_plot_path:
        fig.savefig(save_plot_path)
    return fig


def model_correlation(models, frame, cluster_models=True, use_pandas=True):
    ms = _models(models)
    cls = ms[0]._spec.is_classification
    preds = [m.predict(frame).as_data_frame()["predict"].values for m in ms]
    n = len(ms)
    C = np.ones((n, n))
    for i in range(n):
        for j in range(i + 1, n):
            if cls:
                C[i, j] = C[j, i] = float(np.mean(preds[i] == preds[j]))
            else:
                C[i, j] = C[j, i] = float(np.corrcoef(preds[i].astype(float), preds[j].astype(float))[0, 1])
    if cluster_models and n > 1:
        o = _clustering_order(C)
        C = C[o][:, o]
        ms = [ms[i] for i in o]
    ids = _shorten_model_ids([m.model_id for m in ms])
    return pd.DataFrame(C, columns=ids, index=ids) if use_pandas else (C, ids)


def model_correlation_heatmap(models, frame, top_n=None, cluster_models=True, triangular=True, figsize=(13, 13),
                              colormap="RdYlBu_r", save_plot_path=None):
    df = model_correlation(models[:top_n] if top_n and isinstance(models, list) else models, frame, cluster_models)
    M = df.values.copy()
    if triangular:
        M[np.triu_indices_from(M, 1)] = np.nan
    fig = _heatmap(M, list(df.columns), list(df.index), "Model Correlation", 0, 1, figsize)
    if save_plot_path:
        fig.savefig(save_plot_path)
    return fig


def shap_summary_plot(model, frame, columns=None, top_n_features=20, samples=1000, background_frame=None,
                      colorize_factors=True, alpha=1, colormap=None, figsize=(12, 12), jitter=0.35,
                      save_plot_path=None):
    """Beeswarm of per-row contributions, features ordered by mean |contribution|,
    points coloured by the normalized feature value."""
    plt = _plt()
    fr = frame
    if samples and frame.nrows > samples:
        fr = frame.split_frame(ratios=[samples / frame.nrows], seed=42)[0]
    contr = model.predict_contributions(fr).as_data_frame()
    contr = contr[[c for c in contr.columns if c != "BiasTerm"]]
    imp = contr.abs().mean().sort_values(ascending=False)
    cols = list(imp.index[:top_n_features]) if columns is None else list(columns)
    data = fr.as_data_frame()
    rng = np.random.RandomState(0)
    fig, ax = plt.subplots(figsize=figsize)
    for i, c in enumerate(reversed(cols)):
        v = data[c] if c in data else pd.Series(np.zeros(len(contr)))
        if v.dtype.kind in "biuf":
            vv = v.astype(float).values
            lo, hi = np.nanpercentile(vv, 5), np.nanpercentile(vv, 95)
            col = np.clip((vv - lo) / (hi - lo if hi > lo else 1), 0, 1)
        else:
            codes = pd.Categorical(v).codes.astype(float)
            col = codes / max(codes.max(), 1)
        y = i + rng.uniform(-jitter, jitter, len(contr))
        ax.scatter(contr[c].values, y, c=col, cmap=colormap or "RdYlBu_r", s=6, alpha=alpha)
    ax.set_yticks(range(len(cols)))
    ax.set_yticklabels(list(reversed(cols)))
    ax.axvline(0, color="grey", lw=0.5)
    ax.set_xlabel("SHAP value (contribution)")
    ax.set_title(f"SHAP Summary plot for \"{model.model_id}\"")
    fig.tight_layout()
    if save_plot_path:
        fig.savefig(save_plot_path)
    return fig


def shap_explain_row_plot(model, frame, row_index, columns=None, top_n_features=10, figsize=(16, 9),
                          plot_type="barplot", contribution_type="both", save_plot_path=None):
    plt = _plt()
    row = frame[int(row_index), :]
    contr = model.predict_contributions(row).as_data_frame().iloc[0]
    bias = float(contr.get("BiasTerm", 0.0))
    contr = contr.drop(labels=[c for c in contr.index if c == "BiasTerm"])
    order = contr.abs().sort_values(ascending=False).index[:top_n_features] if columns is None else list(columns)
    vals = contr[order][::-1]
    fig, ax = plt.subplots(figsize=figsize)
    ax.barh(list(vals.index), vals.values, color=["#d62728" if v > 0 else "#1f77b4" for v in vals.values])
    ax.set_title(f"SHAP explanation for \"{model.model_id}\" on row {row_index} (bias {bias:.4g})")
    ax.set_xlabel("contribution")
    fig.tight_layout()
    if save_plot_path:
        fig.savefig(save_plot_path)
    return fig


def pd_plot(model, frame, column, row_index=None, target=None, max_levels=30, figsize=(16, 9),
            colormap="Dark2", save_plot_path=None, show_rug=True, include_na=False, **kw):
    from .explain import partial_dependence
    plt = _plt()
    df = partial_dependence(model, frame, column, include_na=include_na, row_index=row_index,
                            targets=[target] if target else None)[0]
    fig, ax = plt.subplots(figsize=figsize)
    x = df.iloc[:, 0]
    if x.dtype.kind in "biuf":
        ax.plot(x, df["mean_response"], marker="o")
        ax.fill_between(x.astype(float), df["mean_response"] - df["stddev_response"],
                        df["mean_response"] + df["stddev_response"], alpha=0.2)
    else:
        ax.bar(x.astype(str), df["mean_response"], yerr=df["stddev_response"])
    ax.set_xlabel(column)
    ax.set_ylabel("Mean Response")
    ax.set_title(f"Partial Dependence plot for \"{column}\"" + ("" if row_index is None else f" (row {row_index})"))
    fig.tight_layout()
    if save_plot_path:
        fig.savefig(save_plot_path)
    return fig


def pd_multi_plot(models, frame, column, best_of_family=True, row_index=None, target=None, max_levels=30,
                  figsize=(16, 9), colormap="Dark2", markers=None, save_plot_path=None, **kw):
    from .explain import partial_dependence
    plt = _plt()
    fig, ax = plt.subplots(figsize=figsize)
    for m in _models(models):
        df = partial_dependence(m, frame, column, row_index=row_index, targets=[target] if target else None)[0]
        x = df.iloc[:, 0]
        ax.plot(x.astype(float) if x.dtype.kind in "biuf" else x.astype(str), df["mean_response"], marker="o",
                label=m.model_id)
    ax.legend()
    ax.set_xlabel(column)
    ax.set_ylabel("Mean Response")
    ax.set_title(f"Partial Dependence plot for \"{column}\"")
    fig.tight_layout()
    if save_plot_path:
        fig.savefig(save_plot_path)
    return fig


def ice_plot(model, frame, column, target=None, max_levels=30, figsize=(16, 9), colormap="plasma",
             save_plot_path=None, show_pdp=True, binary_response_scale="response", centered=False, **kw):
    from .explain import ice, partial_dependence
    plt = _plt()
    df = ice(model, frame, column)
    fig, ax = plt.subplots(figsize=figsize)
    for r, g in df.groupby("row"):
        resp = g["response"].values
        if centered:
            resp = resp - resp[0]
        x = g[column]
        ax.plot(x.astype(float) if x.dtype.kind in "biuf" else x.astype(str), resp, lw=0.8, alpha=0.6)
    if show_pdp:
        pdp = partial_dependence(model, frame, column, targets=[target] if target else None)[0]
        x = pdp.iloc[:, 0]
        mr = pdp["mean_response"].values
        ax.plot(x.astype(float) if x.dtype.kind in "biuf" else x.astype(str), mr - (mr[0] if centered else 0),
                color="black", lw=2, ls="--", label="Partial Dependence")
        ax.legend()
    ax.set_xlabel(column)
    ax.set_ylabel("Response")
    ax.set_title(f"Individual Conditional Expectation for \"{column}\"")
    fig.tight_layout()
    if save_plot_path:
        fig.savefig(save_plot_path)
    return fig


def residual_analysis_plot(model, frame, figsize=(16, 9), save_plot_path=None):
    plt = _plt()
    p = model.predict(frame).as_data_frame()["predict"].values.astype(float)
    y = frame[model._spec.y].as_data_frame().iloc[:, 0].values.astype(float)
    r = y - p
    fig, ax = plt.subplots(figsize=figsize)
    ax.scatter(p, r, s=4, alpha=0.5)
    ax.axhline(0, color="grey")
    if len(p) > 1:
        k, b = np.polyfit(p, r, 1)
        xs = np.linspace(p.min(), p.max(), 10)
        ax.plot(xs, k * xs + b, color="#d62728")
    ax.set_xlabel("Fitted")
    ax.set_ylabel("Residuals")
    ax.set_title(f"Residual Analysis for \"{model.model_id}\"")
    fig.tight_layout()
    if save_plot_path:
        fig.savefig(save_plot_path)
    return fig


def learning_curve_data(model, metric="AUTO"):
    sh = model.scoring_history() if callable(getattr(model, "scoring_history", None)) else model._scoring_history
    df = sh if isinstance(sh, pd.DataFrame) else pd.DataFrame(sh or [])
    if df.empty:
        return df, None, None
    x = next((c for c in ("number_of_trees", "iterations", "epochs", "iteration", "samples") if c in df), None)
    if metric in (None, "AUTO", "auto"):
        for cand in ("logloss", "deviance", "rmse", "mse", "within_cluster_sum_of_squares", "objective"):
            if any(c.endswith(cand) for c in df.columns):
                metric = cand
                break
    return df, x, metric


def learning_curve_plot(model, metric="AUTO", cv_ribbon=None, cv_lines=None, figsize=(16, 9), colormap=None,
                        save_plot_path=None):
    plt = _plt()
    df, x, metric = learning_curve_data(model, metric)
    fig, ax = plt.subplots(figsize=figsize)
    if not df.empty and metric:
        xs = df[x] if x else np.arange(len(df))
        for col in [c for c in df.columns if c.endswith(metric)]:
            ax.plot(xs, df[col], marker="o", label=col)
        ax.legend()
        ax.set_xlabel(x or "scoring event")
        ax.set_ylabel(metric)
    ax.set_title(f"Learning Curve for \"{model.model_id}\"")
    fig.tight_layout()
    if save_plot_path:
        fig.savefig(save_plot_path)
    return fig
