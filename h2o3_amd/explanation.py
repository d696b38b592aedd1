"""`h2o.explanation`: the public explanation surface of the reference client
(h2o-py/h2o/explanation/__init__.py + _explain.py) in one module.

The computations live in models/explain.py (device-side PDP / ICE / SHAP /
permutation importance, batched scoring) and models/explain_plots.py
(matplotlib drawing); this module re-exports them under the reference names
and adds the Pareto front (_explain.py:2702) and the helpers the reference
exports (`no_progress`, `pd_ice_common`).
"""
from __future__ import annotations

import contextlib

import numpy as np

from .models.explain import h_statistic, ice, partial_dependence, permutation_importance  # noqa: F401
from .models.explain_plots import (ice_plot, learning_curve_plot, model_correlation,  # noqa: F401
                                   model_correlation_heatmap, pd_multi_plot, pd_plot, residual_analysis_plot,
                                   shap_explain_row_plot, shap_summary_plot, varimp, varimp_heatmap)

__all__ = ["explain", "explain_row", "varimp_heatmap", "model_correlation_heatmap", "pd_multi_plot", "varimp",
           "model_correlation", "pareto_front", "shap_summary_plot", "shap_explain_row_plot", "pd_plot", "ice_plot",
           "pd_ice_common", "residual_analysis_plot", "learning_curve_plot", "no_progress",
           "register_explain_methods"]


def explain(models, frame, columns=None, top_n_features=5, include_explanations="ALL", exclude_explanations=(),
            plot_overrides=None, figsize=(16, 9), render=True, qualitative_colormap="Dark2",
            sequential_colormap="RdYlBu_r", background_frame=None):
    from .api import explain as _explain
    return _explain(models, frame, columns=columns, top_n_features=top_n_features,
                    include_explanations=include_explanations, exclude_explanations=exclude_explanations,
                    plot_overrides=plot_overrides or {}, figsize=figsize, render=render,
                    qualitative_colormap=qualitative_colormap, sequential_colormap=sequential_colormap,
                    background_frame=background_frame)


def explain_row(models, frame, row_index, columns=None, top_n_features=5, include_explanations="ALL",
                exclude_explanations=(), plot_overrides=None, qualitative_colormap="Dark2", figsize=(16, 9),
                render=True, background_frame=None):
    from .api import explain_row as _explain_row
    return _explain_row(models, frame, row_index, columns=columns, top_n_features=top_n_features,
                        include_explanations=include_explanations, exclude_explanations=exclude_explanations,
                        plot_overrides=plot_overrides or {}, qualitative_colormap=qualitative_colormap,
                        figsize=figsize, render=render, background_frame=background_frame)


@contextlib.contextmanager
def no_progress():
    """Context manager that silences progress output (the reference toggles
    its progress bar; in-process builds here print none)."""
    from . import api
    prev = getattr(api, "_progress_enabled", True)
    api._progress_enabled = False
    try:
        yield
    finally:
        api._progress_enabled = prev


def pd_ice_common(model, frame, column, row_index=None, target=None, max_levels=30, figsize=(16, 9), colormap=None,
                  save_plot_path=None, show_pdp=True, binary_response_scale="response", centered=False, is_ice=False,
                  grouping_column=None, output_graphing_data=False, nbins=100, show_rug=True, **kwargs):
    """Shared entry of pd_plot / ice_plot (_explain.py pd_ice_common)."""
    if is_ice:
        return ice_plot(model, frame, column, target=target, max_levels=max_levels, figsize=figsize,
                        colormap=colormap or "plasma", save_plot_path=save_plot_path, show_pdp=show_pdp,
                        binary_response_scale=binary_response_scale, centered=centered,
                        grouping_column=grouping_column, output_graphing_data=output_graphing_data, nbins=nbins,
                        show_rug=show_rug, **kwargs)
    return pd_plot(model, frame, column, row_index=row_index, target=target, max_levels=max_levels, figsize=figsize,
                   colormap=colormap or "Dark2", save_plot_path=save_plot_path,
                   binary_response_scale=binary_response_scale, grouping_column=grouping_column,
                   output_graphing_data=output_graphing_data, nbins=nbins, show_rug=show_rug, **kwargs)


def pareto_front_indices(x, y, top=True, left=True):
    """Indices of the non-dominated points for the optimum corner (top: larger
    y is better, left: smaller x is better), in x order.  A point is on the
    front when it strictly improves y over every point at least as good in x
    (equal x: the better y is seen first, so exact duplicates keep one)."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    ys = y if top else -y
    xs = x if left else -x
    order = np.lexsort((-ys, xs))           # by x, ties: better y first
    best = -np.inf
    keep = []
    for i in order:
        if ys[i] > best:
            keep.append(int(i))
            best = ys[i]
    return np.asarray(keep, dtype=np.int64)


def pareto_front(frame, x_metric=None, y_metric=None, optimum="top left", title=None, color_col="algo",
                 figsize=(16, 9), colormap="Dark2"):
    """Pareto front of a leaderboard-like frame (_explain.py:2702): the rows no
    other row beats in both metrics, drawn over all rows.  Returns the front's
    rows (H2OFrame, in row order) with `.figure()` giving the plot."""
    import pandas as pd
    from .core.frame import H2OFrame
    from .models.explain_plots import _plt
    if isinstance(frame, H2OFrame):
        lb = frame
        df = frame.as_data_frame()
    else:
        try:
            df = pd.DataFrame(frame)
            lb = H2OFrame(df)
        except Exception as e:  # noqa: BLE001
            raise ValueError("`frame` parameter has to be either H2OAutoML, H2OGrid, list of models or coercible "
                             "to H2OFrame!") from e
    if x_metric not in df.columns:
        raise ValueError(f"x_metric {x_metric} is not in the leaderboard!")
    if y_metric not in df.columns:
        raise ValueError(f"y_metric {y_metric} is not in the leaderboard!")
    opt = optimum.lower()
    if opt not in ("top left", "top right", "bottom left", "bottom right"):
        raise ValueError('Optimum has to be one of "top left", "top right", "bottom left", "bottom right".')
    top, left = "top" in opt, "left" in opt
    x = df[x_metric].to_numpy(dtype=np.float64)
    y = df[y_metric].to_numpy(dtype=np.float64)
    pf = pareto_front_indices(x, y, top=top, left=left)
    plt = _plt()
    fig = plt.figure(figsize=figsize)
    cols = None
    if color_col in df.columns:
        vals = df[color_col].astype(str).to_numpy()
        levels = sorted(set(vals))
        cmap = plt.get_cmap(colormap, max(len(levels), 1))
        to_c = {a: cmap(i) for i, a in enumerate(levels)}
        cols = np.array([to_c[a] for a in vals])
        from matplotlib.lines import Line2D
        plt.legend(handles=[Line2D([0], [0], marker="o", color="w", label=a, markerfacecolor=to_c[a], markersize=10)
                            for a in levels])
    plt.scatter(x, y, c=cols, alpha=0.5)
    plt.plot(x[pf], y[pf], c="k")
    plt.scatter(x[pf], y[pf], c=cols[pf] if cols is not None else None, s=100, zorder=100)
    plt.xlabel(x_metric)
    plt.ylabel(y_metric)
    plt.grid(True)
    plt.title(title if title is not None else "Pareto Front")
    sub = lb[sorted(pf.tolist()), :]
    sub.figure = lambda: fig
    return sub


def register_explain_methods():
    """The reference attaches the explanation functions to its model / AutoML
    classes at import; here the estimator and AutoML classes define them."""
    return None
