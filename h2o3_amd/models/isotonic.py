"""Isotonic regression.

Reference: hex/isotonic/IsotonicRegression.java (+ PoolAdjacentViolators
and IsotonicRegressionModel: thresholds_x / thresholds_y, linear
interpolation between thresholds, out_of_bounds = "NA" | "clip").

MI355X design: rows are sorted on the device (one argsort), rows sharing an
x are pre-merged with a segmented sum, and only the (much shorter) unique-x
sequence goes through the inherently sequential pool-adjacent-violators
pass on the host.  Scoring is a device searchsorted + lerp.
"""
from __future__ import annotations

import numpy as np
import torch

from ..parallel import collectives as coll
from .base import H2OEstimator
from ..core.groupsum import index_add as _ia

ISO_DEFAULTS = dict(out_of_bounds="NA", custom_metric_func=None)


def pava(y: np.ndarray, w: np.ndarray):
    """Pool adjacent violators (non-decreasing).  Returns block (start, y, w)."""
    ys, ws, starts = [], [], []
    for i in range(len(y)):
        ys.append(float(y[i])); ws.append(float(w[i])); starts.append(i)
        while len(ys) > 1 and ys[-2] > ys[-1]:
            wt = ws[-2] + ws[-1]
            yv = (ys[-2] * ws[-2] + ys[-1] * ws[-1]) / wt
            ys.pop(); ws.pop(); starts.pop()
            ys[-1], ws[-1] = yv, wt
    return np.asarray(starts), np.asarray(ys), np.asarray(ws)


class H2OIsotonicRegressionEstimator(H2OEstimator):
    algo = "isotonicregression"
    _defaults = ISO_DEFAULTS

    def _fit(self, spec):
        if len(spec.x) != 1:
            raise ValueError("Isotonic regression requires exactly one predictor column")
        if spec.is_classification:
            raise ValueError("Isotonic regression requires a numeric response")
        x = spec.frame.vec(spec.x[0]).as_float(torch.float64)
        y = spec.y_tensor(dtype=torch.float64)
        w = spec.w_tensor()
        w = torch.ones_like(y) if w is None else w.to(torch.float64)
        ok = ~torch.isnan(x) & ~torch.isnan(y) & (w > 0)
        x, y, w = x[ok], y[ok], w[ok]
        x, y, w = coll.all_gather_var(x), coll.all_gather_var(y), coll.all_gather_var(w)
        o = torch.argsort(x)
        x, y, w = x[o], y[o], w[o]
        ux, inv = torch.unique_consecutive(x, return_inverse=True)
        sw = _ia(torch.zeros(ux.numel(), dtype=torch.float64, device=x.device), inv, w)
        swy = _ia(torch.zeros(ux.numel(), dtype=torch.float64, device=x.device), inv, w * y)
        uxh, yh, wh = ux.cpu().numpy(), (swy / sw).cpu().numpy(), sw.cpu().numpy()
        starts, by, _ = pava(yh, wh)
        ends = np.concatenate([starts[1:], [len(uxh)]]) - 1
        # thresholds: block endpoints (both ends when the block spans > 1 x)
        tx, ty = [], []
        for s, e, v in zip(starts, ends, by):
            tx.append(uxh[s]); ty.append(v)
            if e > s:
                tx.append(uxh[e]); ty.append(v)
        self._tx = np.asarray(tx)
        self._ty = np.asarray(ty)
        self._output["thresholds_x"] = self._tx.tolist()
        self._output["thresholds_y"] = self._ty.tolist()
        self._output["min_x"], self._output["max_x"] = float(uxh[0]), float(uxh[-1])

    def _predict_raw(self, frame):
        x = frame.vec(self._spec.x[0]).as_float(torch.float64)
        tx = torch.as_tensor(self._tx, device=x.device)
        ty = torch.as_tensor(self._ty, device=x.device)
        clip = str(self._parms.get("out_of_bounds", "NA")).lower() == "clip"
        xc = x.clamp(float(tx[0]), float(tx[-1]))
        i = torch.searchsorted(tx, xc, right=True).clamp(1, max(1, tx.numel() - 1))
        x0, x1 = tx[i - 1], tx[i] if tx.numel() > 1 else tx[i - 1]
        y0, y1 = ty[i - 1], ty[i] if ty.numel() > 1 else ty[i - 1]
        t = torch.where(x1 > x0, (xc - x0) / (x1 - x0).clamp_min(1e-300), torch.zeros_like(xc))
        pred = y0 + t * (y1 - y0)
        pred = torch.where(xc == x1, y1, pred)
        if not clip:
            oob = (x < tx[0]) | (x > tx[-1])
            pred = torch.where(oob, torch.full_like(pred, float("nan")), pred)
        pred = torch.where(torch.isnan(x), torch.full_like(pred, float("nan")), pred)
        return pred.to(torch.float32).view(-1, 1)
