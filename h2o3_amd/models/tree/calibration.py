"""Probability calibration for binomial tree models.

Reference: hex/tree/CalibrationHelper.java (calibrate_model +
calibration_frame; calibration_method PlattScaling = binomial GLM of the
response on the model's p1, IsotonicRegression = isotonic fit of the
response on p1 (out_of_bounds clip); calibrated probabilities are added
to predict() as cal_p0 / cal_p1 columns).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ...parallel import collectives as coll


def fit_calibration(model, frame, method="auto"):
    spec = model._spec
    if spec.nclasses != 2:
        raise ValueError("calibration is only supported for binomial models")
    raw = model._predict_raw(frame)
    p1 = raw[:, 1].to(torch.float64)
    y = model._adapt_enum(frame.vec(spec.y), spec.response_domain).long()
    ok = (y >= 0) & ~torch.isnan(p1)
    x, t = p1[ok], (y[ok] == 1).to(torch.float64)
    m = str(method or "auto").lower()
    if m in ("auto", "plattscaling", "platt"):
        # 2-parameter logistic regression by Newton (GLM binomial on p1)
        a, b = 0.0, 0.0
        for _ in range(50):
            z = a * x + b
            mu = torch.sigmoid(z)
            wgt = (mu * (1 - mu)).clamp_min(1e-12)
            g = torch.stack([((t - mu) * x).sum(), (t - mu).sum()])
            H = torch.stack([torch.stack([(wgt * x * x).sum(), (wgt * x).sum()]),
                             torch.stack([(wgt * x).sum(), wgt.sum()])])
            st = torch.cat([g, H.reshape(-1)])
            coll.allreduce_(st)
            g, H = st[:2], st[2:].view(2, 2)
            d = torch.linalg.solve(H, g)
            a, b = a + float(d[0]), b + float(d[1])
            if float(d.abs().max()) < 1e-10:
                break
        model._calibrator = lambda q, a=a, b=b: torch.sigmoid(a * q.to(torch.float64) + b).to(q.dtype)
        model._output["calibration"] = {"method": "PlattScaling", "coef": a, "intercept": b}
    elif m in ("isotonicregression", "isotonic"):
        from ..isotonic import pava
        xs, ts = coll.all_gather_var(x), coll.all_gather_var(t)
        o = torch.argsort(xs)
        xs, ts = xs[o].cpu().numpy(), ts[o].cpu().numpy()
        ux, inv = np.unique(xs, return_inverse=True)
        sw = np.bincount(inv).astype(float)
        sy = np.bincount(inv, weights=ts)
        starts, by, _ = pava(sy / sw, sw)
        ends = np.concatenate([starts[1:], [len(ux)]]) - 1
        tx, ty = [], []
        for s_, e_, v in zip(starts, ends, by):
            tx.append(ux[s_]); ty.append(v)
            if e_ > s_:
                tx.append(ux[e_]); ty.append(v)
        tx_t, ty_t = torch.as_tensor(tx), torch.as_tensor(ty)

        def iso(q, tx_t=tx_t, ty_t=ty_t):
            dev = q.device
            xx, yy = tx_t.to(dev), ty_t.to(dev)
            qc = q.to(torch.float64).clamp(float(xx[0]), float(xx[-1]))
            i = torch.searchsorted(xx, qc, right=True).clamp(1, max(1, xx.numel() - 1))
            x0, x1 = xx[i - 1], xx[i] if xx.numel() > 1 else xx[i - 1]
            y0, y1 = yy[i - 1], yy[i] if yy.numel() > 1 else yy[i - 1]
            w = torch.where(x1 > x0, (qc - x0) / (x1 - x0).clamp_min(1e-300), torch.zeros_like(qc))
            return (y0 + w * (y1 - y0)).to(q.dtype)
        model._calibrator = iso
        model._output["calibration"] = {"method": "IsotonicRegression", "thresholds_x": tx, "thresholds_y": ty}
    else:
        raise ValueError(f"unknown calibration_method {method}")
