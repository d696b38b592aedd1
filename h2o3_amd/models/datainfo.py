"""DataInfo: design-matrix expansion for linear / neural / clustering models.

Reference: h2o-algos/src/main/java/hex/DataInfo.java (categorical one-hot
expansion with `useAllFactorLevels`, numeric standardization with
`_normMul/_normSub`, missing value handling MeanImputation / Skip /
PlugValues, interactions) — the reference expands rows lazily per chunk;
here the expanded dense design matrix is materialized ONCE in HBM as a
row-major f32 [N, P] tensor (P padded to a multiple of 32 for the MFMA
Gram kernel), because 288 GB of HBM fits it and every iteration then
streams it at full bandwidth.
"""
from __future__ import annotations

import numpy as np
import torch

from ..core.vec import T_ENUM
from ..parallel import cloud


class DataInfo:
    def __init__(self, frame, x, standardize=True, use_all_factor_levels=False, missing_values_handling="MeanImputation",
                 plug_values=None, pad_to=32, max_cat_levels=None, intercept=True, pad_extra=0, interactions=None):
        # interactions: list of (a, b) column pairs -> extra features (glm/interactions.py)
        self.ia_recipe = None
        if interactions:
            from .glm.interactions import apply_recipe, build_recipe
            self.ia_recipe = build_recipe(frame, interactions)
            frame, new_x = apply_recipe(frame, self.ia_recipe)
            x = list(x) + new_x
        self.x = list(x)
        self.standardize = standardize
        self.use_all = use_all_factor_levels
        self.mvh = (missing_values_handling or "MeanImputation").lower()
        self.cat_cols = [c for c in x if frame.vec(c).type == T_ENUM]
        self.num_cols = [c for c in x if frame.vec(c).type != T_ENUM and not frame.vec(c).on_host]
        self.domains = {c: list(frame.vec(c).domain) for c in self.cat_cols}
        self.cat_offsets = {}
        self.coef_names = []
        off = 0
        for c in self.cat_cols:
            dom = self.domains[c]
            lv = dom if self.use_all else dom[1:]
            self.cat_offsets[c] = off
            self.coef_names += [f"{c}.{d}" for d in lv]
            off += len(lv)
        self.n_cat_expanded = off
        self.means, self.sigmas = [], []
        plug = plug_values if plug_values is not None else {}
        if hasattr(plug, "as_data_frame"):
            # the reference takes plug values as a one-row frame (GLM.java:970)
            pdf = plug.as_data_frame()
            if len(pdf) != 1:
                raise ValueError("ERRR on field: _plug_values: Plug values frame needs to have exactly 1 row.")
            plug = {c: float(pdf[c].iloc[0]) for c in pdf.columns if pdf[c].dtype.kind in "fiub"}
        from ..ops import frame_ops
        frame_ops.rollups_many([frame.vec(c) for c in self.num_cols])
        for c in self.num_cols:
            v = frame.vec(c)
            r = v.rollups()
            mu = r["mean"] if r["mean"] == r["mean"] else 0.0
            sd = r["sigma"] if r["sigma"] and r["sigma"] == r["sigma"] and r["sigma"] > 0 else 1.0
            self.means.append(mu)
            self.sigmas.append(sd)
            self.coef_names.append(c)
        self.plug = [float(plug.get(c, m)) for c, m in zip(self.num_cols, self.means)]
        # mode for categorical imputation
        self.cat_modes = {}
        for c in self.cat_cols:
            d = frame.vec(c).data
            ok = d[d >= 0]
            if ok.numel():
                cnt = torch.bincount(ok.long(), minlength=len(self.domains[c]))
                from ..parallel import collectives as coll
                coll.allreduce_(cnt)
                self.cat_modes[c] = int(torch.argmax(cnt))
            else:
                self.cat_modes[c] = 0
        self.P = len(self.coef_names)
        self.Pp = ((self.P + pad_extra + pad_to - 1) // pad_to) * pad_to if pad_to else self.P

    def expand(self, frame, dtype=torch.float32, pad=True, width=None):
        """Returns (X [n, P or Pp, or `width` columns], row_ok mask) on device."""
        if self.ia_recipe:
            from .glm.interactions import apply_recipe
            frame = apply_recipe(frame, self.ia_recipe)[0]
        n = frame.nlocal
        dev = cloud.device()
        P = int(width) if width else (self.Pp if pad else self.P)
        X = torch.zeros((n, P), dtype=dtype, device=dev)
        ok = torch.ones(n, dtype=torch.bool, device=dev)
        for c in self.cat_cols:
            if c in frame.names:
                v = frame.vec(c)
                codes = _adapt(v, self.domains[c])
            else:
                codes = torch.full((n,), -1, dtype=torch.int32, device=dev)
            na = codes < 0
            if self.mvh == "skip":
                ok &= ~na
            codes = torch.where(na, torch.full_like(codes, self.cat_modes[c]), codes).long()
            if not self.use_all:
                codes = codes - 1
            m = codes >= 0
            rows = torch.nonzero(m).flatten()
            X[rows, self.cat_offsets[c] + codes[rows]] = 1.0
        base = self.n_cat_expanded
        fast = self._expand_numeric_fast(frame, X, base, n)
        for j, c in enumerate(self.num_cols):
            if fast and self.mvh != "skip":
                break
            if c in frame.names:
                x = frame.vec(c).as_float(torch.float64)
            else:
                x = torch.full((n,), float("nan"), dtype=torch.float64, device=dev)
            na = torch.isnan(x)
            if self.mvh == "skip":
                ok &= ~na
            if fast:
                continue             # the kernel filled the column; only the skip mask is needed
            x = torch.where(na, torch.full_like(x, self.plug[j]), x)
            if self.standardize:
                x = (x - self.means[j]) / self.sigmas[j]
            X[:, base + j] = x.to(dtype)
        return X, ok

    def _expand_numeric_fast(self, frame, X, base, n):
        """The numeric block by the tiled HIP kernel (ops/csrc/frame.hip):
        every numeric column present, float32 / float64 on the device."""
        if not self.num_cols or not X.is_cuda or any(c not in frame.names for c in self.num_cols):
            return False
        from ..ops import frame_ops
        vs = [frame.vec(c) for c in self.num_cols]
        if not all(frame_ops.batchable(v) and v.data.numel() == n for v in vs):
            return False
        k = len(vs)
        mean = self.means if self.standardize else [0.0] * k
        sd = self.sigmas if self.standardize else [1.0] * k
        return frame_ops.expand_numeric([v.data for v in vs], self.plug, mean, sd, X, base)

    def destandardize(self, beta_std, icpt_std):
        """Convert standardized-space coefficients to original scale."""
        beta = np.array(beta_std, dtype=np.float64).copy()
        icpt = float(icpt_std)
        if self.standardize:
            base = self.n_cat_expanded
            for j in range(len(self.num_cols)):
                b = beta[base + j] / self.sigmas[j]
                icpt -= b * self.means[j]
                beta[base + j] = b
        return beta, icpt


def _adapt(v, domain):
    if v.type == T_ENUM:
        if v.domain == domain:
            return v.data
        idx = {d: i for i, d in enumerate(domain)}
        remap = torch.tensor([idx.get(d, -1) for d in v.domain] or [-1], dtype=torch.int32, device=v.data.device)
        return torch.where(v.data < 0, v.data, remap[v.data.clamp(min=0).long()])
    x = v.as_float(torch.float64)
    idx = {}
    for i, d in enumerate(domain):
        try:
            idx[float(d)] = i
        except ValueError:
            pass
    out = torch.full(x.shape, -1, dtype=torch.int32, device=x.device)
    for k, i in idx.items():
        out[x == k] = i
    return out
