"""Target encoding.

Reference: h2o-extensions/target-encoder (ai/h2o/targetencoding/
TargetEncoder.java, TargetEncoderModel.java, TargetEncoderHelper.java):
per-level response statistics (numerator / denominator) computed with
group-by; data_leakage_handling None | KFold (out-of-fold statistics) |
LeaveOneOut (subtract the row's own contribution); blending
lambda = 1 / (1 + exp((k - n) / f)) with inflection_point k and smoothing
f; uniform noise in [-noise, noise] on training transforms; multinomial
responses produce one encoded column per non-first class
(`<col>_<class>_te`), others `<col>_te`; NA is its own level.

MI355X design: the per-level sums are a device bincount over the level
codes (all-reduced across ranks); per-fold tables are a 2-D bincount
(fold x level); encoding is a gather.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_ENUM, T_REAL, Vec
from ..parallel import cloud
from ..parallel import collectives as coll
from .base import H2OEstimator
from ..core.groupsum import index_add as _ia

TE_DEFAULTS = dict(columns_to_encode=None, keep_original_categorical_columns=True, blending=False,
                   inflection_point=10.0, smoothing=20.0, data_leakage_handling="None", noise=0.01, seed=-1,
                   fold_column=None)


def _sanitize(name):
    """StringUtils.sanitizeIdentifier: non-identifier chars after the first -> '_'."""
    s = str(name)
    return s[:1] + "".join(ch if (ch.isalnum() or ch in "_$") else "_" for ch in s[1:])


def _dlh(v):
    return str(v or "None").lower().replace("_", "").replace("-", "")


class H2OTargetEncoderEstimator(H2OEstimator):
    algo = "targetencoder"
    _defaults = TE_DEFAULTS

    def _wants_categorical_response(self):
        return False

    def train(self, x=None, y=None, training_frame=None, fold_column=None, **kw):
        if fold_column is not None:
            self._parms["fold_column"] = fold_column
        return super().train(x=x, y=y, training_frame=training_frame, **kw)

    def _targets(self, spec):
        """Returns (list of per-row target channels [n], channel suffixes)."""
        if spec.nclasses > 2:
            y = spec.y_tensor().long()
            return [(y == k).to(torch.float64) for k in range(1, spec.nclasses)], \
                [f"_{_sanitize(spec.response_domain[k])}" for k in range(1, spec.nclasses)], y >= 0
        if spec.nclasses == 2:
            y = spec.y_tensor().long()
            return [(y == 1).to(torch.float64)], [""], y >= 0
        yv = spec.y_tensor(dtype=torch.float64)
        return [yv], [""], ~torch.isnan(yv)

    def _fit(self, spec):
        p = self._parms
        cols = p.get("columns_to_encode") or [c for c in spec.x if spec.frame.vec(c).type == T_ENUM]
        cols = [c if isinstance(c, str) else c[0] for c in cols]
        self._cols = cols
        chans, suf, ok = self._targets(spec)
        self._suffix = suf
        fc = p.get("fold_column")
        folds = spec.frame.vec(fc).data.long() if fc else None
        nf = int(coll.allreduce_scalar(float(folds.max()) + 1, "max")) if folds is not None else 0
        self._tables = {}
        self._fold_tables = {}
        self._prior = []
        for t in chans:
            tt = torch.where(ok, t, torch.zeros_like(t))
            s = torch.stack([tt.sum(), ok.to(torch.float64).sum()])
            coll.allreduce_(s)
            self._prior.append(float(s[0] / s[1]))
        for c in cols:
            v = spec.frame.vec(c)
            L = len(v.domain) + 1  # last slot = NA level
            codes = torch.where(v.data >= 0, v.data.long(), torch.full_like(v.data.long(), L - 1))
            per = []
            for t in chans:
                num = _ia(torch.zeros(L, dtype=torch.float64, device=t.device), codes[ok], t[ok])
                den = _ia(torch.zeros(L, dtype=torch.float64, device=t.device),
                          codes[ok], torch.ones_like(t[ok]))
                st = torch.stack([num, den])
                coll.allreduce_(st)
                per.append(st)
            self._tables[c] = (list(v.domain), per)
            if folds is not None:
                fper = []
                for t in chans:
                    key = folds[ok] * L + codes[ok]
                    num = _ia(torch.zeros(nf * L, dtype=torch.float64, device=t.device), key, t[ok])
                    den = _ia(torch.zeros(nf * L, dtype=torch.float64, device=t.device),
                              key, torch.ones_like(t[ok]))
                    st = torch.stack([num.view(nf, L), den.view(nf, L)])
                    coll.allreduce_(st)
                    fper.append(st)
                self._fold_tables[c] = fper
        self._output["encoded_columns"] = [f"{c}{s}_te" for c in cols for s in suf]
        self._train_names = list(spec.frame.names)
        self._output["priors"] = self._prior

    def _blend(self, num, den, prior):
        p = self._parms
        mean = torch.where(den > 0, num / den.clamp_min(1e-300), torch.full_like(num, prior))
        if not p.get("blending"):
            return mean
        k, f = float(p.get("inflection_point", 10.0)), float(p.get("smoothing", 20.0))
        lam = 1.0 / (1.0 + torch.exp((k - den) / max(f, 1e-12)))
        return lam * mean + (1 - lam) * prior

    def transform(self, frame: H2OFrame, as_training=False, blending=None, inflection_point=None, smoothing=None,
                  noise=None):
        p = dict(self._parms)
        for k, v in (("blending", blending), ("inflection_point", inflection_point), ("smoothing", smoothing)):
            if v is not None:
                self._parms[k] = v
        try:
            return self._transform(frame, as_training, noise)
        finally:
            self._parms.update({k: p[k] for k in ("blending", "inflection_point", "smoothing")})

    def _transform(self, frame, as_training, noise):
        p = self._parms
        dlh = _dlh(p.get("data_leakage_handling"))
        if noise is None:
            noise = float(p.get("noise", 0.01)) if as_training else 0.0
        seed = p.get("seed", -1)
        gen = torch.Generator(device="cpu").manual_seed(int(seed) if seed not in (-1, None) else 1234 + cloud.rank())
        out_vecs = [frame.vec(n) for n in frame.names]
        out_names = list(frame.names)
        spec = self._spec
        if as_training and dlh == "leaveoneout":
            ysp = spec.__class__(frame, spec.x, spec.y)
            chans, _, ok = self._targets(ysp)
        for c in self._cols:
            if c not in frame.names:
                continue
            dom, per = self._tables[c]
            L = len(dom) + 1
            codes = self._adapt_enum(frame.vec(c), dom).long()
            codes = torch.where(codes >= 0, codes, torch.full_like(codes, L - 1))
            for ci, (st, suf) in enumerate(zip(per, self._suffix)):
                num, den = st[0][codes], st[1][codes]
                if as_training and dlh == "kfold":
                    fc = p.get("fold_column")
                    fo = frame.vec(fc).data.long()
                    fst = self._fold_tables[c][ci]
                    num = num - fst[0][fo, codes]
                    den = den - fst[1][fo, codes]
                elif as_training and dlh == "leaveoneout":
                    t = chans[ci]
                    num = num - torch.where(ok, t, torch.zeros_like(t))
                    den = den - ok.to(torch.float64)
                enc = self._blend(num, den, self._prior[ci])
                if noise and noise > 0:
                    r = (torch.rand(enc.shape[0], generator=gen, dtype=torch.float64) * 2 - 1) * noise
                    enc = enc + r.to(enc.device)
                out_vecs.append(Vec(enc.to(torch.float64).contiguous(), T_REAL))  # doubles, as the reference
                out_names.append(f"{c}{suf}_te")
            if not p.get("keep_original_categorical_columns", True):
                i = out_names.index(c)
                out_vecs.pop(i)
                out_names.pop(i)
        return self._reorder(H2OFrame.from_vecs(out_vecs, out_names))

    def _reorder(self, fr):
        """TargetEncoderModel.reorderColumns: non-categorical training
        columns, TE columns, remaining categoricals, columns not seen in
        training, then non-predictors (weights, offset, fold, response)."""
        spec = self._spec
        tail = [c for c in (spec.weights_column, spec.offset_column, self._parms.get("fold_column"), spec.y) if c]
        train_cols = list(self._train_names)
        enc = [n for n in self._output["encoded_columns"] if n in fr.names]
        first, later = [], []
        for c in train_cols:
            if c in fr.names and c not in tail:
                (later if fr.vec(c).type == T_ENUM else first).append(c)
        seen = set(train_cols) | set(enc)
        later += [c for c in fr.names if c not in seen]
        later += [c for c in tail if c in fr.names]
        order = first + enc + later
        return fr[order] if order != list(fr.names) else fr

    def _cross_validate(self, spec):
        pass  # the fold column drives out-of-fold encoding, not model CV

    def _predict_raw(self, frame):
        raise NotImplementedError("use transform()")

    def predict(self, test_data, **kw):
        return self.transform(test_data)

    def _score_all(self, spec):
        pass
