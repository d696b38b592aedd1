"""Infogram (admissible machine learning).

Reference: h2o-admissibleml (hex/Infogram/Infogram.java, InfogramModel.java,
InfogramUtils.java, EstimateCMI.java): core infogram -- total information
(relevance) = normalised variable importance of a model on all
predictors, net information = normalised conditional mutual information
I(y; x_j | x_-j) estimated from the log-likelihood gain of the model with
x_j over the model without it; fair infogram (protected_columns) --
relevance from the model on the unprotected predictors, safety index =
I(y; x_j | protected) from models on protected+x_j vs protected only.
Admissible when both indices exceed their thresholds (default 0.1);
admissible_index = distance from the origin / sqrt(2).  Output frame
columns: column, admissible, admissible_index, total_information /
relevance_index, net_information / safety_index, cmi_raw.

MI355X design: every sub-model is a device GBM (histogram kernels), and
the CMI estimate is a fused log-likelihood reduction over the device
predictions; no per-row host work.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from ..core.frame import H2OFrame
from ..parallel import collectives as coll
from .base import H2OEstimator

INFOGRAM_DEFAULTS = dict(algorithm="AUTO", algorithm_params=None, protected_columns=None, total_information_threshold=-1.0,
                         net_information_threshold=-1.0, relevance_index_threshold=-1.0, safety_index_threshold=-1.0,
                         data_fraction=1.0, top_n_features=50, seed=-1,
                         # forwarded to the infogram's models when the algorithm takes them
                         standardize=True, plug_values=None, max_iterations=0, balance_classes=False,
                         class_sampling_factors=None, max_after_balance_size=5.0)

_FORWARD = {"glm": ("standardize", "plug_values", "max_iterations", "balance_classes", "class_sampling_factors",
                    "max_after_balance_size"),
            "deeplearning": ("standardize", "balance_classes", "class_sampling_factors", "max_after_balance_size"),
            "gbm": ("balance_classes", "class_sampling_factors", "max_after_balance_size"),
            "drf": ("balance_classes", "class_sampling_factors", "max_after_balance_size")}


class H2OInfogram(H2OEstimator):
    algo = "infogram"
    _defaults = INFOGRAM_DEFAULTS

    def _model(self, spec, xs):
        from .tree.drf import H2ORandomForestEstimator
        from .tree.gbm import H2OGradientBoostingEstimator
        from .glm.glm import H2OGeneralizedLinearEstimator
        from .deeplearning import H2ODeepLearningEstimator
        p = self._parms
        algo = str(p.get("algorithm") or "AUTO").lower()
        kw = dict(p.get("algorithm_params") or {})
        if p.get("seed", -1) not in (-1, None):
            kw.setdefault("seed", p["seed"])
        for k in _FORWARD.get("gbm" if algo == "auto" else algo, ()):
            if k == "max_iterations" and not p.get(k):
                continue
            if p.get(k) is not None:
                kw.setdefault(k, p[k])
        if algo == "glm" and kw.get("plug_values") is not None:
            kw.setdefault("missing_values_handling", "PlugValues")    # plug values imply PlugValues imputation
        cls = {"auto": H2OGradientBoostingEstimator, "gbm": H2OGradientBoostingEstimator,
               "drf": H2ORandomForestEstimator, "glm": H2OGeneralizedLinearEstimator,
               "deeplearning": H2ODeepLearningEstimator}[algo]
        m = cls(**kw)
        if xs:
            m.train(x=list(xs), y=spec.y, training_frame=spec.frame, weights_column=spec.weights_column)
        return m

    def _loglik(self, spec, m, xs):
        """Mean per-row log-likelihood of the response under model m (no x -> prior)."""
        fr = spec.frame
        if spec.nclasses >= 2:
            y = spec.y_tensor().long()
            ok = y >= 0
            if not xs:
                cnt = torch.bincount(y[ok], minlength=spec.nclasses).to(torch.float64)
                coll.allreduce_(cnt)
                pr = (cnt / cnt.sum())[y.clamp(min=0)]
            else:
                raw = m._predict_raw(fr).to(torch.float64)
                pr = raw.gather(1, y.clamp(min=0).view(-1, 1)).view(-1)
            s = torch.stack([torch.log(pr.clamp_min(1e-12))[ok].sum(), ok.sum().to(torch.float64)])
            coll.allreduce_(s)
            return float(s[0] / s[1])
        y = spec.y_tensor(dtype=torch.float64)
        ok = ~torch.isnan(y)
        if not xs:
            mu = torch.full_like(y, float(y[ok].mean()))
        else:
            mu = m._predict_raw(fr)[:, 0].to(torch.float64)
        r = (y - mu)[ok]
        s = torch.stack([(r * r).sum(), ok.sum().to(torch.float64)])
        coll.allreduce_(s)
        return -0.5 * math.log(max(float(s[0] / s[1]), 1e-300))

    def _fit(self, spec):
        p = self._parms
        frac = float(p.get("data_fraction", 1.0))
        if not 0 < frac <= 1:
            raise ValueError("ERRR on field: data_fraction: must be in (0, 1].")
        if frac < 1:
            # data_fraction (Infogram.java): the infogram's models see a seeded
            # row sample of the training frame (each rank samples its shard)
            import copy
            from ..parallel import cloud
            seed = p.get("seed", -1)
            g = torch.Generator(device=cloud.device())
            g.manual_seed(((int(seed) if seed not in (None, -1) else 1234) * 1000003 + cloud.rank()) & 0x7FFFFFFF)
            keep = torch.rand(spec.frame.nlocal, generator=g, device=cloud.device()) < frac
            spec = copy.copy(spec)
            spec.frame = spec.frame[keep]
        prot = list(p.get("protected_columns") or [])
        xs = [c for c in spec.x if c not in prot]
        fair = bool(prot)
        base = self._model(spec, xs)
        vi = base.varimp(use_pandas=True)
        rel = dict(zip(vi["variable"], vi["scaled_importance"])) if vi is not None else {c: 0.0 for c in xs}
        rel = {c: float(rel.get(c, 0.0)) for c in xs}
        mx = max(rel.values()) if rel else 1.0
        rel = {c: v / mx if mx > 0 else 0.0 for c, v in rel.items()}
        top = sorted(xs, key=lambda c: -rel[c])[: int(p.get("top_n_features", 50))]
        cmi = {}
        if fair:
            ll_p = self._loglik(spec, self._model(spec, prot), prot)
            for c in top:
                ll = self._loglik(spec, self._model(spec, prot + [c]), prot + [c])
                cmi[c] = max(ll - ll_p, 0.0)
        else:
            ll_full = self._loglik(spec, base, xs)
            for c in top:
                rest = [z for z in xs if z != c]
                ll = self._loglik(spec, self._model(spec, rest), rest)
                cmi[c] = max(ll_full - ll, 0.0)
        cmax = max(cmi.values()) if cmi else 1.0
        ncmi = {c: (v / cmax if cmax > 0 else 0.0) for c, v in cmi.items()}
        t_rel = float(p.get("relevance_index_threshold" if fair else "total_information_threshold", -1))
        t_cmi = float(p.get("safety_index_threshold" if fair else "net_information_threshold", -1))
        t_rel = 0.1 if t_rel < 0 else t_rel
        t_cmi = 0.1 if t_cmi < 0 else t_cmi
        rows = []
        for c in top:
            r, s = rel[c], ncmi[c]
            rows.append((c, int(r >= t_rel and s >= t_cmi), math.sqrt(r * r + s * s) / math.sqrt(2), r, s, cmi[c]))
        cols = ["column", "admissible", "admissible_index", "relevance_index" if fair else "total_information",
                "safety_index" if fair else "net_information", "cmi_raw"]
        df = pd.DataFrame(rows, columns=cols).sort_values("admissible_index", ascending=False).reset_index(drop=True)
        self._table = df
        self._output["admissible_features"] = list(df.loc[df.admissible == 1, "column"])
        self._base = base

    def get_admissible_score_frame(self):
        return H2OFrame(self._table)

    def get_admissible_features(self):
        return self._output["admissible_features"]

    def get_admissible_relevance(self):
        return list(self._table.iloc[:, 3])

    def get_admissible_cmi(self):
        return list(self._table.iloc[:, 4])

    def get_admissible_cmi_raw(self):
        return list(self._table["cmi_raw"])

    def _predict_raw(self, frame):
        return self._base._predict_raw(frame)

    def _score_all(self, spec):
        self._training_metrics = self._base._training_metrics
