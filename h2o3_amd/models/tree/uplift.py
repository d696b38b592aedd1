"""Uplift Distributed Random Forest.

Reference: hex/tree/uplift/UpliftDRF.java, UpliftDRFModel.java,
hex/tree/uplift/Divergence.java (KL / Euclidean / ChiSquared divergence
between the treatment and control response distributions; split gain =
weighted child divergence - parent divergence), hex/AUUC.java and
hex/ModelMetricsBinomialUplift.java (uplift curves qini / lift / gain over
quantile thresholds of the prediction, AUUC = sum(uplift_j *
frequency_j) / (n+1), normalised AUUC, AECU = AUUC - random AUUC (= Qini
for qini), ATE / ATT / ATC).  Predictions: uplift_predict =
p(y=1 | treatment) - p(y=1 | control), plus both probabilities.

MI355X design: same tree engine as DRF/GBM -- the histogram kernel runs
twice per node batch (treatment-weighted and control-weighted (w, w*y)
channels) and the 4-channel histograms go through the divergence split
search; sibling subtraction and partitioning are unchanged.
"""
from __future__ import annotations

import copy
import math

import numpy as np
import torch

from ...core.frame import H2OFrame
from ...core.vec import T_ENUM, T_REAL, Vec
from ...parallel import cloud
from ...parallel import collectives as coll
from .. import metrics as mm
from .engine import GrowParams, TreeGrower
from .shared import Forest, SharedTreeEstimator
from ...core.groupsum import index_add as _ia

UPLIFT_DEFAULTS = dict(ntrees=50, max_depth=20, min_rows=1.0, nbins=20, nbins_top_level=1024, nbins_cats=1024,
                       seed=-1, mtries=-2, sample_rate=0.632, col_sample_rate_per_tree=1.0,
                       col_sample_rate_change_per_level=1.0, histogram_type="auto", categorical_encoding="auto",
                       distribution="bernoulli", treatment_column="treatment", uplift_metric="AUTO",
                       auuc_type="AUTO", auuc_nbins=-1, score_tree_interval=0, check_constant_response=True,
                       custom_metric_func=None, stopping_rounds=0, sample_rate_per_class=None)


def auuc_metrics(uplift: torch.Tensor, y: torch.Tensor, treat: torch.Tensor, nbins=1000, auuc_type="qini"):
    """AUUC.java on device tensors (global across ranks)."""
    u = coll.all_gather_var(uplift.to(torch.float64))
    yy = coll.all_gather_var(y.to(torch.float64))
    tt = coll.all_gather_var(treat.to(torch.float64))
    n = u.numel()
    probs = torch.tensor([(nbins - i - 1.0) / nbins for i in range(nbins)], dtype=torch.float64, device=u.device)
    ths = torch.unique(torch.quantile(u, probs.clamp(0, 1)) if n else probs)
    ths = torch.flip(torch.sort(ths).values, [0])       # descending
    nb = ths.numel()
    # bin = first (largest) threshold <= prediction
    idx = torch.searchsorted(-ths, -u, right=False).clamp(max=nb - 1)
    def cnt(v):
        return _ia(torch.zeros(nb, dtype=torch.float64, device=u.device), idx, v)
    T = torch.cumsum(cnt(tt), 0)
    C = torch.cumsum(cnt(1 - tt), 0)
    YT = torch.cumsum(cnt(tt * yy), 0)
    YC = torch.cumsum(cnt((1 - tt) * yy), 0)
    freq = cnt(torch.ones_like(u))
    fcs = torch.cumsum(freq, 0)
    curves = {"qini": YT - YC * T / C, "lift": YT / T - YC / C}
    curves["gain"] = curves["lift"] * (T + C)
    out = {}
    for k, c in curves.items():
        c = c.cpu().numpy()
        ok = np.isfinite(c)
        if not ok.all():
            xi = np.arange(len(c))
            c = np.interp(xi, xi[ok], c[ok]) if ok.any() else np.zeros_like(c)
        f = freq.cpu().numpy()
        rnd = c[-1] / fcs[-1].item() * fcs.cpu().numpy()
        norm = 1.0 if k == "lift" or c[-1] == 0 else abs(c[-1])
        a = float((c * f).sum() / (n + 1))
        ar = float((rnd * f).sum() / (n + 1))
        out[k] = {"auuc": a, "auuc_random": ar, "aecu": a - ar, "auuc_normalized": float((c / norm * f).sum() / (n + 1)),
                  "curve": c, "thresholds": ths.cpu().numpy()}
    return out


class ModelMetricsBinomialUplift(mm.ModelMetrics):
    kind = "binomial_uplift"

    def auuc(self, auuc_type=None):
        t = (auuc_type or self._m.get("auuc_type", "qini")).lower()
        t = "qini" if t == "auto" else t
        return self._m["auuc_table"][t]["auuc"]

    def auuc_normalized(self, auuc_type=None):
        t = (auuc_type or self._m.get("auuc_type", "qini")).lower()
        t = "qini" if t == "auto" else t
        return self._m["auuc_table"][t]["auuc_normalized"]

    def qini(self):
        return self._m["auuc_table"]["qini"]["aecu"]

    def aecu(self, auuc_type="qini"):
        return self._m["auuc_table"][auuc_type]["aecu"]

    def ate(self):
        return self._m["ate"]

    def att(self):
        return self._m["att"]

    def atc(self):
        return self._m["atc"]

    def uplift(self, metric="qini"):
        return list(self._m["auuc_table"][metric]["curve"])


class H2OUpliftRandomForestEstimator(SharedTreeEstimator):
    algo = "upliftdrf"
    _defaults = UPLIFT_DEFAULTS

    def _wants_categorical_response(self):
        return True

    def _resolve_columns(self, x, y, training_frame):
        tc = self._parms.get("treatment_column")
        x, y = super()._resolve_columns(x, y, training_frame)
        return [c for c in x if c != tc], y

    def _n_tree_classes(self):
        return 2

    def _treat(self, frame):
        v = frame.vec(self._parms["treatment_column"])
        if v.type == T_ENUM:
            dom = self._treat_dom if hasattr(self, "_treat_dom") else list(v.domain)
            codes = self._adapt_enum(v, dom) if hasattr(self, "_treat_dom") else v.data
            return (codes.long() == 1).to(torch.float32)
        return (v.as_float(torch.float32) > 0).to(torch.float32)

    def _fit(self, spec):
        dist = str(self._parms.get("distribution") or "bernoulli").lower()
        if dist not in ("auto", "bernoulli"):
            raise ValueError(f"ERRR on field: _distribution: Distribution {dist} is not supported for Uplift DRF; "
                             "only bernoulli (binomial response) is.")
        p = self._parms
        if spec.nclasses != 2:
            raise ValueError("UpliftDRF supports binomial responses only")
        tv = spec.frame.vec(p["treatment_column"])
        if tv.type == T_ENUM:
            self._treat_dom = list(tv.domain)
        bd = self._bin(spec)
        dev = cloud.device()
        N, F = bd.nrows_local, bd.F
        mtries = int(p.get("mtries", -2))
        if mtries == -2:
            mtries = F
        elif mtries == -1:
            mtries = max(1, int(math.sqrt(F)))
        metric = str(p.get("uplift_metric") or "AUTO").lower()
        crit = {"auto": "uplift_kl", "kl": "uplift_kl", "euclidean": "uplift_euclidean",
                "chisquared": "uplift_chisquared"}[metric]
        gp = GrowParams(criterion=crit, max_depth=int(p["max_depth"]) if p["max_depth"] > 0 else 64,
                        min_rows=float(p["min_rows"]), min_split_improvement=0.0,
                        mtries=mtries if mtries < F else -1, seed=self._seed())
        grower = TreeGrower(bd, gp)
        y = (spec.y_tensor().long() == 1).to(torch.float32)
        valid = spec.y_tensor().long() >= 0
        w = spec.w_tensor()
        base_w = torch.ones(N, dtype=torch.float32, device=dev) if w is None else w.to(torch.float32)
        base_w = torch.where(valid, base_w, torch.zeros_like(base_w))
        T = self._treat(spec.frame)
        gen = torch.Generator(device=dev)
        gen.manual_seed(self._seed() + cloud.rank())
        forest = Forest()
        sr = float(p["sample_rate"])
        srpc = p.get("sample_rate_per_class")
        if srpc is not None:
            # per-class row sampling rates (SharedTree sample_rate_per_class)
            ycls = y.clamp(min=0).long()
            sr_row = torch.tensor([float(r) for r in srpc], dtype=torch.float32, device=dev)[ycls]
        for t in range(int(p["ntrees"])):
            u = torch.rand(N, generator=gen, device=dev)
            inbag = u < (sr_row if srpc is not None else sr)
            wt = (base_w * inbag * T).contiguous()
            wc = (base_w * inbag * (1 - T)).contiguous()
            tree, nid, leaves, tot = grower.grow(y.contiguous(), (wt, wc), 3)
            tot = tot.numpy() if isinstance(tot, torch.Tensor) else np.asarray(tot)
            pt = np.where(tot[:, 0] > 0, tot[:, 1] / np.maximum(tot[:, 0], 1e-300), 0.0)
            pc = np.where(tot[:, 2] > 0, tot[:, 3] / np.maximum(tot[:, 2], 1e-300), 0.0)
            tc = copy.deepcopy(tree)
            for li, node in enumerate(leaves):
                tree.value[node] = float(pt[li])
                tc.value[node] = float(pc[li])
            forest.add(tree, 0)
            forest.add(tc, 1)
        self._forest = forest
        self._output["variable_importances"] = self._varimp_from_forest(_only_class(forest, 0), spec.x)
        self._output["model_summary"] = {"number_of_trees": len(forest) // 2}

    def _seed(self):
        s = self._parms.get("seed", -1)
        return 4321 if s is None or s == -1 else int(s) & 0x7FFFFFFF

    def _predict_raw(self, frame):
        X = self._score_matrix(frame)
        s = self._forest.predict(X, 2) / max(1, len(self._forest) // 2)
        return torch.stack([s[:, 0] - s[:, 1], s[:, 0], s[:, 1]], 1)

    def predict(self, test_data, **kw):
        r = self._predict_raw(test_data)
        return H2OFrame.from_vecs([Vec(r[:, i].contiguous(), T_REAL) for i in range(3)],
                                  ["uplift_predict", "p_y1_with_treatment", "p_y1_without_treatment"])

    def _uplift_metrics(self, frame, raw):
        spec = self._spec
        y = self._adapt_enum(frame.vec(spec.y), spec.response_domain).long()
        ok = y >= 0
        T = self._treat(frame)
        u = raw[:, 0]
        nb = int(self._parms.get("auuc_nbins", -1))
        tab = auuc_metrics(u[ok], (y[ok] == 1), T[ok], nbins=1000 if nb <= 0 else nb)
        def gmean(v):
            s = torch.stack([v.sum().double(), torch.tensor(float(v.numel()), dtype=torch.float64, device=v.device)])
            coll.allreduce_(s)
            return float(s[0] / s[1]) if float(s[1]) > 0 else float("nan")
        return ModelMetricsBinomialUplift(auuc_table=tab, auuc_type=str(self._parms.get("auuc_type") or "AUTO"),
                                          ate=gmean(u[ok]), att=gmean(u[ok & (T > 0)]), atc=gmean(u[ok & (T == 0)]),
                                          nobs=int(ok.sum()))

    def _score_all(self, spec):
        self._training_metrics = self._uplift_metrics(spec.frame, self._predict_raw(spec.frame))
        if spec.valid is not None:
            self._validation_metrics = self._uplift_metrics(spec.valid, self._predict_raw(spec.valid))

    def model_performance(self, test_data=None, train=False, valid=False, **kw):
        if test_data is None:
            return self._validation_metrics if valid else self._training_metrics
        return self._uplift_metrics(test_data, self._predict_raw(test_data))

    def auuc(self, train=False, valid=False):
        m = self._validation_metrics if valid else self._training_metrics
        return m.auuc()

    def qini(self, train=False, valid=False):
        m = self._validation_metrics if valid else self._training_metrics
        return m.qini()


def _only_class(forest, k):
    f = Forest()
    for t, c in zip(forest.trees, forest.tclass):
        if c == k:
            f.add(t, 0)
    return f
