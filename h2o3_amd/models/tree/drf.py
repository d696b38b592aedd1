"""Distributed Random Forest (and Extremely Randomized Trees).

Reference: hex/tree/drf/DRF.java — per tree: row sample without
replacement at `sample_rate` (0.632), `mtries` random columns per split
(sqrt(p) classification / p/3 regression), squared-error splits on the class
indicator (one tree per class, or one for binomial unless
`binomial_double_trees`), leaf = mean response; predictions average the
trees; training metrics are out-of-bag (DRF.java: "OOB" scoring).
histogram_type="Random" gives XRT (random split points).

MI355X design: identical engine to GBM (TreeGrower); the OOB bookkeeping is
a per-row running sum + count on the device, updated from the per-row leaf
ids the grower already produces.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ...parallel import cloud
from ...parallel import collectives as coll
from .. import metrics as mm
from ..base import ScoreKeeper, ScoreSchedule, _LESS_IS_BETTER
from .engine import GrowParams, TreeGrower
from .shared import Forest, SharedTreeEstimator

DRF_DEFAULTS = dict(ntrees=50, max_depth=20, min_rows=1.0, nbins=20, nbins_top_level=1024, nbins_cats=1024,
                    r2_stopping=1.79e308, seed=-1, build_tree_one_node=False, mtries=-1, sample_rate=0.632,
                    sample_rate_per_class=None, binomial_double_trees=False, checkpoint=None,
                    col_sample_rate_change_per_level=1.0, col_sample_rate_per_tree=1.0, min_split_improvement=1e-5,
                    histogram_type="auto", categorical_encoding="auto", calibrate_model=False,
                    calibration_frame=None, calibration_method="auto", distribution="auto",
                    check_constant_response=True, score_tree_interval=0, balance_classes=False,
                    class_sampling_factors=None, max_after_balance_size=5.0, max_confusion_matrix_size=20,
                    custom_metric_func=None, stopping_rounds=0, stopping_metric="auto", stopping_tolerance=0.001)


class H2ORandomForestEstimator(SharedTreeEstimator):
    algo = "drf"
    _defaults = DRF_DEFAULTS

    def _n_tree_classes(self):
        return self._K

    def _fit(self, spec):
        p = self._parms
        drv = DRFDriver(self, spec)
        ntrees = int(p["ntrees"])
        start = 0
        if p.get("checkpoint") is not None:
            start = self._resume_from(drv, p["checkpoint"])
        t0 = time.time()
        max_rt = float(p.get("max_runtime_secs") or 0)
        self._scoring_history = []
        stop_rounds = int(p.get("stopping_rounds") or 0)
        metric_name = self._stopping_metric(spec)
        history = []
        sched = ScoreSchedule(p)
        for t in range(start, ntrees):
            drv.step()
            # a max_runtime_secs stop scores the last tree into the history too
            score, timed_out = self._tick(t + 1, ntrees, sched, t + 1 == ntrees, t0, max_rt)
            if score:
                entry = {"number_of_trees": t + 1}
                sched.started()
                self._forest = drv.forest
                self._score_entry(entry, spec, drv.oob_sum, drv.oob_cnt)
                sched.ended()
                self._scoring_history.append(entry)
                if stop_rounds:
                    key = ("validation_" if spec.valid is not None else "training_") + \
                        ("custom" if metric_name.startswith("custom") else metric_name)
                    history.append(entry.get(key))
                    if ScoreKeeper.stop_early(history, stop_rounds, float(p.get("stopping_tolerance", 0.001)),
                                              metric_name in _LESS_IS_BETTER, metric=metric_name):
                        break
            if timed_out:
                break
        forest, K = drv.forest, drv.K
        self._forest = forest
        self._output["variable_importances"] = self._varimp_from_forest(forest, spec.x)
        self._output["model_summary"] = {"number_of_trees": len(forest) // K,
                                         "number_of_internal_trees": len(forest),
                                         "max_depth": max((tt.max_depth() for tt in forest.trees), default=0),
                                         "mean_leaves": float(np.mean([len(tt.leaves()) for tt in forest.trees]))}
        # out-of-bag predictions -> training metrics (reference reports OOB)
        self._oob_state = (drv.oob_sum, drv.oob_cnt)     # kept for checkpoint continuation
        cnt = drv.oob_cnt.clamp_min(1).view(-1, 1)
        oobp = drv.oob_sum / cnt
        self._oob_raw = self._normalize(oobp)
        self._oob_mask = drv.oob_cnt > 0
        if p.get("calibrate_model") and p.get("calibration_frame") is not None:
            from .calibration import fit_calibration
            fit_calibration(self, p["calibration_frame"], p.get("calibration_method", "auto"))

    def _stopping_metric(self, spec):
        m = (self._parms.get("stopping_metric") or "auto").lower()
        if m == "auto":
            return "logloss" if spec.is_classification else "deviance"
        return m

    def _resume_from(self, drv, ck):
        """Continue a forest (SharedTree.java:144): the checkpoint's trees are
        kept, the OOB state is the checkpoint's when it was trained on these
        rows (else rebuilt from its trees' in-bag draws is impossible: start
        from its predictions as OOB estimates), and the iteration counter
        resumes so the per-tree randomness continues the same stream."""
        from .shared import checkpoint_model
        prev, done = checkpoint_model(ck, "drf", self)
        if prev._K != drv.K:
            raise ValueError("checkpoint: the checkpoint model has a different number of classes / tree classes")
        for t, k in zip(prev._forest.trees, prev._forest.tclass):
            drv.forest.add(t, k)
        st = getattr(prev, "_oob_state", None)
        if st is not None and st[0].shape == drv.oob_sum.shape:
            drv.oob_sum.copy_(st[0])
            drv.oob_cnt.copy_(st[1])
        drv.iter = done
        return done

    def _score_entry(self, entry, spec, oob_sum, oob_cnt):
        """Scoring-history row: OOB training metrics (DRF.java scores OOB) plus
        validation metrics of the forest so far."""
        from .gbm import H2OGradientBoostingEstimator as _G
        has = oob_cnt > 0
        # branch on the GLOBAL state: a rank-local any()/all() would split the
        # SPMD sequence (metrics collectives, frame keys) when one rank's shard
        # happens to be fully covered
        n_has = coll.allreduce_scalar(float(has.sum()))
        if n_has > 0:
            oobp = self._normalize(oob_sum / oob_cnt.clamp_min(1).view(-1, 1))
            sub = spec.frame[has] if n_has < spec.frame.nrows else spec.frame
            m = self._metrics_from_raw(spec, sub, oobp[has])
            _G._add_metrics(entry, "training", m)
        if spec.valid is not None:
            _G._add_metrics(entry, "validation", self._metrics_from_raw(spec, spec.valid,
                                                                        self._predict_raw(spec.valid)))

    def _seed(self):
        s = self._parms.get("seed", -1)
        return 4321 if s is None or s == -1 else int(s) & 0x7FFFFFFF

    def _normalize(self, sums):
        spec = self._spec
        if spec.nclasses == 2 and self._binomial_single:
            p1 = sums[:, 0].clamp(0, 1)
            return torch.stack([1 - p1, p1], 1)
        if spec.nclasses > 1:
            s = sums.clamp_min(0)
            tot = s.sum(1, keepdim=True)
            return torch.where(tot > 0, s / tot.clamp_min(1e-30), torch.full_like(s, 1.0 / s.shape[1]))
        return sums[:, :1]

    def _predict_raw(self, frame):
        X = self._score_matrix(frame)
        K = self._K
        sums = self._forest.predict(X, K)
        ntrees = max(1, len(self._forest) // K)
        return self._normalize(sums / ntrees)

    def predict_contributions(self, test_data, output_format="Original", top_n=None, bottom_n=None,
                              compare_abs=False, background_frame=None):
        from .shap import tree_contributions
        return tree_contributions(self, test_data, top_n=top_n, bottom_n=bottom_n, compare_abs=compare_abs)

    def _score_all(self, spec):
        raw = self._predict_raw(spec.frame)
        if getattr(self, "_oob_raw", None) is not None and not getattr(self, "_in_cv", False):
            oob = torch.where(self._oob_mask.view(-1, 1), self._oob_raw.to(raw.dtype), raw)
            self._training_metrics = self._metrics_from_raw(spec, spec.frame, oob)
        else:
            self._training_metrics = self._metrics_from_raw(spec, spec.frame, raw)
        if spec.valid is not None:
            self._validation_metrics = self._metrics_from_raw(spec, spec.valid, self._predict_raw(spec.valid))


class DRFDriver:
    """Random-forest state; `step()` grows one forest iteration (K class trees)
    on a fresh row sample and folds its out-of-bag predictions in."""

    def __init__(self, est, spec):
        p = est._parms
        self.est, self.spec = est, spec
        # AUTO -> 254 global quantile bins: the reference re-bins every node
        # adaptively (nbins_top_level -> nbins), a global 20-bin grid would be
        # far coarser than that at depth (measured: 79% vs 99% train accuracy)
        bd = est._bin(spec)
        self.bd = bd
        dev = cloud.device()
        self.dev = dev
        N = bd.nrows_local
        F = bd.F
        ncls = spec.nclasses
        double = bool(p.get("binomial_double_trees"))
        K = ncls if (ncls > 2 or (ncls == 2 and double)) else 1
        self.K = est._K = K
        est._binomial_single = ncls == 2 and K == 1
        mtries = int(p.get("mtries", -1))
        if mtries == -1:
            mtries = max(1, int(math.floor(math.sqrt(F)))) if ncls > 1 else max(1, F // 3)
        elif mtries == -2:
            mtries = F
        self.gp = GrowParams(criterion="se", max_depth=int(p["max_depth"]) if p["max_depth"] > 0 else 64,
                             min_rows=float(p["min_rows"]), min_split_improvement=float(p["min_split_improvement"]),
                             mtries=mtries if mtries < F else -1,
                             col_sample_rate_change_per_level=float(p["col_sample_rate_change_per_level"]),
                             seed=est._seed())
        self.grower = TreeGrower(bd, self.gp)
        y = spec.y_tensor()
        w = spec.w_tensor()
        base_w = torch.ones(N, dtype=torch.float32, device=dev) if w is None else w.to(torch.float32)
        if spec.is_classification:
            self.ycode = y.to(torch.int64)
            valid = self.ycode >= 0
            self.targets = [((self.ycode == (1 if est._binomial_single else k)).to(torch.float32))
                            for k in range(K)]
        else:
            yf = y.to(torch.float32)
            valid = ~torch.isnan(yf)
            self.targets = [torch.nan_to_num(yf)]
        self.base_w = torch.where(valid, base_w, torch.zeros_like(base_w))
        # caller-known histogram bounds (grow() would otherwise run two
        # full-column reductions + device syncs per tree): the in-bag weights
        # are base_w * {0, 1}, so the base weights' bounds hold for every tree
        self._unit_w = bool(((self.base_w == 0) | (self.base_w == 1)).all())
        self._vmax = [max(float(self.base_w.abs().max()) if N else 1.0, 1e-30),
                      max([float((self.base_w * t.abs()).max()) if N else 0.0 for t in self.targets] + [1e-30])]
        self.forest = Forest()
        self.oob_sum = torch.zeros((N, K), dtype=torch.float32, device=dev)
        self.oob_cnt = torch.zeros(N, dtype=torch.float32, device=dev)
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(est._seed() + cloud.rank())
        self.rng = np.random.RandomState(est._seed())
        self.iter = 0

    def step(self):
        p, spec, dev = self.est._parms, self.spec, self.dev
        N, F = self.bd.nrows_local, self.bd.F
        from .shared import reseed_iteration
        reseed_iteration(self, self.est._seed(), self.iter)
        srpc = p.get("sample_rate_per_class")
        if srpc is not None and spec.is_classification:
            rates = torch.tensor(srpc, dtype=torch.float32, device=dev)[self.ycode.clamp(min=0)]
            inbag = torch.rand(N, generator=self.gen, device=dev) < rates
        else:
            inbag = torch.rand(N, generator=self.gen, device=dev) < float(p["sample_rate"])
        wt = (self.base_w * inbag).contiguous()
        r = float(p.get("col_sample_rate_per_tree", 1.0))
        if r < 1.0:
            kk = max(1, int(math.floor(r * F + 0.5)))
            m = np.zeros(F, dtype=bool)
            m[self.rng.choice(F, size=kk, replace=False)] = True
            self.gp.tree_col_mask = m
        oob = ~inbag
        for k in range(self.K):
            tree, nid, leaves, tot = self.grower.grow(self.targets[k].contiguous(), wt, 0, vmax=self._vmax,
                                                      unit_w=self._unit_w)
            tot = tot.numpy() if isinstance(tot, torch.Tensor) else np.asarray(tot)
            vals = np.where(tot[:, 0] > 0, tot[:, 1] / np.where(tot[:, 0] > 0, tot[:, 0], 1), 0.0)
            if isinstance(tree.value, np.ndarray):
                tree.value[np.asarray(leaves, dtype=np.int64)] = vals[:len(leaves)]
            else:
                for li, node in enumerate(leaves):
                    tree.value[node] = float(vals[li])
            vt = torch.tensor(vals, dtype=torch.float32, device=dev)
            self.oob_sum[:, k] += torch.where(oob, vt[nid.long()], torch.zeros(N, device=dev))
            self.forest.add(tree, k)
        self.oob_cnt += oob.to(torch.float32)
        self.iter += 1


class H2OExtremelyRandomizedTreesEstimator(H2ORandomForestEstimator):
    """XRT = DRF with histogram_type="Random" (reference: DRF docs)."""

    def __init__(self, **kw):
        kw.setdefault("histogram_type", "Random")
        super().__init__(**kw)
