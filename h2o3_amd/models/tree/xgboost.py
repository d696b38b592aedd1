"""XGBoost-style second-order gradient boosting.

Reference: h2o-extensions/xgboost (hex/tree/xgboost/XGBoost.java,
BoosterParms.java) which wraps native XGBoost (tree_method hist/approx,
grow_policy depthwise/lossguide, booster gbtree/dart/gblinear).  Here the
booster is native to this framework: the same GPU tree engine with
(g, h) histogram channels, gain = 1/2 [G_L^2/(H_L+l) + G_R^2/(H_R+l) -
G^2/(H+l)] - gamma (with L1 soft-thresholding by alpha), leaf weight
-G/(H+lambda) * eta, max_delta_step clipping, row/column subsampling and
DART dropout.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ...parallel import cloud
from ...parallel import collectives as coll
from ...ops import tree_ops
from ..distributions import get_distribution
from .engine import GrowParams, TreeGrower
from ..base import ScoreKeeper, ScoreSchedule, _LESS_IS_BETTER
from .shared import Forest, SharedTreeEstimator

XGB_DEFAULTS = dict(ntrees=50, max_depth=6, min_rows=1.0, min_child_weight=1.0, learn_rate=0.3, eta=0.3,
                    sample_rate=1.0, subsample=1.0, col_sample_rate=1.0, colsample_bylevel=1.0,
                    col_sample_rate_per_tree=1.0, colsample_bytree=1.0, colsample_bynode=1.0,
                    max_abs_leafnode_pred=0.0, max_delta_step=0.0, monotone_constraints=None,
                    interaction_constraints=None, score_tree_interval=0, min_split_improvement=0.0, gamma=0.0,
                    nthread=-1, save_matrix_directory=None, build_tree_one_node=False, calibrate_model=False,
                    calibration_frame=None, calibration_method="auto", max_bins=256, max_leaves=0,
                    tree_method="auto", grow_policy="depthwise", booster="gbtree", reg_lambda=1.0, reg_alpha=0.0,
                    dmatrix_type="auto", backend="auto", gpu_id=None, gainslift_bins=-1, sample_type="uniform",
                    normalize_type="tree", rate_drop=0.0, one_drop=False, skip_drop=0.0, scale_pos_weight=1.0,
                    distribution="auto", tweedie_power=1.5, categorical_encoding="auto", quiet_mode=True,
                    checkpoint=None, stopping_rounds=0, stopping_metric="auto", stopping_tolerance=0.001,
                    seed=-1, eval_metric=None, score_eval_metric_only=False)


class H2OXGBoostEstimator(SharedTreeEstimator):
    algo = "xgboost"
    _defaults = XGB_DEFAULTS

    def __init__(self, **kw):
        # XGBoost-native aliases (reference BoosterParms maps both spellings)
        alias = {"eta": "learn_rate", "subsample": "sample_rate", "colsample_bylevel": "col_sample_rate",
                 "colsample_bytree": "col_sample_rate_per_tree", "min_child_weight": "min_rows",
                 "gamma": "min_split_improvement", "max_bin": "max_bins"}
        for a, b in alias.items():
            if a in kw and b not in kw:
                kw[b] = kw[a]
        super().__init__(**kw)

    @staticmethod
    def available():
        return True

    def _n_tree_classes(self):
        return self._K

    def _fit(self, spec):
        p = self._parms
        dev = cloud.device()
        bd = self._bin(spec, hist_type="QuantilesGlobal", nbins=max(2, int(p.get("max_bins", 256)) - 1))
        N = bd.nrows_local
        nc = spec.nclasses
        dist_name = (p.get("distribution") or "auto").lower()
        if dist_name == "auto":
            dist_name = "bernoulli" if nc == 2 else ("multinomial" if nc > 2 else "gaussian")
        self._dist = get_distribution(dist_name, nc, tweedie_power=p.get("tweedie_power", 1.5))
        K = nc if nc > 2 else 1
        self._K = K
        y = spec.y_tensor()
        w = spec.w_tensor()
        base_w = torch.ones(N, dtype=torch.float32, device=dev) if w is None else w.to(torch.float32)
        if spec.is_classification:
            yc = y.to(torch.int64)
            valid = yc >= 0
            yv = (yc == 1).to(torch.float32) if K == 1 else None
            Y = torch.nn.functional.one_hot(yc.clamp(min=0), K).to(torch.float32) if K > 1 else None
            if K == 1 and float(p.get("scale_pos_weight", 1.0)) != 1.0:
                base_w = torch.where(yc == 1, base_w * float(p["scale_pos_weight"]), base_w)
        else:
            yv = torch.nan_to_num(y.to(torch.float32))
            Y = None
            valid = ~torch.isnan(y.to(torch.float32))
        base_w = torch.where(valid, base_w, torch.zeros_like(base_w))
        # base score: 0.5 probability / mean (XGBoost default base_score=0.5)
        if K == 1:
            if self._dist.link == "logit":
                f0 = 0.0
            elif self._dist.link == "log":
                mu = coll.allreduce_scalar(float((base_w * yv).sum())) / max(coll.allreduce_scalar(float(base_w.sum())), 1e-12)
                f0 = math.log(max(mu, 1e-10))
            else:
                f0 = coll.allreduce_scalar(float((base_w * yv).sum())) / max(coll.allreduce_scalar(float(base_w.sum())), 1e-12)
            self._init_f = [f0]
        else:
            self._init_f = [0.0] * K
        f = torch.tensor(self._init_f, dtype=torch.float32, device=dev).view(1, -1).repeat(N, 1)
        self._gblinear = None
        if (p.get("booster") or "gbtree").lower() == "gblinear":
            return self._fit_gblinear(spec, yv, Y, base_w, f, K)
        tm = (p.get("tree_method") or "auto").lower()
        if tm not in ("auto", "hist", "approx"):
            raise ValueError(f"tree_method '{p.get('tree_method')}' is not supported: the trees are grown from "
                             "quantile histograms (tree_method hist / approx); exact split enumeration is not "
                             "implemented")
        gp = GrowParams(criterion="xgb", max_depth=int(p["max_depth"]) if int(p["max_depth"]) > 0 else 64,
                        min_rows=float(p["min_rows"]), reg_lambda=float(p["reg_lambda"]),
                        reg_alpha=float(p["reg_alpha"]), gamma=float(p["min_split_improvement"]),
                        col_sample_rate=float(p["col_sample_rate"]) * float(p.get("colsample_bynode", 1.0)),
                        max_leaves=int(p.get("max_leaves") or 0), seed=self._seed())
        from . import constraints as cons
        gp.monotone = cons.monotone_vector(p.get("monotone_constraints"), list(spec.x))
        if p.get("interaction_constraints"):
            gp.interaction_sets = cons.interaction_sets(p["interaction_constraints"], list(spec.x), p)
        policy = (p.get("grow_policy") or "depthwise").lower()
        if policy not in ("depthwise", "lossguide"):
            raise ValueError(f"grow_policy must be depthwise or lossguide, got {p.get('grow_policy')}")
        if policy == "lossguide":
            # best-first: the leaf budget goes to the largest loss reductions;
            # max_depth 0 means unlimited under lossguide (XGBoostModel.java:54)
            gp.leaf_budget_by_gain = True
            if int(p["max_depth"]) <= 0:
                gp.max_depth = 64
        grower = TreeGrower(bd, gp)
        forest = Forest()
        self._vinc = None          # incremental validation link (gbm._valid_raw_incremental)
        eta = float(p["learn_rate"])
        mds = float(p.get("max_delta_step") or 0.0)
        mabs = float(p.get("max_abs_leafnode_pred") or 0.0)
        booster = (p.get("booster") or "gbtree").lower()
        dart = booster == "dart"
        tree_w = []  # dart weights
        ntrees = int(p["ntrees"])
        weighted_drop = (p.get("sample_type") or "uniform").lower() == "weighted"
        if (p.get("sample_type") or "uniform").lower() not in ("uniform", "weighted"):
            raise ValueError(f"sample_type must be uniform or weighted, got {p.get('sample_type')}")
        start = 0
        if p.get("checkpoint") is not None:
            start, f, tree_w = self._resume_from(p["checkpoint"], forest, f, K)
        from .shared import iter_seed
        sr = float(p["sample_rate"])
        F = bd.F
        interval = int(p.get("score_tree_interval") or 0)
        stop_rounds = int(p.get("stopping_rounds") or 0)
        metric_name = (p.get("stopping_metric") or "auto").lower()
        if metric_name == "auto":
            metric_name = "logloss" if spec.is_classification else "deviance"
        history = []
        self._scoring_history = []
        max_rt = float(p.get("max_runtime_secs") or 0)
        t0 = time.time()
        sched = ScoreSchedule(p)
        for it in range(start, ntrees):
            # per-iteration randomness (checkpoint continuation draws what an
            # uninterrupted build draws)
            gen = torch.Generator(device=dev)
            gen.manual_seed(iter_seed(self._seed(), it, 1) + cloud.rank())
            rng = np.random.RandomState(iter_seed(self._seed(), it, 2))
            grower.rng = np.random.RandomState(iter_seed(self._seed(), it, 3))
            wt = base_w
            if sr < 1.0:
                wt = base_w * (torch.rand(N, generator=gen, device=dev) < sr)
            r = float(p.get("col_sample_rate_per_tree", 1.0))
            if r < 1.0:
                kk = max(1, int(math.floor(r * F + 0.5)))
                m = np.zeros(F, dtype=bool)
                m[rng.choice(F, size=kk, replace=False)] = True
                gp.tree_col_mask = m
            dropped = []
            f_use = f
            if dart and len(forest) and rng.rand() >= float(p.get("skip_drop", 0.0)):
                nit = len(forest) // K
                rd = float(p.get("rate_drop", 0.0))
                if weighted_drop:
                    # sample_type weighted: drop probability proportional to the tree weight
                    tw = np.asarray(tree_w[:nit], dtype=np.float64)
                    pr = rd * nit * tw / max(tw.sum(), 1e-300)
                    dropped = [i for i in range(nit) if rng.rand() < pr[i]]
                else:
                    dropped = [i for i in range(nit) if rng.rand() < rd]
                if not dropped and p.get("one_drop"):
                    dropped = [int(rng.randint(nit))]
                if dropped:
                    f_use = f - self._contrib(forest, tree_w, dropped, K, bd, N)
            if K == 1:
                g, h = self._dist.grad_hess(yv, f_use[:, 0])
                g, h = (g * wt).to(torch.float32).contiguous(), (h * wt).to(torch.float32).contiguous()
                tree, nid, leaves, tot = grower.grow(g, h, 1)
                vals = self._leaf_values(tot, eta, mds, mabs, gp, tree, leaves)
                for li, node in enumerate(leaves):
                    tree.value[node] = float(vals[li])
                delta = torch.tensor(vals, dtype=torch.float32, device=dev)[nid.long()].view(-1, 1)
                trees_it = [tree]
                deltas = [delta]
            else:
                P = torch.softmax(f_use, 1)
                trees_it, deltas = [], []
                for k in range(K):
                    g = ((P[:, k] - Y[:, k]) * wt).contiguous()
                    h = (torch.clamp(2 * P[:, k] * (1 - P[:, k]), min=1e-16) * wt).contiguous()
                    tree, nid, leaves, tot = grower.grow(g, h, 1)
                    vals = self._leaf_values(tot, eta, mds, mabs, gp, tree, leaves)
                    for li, node in enumerate(leaves):
                        tree.value[node] = float(vals[li])
                    trees_it.append(tree)
                    deltas.append(torch.tensor(vals, dtype=torch.float32, device=dev)[nid.long()])
            if dart and dropped:
                kd = len(dropped)
                nt = 1.0 / (kd + 1) if (p.get("normalize_type") or "tree") == "tree" else 1.0 / (1 + eta)
                for tt in trees_it:
                    for i in range(tt.n_nodes):
                        tt.value[i] *= nt
                scale = kd / (kd + 1.0) if (p.get("normalize_type") or "tree") == "tree" else 1.0 / (1 + eta)
                contrib = self._contrib(forest, tree_w, dropped, K, bd, N)
                for d in dropped:
                    tree_w[d] *= scale
                f = f - contrib * (1 - scale)
                deltas = [d * nt for d in deltas]
            for k, tt in enumerate(trees_it):
                forest.add(tt, k)
            tree_w.append(1.0)
            if K == 1:
                f = f + deltas[0]
            else:
                f = f + torch.stack(deltas, 1)
            n_it = it + 1
            # a max_runtime_secs stop scores the last iteration into the history too
            score, timed_out = self._tick(n_it, ntrees, sched, n_it == ntrees, t0, max_rt)
            if score:
                entry = {"number_of_trees": n_it}
                self._forest = forest
                sched.started()
                self._score_entry(entry, spec, f)
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
        if dart:
            # bake DART weights into leaf values
            for it, wgt in enumerate(tree_w):
                for k in range(K):
                    tt = forest.trees[it * K + k]
                    for i in range(tt.n_nodes):
                        tt.value[i] *= wgt
        self._forest = forest
        self._train_f = f
        self._vinc = None
        from .shared import forest_varimp
        self._output["variable_importances"] = forest_varimp(forest, spec.x)
        self._output["model_summary"] = {"number_of_trees": len(forest) // K, "booster": booster}

    @staticmethod
    def _coord_delta(G, H, w, alpha, lam):
        """XGBoost's CoordinateDelta (src/linear/coordinate_common.h): the L1/L2
        regularised Newton step of one coefficient, never crossing zero."""
        Gl = G + lam * w
        Hl = H + lam
        tmp = w - Gl / torch.where(Hl > 0, Hl, torch.ones_like(Hl))
        up = torch.maximum(-(Gl + alpha) / Hl, -w)
        dn = torch.minimum(-(Gl - alpha) / Hl, -w)
        d = torch.where(tmp >= 0, up, dn)
        return torch.where(H < 1e-5, torch.zeros_like(d), d)

    def _fit_gblinear(self, spec, yv, Y, base_w, f, K):
        """booster = gblinear (XGBoostModel.java:54): boosted linear model.
        Each round: the bias Newton step, then every coefficient's
        regularised coordinate step from the same gradient pairs (XGBoost's
        shotgun updater, done as two GEMVs over the design in HBM: X^T g and
        (X.X)^T h), all scaled by eta.  Penalties are denormalised by the
        total row weight as XGBoost does (LinearTrainParam)."""
        from ..datainfo import DataInfo
        p = self._parms
        di = DataInfo(spec.frame, spec.x, standardize=False, use_all_factor_levels=True, pad_to=1)
        X = di.expand(spec.frame, pad=False)[0].to(torch.float32)
        self._gbl_di = di
        P = X.shape[1]
        dev = X.device
        wsum = coll.allreduce_scalar(float(base_w.sum()))
        lam = float(p.get("reg_lambda", 1.0)) * wsum
        alpha = float(p.get("reg_alpha", 0.0)) * wsum
        eta = float(p["learn_rate"])
        W = torch.zeros((P, K), dtype=torch.float64, device=dev)
        b = torch.tensor(self._init_f, dtype=torch.float64, device=dev)
        X2 = X * X
        ntrees = int(p["ntrees"])
        t0 = time.time()
        max_rt = float(p.get("max_runtime_secs") or 0)
        sched = ScoreSchedule(p)
        self._scoring_history = []
        f = f.to(torch.float64)
        for it in range(ntrees):
            if K == 1:
                g, h = self._dist.grad_hess(yv, f[:, 0].to(torch.float32))
                g, h = (g * base_w).to(torch.float64).view(-1, 1), (h * base_w).to(torch.float64).view(-1, 1)
            else:
                Pm = torch.softmax(f, 1)
                g = ((Pm - Y) * base_w.view(-1, 1)).to(torch.float64)
                h = (torch.clamp(2 * Pm * (1 - Pm), min=1e-16) * base_w.view(-1, 1)).to(torch.float64)
            sg = torch.cat([g.sum(0), h.sum(0)])
            coll.allreduce_(sg)
            db = eta * torch.where(sg[K:] > 0, -sg[:K] / sg[K:].clamp_min(1e-300), torch.zeros_like(sg[:K]))
            b = b + db
            f = f + db.view(1, -1)
            g = g + h * db.view(1, -1)                      # gradient pairs after the bias step
            G = X.T.to(torch.float64) @ g
            Hs = X2.T.to(torch.float64) @ h
            coll.allreduce_many_([G, Hs])
            dW = eta * self._coord_delta(G, Hs, W, alpha, lam)
            W = W + dW
            f = f + (X.to(torch.float64) @ dW)
            score, timed_out = self._tick(it + 1, ntrees, sched, it + 1 == ntrees, t0, max_rt)
            if score:
                self._gblinear = (W, b)
                entry = {"number_of_trees": it + 1}
                self._score_entry(entry, spec, f.to(torch.float32))
                self._scoring_history.append(entry)
            if timed_out:
                break
        self._gblinear = (W, b)
        self._forest = Forest()
        self._train_f = f.to(torch.float32)
        names = di.coef_names
        imp = W.abs().sum(1).cpu().numpy()
        order = np.argsort(-imp)
        mx = float(imp.max()) if imp.size and imp.max() > 0 else 1.0
        tot = float(imp.sum()) or 1.0
        self._output["variable_importances"] = {"variable": [names[i] for i in order],
                                                "relative_importance": [float(imp[i]) for i in order],
                                                "scaled_importance": [float(imp[i] / mx) for i in order],
                                                "percentage": [float(imp[i] / tot) for i in order]}
        self._output["model_summary"] = {"number_of_trees": 0, "booster": "gblinear"}
        self._output["coefficients"] = {n: W[i].cpu().tolist() for i, n in enumerate(names)}
        self._output["intercept"] = b.cpu().tolist()

    def _raw_from_f(self, f):
        if self._K > 1:
            return torch.softmax(f, 1)
        mu = self._dist.linkinv(f[:, 0])
        if self._spec.nclasses == 2:
            return torch.stack([1 - mu, mu], 1)
        return mu.view(-1, 1)

    def _score_entry(self, entry, spec, f):
        self._lite_metrics = True
        try:
            self._score_entry_inner(entry, spec, f)
        finally:
            self._lite_metrics = False

    def _score_entry_inner(self, entry, spec, f):
        from .gbm import H2OGradientBoostingEstimator as _G
        _G._add_metrics(entry, "training", self._metrics_from_raw(spec, spec.frame, self._raw_from_f(f)))
        if spec.valid is not None:
            # gbtree: the validation link grows by the new trees only (DART
            # rescales earlier trees, so it re-predicts the forest)
            dart = (self._parms.get("booster") or "gbtree").lower() == "dart"
            vr = self._predict_raw(spec.valid) if dart else _G._valid_raw_incremental(self, spec.valid)
            _G._add_metrics(entry, "validation", self._metrics_from_raw(spec, spec.valid, vr))

    def _contrib(self, forest, tree_w, dropped, K, bd, N):
        X = self._score_matrix(self._spec.frame)
        out = torch.zeros((N, K), dtype=torch.float32, device=X.device)
        sub = Forest()
        for d in dropped:
            for k in range(K):
                sub.add(forest.trees[d * K + k], k)
        s = sub.predict(X, K)
        # weights of dropped trees
        return s * torch.tensor([tree_w[d] for d in dropped], device=X.device).mean() if dropped else out

    @staticmethod
    def _leaf_values(tot, eta, mds, mabs, gp, tree=None, leaves=None):
        tot = tot.numpy() if isinstance(tot, torch.Tensor) else np.asarray(tot)
        G, H = tot[:, 0], tot[:, 1]
        if gp.reg_alpha > 0:
            G = np.sign(G) * np.maximum(np.abs(G) - gp.reg_alpha, 0)
        v = -G / (H + gp.reg_lambda)
        if mds > 0:
            v = np.clip(v, -mds, mds)
        if gp.monotone is not None and tree is not None:
            # XGBoost's monotone bounds (mid-point of the children's weights),
            # leaf weights clamped into them
            from .constraints import monotone_clamp
            v = monotone_clamp(tree, leaves, v, H + gp.reg_lambda, gp.monotone)
        v = v * eta
        if mabs > 0:
            v = np.clip(v, -mabs, mabs)
        return v

    def _resume_from(self, ck, forest, f, K):
        """checkpoint (XGBoost.java:126, :429): the checkpoint's trees, its raw
        predictions on the training rows, and the iteration counter."""
        from .shared import checkpoint_model
        prev, done = checkpoint_model(ck, "xgboost", self)
        if prev._K != K:
            raise ValueError("checkpoint: the checkpoint model has a different number of tree classes")
        if (prev._parms.get("booster") or "gbtree").lower() != (self._parms.get("booster") or "gbtree").lower():
            raise ValueError("checkpoint: booster must match the checkpoint model's")
        for t, k in zip(prev._forest.trees, prev._forest.tclass):
            forest.add(t, k)
        X = self._score_matrix(self._spec.frame)
        f = f + prev._forest.predict(X, K)
        return done, f, [1.0] * done

    def _seed(self):
        s = self._parms.get("seed", -1)
        return 777 if s is None or s == -1 else int(s) & 0x7FFFFFFF

    def _predict_raw(self, frame):
        K = self._K
        if getattr(self, "_gblinear", None) is not None:
            W, b = self._gblinear
            Xd = self._gbl_di.expand(frame, pad=False)[0].to(torch.float64)
            f = (Xd @ W + b.view(1, -1)).to(torch.float32)
        else:
            X = self._score_matrix(frame)
            f = self._forest.predict(X, K) + torch.tensor(self._init_f, dtype=torch.float32,
                                                          device=X.device).view(1, -1)
        if K > 1:
            return torch.softmax(f, 1)
        mu = self._dist.linkinv(f[:, 0])
        if self._spec.nclasses == 2:
            return torch.stack([1 - mu, mu], 1)
        return mu.view(-1, 1)

    def predict_contributions(self, test_data, **kw):
        if getattr(self, "_gblinear", None) is not None:
            raise NotImplementedError("predict_contributions is not available for booster=gblinear (no trees)")
        from .shap import tree_contributions
        return tree_contributions(self, test_data)
