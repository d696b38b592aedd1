"""Gradient Boosting Machine.

Reference: hex/tree/gbm/GBM.java — per iteration: compute the negative
half-gradient residuals (GBM.ComputePredAndRes / Distribution.negHalfGradient),
grow K regression trees on them with the squared-error histogram
criterion (SharedTree + DTree.findBestSplitPoint), then set terminal node
values with the distribution-specific Newton step (GBM.GammaPass,
gbm/GBM.java:1286: gamma = sum(w*num)/sum(w*denom)) and add
learn_rate * gamma to the predictions.

MI355X design: residuals, weights and predictions are device tensors; the
tree is grown by TreeGrower (LDS histogram kernel + GPU partition) and the
leaf rows are contiguous segments, so the gamma pass is two index_add
reductions over the per-row leaf ids and the prediction update one gather.
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from ...core.frame import H2OFrame
from ...parallel import cloud
from ...parallel import collectives as coll
from ..base import ScoreKeeper, ScoreSchedule, _LESS_IS_BETTER
from ..distributions import get_distribution
from .engine import GrowParams, TreeGrower
from ...ops import tree_ops
from ...utils.timer import phase
from .shared import Forest, SharedTreeEstimator
from ...core.groupsum import index_add as _ia

GBM_DEFAULTS = dict(ntrees=50, max_depth=5, min_rows=10.0, nbins=20, nbins_top_level=1024, nbins_cats=1024,
                    r2_stopping=1.79e308, stopping_rounds=0, stopping_metric="auto", stopping_tolerance=0.001,
                    seed=-1, build_tree_one_node=False, learn_rate=0.1, learn_rate_annealing=1.0,
                    distribution="auto", quantile_alpha=0.5, tweedie_power=1.5, huber_alpha=0.9,
                    checkpoint=None, sample_rate=1.0, sample_rate_per_class=None, col_sample_rate=1.0,
                    col_sample_rate_change_per_level=1.0, col_sample_rate_per_tree=1.0,
                    min_split_improvement=1e-5, histogram_type="auto", max_abs_leafnode_pred=1.79e308,
                    pred_noise_bandwidth=0.0, categorical_encoding="auto", calibrate_model=False,
                    calibration_frame=None, calibration_method="auto", custom_distribution_func=None,
                    monotone_constraints=None, check_constant_response=True, interaction_constraints=None,
                    score_tree_interval=0, balance_classes=False, class_sampling_factors=None,
                    max_after_balance_size=5.0, max_confusion_matrix_size=20, in_training_checkpoints_dir=None,
                    in_training_checkpoints_tree_interval=1)


class GBMDriver:
    """Stateful boosting loop (one `step()` = one boosting iteration = K trees)."""

    def __init__(self, est, spec, bd=None):
        self.est = est
        p = est._parms
        self.spec = spec
        self.K = spec.nclasses if spec.nclasses > 2 else 1
        dist_name = p.get("distribution", "auto")
        if spec.nclasses == 2 and dist_name in ("auto", "AUTO"):
            dist_name = "bernoulli"
        self.dist = get_distribution(dist_name, spec.nclasses, tweedie_power=p.get("tweedie_power", 1.5),
                                     quantile_alpha=p.get("quantile_alpha", 0.5),
                                     huber_alpha=p.get("huber_alpha", 0.9),
                                     custom_distribution_func=p.get("custom_distribution_func"))
        est._dist = self.dist
        dev = cloud.device()
        self.dev = dev
        self.bd = bd if bd is not None else est._bin(spec)
        N = self.bd.nrows_local
        y = spec.y_tensor()
        w = spec.w_tensor()
        self.w_user = w
        if spec.is_classification:
            self.ycode = y.to(torch.int64)
            valid = self.ycode >= 0
        else:
            self.yf = y.to(torch.float32)
            valid = ~torch.isnan(self.yf)
        base_w = torch.ones(N, dtype=torch.float32, device=dev) if w is None else w.to(torch.float32)
        self.base_w = torch.where(valid, base_w, torch.zeros_like(base_w))
        pp = est._parms
        self._unit_weights = bool((self.base_w == 1).all()) and float(pp.get("sample_rate", 1.0)) >= 1.0 and \
            pp.get("sample_rate_per_class") is None
        self.offset = spec.offset_tensor()
        # init prediction (reference: GBM.init -> initial value by distribution)
        if self.K == 1:
            if spec.nclasses == 2:
                yv = (self.ycode == 1).to(torch.float32)
                self.yb = yv
            else:
                yv = torch.nan_to_num(self.yf)
            sw = coll.allreduce_scalar(float(self.base_w.sum()))
            sy = coll.allreduce_scalar(float((self.base_w * yv).sum()))
            mu = sy / sw if sw > 0 else 0.0
            if self.dist.family == "custom":
                f0 = self.dist.init_f(yv, self.base_w, self.offset)
            elif self.dist.family in ("laplace", "quantile", "huber"):
                f0 = _weighted_quantile(yv[self.base_w > 0], self.base_w[self.base_w > 0],
                                        0.5 if self.dist.family != "quantile" else self.dist.quantile_alpha)
            elif self.dist.link == "logit":
                mu = min(max(mu, 1e-10), 1 - 1e-10)
                f0 = math.log(mu / (1 - mu))
            elif self.dist.link == "log":
                f0 = math.log(max(mu, 1e-10))
            else:
                f0 = mu
            if self.offset is not None and self.dist.link != "identity" and self.dist.family != "custom":
                f0 = self._newton_init(f0, yv)
            self.init_f = [f0]
        else:
            # multinomial: reference initialises f_k = log(prior_k) - mean
            ok = self.ycode >= 0
            from ...core.groupsum import group_sum
            cnt = group_sum(self.ycode[ok], self.base_w[ok], self.K)
            coll.allreduce_(cnt)
            pri = (cnt / cnt.sum()).clamp_min(1e-10)
            lp = torch.log(pri)
            self.init_f = (lp - lp.mean()).cpu().tolist()
            self.Y = torch.nn.functional.one_hot(self.ycode.clamp(min=0), self.K).to(torch.float32)
        self.f = torch.tensor(self.init_f, dtype=torch.float32, device=dev).view(1, -1).repeat(N, 1)
        if self.offset is not None:
            self.f += self.offset.view(-1, 1)
        gp = GrowParams(criterion="se", max_depth=int(p["max_depth"]) if p["max_depth"] > 0 else 64,
                        min_rows=float(p["min_rows"]), min_split_improvement=float(p["min_split_improvement"]),
                        col_sample_rate=float(p["col_sample_rate"]),
                        col_sample_rate_change_per_level=float(p["col_sample_rate_change_per_level"]),
                        seed=self._seed())
        from . import constraints as cons
        gp.monotone = cons.monotone_vector(p.get("monotone_constraints"), list(spec.x))
        self.mono_on = gp.monotone is not None
        if self.mono_on:
            cons.check_monotone_family(self.dist.family)
        ic = p.get("interaction_constraints")
        if ic:
            from ..catenc import canon
            if canon(p.get("categorical_encoding")) not in ("AUTO", "OneHotInternal"):
                raise ValueError("interaction_constraints: Interaction constraints can be used when the "
                                 "categorical encoding is set to AUTO (one_hot_internal or OneHotInternal) only.")
            gp.interaction_sets = cons.interaction_sets(ic, list(spec.x), p)
        self.noise_bw = float(p.get("pred_noise_bandwidth") or 0.0)
        self.gp = gp
        self.grower = TreeGrower(self.bd, gp)
        self._pending = None
        self.forest = Forest()
        self.lr = float(p["learn_rate"])
        self.iter = 0
        self.rng = np.random.RandomState(self._seed())
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(self._seed() + cloud.rank())
        if self.dist.family == "huber":
            self.dist.huber_delta = None

    def _seed(self):
        s = self.est._parms.get("seed", -1)
        return 1234 if s is None or s == -1 else int(s) & 0x7FFFFFFF

    def _newton_init(self, f0, yv):
        for _ in range(20):
            ff = f0 + self.offset
            z = self.dist.neg_half_gradient(yv, ff)
            num = coll.allreduce_scalar(float(self.dist.gamma_num(self.base_w, yv, z, ff).sum()))
            den = coll.allreduce_scalar(float(self.dist.gamma_denom(self.base_w, yv, z, ff).sum()))
            if self.dist.link == "logit":
                step = num / den if den != 0 else 0.0
                f0 += step
                if abs(step) < 1e-8:
                    break
            else:
                g = self.dist.gamma(num, den)
                f0 += g
                if abs(g) < 1e-8:
                    break
        return f0

    @property
    def forest(self):
        self._resolve_pending()
        return self._forest_obj

    @forest.setter
    def forest(self, fo):
        self._pending = None
        self._forest_obj = fo

    def _resolve_pending(self):
        """Fill the last tree's leaf values from its async device->host copy."""
        pend = getattr(self, "_pending", None)
        if pend is None:
            return
        self._pending = None
        if pend[0] == "dev":
            # device-resident tree: the whole tree arrives as one heap record
            _, hrec, ev = pend
            ev.synchronize()
            self._forest_obj.add(self._devtree.decode(hrec.numpy()), 0)
            return
        tree, leaves, hv, ev = pend
        ev.synchronize()
        v = hv.numpy().tolist()
        for li, node in enumerate(leaves):
            tree.value[node] = float(v[li])
        # a pack taken before the values landed holds zero leaf values: drop it
        if self._forest_obj is not None:
            self._forest_obj._packed = None

    def _row_weights(self):
        p = self.est._parms
        w = self.base_w
        sr = float(p.get("sample_rate", 1.0))
        srpc = p.get("sample_rate_per_class")
        if srpc is not None and self.spec.is_classification:
            rates = torch.tensor(srpc, dtype=torch.float32, device=self.dev)[self.ycode.clamp(min=0)]
            keep = torch.rand(w.shape, generator=self.gen, device=self.dev) < rates
            return w * keep
        if sr < 1.0:
            keep = torch.rand(w.shape, generator=self.gen, device=self.dev) < sr
            return w * keep
        return w

    def _tree_col_mask(self):
        r = float(self.est._parms.get("col_sample_rate_per_tree", 1.0))
        F = self.bd.F
        if r >= 1.0:
            return None
        k = max(1, int(math.floor(r * F + 0.5)))
        m = np.zeros(F, dtype=bool)
        m[self.rng.choice(F, size=k, replace=False)] = True
        return m

    # f: the running raw prediction [N, K].  With the scatter leaf update the
    # last tree's per-row leaf values wait in _dpend and are folded into f by
    # the next residual pass; any other reader of f flushes them first.
    @property
    def f(self):
        d = self.__dict__.get("_dpend")
        if d is not None:
            self._dpend = None
            self._f[:, 0].add_(d)
        return self._f

    @f.setter
    def f(self, v):
        self._dpend = None
        self._f = v

    def _scatter_ok(self, st, ct):
        """The scatter update writes every row: only when the leaf segments
        tile all N positions of the row permutation."""
        if os.environ.get("H2O3_LEAF_SCATTER", "1") != "1":
            return False
        st = np.asarray(st, dtype=np.int64)
        ct = np.asarray(ct, dtype=np.int64)
        m = ct > 0
        st, ct = st[m], ct[m]
        if st.size == 0:
            return False
        o = np.argsort(st, kind="stable")
        st, ct = st[o], ct[o]
        return bool(st[0] == 0 and st[-1] + ct[-1] == self._f.shape[0] and
                    (st.size == 1 or np.array_equal(st[1:], st[:-1] + ct[:-1])))

    def step(self):
        """One boosting iteration."""
        p = self.est._parms
        from .shared import reseed_iteration
        reseed_iteration(self, self._seed(), self.iter)
        w = self._row_weights()
        self.gp.tree_col_mask = self._tree_col_mask()
        # GBM.effective_learning_rate (GBM.java:726): learn_rate *
        # annealing^(trees already built - 1) while the leaves of the next tree
        # are fitted -- the first tree uses learn_rate / annealing
        lr = self.lr * (float(p.get("learn_rate_annealing", 1.0)) ** (self.iter - 1))
        maxabs = float(p.get("max_abs_leafnode_pred", 1.79e308))
        if self.K == 1 and self._devtree_ok():
            self._step_devtree(lr, w)
            return
        if self.K == 1:
            dpend = self.__dict__.get("_dpend")
            self._dpend = None
            f = self._f[:, 0]
            y = self.yb if self.spec.nclasses == 2 else torch.nan_to_num(self.yf)
            # monotone bounds / prediction noise need the leaf values on the host
            # before the prediction update: not the device-resident leaf path
            simple = self.dev.type == "cuda" and self.dist.family in ("gaussian", "bernoulli") and \
                self.dist.link in ("identity", "logit") and not self.mono_on and self.noise_bw == 0
            fused = simple and os.environ.get("H2O3_FUSED_LEAF", "0") == "1"
            # position-ordered residual payload + segment update: no per-row leaf ids at all
            posleaf = simple and not fused and self.K == 1 and self.f.shape[1] == 1 and \
                os.environ.get("H2O3_POS_LEAF", "1") == "1"
            if getattr(self, "_base_unit", None) is None:
                bw = self.base_w
                self._base_unit = bool(((bw == 0) | (bw == 1)).all())
            # one-pass residual straight into the grower's root payload (NaN =
            # weight 0): the 0/1-weight position-ordered path of grow()
            onepass = posleaf and self._base_unit and self.grower.pos_payload_ok() and \
                os.environ.get("H2O3_GBM_GRAD", "1") == "1"
            if dpend is not None and not onepass:
                f.add_(dpend)
                dpend = None
            with phase("gbm.grad"):
                if onepass:
                    z = tree_ops.gbm_grad(y, f, None if self._unit_weights else w, self.dist.family, d=dpend)
                else:
                    z = self.dist.neg_half_gradient(y, f).to(torch.float32)
            if self.dist.family == "huber":
                self._update_huber_delta(y, f, w)
                z = self.dist.neg_half_gradient(y, f).to(torch.float32)
            # bernoulli residuals y - p lie in (-1, 1): with 0/1 weights both
            # histogram channels are bounded by 1 (no per-tree max reduction)
            vmax_h = [1.0, 1.0] if (self.dist.family == "bernoulli" and self._base_unit) else None
            with phase("gbm.grow"):
                if onepass:
                    tree, nid, leaves, tot = self.grower.grow(z, None, 0, want_nid=False, vmax=vmax_h,
                                                              unit_w=True, va_scratch=True)
                else:
                    tree, nid, leaves, tot = self.grower.grow(z.contiguous(), w.contiguous(), 0,
                                                              want_nid=not (fused or posleaf), vmax=vmax_h,
                                                              unit_w=self._base_unit)
            zpos = self.grower._pos1[0] if (posleaf and getattr(self.grower, "_pos1", None) is not None) else None
            if posleaf and zpos is None:
                posleaf = False
                nid = tree_ops.fill_nid(self.grower.ridx, *self.grower.last_segs, z.shape[0])
            if posleaf:
                # leaf values stay on the device: the prediction update runs
                # without a host round trip and the tree's host copy of the
                # values arrives by an async pinned copy, resolved the next time
                # the forest is touched (no GPU bubble between trees)
                lids, st, ct = self.grower.last_segs
                with phase("gbm.gamma"):
                    s_ = tree_ops.leaf_pos_sums(zpos, lids, st, ct, len(leaves),
                                                1 if self.dist.family == "bernoulli" else 0)
                    coll.allreduce_(s_)
                    den = s_[:, 1]
                    vals_d = torch.where(den != 0, s_[:, 0] / torch.where(den == 0, torch.ones_like(den), den),
                                         torch.zeros_like(den)).clamp(-maxabs, maxabs) * lr
                with phase("gbm.update"):
                    if onepass and self._scatter_ok(st, ct):
                        # write-only scatter of the per-row leaf value; the next
                        # residual pass adds it into f (no random read-modify-write)
                        db = self.__dict__.get("_dbuf")
                        if db is None or db.numel() != f.numel():
                            db = self._dbuf = torch.empty_like(f)
                        tree_ops.leaf_scatter(self.grower.ridx, db, vals_d.to(torch.float32), lids, st, ct)
                        self._dpend = db
                    else:
                        tree_ops.leaf_update(self.grower.ridx, self._f, vals_d.to(torch.float32), lids, st, ct)
                # two reusable pinned slots: tree t's values land in one while
                # tree t-1's (read by _resolve_pending below) sit in the other
                ring = self.__dict__.setdefault("_hv_ring", [None, None])
                k_ = self.iter & 1
                if ring[k_] is None or ring[k_].numel() < vals_d.numel():
                    ring[k_] = torch.empty(max(vals_d.numel(), 1024), dtype=torch.float64, pin_memory=True)
                hv = ring[k_][:vals_d.numel()]
                hv.copy_(vals_d, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                self._resolve_pending()
                self._forest_obj.add(tree, 0)
                self._pending = (tree, list(leaves), hv, ev)
                self.iter += 1
                return
            with phase("gbm.gamma"):
                if fused:
                    # one walk over the leaf segments: nid fill + gamma sums
                    lids, st, ct = self.grower.last_segs
                    nid, s_ = tree_ops.leaf_pass(self.grower.ridx, z, w, lids, st, ct, len(leaves), z.shape[0],
                                                 1 if self.dist.family == "bernoulli" else 0)
                    coll.allreduce_(s_)
                    sh = s_.cpu().numpy()
                    vals = np.where(sh[:, 1] != 0, sh[:, 0] / np.where(sh[:, 1] == 0, 1, sh[:, 1]), 0.0)
                elif self.dev.type == "cuda" and self.dist.family in ("gaussian", "bernoulli") and \
                        self.dist.link in ("identity", "logit"):
                    # gamma sums straight from the residual: den is w for gaussian and
                    # w |z| (1 - |z|) = w p (1 - p) for bernoulli -> one gather per row
                    lids, st, ct = self.grower.last_segs
                    wu = None if self._unit_weights else w
                    _, s_ = tree_ops.leaf_pass(self.grower.ridx, z, wu, lids, st, ct, len(leaves), z.shape[0],
                                               1 if self.dist.family == "bernoulli" else 0, want_nid=False)
                    coll.allreduce_(s_)
                    sh = s_.cpu().numpy()
                    vals = np.where(sh[:, 1] != 0, sh[:, 0] / np.where(sh[:, 1] == 0, 1, sh[:, 1]), 0.0)
                    self._last_den = sh[:, 1]
                else:
                    self._last_den = None
                    vals = self._gamma(tree, nid, leaves, w, y, z, f, 0)
            vals = np.clip(vals, -maxabs, maxabs)
            if self.mono_on:
                from .constraints import monotone_clamp
                dens = self._last_den if self._last_den is not None else np.asarray(tree.weight)[leaves]
                vals = monotone_clamp(tree, leaves, vals, dens, self.gp.monotone)
            for li, node in enumerate(leaves):
                tree.value[node] = float(lr * vals[li])
            with phase("gbm.update"):
                vt = torch.tensor(lr * vals * self._noise(0, len(leaves)), dtype=torch.float32, device=self.dev)
                if posleaf:
                    lids, st, ct = self.grower.last_segs
                    tree_ops.leaf_update(self.grower.ridx, self.f, vt, lids, st, ct)
                else:
                    self.f[:, 0] += vt[nid.long()]
            self.forest.add(tree, 0)
        else:
            P = torch.softmax(self.f, 1)
            if getattr(self, "_base_unit", None) is None:
                bw = self.base_w
                self._base_unit = bool(((bw == 0) | (bw == 1)).all())
            if self.dev.type == "cuda" and self._base_unit and self.noise_bw == 0 and \
                    self.grower.pos_payload_ok() and os.environ.get("H2O3_POS_LEAF", "1") == "1":
                self._step_multi_dev(P, w, lr, maxabs)
                self.iter += 1
                return
            new = []
            for k in range(self.K):
                z = (self.Y[:, k] - P[:, k]).contiguous()
                tree, nid, leaves, tot = self.grower.grow(z, w.contiguous(), 0)
                vals = self._gamma_multi(nid, len(leaves), w, z)
                vals = np.clip(vals, -maxabs, maxabs)
                for li, node in enumerate(leaves):
                    tree.value[node] = float(lr * vals[li])
                vt = torch.tensor(lr * vals * self._noise(k, len(leaves)), dtype=torch.float32, device=self.dev)
                new.append(vt[nid.long()])
                self.forest.add(tree, k)
            for k in range(self.K):
                self.f[:, k] += new[k]
        self.iter += 1

    def _devtree_ok(self):
        """The device-resident tree (devtree.py) serves this configuration."""
        dt = self.__dict__.get("_devtree")
        if dt is not None:
            return True
        if self.__dict__.get("_devtree_why") is not None:
            return False
        if getattr(self, "_base_unit", None) is None:
            bw = self.base_w
            self._base_unit = bool(((bw == 0) | (bw == 1)).all())
        from . import devtree
        why = devtree.supported(self)
        if why is None:
            self._devtree = devtree.DevTreeGBM(self)
            return True
        self._devtree_why = why
        return False

    def _step_devtree(self, lr, w=None):
        """One boosting iteration as one device-resident tree (graph replay on
        one rank): residual, every level, leaf values and the per-row leaf
        scatter without a host round trip; the tree's record is decoded on the
        host while the GPU grows the next one."""
        dt = self._devtree
        dt.set_tree_cols(self.gp.tree_col_mask)
        dt.set_col_sampling(self.gp.tree_col_mask)
        pending = self.__dict__.get("_dpend") is not None
        self._dpend = None
        with phase("gbm.devtree"):
            hrec, ev = dt.run(lr, pending, w)
        self._dpend = dt.dbuf
        self._resolve_pending()
        self._pending = ("dev", hrec, ev)
        self.iter += 1

    def _step_multi_dev(self, P, w, lr, maxabs):
        """Multinomial iteration on the position-ordered path: each class tree
        keeps its NaN-masked residual as the grower's payload, the gamma sums
        ((K-1)/K * sum z / sum |z|(1-|z|)) come from contiguous reads of it,
        the leaf values stay on the device and are scattered into a per-class
        delta -- no per-row leaf ids, no host gamma -- and ONE host copy per
        iteration brings every class tree's leaf values back."""
        K = self.K
        wc = w.contiguous()
        deltas, vals_l, trees = [], [], []
        for k in range(K):
            z = (self.Y[:, k] - P[:, k]).contiguous()
            tree, nid, leaves, tot = self.grower.grow(z, wc, 0, want_nid=False, vmax=[1.0, 1.0], unit_w=True)
            zpos = self.grower._pos1[0] if getattr(self.grower, "_pos1", None) is not None else None
            lids, st, ct = self.grower.last_segs
            L = len(leaves)
            if zpos is not None:
                s_ = tree_ops.leaf_pos_sums(zpos, lids, st, ct, L, 1)
            else:
                s_ = tree_ops.seg_sum2(self.grower.ridx, wc * z, wc * z.abs() * (1 - z.abs()), lids, st, ct, L)
            coll.allreduce_(s_)
            den = s_[:, 1]
            v = torch.where(den > 1e-300, s_[:, 0] / torch.where(den > 1e-300, den, torch.ones_like(den)),
                            torch.zeros_like(den))
            v = ((K - 1.0) / K * v).clamp(-maxabs, maxabs) * lr
            d = torch.empty(self.f.shape[0], dtype=torch.float32, device=self.dev) if self._scatter_ok(st, ct) \
                else torch.zeros(self.f.shape[0], dtype=torch.float32, device=self.dev)
            vf = v.to(torch.float32)
            if self._scatter_ok(st, ct):
                tree_ops.leaf_scatter(self.grower.ridx, d, vf, lids, st, ct)
            else:
                tree_ops.leaf_update(self.grower.ridx, d, vf, lids, st, ct)
            deltas.append(d)
            vals_l.append(v)
            trees.append((tree, list(leaves)))
        for k in range(K):
            self.f[:, k] += deltas[k]
        host = torch.cat(vals_l).cpu().numpy()
        o = 0
        for k, (tree, leaves) in enumerate(trees):
            for li, node in enumerate(leaves):
                tree.value[node] = float(host[o + li])
            o += len(leaves)
            self.forest.add(tree, k)

    def _noise(self, k, nleaves):
        """pred_noise_bandwidth factors of this tree's leaves (1 when off)."""
        if self.noise_bw == 0:
            return 1.0
        from .constraints import noise_factors
        return noise_factors(self._seed(), k, int(self.est._parms.get("ntrees", 0)), self.iter, nleaves,
                             self.noise_bw)

    def _update_huber_delta(self, y, f, w):
        r = (y - f).abs()
        m = w > 0
        self.dist.huber_delta = _weighted_quantile(r[m], w[m], self.dist.huber_alpha)

    def _gamma(self, tree, nid, leaves, w, y, z, f, k):
        L = len(leaves)
        idx = nid.long()
        fam = self.dist.family
        if fam in ("laplace", "quantile"):
            alpha = 0.5 if fam == "laplace" else self.dist.quantile_alpha
            return _segmented_wquantile(idx, (y - f).to(torch.float64), w.to(torch.float64), L, alpha)
        if fam == "huber":
            res = (y - f).to(torch.float64)
            med = _segmented_wquantile(idx, res, w.to(torch.float64), L, 0.5)
            mt = torch.tensor(med, dtype=torch.float64, device=self.dev)
            d = res - mt[idx]
            delta = self.dist.huber_delta
            corr = torch.sign(d) * torch.minimum(d.abs(), torch.full_like(d, delta))
            num = _ia(torch.zeros(L, dtype=torch.float64, device=self.dev), idx, w.to(torch.float64) * corr)
            den = _ia(torch.zeros(L, dtype=torch.float64, device=self.dev), idx, w.to(torch.float64))
            s = torch.cat([num, den])
            coll.allreduce_(s)
            num, den = s[:L], s[L:]
            return (mt + torch.where(den > 0, num / den.clamp_min(1e-300), torch.zeros_like(num))).cpu().numpy()
        num_r = self.dist.gamma_num(w, y, z, f)
        den_r = self.dist.gamma_denom(w, y, z, f)
        lids, st, ct = self.grower.last_segs
        s = tree_ops.seg_sum2(self.grower.ridx, num_r, den_r, lids, st, ct, L)
        coll.allreduce_(s)
        sh = s.cpu().numpy()
        num, den = sh[:, 0], sh[:, 1]
        self._last_den = den
        if self.dist.link == "log" or self.dist.family in ("poisson", "gamma", "tweedie"):
            return np.array([self.dist.gamma(float(a), float(b)) for a, b in zip(num, den)])
        out = np.where(den != 0, num / np.where(den == 0, 1, den), 0.0)
        return out

    def _gamma_multi(self, nid, L, w, z):
        K = self.K
        lids, st, ct = self.grower.last_segs
        s = tree_ops.seg_sum2(self.grower.ridx, w * z, w * z.abs() * (1 - z.abs()), lids, st, ct, L)
        coll.allreduce_(s)
        sh = s.cpu().numpy()
        num, den = sh[:, 0], sh[:, 1]
        return (K - 1.0) / K * np.where(den > 1e-300, num / np.where(den > 1e-300, den, 1), 0.0)

    def predictions(self):
        if self.K == 1:
            return self.dist.linkinv(self.f[:, 0])
        return torch.softmax(self.f, 1)


class H2OGradientBoostingEstimator(SharedTreeEstimator):
    algo = "gbm"
    _defaults = GBM_DEFAULTS

    def _n_tree_classes(self):
        return self._K

    def _fit(self, spec):
        p = self._parms
        t0 = time.time()
        drv = GBMDriver(self, spec)
        self._K = drv.K
        self._driver = drv
        self._vinc = None          # incremental validation link (_valid_raw_incremental)
        ntrees = int(p["ntrees"])
        if p.get("checkpoint") is not None:
            self._resume_from(drv, p["checkpoint"])
        interval = int(p.get("score_tree_interval") or 0)
        stop_rounds = int(p.get("stopping_rounds") or 0)
        metric_name = self._stopping_metric(spec)
        history = []
        max_rt = float(p.get("max_runtime_secs") or 0)
        self._scoring_history = []
        sched = ScoreSchedule(p)
        anneal = float(p.get("learn_rate_annealing", 1.0))
        while drv.iter < ntrees:
            drv.step()
            # GBM.java:586: stop once the effective learning rate of the next
            # tree, learn_rate * annealing^(ntrees - 1), drops below 1e-6
            lr_stop = anneal < 1.0 and float(p["learn_rate"]) * anneal ** (drv.iter - 1) < 1e-6
            # a max_runtime_secs stop scores the last tree into the history too
            score, timed_out = self._tick(drv.iter, ntrees, sched, drv.iter == ntrees or lr_stop, t0, max_rt)
            if score:
                sched.started()
                entry = self._score_iteration(drv, spec)
                sched.ended()
                self._scoring_history.append(entry)
                if stop_rounds > 0:
                    suffix = "custom" if metric_name.startswith("custom") else metric_name
                    key = ("validation_" if spec.valid is not None else "training_") + suffix
                    history.append(entry.get(key))
                    if ScoreKeeper.stop_early(history, stop_rounds, float(p["stopping_tolerance"]),
                                              metric_name in _LESS_IS_BETTER, metric=metric_name):
                        break
            if timed_out or lr_stop:
                break
            ckdir = p.get("in_training_checkpoints_dir")
            if ckdir and drv.iter % max(1, int(p.get("in_training_checkpoints_tree_interval") or 1)) == 0 and \
                    drv.iter < ntrees:
                self._in_training_checkpoint(drv, ckdir)
        self._forest = drv.forest
        self._init_f = drv.init_f
        self._output["variable_importances"] = self._varimp_from_forest(drv.forest, spec.x)
        self._output["model_summary"] = {"number_of_trees": len(drv.forest),
                                         "number_of_internal_trees": len(drv.forest),
                                         "min_depth": min((t.max_depth() for t in drv.forest.trees), default=0),
                                         "max_depth": max((t.max_depth() for t in drv.forest.trees), default=0),
                                         "mean_leaves": float(np.mean([len(t.leaves()) for t in drv.forest.trees]))
                                         if len(drv.forest) else 0.0}
        self._output["init_f"] = drv.init_f
        self._train_f = drv.f
        self._vinc = None
        self._used_devtree = drv.__dict__.get("_devtree") is not None
        del drv.grower
        self._driver = None
        if p.get("calibrate_model") and p.get("calibration_frame") is not None:
            from .calibration import fit_calibration
            fit_calibration(self, p["calibration_frame"], p.get("calibration_method", "auto"))

    def _in_training_checkpoint(self, drv, ckdir):
        """GBM.java:921 doInTrainingCheckpoint: the model so far, exported as a
        binary model `<dir>/<model_id>.ntrees_<n>` under key `<model_id>.<n>`
        (reloadable with h2o.load_model, usable as a `checkpoint`)."""
        import copy
        import os
        from ..persist import save_model
        n = drv.iter
        snap = copy.copy(self)
        snap.__dict__ = dict(self.__dict__)
        snap._parms = dict(self._parms)
        snap._output = dict(self._output)
        f = Forest()
        for t, k in zip(drv.forest.trees, drv.forest.tclass):
            f.add(t, k)
        snap._forest, snap._init_f, snap._K = f, list(drv.init_f), drv.K
        snap._id = f"{self._id}.{n}"
        snap._driver = None
        snap._output["model_summary"] = {"number_of_trees": n}
        os.makedirs(ckdir, exist_ok=True)
        save_model(snap, path=ckdir, force=True, filename=f"{self._id}.ntrees_{n}")

    def _cv_optimal_params(self, cv_models):
        if int(self._parms.get("stopping_rounds") or 0) > 0 and cv_models:
            nt = [len(m._forest) // max(1, m._K) for m in cv_models]
            self._parms["ntrees"] = int(math.ceil(np.mean(nt)))
            self._parms["stopping_rounds"] = 0

    def _stopping_metric(self, spec):
        m = (self._parms.get("stopping_metric") or "auto").lower()
        if m == "auto":
            return "logloss" if spec.is_classification else "deviance"
        if m == "custom_increasing":
            return "custom_increasing"
        return m

    def _score_iteration(self, drv, spec):
        self._lite_metrics = True
        try:
            return self._score_iteration_inner(drv, spec)
        finally:
            self._lite_metrics = False

    def _score_iteration_inner(self, drv, spec):
        entry = {"number_of_trees": drv.iter}
        pred = drv.predictions()
        raw = pred.view(-1, 1) if pred.dim() == 1 else pred
        if spec.nclasses == 2:
            raw = torch.stack([1 - raw[:, 0], raw[:, 0]], 1)
        m = self._metrics_from_raw(spec, spec.frame, raw, w=drv.w_user)
        self._add_metrics(entry, "training", m)
        if spec.valid is not None:
            self._forest = drv.forest
            self._init_f = drv.init_f
            vm = self._metrics_from_raw(spec, spec.valid, self._valid_raw_incremental(spec.valid))
            self._add_metrics(entry, "validation", vm)
        return entry

    def _valid_raw_incremental(self, frame):
        """Validation predictions at a scoring round from the running link of
        the trees already scored plus the trees grown since (the forest kernel
        over the new trees only): scoring every score_tree_interval trees
        costs O(new trees), not O(all trees) per round."""
        fo = self._forest
        T = len(fo)
        st = self.__dict__.get("_vinc")
        if st is None or st[0] is not frame or st[1] > T:
            X = self._score_matrix(frame)
            f = torch.zeros((X.shape[1], self._K), dtype=torch.float32, device=X.device)
            st = self._vinc = [frame, 0, f, X]
        _, t0, f, X = st
        if T > t0:
            f += fo.predict_range(X, self._K, t0, T)
            st[1] = T
        link = f + torch.tensor(self._init_f, dtype=torch.float32, device=f.device).view(1, -1)
        off = self._spec.offset_column
        if off and off in frame.names:
            link = link + torch.nan_to_num(frame.vec(off).as_float()).view(-1, 1)
        if self._K > 1:
            return torch.softmax(link, 1)
        mu = self._dist.linkinv(link[:, 0])
        if self._spec.nclasses == 2:
            return torch.stack([1 - mu, mu], 1)
        return mu.view(-1, 1)

    @staticmethod
    def _add_metrics(entry, prefix, m):
        if m is None:
            return
        for k, name in (("RMSE", "rmse"), ("logloss", "logloss"), ("AUC", "auc"), ("mae", "mae"),
                        ("mean_residual_deviance", "deviance"), ("MSE", "mse"), ("pr_auc", "aucpr"),
                        ("mean_per_class_error", "mean_per_class_error"), ("r2", "r2")):
            v = m.get(k)
            if v is not None:
                entry[f"{prefix}_{name}"] = v
        if m.get("custom_metric_value") is not None:
            entry[f"{prefix}_custom"] = m["custom_metric_value"]
        if m.get("cm") is not None and m.kind in ("binomial", "multinomial"):
            entry[f"{prefix}_classification_error"] = m["cm"]["total_error"]
            entry[f"{prefix}_misclassification"] = m["cm"]["total_error"]

    def _resume_from(self, drv, ck):
        from .shared import checkpoint_model
        prev, _ = checkpoint_model(ck, "gbm", self)
        drv.forest = Forest()
        for t, k in zip(prev._forest.trees, prev._forest.tclass):
            drv.forest.add(t, k)
        drv.init_f = list(prev._init_f)
        X = self._score_matrix(drv.spec.frame)
        drv.f = torch.tensor(drv.init_f, dtype=torch.float32, device=drv.dev).view(1, -1).repeat(X.shape[1], 1)
        drv.f += drv.forest.predict(X, drv.K)
        drv.iter = len(drv.forest) // drv.K

    def _predict_link(self, frame, ntrees=None):
        X = self._score_matrix(frame)
        K = self._K
        upto = None if ntrees is None else ntrees * K
        f = self._forest.predict(X, K, upto=upto)
        f = f + torch.tensor(self._init_f, dtype=torch.float32, device=f.device).view(1, -1)
        off = self._spec.offset_column
        if off and off in frame.names:
            f = f + torch.nan_to_num(frame.vec(off).as_float()).view(-1, 1)
        return f

    def _predict_raw(self, frame):
        f = self._predict_link(frame)
        if self._K > 1:
            return torch.softmax(f, 1)
        mu = self._dist.linkinv(f[:, 0])
        if self._spec.nclasses == 2:
            return torch.stack([1 - mu, mu], 1)
        return mu.view(-1, 1)

    def staged_predict_proba(self, test_data):
        out = []
        K = self._K
        for t in range(1, len(self._forest) // K + 1):
            f = self._predict_link(test_data, ntrees=t)
            if K > 1:
                pr = torch.softmax(f, 1)
            else:
                pr = self._dist.linkinv(f[:, 0]).view(-1, 1)
            out.append(pr)
        from ...core.vec import Vec, T_REAL
        vecs, names = [], []
        for t, pr in enumerate(out):
            for k in range(pr.shape[1]):
                vecs.append(Vec(pr[:, k].contiguous(), T_REAL))
                names.append(f"T{t + 1}.C{k + 1}")
        return H2OFrame.from_vecs(vecs, names)

    def predict_contributions(self, test_data, output_format="Original", top_n=None, bottom_n=None,
                              compare_abs=False, background_frame=None):
        from .shap import tree_contributions
        return tree_contributions(self, test_data, top_n=top_n, bottom_n=bottom_n, compare_abs=compare_abs)


def _weighted_quantile(x, w, q):
    if x.numel() == 0:
        return 0.0
    if cloud.is_distributed():
        x = coll.all_gather_var(x)
        w = coll.all_gather_var(w)
    o = torch.argsort(x)
    xs, ws = x[o].to(torch.float64), w[o].to(torch.float64)
    cw = torch.cumsum(ws, 0)
    t = q * float(cw[-1])
    i = int(torch.searchsorted(cw, torch.tensor([t], dtype=cw.dtype, device=cw.device)).clamp(max=xs.numel() - 1))
    return float(xs[i])


def _segmented_wquantile(idx, x, w, L, q):
    """Weighted q-quantile of x within each segment id (host loop over leaves
    after one device sort by (segment, value))."""
    if cloud.is_distributed():
        idx = coll.all_gather_var(idx)
        x = coll.all_gather_var(x)
        w = coll.all_gather_var(w)
    m = w > 0
    idx, x, w = idx[m], x[m], w[m]
    key = idx.to(torch.float64) * 0 + x
    o = torch.argsort(x)
    idx, x, w = idx[o], x[o], w[o]
    o2 = torch.argsort(idx, stable=True)
    idx, x, w = idx[o2], x[o2], w[o2]
    out = np.zeros(L)
    counts = torch.bincount(idx, minlength=L).cpu().numpy()
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    xh, wh = x.cpu().numpy(), w.cpu().numpy()
    for l in range(L):
        s, c = starts[l], counts[l]
        if c == 0:
            continue
        cw = np.cumsum(wh[s:s + c])
        j = int(np.searchsorted(cw, q * cw[-1]))
        out[l] = xh[s + min(j, c - 1)]
    return out
