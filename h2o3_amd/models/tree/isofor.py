"""Isolation Forest and Extended Isolation Forest.

Reference: hex/tree/isofor/IsolationForest.java (random column, random
split in [min,max] of the node, sample_size rows per tree, path length with
the c(n) adjustment, normalized score from training min/max mean length,
optional contamination threshold) and
hex/tree/isoforextended/ExtendedIsolationForest.java (random hyperplane
splits with `extension_level`, anomaly score 2^(-E[h]/c(psi))).

Trees are grown on a small row sample (default 256 rows) — that is host
work; scoring every row against the forest is the hot path and runs on the
GPU (forest traversal kernel for IF; batched hyperplane traversal for EIF).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ...core.frame import H2OFrame
from ...core.vec import T_ENUM, T_REAL, Vec
from ...parallel import cloud
from ...parallel import collectives as coll
from .. import metrics as mm
from ..base import H2OEstimator
from .engine import Tree
from .shared import Forest, SharedTreeEstimator


def c_factor(n):
    """Average path length of an unsuccessful BST search (Liu et al.)."""
    if n <= 1:
        return 0.0
    if n == 2:
        return 1.0
    return 2.0 * (math.log(n - 1) + 0.5772156649) - 2.0 * (n - 1) / n


IF_DEFAULTS = dict(ntrees=50, max_depth=8, min_rows=1.0, max_runtime_secs=0.0, seed=-1, build_tree_one_node=False,
                   mtries=-1, sample_size=256, sample_rate=-1.0, col_sample_rate_change_per_level=1.0,
                   col_sample_rate_per_tree=1.0, categorical_encoding="auto", stopping_rounds=0,
                   stopping_metric="auto", stopping_tolerance=0.01, export_checkpoints_dir=None,
                   contamination=-1.0, validation_response_column=None, score_each_iteration=False,
                   score_tree_interval=0)


def _floyd_sample(n, k, rng):
    """k distinct sorted indices of range(n) in O(k) draws (Floyd's
    algorithm): RandomState.choice(replace=False) permutes all n rows per
    tree (7 ms per tree at 1M rows)."""
    chosen = set()
    for j in range(n - k, n):
        t = int(rng.randint(0, j + 1))
        chosen.add(j if t in chosen else t)
    return np.fromiter(sorted(chosen), dtype=np.int64, count=len(chosen))


def _sample_rows(X, n, k, rng):
    """Gather k random rows (global) of X [F, n_local] to the host."""
    if cloud.is_distributed():
        ntot = int(coll.allreduce_scalar(n))
    else:
        ntot = n
    idx = _floyd_sample(ntot, min(k, ntot), rng)
    if cloud.is_distributed():
        off = int(coll.all_gather_dim0(torch.tensor([n], device=X.device)).cumsum(0)[cloud.rank()].item()) - n
        loc = idx[(idx >= off) & (idx < off + n)] - off
        part = X[:, torch.as_tensor(loc, device=X.device)].T
        return coll.all_gather_var(part).cpu().numpy().astype(np.float64)
    return X[:, torch.as_tensor(idx, device=X.device)].T.cpu().numpy().astype(np.float64)


class H2OIsolationForestEstimator(SharedTreeEstimator):
    algo = "isolationforest"
    supervised_learning = False
    _defaults = IF_DEFAULTS

    def _n_tree_classes(self):
        return 1

    def _fit(self, spec):
        p = self._parms
        fr = spec.frame
        feats, is_cat, cards, domains = self._feature_inputs(fr, spec.x)
        self._x_domains = domains
        self._x_is_cat = is_cat
        X = self._score_matrix(fr)
        seed = p.get("seed", -1)
        rng = np.random.RandomState(1234 if seed in (None, -1) else int(seed) & 0x7FFFFFFF)
        n = fr.nlocal
        ntot = fr.nrows
        k = int(p.get("sample_size", 256))
        if float(p.get("sample_rate", -1)) > 0:
            k = max(2, int(float(p["sample_rate"]) * ntot))
        max_depth = int(p.get("max_depth", 8))
        if max_depth <= 0:
            max_depth = int(math.ceil(math.log2(max(k, 2))))
        forest = Forest()
        F = X.shape[0]
        for t in range(int(p["ntrees"])):
            S = _sample_rows(X, n, k, rng)
            cols = np.arange(F)
            r = float(p.get("col_sample_rate_per_tree", 1.0))
            if r < 1.0:
                cols = np.sort(rng.choice(F, size=max(1, int(round(r * F))), replace=False))
            forest.add(self._grow(S, cols, max_depth, float(p.get("min_rows", 1.0)), rng), 0)
        self._forest = forest
        ml = self._mean_length(X)
        self._min_len = coll.allreduce_scalar(float(ml.min()), "min")
        self._max_len = -coll.allreduce_scalar(-float(ml.max()), "min")
        self._output["model_summary"] = {"number_of_trees": len(forest), "sample_size": k, "max_depth": max_depth}
        cont = float(p.get("contamination", -1))
        self._threshold = None
        if cont > 0:
            sc = self._score_from_len(ml)
            self._threshold = float(torch.quantile(sc.to(torch.float64)[: 1 << 24], 1 - cont))
        vi = {nm: 0.0 for nm in spec.x}
        for tt in forest.trees:
            for i in range(tt.n_nodes):
                if tt.left[i] >= 0:
                    vi[spec.x[tt.feat[i]]] += 1.0
        self._output["variable_importances"] = vi

    @staticmethod
    def _grow(S, cols, max_depth, min_rows, rng):
        tree = Tree()
        root = tree.add_node(0, len(S))
        stack = [(root, np.arange(len(S)), 0)]
        while stack:
            nd, idx, d = stack.pop()
            rows = S[idx]
            if d >= max_depth or len(idx) <= max(1, min_rows):
                tree.value[nd] = d + c_factor(len(idx))
                continue
            cand = []
            for c in cols:
                v = rows[:, c]
                v = v[~np.isnan(v)]
                if v.size and v.min() < v.max():
                    cand.append((c, v.min(), v.max()))
            if not cand:
                tree.value[nd] = d + c_factor(len(idx))
                continue
            c, lo, hi = cand[rng.randint(len(cand))]
            thr = rng.uniform(lo, hi)
            x = rows[:, c]
            left = np.where(np.isnan(x), True, x < thr)
            if left.all() or (~left).all():
                tree.value[nd] = d + c_factor(len(idx))
                continue
            tree.feat[nd] = int(c)
            tree.thr[nd] = float(thr)
            tree.na_left[nd] = True
            l = tree.add_node(d + 1, int(left.sum()))
            r = tree.add_node(d + 1, int((~left).sum()))
            tree.left[nd], tree.right[nd] = l, r
            stack.append((l, idx[left], d + 1))
            stack.append((r, idx[~left], d + 1))
        return tree

    def _mean_length(self, X):
        s = self._forest.predict(X, 1)[:, 0]
        return s / max(1, len(self._forest))

    def _score_from_len(self, ml):
        rng = self._max_len - self._min_len
        return (self._max_len - ml) / rng if rng > 0 else torch.zeros_like(ml)

    def _predict_raw(self, frame):
        X = self._score_matrix(frame)
        ml = self._mean_length(X)
        return torch.stack([self._score_from_len(ml), ml], 1)

    def predict(self, test_data, **kw):
        raw = self._predict_raw(test_data)
        vecs = [Vec(raw[:, 0].contiguous(), T_REAL), Vec(raw[:, 1].contiguous(), T_REAL)]
        names = ["predict", "mean_length"]
        if self._threshold is not None:
            lab = (raw[:, 0] >= self._threshold).to(torch.int32)
            vecs = [Vec(lab, T_ENUM, ["0", "1"])] + [Vec(raw[:, 0].contiguous(), T_REAL), Vec(raw[:, 1].contiguous(), T_REAL)]
            names = ["predict", "score", "mean_length"]
        return H2OFrame.from_vecs(vecs, names)

    def _score_unsupervised(self, spec):
        raw = self._predict_raw(spec.frame)
        self._training_metrics = mm.ModelMetricsAnomaly(mean_score=float(raw[:, 0].mean()),
                                                        mean_normalized_score=float(raw[:, 0].mean()),
                                                        mean_length=float(raw[:, 1].mean()), nobs=spec.frame.nrows)
        vr = self._parms.get("validation_response_column")
        if spec.valid is not None and vr:
            vraw = self._predict_raw(spec.valid)
            y = spec.valid.vec(vr)
            yy = (y.data == (y.domain.index("1") if y.domain and "1" in y.domain else 1)).to(torch.float64) \
                if y.type == T_ENUM else y.as_float(torch.float64)
            self._validation_metrics = mm.binomial_metrics(yy, vraw[:, 0], None, ["0", "1"])

    def _unsupervised_perf(self, frame):
        raw = self._predict_raw(frame)
        return mm.ModelMetricsAnomaly(mean_score=float(raw[:, 0].mean()), mean_length=float(raw[:, 1].mean()),
                                      nobs=frame.nrows)


EIF_DEFAULTS = dict(ntrees=100, sample_size=256, extension_level=0, seed=-1, categorical_encoding="auto",
                    score_tree_interval=0, disable_training_metrics=True)


class H2OExtendedIsolationForestEstimator(H2OEstimator):
    algo = "extendedisolationforest"
    supervised_learning = False
    _defaults = EIF_DEFAULTS

    def _fit(self, spec):
        from ..datainfo import DataInfo
        p = self._parms
        self._dinfo = DataInfo(spec.frame, spec.x, standardize=False, use_all_factor_levels=True, pad_to=1)
        X, _ = self._dinfo.expand(spec.frame, pad=False)
        seed = p.get("seed", -1)
        rng = np.random.RandomState(4321 if seed in (None, -1) else int(seed) & 0x7FFFFFFF)
        n, P = X.shape
        k = min(int(p["sample_size"]), fr_n := spec.frame.nrows)
        ext = int(p.get("extension_level", 0))
        self._psi = k
        self._height = int(math.ceil(math.log2(max(k, 2))))
        trees = []
        Xt = X.T.contiguous()
        for t in range(int(p["ntrees"])):
            S = _sample_rows(Xt, n, k, rng)
            trees.append(self._grow(S, ext, rng))
        self._trees = trees
        self._pack(X.device)
        self._output["model_summary"] = {"number_of_trees": len(trees), "sample_size": k, "extension_level": ext}

    def _grow(self, S, ext, rng):
        P = S.shape[1]
        nodes = []  # (normal[P], point[P], left, right, value, rows)

        def build(idx, d):
            me = len(nodes)
            nodes.append(None)
            rows = S[idx]
            if d >= self._height or len(idx) <= 1:
                nodes[me] = (None, None, -1, -1, d + c_factor(len(idx)), len(idx))
                return me
            nvec = rng.normal(size=P)
            zero = rng.choice(P, size=max(0, P - ext - 1), replace=False)
            nvec[zero] = 0.0
            lo, hi = np.nanmin(rows, 0), np.nanmax(rows, 0)
            pt = rng.uniform(lo, hi)
            proj = (np.nan_to_num(rows) - pt) @ nvec
            left = proj <= 0
            if left.all() or (~left).all():
                nodes[me] = (None, None, -1, -1, d + c_factor(len(idx)), len(idx))
                return me
            l = build(idx[left], d + 1)
            r = build(idx[~left], d + 1)
            nodes[me] = (nvec, pt, l, r, 0.0, len(idx))
            return me
        build(np.arange(len(S)), 0)
        return nodes

    def _pack(self, dev):
        P = None
        normals, points, lefts, rights, vals, roots = [], [], [], [], [], []
        base = 0
        for tr in self._trees:
            roots.append(base)
            for nd in tr:
                if P is None and nd[0] is not None:
                    P = len(nd[0])
            base += len(tr)
        P = P or 1
        base = 0
        for ti, tr in enumerate(self._trees):
            for nd in tr:
                nv, pt, l, r, v = nd[:5]
                normals.append(nv if nv is not None else np.zeros(P))
                points.append(pt if pt is not None else np.zeros(P))
                lefts.append(l + base if l >= 0 else -1)
                rights.append(r + base if r >= 0 else -1)
                vals.append(v)
            base += len(tr)
        self._packed = {k: torch.tensor(np.asarray(v), device=dev) for k, v in
                        dict(normal=normals, point=points, left=lefts, right=rights, value=vals, roots=roots).items()}

    def _predict_raw(self, frame):
        X, _ = self._dinfo.expand(frame, pad=False)
        X = torch.nan_to_num(X.to(torch.float64))
        P = self._packed
        n = X.shape[0]
        tot = torch.zeros(n, dtype=torch.float64, device=X.device)
        for r in P["roots"].tolist():
            nd = torch.full((n,), r, dtype=torch.int64, device=X.device)
            for _ in range(self._height + 1):
                l = P["left"][nd]
                act = l >= 0
                if not bool(act.any()):
                    break
                proj = ((X - P["point"][nd]) * P["normal"][nd]).sum(1)
                nxt = torch.where(proj <= 0, l, P["right"][nd])
                nd = torch.where(act, nxt, nd)
            tot += P["value"][nd]
        ml = tot / len(self._trees)
        score = torch.pow(2.0, -ml / c_factor(self._psi))
        return torch.stack([score, ml], 1)

    def predict(self, test_data, **kw):
        raw = self._predict_raw(test_data)
        return H2OFrame.from_vecs([Vec(raw[:, 0].to(torch.float32).contiguous(), T_REAL),
                                   Vec(raw[:, 1].to(torch.float32).contiguous(), T_REAL)],
                                  ["anomaly_score", "mean_length"])

    def _score_unsupervised(self, spec):
        raw = self._predict_raw(spec.frame)
        self._training_metrics = mm.ModelMetricsAnomaly(mean_score=float(raw[:, 0].mean()),
                                                        mean_length=float(raw[:, 1].mean()), nobs=spec.frame.nrows)
