"""Shared tree model machinery: feature prep, binning, forest packing and
GPU scoring, variable importance, leaf-node assignment.

Reference: hex/tree/SharedTree.java (driver skeleton),
hex/tree/SharedTreeModel.java (score0, varimp, predictLeafNodeAssignment),
hex/tree/CompressedForest.java.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import pandas as pd
import torch

from ...core.frame import H2OFrame
from ...core.vec import T_ENUM, T_INT, T_REAL, Vec
from ...ops import _native
from ...parallel import cloud
from ..base import H2OEstimator
from .binning import bin_frame_tensors
from .engine import Tree

_c_void = ctypes.c_void_p


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def iter_seed(seed, it, salt=0):
    """Seed of boosting / forest iteration `it`: every tree's randomness
    (row sample, per-tree and per-node column samples) is a function of
    (seed, iteration) only, so a build continued from a checkpoint draws
    exactly what an uninterrupted build draws for the same trees
    (SharedTree.java:144 checkpoint restart)."""
    return (int(seed) * 1000003 + int(it) * 7919 + int(salt) * 104729 + 12345) & 0x7FFFFFFF


def reseed_iteration(drv, seed, it):
    """Re-seed a driver's generators for iteration `it` (row sampling:
    rank-dependent torch generator; host column sampling: rank-independent)."""
    from ...parallel import cloud
    drv.gen.manual_seed(iter_seed(seed, it, 1) + cloud.rank())
    drv.rng = np.random.RandomState(iter_seed(seed, it, 2))
    drv.grower.rng = np.random.RandomState(iter_seed(seed, it, 3))


def checkpoint_model(ck, algo, est):
    """The checkpoint model a build continues (hex/ModelBuilder checkpoint
    checks: same algorithm, same response, the new ntrees must exceed the
    checkpoint's)."""
    from ...core import dkv
    prev = dkv.get(ck) if isinstance(ck, str) else ck
    if prev is None:
        raise ValueError(f"checkpoint: model {ck} not found")
    if getattr(prev, "algo", None) != algo:
        raise ValueError(f"checkpoint: model {getattr(prev, 'model_id', ck)} is a {getattr(prev, 'algo', '?')} "
                         f"model, not {algo}")
    done = len(prev._forest) // max(1, prev._n_tree_classes())
    if int(est._parms["ntrees"]) <= done:
        raise ValueError(f"checkpoint: ntrees ({est._parms['ntrees']}) must be larger than the checkpoint "
                         f"model's number of trees ({done})")
    return prev, done


def forest_varimp(forest, names):
    """Sum of positive split gains per feature over every split node
    (vectorized over each tree's node arrays)."""
    acc = np.zeros(len(names), dtype=np.float64)
    for t in forest.trees:
        l_ = np.asarray(t.left, dtype=np.int64)
        if l_.size == 0:
            continue
        sp = l_ >= 0
        f_ = np.asarray(t.feat, dtype=np.int64)[sp]
        g_ = np.maximum(np.asarray(t.gain, dtype=np.float64)[sp], 0.0)
        np.add.at(acc, f_, g_)
    return {n: float(acc[j]) for j, n in enumerate(names)}


class Forest:
    """Flattened struct-of-arrays forest for the scoring kernel."""

    def __init__(self):
        self.trees: list[Tree] = []
        self.tclass: list[int] = []
        self._packed = None

    def add(self, tree: Tree, k: int = 0):
        self.trees.append(tree)
        self.tclass.append(k)
        self._packed = None

    def __len__(self):
        return len(self.trees)

    def pack(self, device, upto=None):
        trees = self.trees if upto is None else self.trees[:upto]
        key = (str(device), len(trees))
        if self._packed is not None and self._packed[0] == key:
            return self._packed[1]
        # vectorized per tree (trees of deep DRF models have ~10^5 nodes; a
        # per-node Python loop here cost seconds per scoring)
        feat, thr, left, right, nal, coff, clen, val, roots, bits = [], [], [], [], [], [], [], [], [], []
        base = 0
        nb = 0
        for t in trees:
            n = t.n_nodes
            roots.append(base)
            f_ = np.asarray(t.feat, dtype=np.int64)
            th = np.asarray(t.thr, dtype=np.float64)
            l_ = np.asarray(t.left, dtype=np.int64)
            r_ = np.asarray(t.right, dtype=np.int64)
            feat.append(np.maximum(f_, 0))
            thr.append(np.where(np.isnan(th), 0.0, th))
            left.append(np.where(l_ >= 0, l_ + base, -1))
            right.append(np.where(r_ >= 0, r_ + base, -1))
            nal.append(np.asarray(t.na_left, dtype=bool).astype(np.uint8))
            co = np.full(n, -1, dtype=np.int64)
            cl = np.zeros(n, dtype=np.int64)
            for i in np.nonzero(np.asarray(t.is_cat, dtype=bool))[0]:
                m = t.cat_left[i]
                if m is None:
                    continue
                mb = np.asarray(m).astype(np.uint8).reshape(-1)
                co[i] = nb
                cl[i] = mb.size
                bits.append(mb)
                nb += mb.size
            coff.append(co)
            clen.append(cl)
            val.append(np.asarray(t.value, dtype=np.float64))
            base += n

        def cat(parts, dt):
            return np.concatenate(parts).astype(dt) if parts else np.zeros(0, dtype=dt)
        d = device
        # packed 16-byte nodes for the HIP kernel: feature | NA-left << 30 |
        # categorical << 31, threshold bits, left, right
        f32 = cat(thr, np.float32)
        cof = cat(coff, np.int32)
        node = np.stack([(cat(feat, np.int64) & 0x3FFFFFFF) | (cat(nal, np.int64) << 30) |
                         ((cof >= 0).astype(np.int64) << 31),
                         f32.view(np.int32).astype(np.int64), cat(left, np.int64), cat(right, np.int64)], 1)
        node = node.astype(np.uint32).view(np.int32) if node.size else np.zeros((0, 4), dtype=np.int32)
        P = {"node": torch.as_tensor(np.ascontiguousarray(node), device=d),
             "feat": torch.as_tensor(cat(feat, np.int32), device=d),
             "thr": torch.as_tensor(cat(thr, np.float32), device=d),
             "left": torch.as_tensor(cat(left, np.int32), device=d),
             "right": torch.as_tensor(cat(right, np.int32), device=d),
             "na_left": torch.as_tensor(cat(nal, np.uint8), device=d),
             "cat_off": torch.as_tensor(cat(coff, np.int32), device=d),
             "cat_len": torch.as_tensor(cat(clen, np.int32), device=d),
             "cat_bits": torch.as_tensor(cat(bits, np.uint8) if bits else np.zeros(1, dtype=np.uint8), device=d),
             "value": torch.as_tensor(cat(val, np.float32), device=d),
             "roots": torch.tensor(roots, dtype=torch.int32, device=d),
             "tclass": torch.tensor(self.tclass[: len(trees)], dtype=torch.int32, device=d),
             "T": len(trees)}
        self._packed = (key, P)
        return P

    def predict_range(self, X: torch.Tensor, K: int, start: int, end: int):
        """[N, K] sums of trees [start, end) only (incremental scoring: the
        pack covers just these trees)."""
        sub = Forest()
        sub.trees = self.trees[start:end]
        sub.tclass = self.tclass[start:end]
        return sub.predict(X, K)

    def predict(self, X: torch.Tensor, K: int, upto=None, leaf=False):
        """X: [F, N] float32 column-major.  Returns [N, K] sums (or leaf ids)."""
        N = X.shape[1]
        P = self.pack(X.device, upto)
        T = P["T"]
        out = torch.zeros((N, K), dtype=torch.float32, device=X.device)
        leaf_out = torch.empty((N, T), dtype=torch.int32, device=X.device) if leaf else None
        if T == 0:
            return leaf_out if leaf else out
        if X.device.type == "cuda":
            lib = _native.get_lib("tree_predict")
            if not getattr(lib, "_typed2", False):
                lib.h2o_forest_predict.argtypes = [_c_void, ctypes.c_longlong] + [_c_void] * 7 + \
                    [ctypes.c_int, ctypes.c_int, _c_void, _c_void, _c_void]
                lib._typed2 = True
            X = X.contiguous().to(torch.float32)
            rc = lib.h2o_forest_predict(_ptr(X), N, _ptr(P["node"]), _ptr(P["cat_off"]),
                                        _ptr(P["cat_len"]), _ptr(P["cat_bits"]), _ptr(P["value"]),
                                        _ptr(P["roots"]), _ptr(P["tclass"]), T, K,
                                        _ptr(out) if not leaf else ctypes.c_void_p(0),
                                        _ptr(leaf_out) if leaf else ctypes.c_void_p(0),
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            if rc != 0:
                raise RuntimeError(f"h2o_forest_predict failed: {rc}")
            return leaf_out if leaf else out
        return self._predict_torch(X, K, P, leaf)

    @staticmethod
    def _predict_torch(X, K, P, leaf=False):
        N = X.shape[1]
        T = P["T"]
        out = torch.zeros((N, K), dtype=torch.float32, device=X.device)
        leaf_out = torch.empty((N, T), dtype=torch.int32, device=X.device) if leaf else None
        ar = torch.arange(N, device=X.device)
        for t in range(T):
            nd = torch.full((N,), int(P["roots"][t]), dtype=torch.int64, device=X.device)
            while True:
                l = P["left"][nd].long()
                active = l >= 0
                if not bool(active.any()):
                    break
                f = P["feat"][nd].long()
                x = X[f, ar]
                isnan = torch.isnan(x)
                co = P["cat_off"][nd].long()
                cl = P["cat_len"][nd].long()
                code = torch.nan_to_num(x, nan=-1).long()
                in_rng = (code >= 0) & (code < cl)
                bit = P["cat_bits"][(co + code.clamp(min=0)).clamp(min=0, max=P["cat_bits"].numel() - 1)] != 0
                nal = P["na_left"][nd] != 0
                go_cat = torch.where(isnan | ~in_rng, nal, bit)
                go_num = torch.where(isnan, nal, x < P["thr"][nd])
                go = torch.where(co >= 0, go_cat, go_num)
                nxt = torch.where(go, l, P["right"][nd].long())
                nd = torch.where(active, nxt, nd)
            if leaf:
                leaf_out[:, t] = (nd - int(P["roots"][t])).to(torch.int32)
            else:
                out[ar, int(P["tclass"][t])] += P["value"][nd]
        return leaf_out if leaf else out


class SharedTreeEstimator(H2OEstimator):
    def _check_response(self, frame, y):
        """SharedTree.init: a constant response is an error unless
        check_constant_response is off; r2_stopping is deprecated there and
        ignored with a warning."""
        p = self._parms
        if y is not None and p.get("check_constant_response", True) and y in frame.names:
            v = frame.vec(y)
            if v.type == "enum":
                codes = v.data
                import torch as _t
                # level counts by bincount: an f64 index_add_ onto 2-3 slots
                # serialises on atomics (2.2 s at 10M rows)
                present = _t.bincount((codes.long() + 1).clamp_min(0),
                                      minlength=len(v.domain or []) + 1).to(_t.float64)
                from ...parallel import collectives as _coll
                _coll.allreduce_(present)
                if int((present[1:] > 0).sum()) < 2:
                    raise ValueError("ERRR on field: _response: Response cannot be constant.")
            elif v.is_const():
                raise ValueError("ERRR on field: _response: Response cannot be constant.")
        r2 = p.get("r2_stopping")
        if r2 is not None and float(r2) < 1.79e308:
            import warnings
            warnings.warn("r2_stopping is no longer supported and will be ignored if set - please use "
                          "stopping_rounds, stopping_metric and stopping_tolerance instead.")

    """Base of GBM / DRF / XGBoost / IsolationForest / UpliftDRF."""

    def _cv_optimal_params(self, cv_models):
        """Main model trains the mean number of trees the early-stopped CV models
        kept (ModelBuilder.cv_computeAndSetOptimalParameters / SharedTree)."""
        import math as _m
        if int(self._parms.get("stopping_rounds") or 0) > 0 and cv_models and \
                all(getattr(m, "_forest", None) is not None for m in cv_models):
            nt = [len(m._forest) // max(1, getattr(m, "_K", 1)) for m in cv_models]
            self._parms["ntrees"] = max(1, int(_m.ceil(sum(nt) / len(nt))))
            self._parms["stopping_rounds"] = 0

    def _feature_inputs(self, frame: H2OFrame, x):
        feats, is_cat, cards = [], [], []
        domains = {}
        for n in x:
            v = frame.vec(n)
            if v.type == T_ENUM:
                feats.append(v.data)
                is_cat.append(True)
                cards.append(len(v.domain))
                domains[n] = list(v.domain)
            else:
                feats.append(v.as_float(torch.float32) if v.data.dtype != torch.float64 else v.data.to(torch.float32))
                is_cat.append(False)
                cards.append(0)
        return feats, is_cat, cards, domains

    def _bin(self, spec, hist_type=None, nbins=None, want_col_major=True):
        p = self._parms
        feats, is_cat, cards, domains = self._feature_inputs(spec.frame, spec.x)
        self._x_domains = domains
        self._x_is_cat = is_cat
        bd = bin_frame_tensors(feats, is_cat, cards, spec.x,
                               hist_type=hist_type or p.get("histogram_type", "AUTO"),
                               nbins=nbins or p.get("nbins", 20), nbins_top_level=p.get("nbins_top_level", 1024),
                               nbins_cats=p.get("nbins_cats", 1024),
                               seed=(p.get("seed") if p.get("seed") not in (None, -1) else 1234),
                               want_col_major=want_col_major)
        return bd

    def _score_matrix(self, frame: H2OFrame) -> torch.Tensor:
        """[F, N] float32 column-major scoring matrix adapted to training."""
        x = self._spec.x
        cols = []
        for n in x:
            if n not in frame.names:
                cols.append(torch.full((frame.nlocal,), float("nan"), device=cloud.device()))
                continue
            v = frame.vec(n)
            if n in self._x_domains:
                codes = self._adapt_enum(v, self._x_domains[n])
                c = codes.to(torch.float32)
                cols.append(torch.where(codes < 0, torch.full_like(c, float("nan")), c))
            else:
                cols.append(v.as_float(torch.float32) if not v.on_host else
                            torch.full((frame.nlocal,), float("nan"), device=cloud.device()))
        if not cols:
            return torch.zeros((0, frame.nlocal), device=cloud.device())
        return torch.stack(cols, 0).contiguous()

    def _varimp_from_forest(self, forest: Forest, names):
        return forest_varimp(forest, names)

    def predict_leaf_node_assignment(self, test_data, type="Path"):
        X = self._score_matrix(test_data)
        K = self._n_tree_classes()
        leaf = self._forest.predict(X, K, leaf=True)
        names = []
        ntrees_iter = len(self._forest) // max(K, 1)
        for t in range(len(self._forest)):
            k = self._forest.tclass[t]
            it = t // max(K, 1)
            cls = "" if K == 1 else f".C{k + 1}"
            names.append(f"T{it + 1}{cls}")
        if type == "Node_ID":
            vecs = [Vec(leaf[:, t].to(torch.float32).contiguous(), T_INT) for t in range(leaf.shape[1])]
            return H2OFrame.from_vecs(vecs, names)
        # Path: string of L/R decisions
        paths = []
        lh = leaf.cpu().numpy()
        for t, tree in enumerate(self._forest.trees):
            pmap = _paths(tree)
            paths.append([pmap.get(int(n), "") for n in lh[:, t]])
        from ...core.vec import make_enum_from_strings
        vecs = [make_enum_from_strings(p) for p in paths]
        return H2OFrame.from_vecs(vecs, names)

    def _n_tree_classes(self):
        return 1

    def staged_predict_proba(self, test_data):
        raise NotImplementedError

    @property
    def ntrees_built(self):
        return len(self._forest) // max(1, self._n_tree_classes())

    def ntrees_actual(self):
        """Trees actually built (early stopping may stop before ntrees)."""
        return self.ntrees_built

    def feature_interaction(self, max_interaction_depth=100, max_tree_depth=100, max_deepening=-1, path=None):
        """Feature interaction tables (hex/FeatureInteractions.java): one
        table per interaction depth, leaf statistics, split value histograms."""
        from .interactions import feature_interactions, interaction_tables
        K = self._n_tree_classes()
        fis = feature_interactions(self._forest, list(self._spec.x), len(self._forest) // max(K, 1), K,
                                   max_interaction_depth, max_tree_depth, max_deepening)
        tables = interaction_tables(fis)
        if path is not None:
            with pd.ExcelWriter(path) as xw:
                for i, t in enumerate(tables):
                    t.to_excel(xw, sheet_name=t.attrs.get("table_header", f"t{i}")[:31], index=False)
        return tables

    def feature_frequencies(self, test_data):
        """Per row: how often each feature is used on its decision paths,
        summed over the trees."""
        from .interactions import feature_frequencies
        X = self._score_matrix(test_data)
        leaf = self._forest.predict(X, self._n_tree_classes(), leaf=True)
        fq = feature_frequencies(self._forest, leaf, len(self._spec.x))
        return H2OFrame.from_vecs([Vec(fq[:, j].contiguous(), T_REAL) for j in range(fq.shape[1])],
                                  list(self._spec.x))

    def update_tree_weights(self, frame, weights_column):
        """Re-populate node covers from `frame` weighted by `weights_column`
        (SharedTreeModel.updateTreeWeights); TreeSHAP then explains that
        sub-population."""
        from .interactions import update_tree_weights
        X = self._score_matrix(frame)
        leaf = self._forest.predict(X, self._n_tree_classes(), leaf=True)
        update_tree_weights(self._forest, leaf, frame.vec(weights_column).as_float(torch.float64))

    def get_tree(self, tree_number=0, tree_class=None):
        K = self._n_tree_classes()
        idx = tree_number * K + (0 if tree_class is None else (tree_class if isinstance(tree_class, int) else
                                                               self._spec.response_domain.index(tree_class)))
        return self._forest.trees[idx]


def _paths(tree: Tree):
    out = {}
    stack = [(0, "")]
    while stack:
        i, p = stack.pop()
        if tree.left[i] < 0:
            out[i] = p
        else:
            stack.append((tree.left[i], p + "L"))
            stack.append((tree.right[i], p + "R"))
    return out
