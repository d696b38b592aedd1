"""XGBoost legacy binary booster ("boosterBytes" inside the reference's
XGBoost MOJO) -- reader, writer and a vectorized numpy scorer.

The reference's XGBoost MOJO (h2o-genmodel-extensions/xgboost,
XGBoostMojoReader.java:36 readblob("boosterBytes"), XGBoostJavaMojoModel.java:48
makePredictor) carries the native XGBoost model in XGBoost's legacy binary
serialization, scored in Java by the xgboost-predictor library.  The layout
(all little endian):

  LearnerModelParam   base_score f32, num_feature u32, num_class i32,
                      contain_extra_attrs i32, contain_eval_metrics i32,
                      major_version u32, minor_version u32, reserved i32[27]
                      (136 bytes; an optional "binf" signature precedes it)
  name_obj, name_gbm  u64 length + bytes ("binary:logistic", "gbtree", ...)
  GBTreeModelParam    num_trees i32, num_roots i32, num_feature i32, pad i32,
                      num_pbuffer i64, num_output_group i32,
                      size_leaf_vector i32, reserved i32[32]   (160 bytes)
  per tree            TreeParam (num_roots, num_nodes, num_deleted, max_depth,
                      num_feature, size_leaf_vector, reserved[31]; 148 bytes),
                      num_nodes x Node (parent i32 | left-child bit 31,
                      cleft i32, cright i32, sindex u32 = feature | default-left
                      bit 31, f32 split_cond / leaf_value), num_nodes x
                      NodeStat (loss_chg f32, sum_hess f32, base_weight f32,
                      leaf_child_cnt i32)
  tree_info           i32[num_trees] (output group of each tree)
  dart only           u64 n + f32[n] weight_drop

Since XGBoost 1.0 base_score is stored as a probability and turned into a
margin by the objective's ProbToMargin on load (earlier versions stored the
margin); scoring: fvalue < split_cond -> left, NaN -> default direction.
"""
from __future__ import annotations

import struct

import numpy as np

_LEARNER_FMT = "<fIiiiII27i"
_GBT_FMT = "<iiiiqii32i"
_TREE_FMT = "<iiiiii31i"
_NODE_DT = np.dtype([("parent", "<i4"), ("cleft", "<i4"), ("cright", "<i4"), ("sindex", "<u4"), ("info", "<f4")])
_STAT_DT = np.dtype([("loss_chg", "<f4"), ("sum_hess", "<f4"), ("base_weight", "<f4"), ("leaf_child_cnt", "<i4")])

# objective -> (margin -> output transform, probability -> margin)
_LOG_OBJ = ("count:poisson", "reg:gamma", "reg:tweedie")


def prob_to_margin(obj: str, p: float) -> float:
    if obj == "binary:logistic":
        return float(-np.log(1.0 / p - 1.0))
    if obj in _LOG_OBJ:
        return float(np.log(p))
    return float(p)


def margin_to_prob(obj: str, m: float) -> float:
    if obj == "binary:logistic":
        return float(1.0 / (1.0 + np.exp(-m)))
    if obj in _LOG_OBJ:
        return float(np.exp(m))
    return float(m)


class Booster:
    """Parsed gbtree / dart booster."""

    def __init__(self):
        self.base_score = 0.5          # as stored
        self.num_feature = 0
        self.num_class = 0
        self.major_version = 0
        self.minor_version = 0
        self.name_obj = "reg:squarederror"
        self.name_gbm = "gbtree"
        self.num_output_group = 1
        self.trees = []                # (nodes structured array, stats structured array)
        self.tree_info = []
        self.weight_drop = None

    @property
    def base_margin(self) -> float:
        if self.major_version >= 1:
            return prob_to_margin(self.name_obj, self.base_score)
        return float(self.base_score)

    # ------------------------------------------------------------- parse
    @classmethod
    def parse(cls, buf: bytes) -> "Booster":
        b = cls()
        p = 0
        if buf[:4] == b"binf":
            p = 4
        lp = struct.unpack_from(_LEARNER_FMT, buf, p)
        p += struct.calcsize(_LEARNER_FMT)
        b.base_score, b.num_feature, b.num_class = lp[0], lp[1], lp[2]
        b.major_version, b.minor_version = lp[5], lp[6]

        def string(p):
            n = struct.unpack_from("<Q", buf, p)[0]
            return buf[p + 8:p + 8 + n].decode("utf-8"), p + 8 + n
        b.name_obj, p = string(p)
        b.name_gbm, p = string(p)
        if b.name_gbm not in ("gbtree", "dart"):
            raise NotImplementedError(f"XGBoost booster '{b.name_gbm}' is not supported (tree boosters only)")
        gp = struct.unpack_from(_GBT_FMT, buf, p)
        p += struct.calcsize(_GBT_FMT)
        num_trees, num_pbuffer, b.num_output_group, leaf_vec = gp[0], gp[4], gp[5], gp[6]
        if leaf_vec != 0:
            raise NotImplementedError("XGBoost trees with leaf vectors are not supported")
        for _ in range(num_trees):
            tp = struct.unpack_from(_TREE_FMT, buf, p)
            p += struct.calcsize(_TREE_FMT)
            nn = tp[1]
            nodes = np.frombuffer(buf, dtype=_NODE_DT, count=nn, offset=p).copy()
            p += nn * _NODE_DT.itemsize
            stats = np.frombuffer(buf, dtype=_STAT_DT, count=nn, offset=p).copy()
            p += nn * _STAT_DT.itemsize
            b.trees.append((nodes, stats))
        b.tree_info = list(np.frombuffer(buf, dtype="<i4", count=num_trees, offset=p)) if num_trees else []
        p += 4 * num_trees
        if num_pbuffer != 0:
            # deprecated prediction buffer (very old models): two f32 blocks
            p += 2 * 4 * num_pbuffer * b.num_output_group
        if b.name_gbm == "dart" and num_trees:
            n = struct.unpack_from("<Q", buf, p)[0]
            b.weight_drop = np.frombuffer(buf, dtype="<f4", count=n, offset=p + 8).astype(np.float64)
        return b

    # ------------------------------------------------------------- write
    def to_bytes(self) -> bytes:
        out = bytearray()
        out += struct.pack(_LEARNER_FMT, float(self.base_score), int(self.num_feature), int(self.num_class),
                           0, 0, int(self.major_version), int(self.minor_version), *([0] * 27))
        for s in (self.name_obj, self.name_gbm):
            e = s.encode("utf-8")
            out += struct.pack("<Q", len(e)) + e
        out += struct.pack(_GBT_FMT, len(self.trees), 1, int(self.num_feature), 0, 0,
                           int(self.num_output_group), 0, *([0] * 32))
        for nodes, stats in self.trees:
            out += struct.pack(_TREE_FMT, 1, len(nodes), 0, 0, int(self.num_feature), 0, *([0] * 31))
            out += nodes.astype(_NODE_DT).tobytes()
            out += stats.astype(_STAT_DT).tobytes()
        out += np.asarray(self.tree_info, dtype="<i4").tobytes()
        if self.name_gbm == "dart" and self.trees:
            wd = np.ones(len(self.trees)) if self.weight_drop is None else np.asarray(self.weight_drop)
            out += struct.pack("<Q", len(wd)) + wd.astype("<f4").tobytes()
        return bytes(out)

    # ------------------------------------------------------------- score
    @staticmethod
    def tree_leaves(nodes, F: np.ndarray) -> np.ndarray:
        """Leaf node index per row of the f32 feature matrix F."""
        n = F.shape[0]
        cur = np.zeros(n, dtype=np.int64)
        cleft = nodes["cleft"].astype(np.int64)
        cright = nodes["cright"].astype(np.int64)
        feat = (nodes["sindex"] & 0x7FFFFFFF).astype(np.int64)
        dleft = (nodes["sindex"] >> 31).astype(bool)
        cond = nodes["info"].astype(np.float32)
        rows = np.arange(n)
        active = cleft[cur] != -1
        while active.any():
            r = rows[active]
            c = cur[r]
            v = F[r, feat[c]]
            go_left = np.where(np.isnan(v), dleft[c], v < cond[c])
            cur[r] = np.where(go_left, cleft[c], cright[c])
            active[r] = cleft[cur[r]] != -1
        return cur

    def _native_acc(self, F, K):
        """f32 tree sums from the native walk (native/mojo_forest.cpp
        h2o_xgb_forest_score: the numpy loop's f32 adds in the same order),
        or None without the library."""
        from .h2o_mojo import _forest_lib
        lib = _forest_lib()
        if lib is None or F.shape[0] < 64 or not self.trees:
            return None
        import ctypes
        if not getattr(lib, "_typed_xgb", False):
            cv = ctypes.c_void_p
            lib.h2o_xgb_forest_score.argtypes = [ctypes.c_longlong, ctypes.c_int, cv, ctypes.c_int] + [cv] * 8 + \
                [ctypes.c_int, cv, ctypes.c_int]
            lib._typed_xgb = True
        pk = self.__dict__.get("_xpack")
        if pk is None:
            nodes = [nd for nd, _ in self.trees]
            sizes = [len(nd) for nd in nodes]
            cat = np.concatenate(nodes) if nodes else np.zeros(0, dtype=_NODE_DT)
            pk = self._xpack = {
                "off": np.ascontiguousarray(np.concatenate([[0], np.cumsum(sizes)]), dtype=np.int64),
                "cleft": np.ascontiguousarray(cat["cleft"], dtype=np.int32),
                "cright": np.ascontiguousarray(cat["cright"], dtype=np.int32),
                "feat": np.ascontiguousarray(cat["sindex"] & 0x7FFFFFFF, dtype=np.int32),
                "dleft": np.ascontiguousarray(cat["sindex"] >> 31, dtype=np.uint8),
                "info": np.ascontiguousarray(cat["info"], dtype=np.float32),
                "group": np.ascontiguousarray(self.tree_info[:len(nodes)], dtype=np.int32),
                "wdrop": None if self.weight_drop is None else
                np.ascontiguousarray(self.weight_drop[:len(nodes)], dtype=np.float32),
            }
        Fc = np.ascontiguousarray(F, dtype=np.float32)
        acc = np.zeros((F.shape[0], K), dtype=np.float32)
        P = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        rc = lib.h2o_xgb_forest_score(Fc.shape[0], Fc.shape[1], P(Fc), len(self.trees), P(pk["off"]), P(pk["cleft"]),
                                      P(pk["cright"]), P(pk["feat"]), P(pk["dleft"]), P(pk["info"]), P(pk["group"]),
                                      P(pk["wdrop"]), K, P(acc), 0)
        if rc != 0:
            raise RuntimeError(f"h2o_xgb_forest_score failed: {rc}")
        return acc

    def margins(self, F: np.ndarray) -> np.ndarray:
        """[n, num_output_group] raw margins (base margin + tree sums)."""
        F = np.asarray(F, dtype=np.float32)
        K = max(1, int(self.num_output_group))
        out = np.full((F.shape[0], K), self.base_margin, dtype=np.float64)
        nacc = self._native_acc(F, K)
        if nacc is not None:
            return out + nacc
        acc = np.zeros((F.shape[0], K), dtype=np.float32)
        for t, (nodes, _) in enumerate(self.trees):
            leaf = self.tree_leaves(nodes, F)
            v = nodes["info"][leaf].astype(np.float32)
            if self.weight_drop is not None:
                v = (v * np.float32(self.weight_drop[t])).astype(np.float32)
            acc[:, int(self.tree_info[t])] += v
        return out + acc

    def predict(self, F: np.ndarray) -> np.ndarray:
        m = self.margins(F)
        if self.name_obj == "binary:logistic":
            return 1.0 / (1.0 + np.exp(-m))
        if self.name_obj in ("multi:softprob", "multi:softmax"):
            z = np.exp(m - m.max(1, keepdims=True))
            return z / z.sum(1, keepdims=True)
        if self.name_obj in _LOG_OBJ:
            return np.exp(m)
        return m


def nodes_from_lists(parent, cleft, cright, feat, default_left, info):
    nodes = np.zeros(len(cleft), dtype=_NODE_DT)
    nodes["parent"] = np.asarray(parent, dtype=np.int64).astype(np.uint32).view(np.int32) \
        if len(parent) else np.zeros(0, np.int32)
    nodes["cleft"] = cleft
    nodes["cright"] = cright
    nodes["sindex"] = (np.asarray(feat, dtype=np.uint64) | (np.asarray(default_left, dtype=np.uint64) << 31)) \
        .astype(np.uint32)
    nodes["info"] = np.asarray(info, dtype=np.float32)
    return nodes


def stats_from_lists(loss_chg, sum_hess, base_weight):
    st = np.zeros(len(sum_hess), dtype=_STAT_DT)
    st["loss_chg"] = loss_chg
    st["sum_hess"] = sum_hess
    st["base_weight"] = base_weight
    return st
