"""Generic model: an imported MOJO served inside the platform.

Reference: hex/generic/Generic.java, GenericModel.java (score / metrics /
contributions of a MOJO read by h2o-genmodel, GenericModel.java:449-498)
and hex/genmodel/attributes/ModelAttributes.java + ModelJsonReader.java (the
original model's metrics, variable importances, model summary and scoring
history from experimental/modelDetails.json).

MI355X design: a tree MOJO (GBM / DRF / XGBoost, either MOJO layout) is
converted once into the platform's Forest, so predict, metrics, leaf
assignment and TreeSHAP contributions run on the device like a native tree
model (forest kernel, torch TreeSHAP); other algorithms score through the
MOJO's vectorised numpy scorer on each rank's row shard.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_ENUM, T_INT, T_REAL, Vec
from ..parallel import cloud
from . import metrics as mm
from .base import H2OEstimator
from .tree.engine import Tree
from .tree.shared import Forest


class _MojoSpec:
    """What scoring and metrics need of a TrainSpec, from a MOJO's columns."""

    def __init__(self, x, y, domain):
        self.x = list(x)
        self.y = y
        self.response_domain = list(domain) if domain else None
        self.nclasses = len(domain) if domain else 1
        self.weights_column = self.offset_column = self.fold_column = None
        self.valid = None
        self.frame = None

    @property
    def is_classification(self):
        return self.nclasses > 1

    def y_tensor(self, frame, dtype=torch.float32):
        v = frame.vec(self.y)
        if self.response_domain:
            if v.type == T_ENUM:
                idx = {d: i for i, d in enumerate(self.response_domain)}
                remap = torch.tensor([idx.get(d, -1) for d in v.domain] or [-1], dtype=torch.int64,
                                     device=v.data.device)
                return torch.where(v.data < 0, v.data.to(torch.int64), remap[v.data.clamp(min=0).long()])
            x = v.as_float(torch.float64)
            return torch.where(torch.isnan(x), torch.full_like(x, -1), x).to(torch.int64)
        return v.as_float(dtype)

    def w_tensor(self, frame=None):
        return None

    def offset_tensor(self, frame=None):
        return None


# ------------------------------------------------------------------ MOJO trees -> Forest
def _tree_from_ref(t, aux, dom_len, version):
    """h2o_mojo._Tree (reference compressed tree + _aux.bin) -> engine Tree:
    numeric splits keep the f32 split point (x < split goes left), bitset
    splits become per-level left masks over the column's domain (levels
    outside the bitset follow the NA direction from MOJO version 1.1), NA vs
    rest splits a +inf threshold."""
    tr = Tree()
    if t.root_leaf is not None:
        tr.add_node(0, 1.0)
        tr.value[0] = float(t.root_leaf)
        return tr, np.zeros(1, dtype=np.int64)
    left, right, cover, value, feat = t.shap_graph(aux)
    nid = t._nid.copy()
    I = len(t.col)
    n = left.size
    depth = np.zeros(n, dtype=np.int64)
    for j in range(I):                         # parents precede children in decode order
        for c in (left[j], right[j]):
            depth[c] = depth[j] + 1
    tr.feat = [int(f) if j < I else -1 for j, f in enumerate(feat)]
    tr.left = left.tolist()
    tr.right = right.tolist()
    tr.value = value.tolist()
    tr.weight = (cover if aux else np.ones(n)).tolist()
    tr.gain = [0.0] * n
    tr.depth = depth.tolist()
    tr.split_code = [-1] * n
    thr, nal, isc, masks = [0.0] * n, [False] * n, [False] * n, [None] * n
    for j in range(I):
        nal[j] = bool(t.na_left[j])
        k = int(t.kind[j])
        if k == 0:
            thr[j] = float(t.split[j])
        elif k == 2:
            thr[j] = math.inf
        else:
            c = int(t.col[j])
            card = int(dom_len[c]) if dom_len is not None and dom_len[c] > 0 else int(t.bs_off[j] + t.bs_n[j])
            lv = np.arange(card)
            rel = lv - t.bs_off[j]
            inr = (rel >= 0) & (rel < t.bs_n[j])
            relc = np.clip(rel, 0, None)
            byte = t.raw[np.minimum(t.bs_pos[j] + (relc >> 3), t.raw.size - 1)]
            contains = ((byte >> (relc & 7)) & 1).astype(bool) & inr
            go_left = np.where(inr, ~contains, nal[j] if version >= 1.1 else True)
            isc[j] = True
            thr[j] = float("nan")
            masks[j] = go_left.astype(np.uint8)
    tr.thr, tr.na_left, tr.is_cat, tr.cat_left = thr, nal, isc, masks
    return tr, nid


def _trees_from_native(A):
    """Packed forest arrays of a native-layout MOJO -> engine Trees."""
    roots = A["forest_roots"].astype(np.int64)
    ends = np.append(roots[1:], A["forest_feat"].size)
    w = A.get("forest_weight")
    out = []
    for t in range(roots.size):
        a, b = int(roots[t]), int(ends[t])
        tr = Tree()
        n = b - a
        l_, r_ = A["forest_left"][a:b].astype(np.int64), A["forest_right"][a:b].astype(np.int64)
        tr.left = np.where(l_ >= 0, l_ - a, -1).tolist()
        tr.right = np.where(r_ >= 0, r_ - a, -1).tolist()
        tr.feat = np.where(l_ >= 0, A["forest_feat"][a:b], -1).astype(np.int64).tolist()
        tr.thr = A["forest_thr"][a:b].astype(np.float64).tolist()
        tr.na_left = (A["forest_na_left"][a:b] != 0).tolist()
        tr.value = A["forest_value"][a:b].astype(np.float64).tolist()
        tr.weight = (w[a:b] if w is not None else np.ones(n)).astype(np.float64).tolist()
        co, cl = A["forest_cat_off"][a:b], A["forest_cat_len"][a:b]
        tr.is_cat = (co >= 0).tolist()
        tr.cat_left = [A["forest_cat_bits"][int(o):int(o) + int(c)].astype(np.uint8) if o >= 0 else None
                       for o, c in zip(co, cl)]
        tr.gain = [0.0] * n
        tr.split_code = [-1] * n
        depth = np.zeros(n, dtype=np.int64)
        for j in range(n):
            if tr.left[j] >= 0:
                depth[tr.left[j]] = depth[tr.right[j]] = depth[j] + 1
        tr.depth = depth.tolist()
        out.append((tr, int(A["forest_tclass"][t])))
    return out


def _twodim_df(t):
    """TwoDimTableV3 JSON -> pandas (row headers dropped when empty)."""
    import pandas as pd
    if not t or "columns" not in t:
        return None
    names = [c["name"] for c in t["columns"]]
    data = t.get("data") or []
    cols = {n: list(data[i]) if i < len(data) else [] for i, n in enumerate(names)}
    df = pd.DataFrame(cols)
    if "" in df.columns and not any(v not in (None, "") for v in df[""]):
        df = df.drop(columns=[""])
    return df


def _metrics_from_json(d, category):
    """ModelMetrics* from a ModelMetrics*V3 JSON block (scalar fields, the
    threshold table and the confusion matrix) -- MojoModelMetrics*."""
    if not d:
        return None
    cls = {"Binomial": mm.ModelMetricsBinomial, "Multinomial": mm.ModelMetricsMultinomial,
           "Ordinal": mm.ModelMetricsOrdinal, "Regression": mm.ModelMetricsRegression,
           "Clustering": mm.ModelMetricsClustering, "AnomalyDetection": mm.ModelMetricsAnomaly,
           "CoxPH": mm.ModelMetricsCoxPH}.get(category, mm.ModelMetrics)
    kw = {k: v for k, v in d.items() if isinstance(v, (int, float, str, bool)) and not k.startswith("__")}
    tt = _twodim_df(d.get("thresholds_and_metric_scores"))
    if tt is not None and len(tt):
        kw["thresholds_and_metric_scores"] = {c: tt[c].tolist() for c in tt.columns}
    gl = _twodim_df(d.get("gains_lift_table"))
    if gl is not None and len(gl):
        kw["gains_lift_table"] = gl
    if d.get("domain") is not None:
        kw["domain"] = list(d["domain"])
    mx = _twodim_df(d.get("max_criteria_and_metric_scores"))
    if mx is not None and "metric" in mx.columns:
        for _, r in mx.iterrows():
            if r["metric"] == "max f1":
                kw["max_f1_threshold"] = float(r["threshold"])
    return cls(**kw)


class H2OGenericEstimator(H2OEstimator):
    algo = "generic"
    _defaults = dict(model_key=None, path=None)

    @classmethod
    def from_file(cls, file=None, model_id=None):
        est = cls(path=file, model_id=model_id)
        est._load(file)
        return est

    def _load(self, path):
        from ..mojo.genmodel import MojoModel
        self._mojo = MojoModel.load(path)
        m = self._mojo.meta
        self._x = list(m["x"])
        self._y = m.get("response")
        self._ncls = self._mojo.nclasses
        self.supervised_learning = self._y is not None
        self._spec = _MojoSpec(self._x, self._y, self._mojo.response_domain) if self._y else None
        self._forest = None
        self._build_forest()
        self._read_details()
        from ..core import dkv
        dkv.put(self.model_id, self)

    def train(self, x=None, y=None, training_frame=None, **kw):
        self._load(self._parms.get("path") or self._parms.get("model_key"))
        return self

    # ------------------------------------------------------------ device forest
    def _build_forest(self):
        mj = self._mojo
        algo = mj.algo
        if algo not in ("gbm", "drf", "xgboost"):
            return
        fo = Forest()
        self._x_domains = {}
        if hasattr(mj, "_arr"):                            # native layout
            A = mj._arr
            if "forest_feat" not in A:
                return
            for tr, k in _trees_from_native(A):
                fo.add(tr, k)
            self._x_domains = dict(mj.meta.get("x_domains") or {})
            self._K = int(mj.meta.get("K", 1))
            self._init_f = list(mj.meta.get("init_f", [0.0] * self._K))
            self._link = mj.meta.get("link", "identity")
            self._p0_trees = False
            self._binomial_single = bool(mj.meta.get("binomial_single", False))
        else:                                               # reference layout
            if algo == "xgboost":
                return
            dl = mj.dom_len if mj.version >= 1.2 else None
            self._nids = []
            K = mj.ntrees_per_group
            for g in range(mj.ntree_groups):
                for k in range(K):
                    t = mj.trees[k][g]
                    if t is None:
                        continue
                    name = "trees/t%02d_%03d_aux.bin" % (k, g)
                    aux = mj.be.read(name) if mj.be.exists(name) else b""
                    tr, nid = _tree_from_ref(t, aux, dl, mj.version)
                    fo.add(tr, k)
                    self._nids.append(nid)
            self._x_domains = {c: d for c, d in zip(mj.features, mj.domains[:len(mj.features)]) if d is not None}
            self._K = K
            self._init_f = [float(getattr(mj, "init_f", 0.0))] * K if algo == "gbm" else [0.0] * K
            self._link = getattr(mj, "link", "identity")
            self._p0_trees = algo == "drf" and mj.nclasses == 2 and not mj.binomial_double_trees
            self._binomial_single = self._p0_trees
        self._forest = fo

    def _score_matrix(self, frame):
        cols = []
        n = frame.nlocal
        for c in self._x:
            if c not in frame.names:
                cols.append(torch.full((n,), float("nan"), device=cloud.device()))
                continue
            v = frame.vec(c)
            if c in self._x_domains:
                codes = self._adapt_enum(v, self._x_domains[c])
                f = codes.to(torch.float32)
                cols.append(torch.where(codes < 0, torch.full_like(f, float("nan")), f))
            else:
                cols.append(v.as_float(torch.float32) if not v.on_host else
                            torch.full((n,), float("nan"), device=cloud.device()))
        return torch.stack(cols, 0).contiguous() if cols else torch.zeros((0, n), device=cloud.device())

    def _forest_raw(self, frame):
        X = self._score_matrix(frame)
        K = self._K
        s = self._forest.predict(X, K).to(torch.float64)
        algo = self._mojo.algo
        if algo in ("gbm", "xgboost"):
            f = s + torch.tensor(self._init_f, dtype=torch.float64, device=s.device).view(1, -1)
            if K > 1:
                return torch.softmax(f, 1)
            mu = torch.sigmoid(f[:, 0]) if self._link == "logit" else \
                (torch.exp(f[:, 0]) if self._link == "log" else f[:, 0])
            return torch.stack([1 - mu, mu], 1) if self._ncls == 2 else mu.view(-1, 1)
        ng = max(1, len(self._forest) // max(K, 1))
        a = s / ng
        if self._ncls == 2 and self._binomial_single:
            p1 = (1.0 - a[:, 0]) if self._p0_trees else a[:, 0].clamp(0, 1)
            return torch.stack([1 - p1, p1], 1)
        if self._ncls > 1:
            a = a.clamp(min=0)
            return a / a.sum(1, keepdim=True).clamp(min=1e-30)
        return a[:, :1]

    def _predict_raw(self, frame):
        if self._forest is not None:
            return self._forest_raw(frame)
        df = frame.as_data_frame(local=True)          # each rank scores its own row shard
        raw = self._mojo.predict_raw(df)
        return torch.as_tensor(np.asarray(raw, dtype=np.float64), device=cloud.device())

    def predict(self, test_data, **kw):
        if self._forest is not None and self._spec is not None:
            return self._pred_frame_from_raw(self._predict_raw(test_data), threshold=self._threshold())
        return H2OFrame(self._mojo.predict(test_data.as_data_frame(local=True)), _local=True)

    def _threshold(self):
        th = getattr(self._mojo, "default_threshold", None)
        if th is None:
            th = float(self._mojo.info.get("default_threshold", 0.5) or 0.5) if hasattr(self._mojo, "info") else 0.5
        return th

    def model_performance(self, test_data=None, train=False, valid=False, xval=False, **kw):
        if test_data is None:
            if valid:
                return self._validation_metrics
            if xval:
                return self._cross_validation_metrics
            return self._training_metrics
        spec = _MojoSpec(self._x, self._y, self._mojo.response_domain)
        return self._metrics_from_raw(spec, test_data, self._predict_raw(test_data))

    # ------------------------------------------------------------ tree extras
    def predict_contributions(self, test_data, output_format="Original", top_n=None, bottom_n=None,
                              compare_abs=False, **kw):
        """TreeSHAP of the imported trees on the device (GenericModel.java:449:
        the MOJO's contribution predictor), same output layout as the MOJO's."""
        if self._forest is None:
            raise ValueError(f"contributions are not available for a {self._mojo.algo} MOJO")
        if self._ncls > 2:
            raise ValueError("Calculating contributions is currently not supported for multinomial models.")
        from .tree.shap import forest_contributions
        X = self._score_matrix(test_data)
        F = len(self._x)
        trees = [t for t, k in zip(self._forest.trees, self._forest.tclass) if k == 0]
        algo = self._mojo.algo
        if algo in ("gbm", "xgboost"):
            phi = forest_contributions(trees, X, F)
            phi[:, -1] += float(self._init_f[0])
        else:
            phi = forest_contributions(trees, X, F, scale=1.0 / max(1, len(trees)))
            if self._ncls == 2 and self._binomial_single:
                r = 1.0 / (F + 1)
                phi = r - phi if self._p0_trees else phi + r
                if not self._p0_trees:
                    phi[:, -1] -= 1.0
        from ..mojo.treeshap_np import contributions_frame
        df = contributions_frame(phi.cpu().numpy(), self._x, top_n=top_n, bottom_n=bottom_n,
                                 compare_abs=compare_abs)
        return H2OFrame(df, _local=True)

    def predict_leaf_node_assignment(self, test_data, type="Path"):
        """Per tree: the leaf's decision path (L/R from the root) or, with
        type="Node_ID", the leaf's node id as the MOJO numbers it."""
        if self._forest is None:
            raise ValueError(f"{self._mojo.algo} MOJO has no trees")
        from ..core.vec import make_enum_from_strings
        from .tree.shared import _paths
        X = self._score_matrix(test_data)
        leaf = self._forest.predict(X, self._K, leaf=True).cpu().numpy()
        K = self._K
        names = [f"T{t // max(K, 1) + 1}" + ("" if K == 1 else f".C{self._forest.tclass[t] + 1}")
                 for t in range(len(self._forest))]
        if type == "Node_ID":
            nids = getattr(self, "_nids", None)
            vecs = []
            for t in range(leaf.shape[1]):
                ids = leaf[:, t] if nids is None else nids[t][leaf[:, t]]
                vecs.append(Vec(torch.as_tensor(ids.astype(np.int32), device=cloud.device()), T_INT))
            return H2OFrame.from_vecs(vecs, names)
        vecs = []
        for t, tree in enumerate(self._forest.trees):
            pm = _paths(tree)
            vecs.append(make_enum_from_strings([pm.get(int(i), "") for i in leaf[:, t]]))
        return H2OFrame.from_vecs(vecs, names)

    @property
    def ntrees(self):
        return len(self._forest) if self._forest is not None else 0

    # ------------------------------------------------------------ model details
    def _read_details(self):
        """Metrics / varimp / summary / scoring history of the ORIGINAL model,
        from the MOJO's experimental/modelDetails.json (ModelAttributes)."""
        d = getattr(self._mojo, "details", None)
        self._details = d
        self._training_metrics = self._validation_metrics = self._cross_validation_metrics = None
        self._varimp_df = None
        self._scoring_history = []
        if not d or not isinstance(d.get("output"), dict):
            return
        o = d["output"]
        cat = o.get("model_category") or (self._mojo.info.get("category") if hasattr(self._mojo, "info") else None)
        self._training_metrics = _metrics_from_json(o.get("training_metrics"), cat)
        self._validation_metrics = _metrics_from_json(o.get("validation_metrics"), cat)
        self._cross_validation_metrics = _metrics_from_json(o.get("cross_validation_metrics"), cat)
        self._varimp_df = _twodim_df(o.get("variable_importances"))
        ms = _twodim_df(o.get("model_summary"))
        if ms is not None:
            self._output["model_summary"] = ms
        sh = _twodim_df(o.get("scoring_history"))
        if sh is not None:
            self._scoring_history = sh
        self._output["original_algo"] = d.get("algo")
        self._output["original_model_id"] = (d.get("model_id") or {}).get("name") \
            if isinstance(d.get("model_id"), dict) else d.get("model_id")

    def varimp(self, use_pandas=False):
        df = getattr(self, "_varimp_df", None)
        if df is None:
            return None
        if use_pandas:
            return df
        return [tuple(r) for r in df.itertuples(index=False)]

    def scoring_history(self):
        import pandas as pd
        sh = getattr(self, "_scoring_history", None)
        return sh if isinstance(sh, pd.DataFrame) else pd.DataFrame(sh or [])
