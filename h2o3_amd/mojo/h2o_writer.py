"""MOJO export in the reference's h2o-genmodel layout.

`build_h2o_mojo(model)` writes GBM, DRF, XGBoost, GLM, K-Means, Isolation
Forest, Extended Isolation Forest, Deep Learning, Word2Vec, PCA and Stacked
Ensemble models as the reference's
MOJO zip -- model.ini ([info] / [columns] / [domains]), domains/dNNN.txt and,
for trees, the compressed tree byte streams trees/tCC_GGG.bin with their
_aux.bin node records -- so the reference's Java scorer (h2o-genmodel
MojoModel / EasyPredictModelWrapper) and any tool built on it can score
models trained here.  mojo/h2o_mojo.py reads the same layout back; the
round-trip tests score both ways.

Format parity (behaviour studied, not translated):
  hex/genmodel/AbstractMojoWriter.java:159   [info] keys written for every model
  hex/genmodel/algos/tree/SharedTreeMojoModel.java:129 + SharedTreeMojoReader.java
                                             tree byte layout read by scoreTree (mojo 1.40)
  hex/genmodel/algos/tree/SharedTreeMojoModel.java:704  AuxInfo records (40 bytes per split)
  hex/genmodel/algos/gbm/GbmMojoModel.java, drf/DrfMojoModel.java, glm/Glm*MojoModel.java
  hex/genmodel/algos/kmeans/KMeansMojoReader.java, isofor/IsolationForestMojoReader.java,
  isoforextended/ExtendedIsolationForestMojoReader.java, deeplearning/DeeplearningMojoReader.java,
  word2vec/Word2VecMojoReader.java, ensemble/StackedEnsembleMojoReader.java
  h2o-genmodel-extensions/xgboost: XGBoostMojoReader.java, OneHotEncoderFactory.java (one-hot feature
                                             space + native booster blob, mojo/xgb_booster.py)
"""
from __future__ import annotations

import io
import struct
import time
import zlib
import zipfile

import numpy as np

TREE_MOJO_VERSION = "1.40"
GLM_MOJO_VERSION = "1.00"
_NSD_NA_VS_REST, _NSD_NA_LEFT, _NSD_NA_RIGHT = 1, 2, 3


def _fmt(v):
    """Java-style stringification for the [info] section."""
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (list, tuple, np.ndarray)):
        return "[" + ", ".join(_fmt(x) for x in v) + "]"
    if isinstance(v, (float, np.floating)):
        f = float(v)
        if f != f:
            return "NaN"
        if f in (float("inf"), float("-inf")):
            return "Infinity" if f > 0 else "-Infinity"
        return repr(f)
    if isinstance(v, (np.integer,)):
        return str(int(v))
    return str(v)


class _Zip:
    def __init__(self):
        self.buf = io.BytesIO()
        self.z = zipfile.ZipFile(self.buf, "w", zipfile.ZIP_DEFLATED)

    def write(self, name, data):
        self.z.writestr(name, data)

    def nested(self, prefix):
        return _Prefixed(self, prefix)

    def close(self) -> bytes:
        self.z.close()
        return self.buf.getvalue()


class _Prefixed:
    """Writes into a parent zip under a directory prefix (Stacked Ensemble
    sub-models: models/<algo>/<key>/...)."""

    def __init__(self, z, prefix):
        self.z, self.prefix = z, prefix

    def write(self, name, data):
        self.z.write(self.prefix + name, data)

    def nested(self, prefix):
        return _Prefixed(self.z, self.prefix + prefix)


def _threshold(model):
    """The labelling threshold predict() uses: max-F1 of the validation (else
    training) metrics, 0.5 without metrics (base.py _pred_frame_from_raw)."""
    if hasattr(model, "_label_threshold"):
        return float(model._label_threshold())
    thr = 0.5
    for m in (getattr(model, "_training_metrics", None), getattr(model, "_validation_metrics", None)):
        if m is not None and m.get("max_f1_threshold") is not None:
            thr = float(m["max_f1_threshold"])
    return thr


def _header(model, algo_short, algo_full, category, columns, nfeatures, nclasses, domains, mojo_version, extra,
            supervised=True):
    info = {
        "h2o_version": "3.46.0.99999", "mojo_version": mojo_version, "license": "Apache License Version 2.0",
        "algo": algo_short, "algorithm": algo_full, "endianness": "LITTLE_ENDIAN", "category": category,
        "uuid": str(zlib.crc32(str(model.model_id).encode()) * 2654435761 % (1 << 62)), "supervised": supervised, "n_features": nfeatures,
        "n_classes": nclasses, "n_columns": len(columns), "n_domains": sum(d is not None for d in domains),
        "balance_classes": False, "default_threshold": _threshold(model),
        "prior_class_distrib": None, "model_class_distrib": None,
        "timestamp": time.strftime("%Y-%m-%dT%H:%M:%S.000+00:00", time.gmtime()), "escape_domain_values": True,
    }
    info.update(extra)
    lines = ["[info]"] + [f"{k} = {_fmt(v)}" for k, v in info.items()] + ["", "[columns]"] + list(columns) + \
        ["", "[domains]"]
    files = {}
    di = 0
    for ci, dom in enumerate(domains):
        if dom is None:
            continue
        fname = f"d{di:03d}.txt"
        lines.append(f"{ci}: {len(dom)} {fname}")
        files["domains/" + fname] = "\n".join(str(x).replace("\n", "\\n") for x in dom) + "\n"
        di += 1
    return "\n".join(lines) + "\n", files


# ------------------------------------------------------------------ trees
def _f32(v):
    return struct.pack("<f", float(np.float32(v)))


def _subtree_counts(left, right):
    """Split nodes under each node (itself included), bottom-up: children are
    always numbered after their parent (Tree.add_children appends)."""
    n = len(left)
    ns = np.zeros(n, dtype=np.int64)
    for i in range(n - 1, -1, -1):
        if left[i] >= 0:
            ns[i] = 1 + ns[left[i]] + ns[right[i]]
    return ns


def _encode_tree(tree, leaf_map=None):
    """Our Tree (x < thr goes left; cat_left = level mask going left) -> the
    reference's pre-order byte stream.  leaf_map(value) transforms leaf values
    (e.g. DRF binomial class-0 probabilities).  Subtree byte sizes are
    computed bottom-up, then the stream is written front to back with an
    explicit stack (deep DRF trees have 10^5-10^6 nodes)."""
    lm = leaf_map or (lambda v: v)
    left = np.asarray(tree.left, dtype=np.int64)
    right = np.asarray(tree.right, dtype=np.int64)
    if left[0] < 0:
        return b"\x00" + struct.pack("<H", 65535) + _f32(lm(tree.value[0]))
    n = len(left)
    thr = np.asarray(tree.thr, dtype=np.float64)
    feat = np.asarray(tree.feat, dtype=np.int64)
    if int(feat[left >= 0].max(initial=0)) >= 65535:
        raise ValueError("reference tree MOJOs address at most 65534 columns")
    heads = [None] * n            # node type byte + column + NA direction + split payload, per split node
    size = np.zeros(n, dtype=np.int64)
    for i in range(n - 1, -1, -1):
        l = left[i]
        if l < 0:
            continue
        r = right[i]
        node_type = 0
        if tree.is_cat[i]:
            mask = np.asarray(tree.cat_left[i]).astype(bool)
            rb = ~mask                            # bitset bit set -> go right
            nbits = len(rb)
            nsd = _NSD_NA_LEFT if tree.na_left[i] else _NSD_NA_RIGHT
            if nbits <= 32:
                node_type |= 8
                bits = np.zeros(32, dtype=bool)
                bits[:nbits] = rb
                split = np.packbits(bits, bitorder="little").tobytes()
            else:
                node_type |= 12
                split = struct.pack("<Hi", 0, nbits) + np.packbits(rb, bitorder="little").tobytes()
        elif not np.isfinite(thr[i]) and thr[i] > 0:
            nsd = _NSD_NA_VS_REST                 # every number left, NA right
            split = b""
        else:
            nsd = _NSD_NA_LEFT if tree.na_left[i] else _NSD_NA_RIGHT
            split = _f32(thr[i])
        sz = 4 + len(split)
        if left[l] < 0:
            node_type |= 48
            sz += 4
        else:
            sl = int(size[l])
            width = 1 if sl < (1 << 8) else 2 if sl < (1 << 16) else 3 if sl < (1 << 24) else 4
            node_type |= width - 1
            sz += width + sl
        if left[r] < 0:
            node_type |= 0xC0
            sz += 4
        else:
            sz += int(size[r])
        size[i] = sz
        heads[i] = bytes([node_type]) + struct.pack("<H", int(feat[i])) + bytes([nsd]) + split
    out = bytearray()
    stack = [("node", 0)]
    while stack:
        kind, i = stack.pop()
        if kind == "leaf":
            out += _f32(lm(tree.value[i]))
            continue
        l, r = int(left[i]), int(right[i])
        out += heads[i]
        if left[l] >= 0:
            sl = int(size[l])
            out += sl.to_bytes((heads[i][0] & 3) + 1, "little")
        # pre-order: left part, then right part (stack: push right first)
        stack.append(("leaf", r) if left[r] < 0 else ("node", r))
        stack.append(("leaf", l) if left[l] < 0 else ("node", l))
    return bytes(out)


_AUX = np.dtype([("nid", "<i4"), ("nsl", "<i4"), ("wl", "<f4"), ("wr", "<f4"), ("pl", "<f4"), ("pr", "<f4"),
                 ("sel", "<f4"), ("ser", "<f4"), ("l", "<i4"), ("r", "<i4")])


def _encode_aux(tree, leaf_map=None):
    """AuxInfo records (pre-order over split nodes): nid, #split nodes in the
    left subtree, child weights, child predictions, squared errors (0: not
    tracked), child node ids -- one structured array, written at once."""
    lm = leaf_map or (lambda v: v)
    left = np.asarray(tree.left, dtype=np.int64)
    right = np.asarray(tree.right, dtype=np.int64)
    if left[0] < 0:
        return b""
    ns = _subtree_counts(left, right)
    order = []
    stack = [0]
    while stack:
        i = stack.pop()
        if left[i] < 0:
            continue
        order.append(i)
        stack.append(int(right[i]))
        stack.append(int(left[i]))
    order = np.asarray(order, dtype=np.int64)
    l, r = left[order], right[order]
    w = np.asarray(tree.weight, dtype=np.float64)
    v = np.asarray(tree.value, dtype=np.float64)
    rec = np.zeros(order.size, dtype=_AUX)
    rec["nid"], rec["nsl"] = order, ns[l]
    rec["wl"], rec["wr"] = w[l], w[r]
    if leaf_map is None:
        rec["pl"], rec["pr"] = v[l], v[r]
    else:
        rec["pl"] = [lm(x) for x in v[l]]
        rec["pr"] = [lm(x) for x in v[r]]
    rec["l"], rec["r"] = l, r
    return rec.tobytes()


def _encoding_kv(model, supervised=True):
    """categorical_encoding of the model in the reference layout
    (SharedTreeMojoWriter / DeepLearningMojoWriter: _genmodel_encoding,
    _orig_names, _orig_domain_values_i, _orig_projection_array); returns
    (info keys, extra files)."""
    enc = getattr(model, "_catenc", None)
    if enc is None:
        return {"_genmodel_encoding": "AUTO"}, {}
    spec = model._spec
    names = list(enc.x_in) + ([spec.y] if supervised and spec.y else [])
    doms = [enc.cols[c]["domain"] if c in enc.cols else None for c in enc.x_in]
    if supervised and spec.y:
        doms.append(list(spec.response_domain) if spec.response_domain else None)
    info = {"_genmodel_encoding": enc.scheme, "_n_orig_names": len(names), "_n_orig_domain_values": len(doms)}
    esc = lambda v: "\n".join(str(x).replace("\n", "\\n") for x in v) + "\n"   # noqa: E731
    files = {"_orig_names": esc(names)}
    for i, d in enumerate(doms):
        info[f"_m_orig_domain_values_{i}"] = 0 if d is None else len(d)
        if d is not None:
            files[f"_orig_domain_values_{i}"] = esc(d)
    if enc.scheme == "Eigen":
        info["_orig_projection_array"] = [float(v) for c in enc.x_in if c in enc.cols
                                          for v in enc.cols[c]["proj"]]
    return info, files


def _tree_model(model, z, algo_short, algo_full, extra, leaf_maps, supervised=True, category=None):
    spec = model._spec
    x = list(spec.x)
    xd = getattr(model, "_x_domains", {}) or {}
    columns = x + ([spec.y] if supervised else [])
    domains = [xd.get(c) for c in x] + ([list(spec.response_domain) if spec.response_domain else None]
                                        if supervised else [])
    K = model._n_tree_classes()
    ng = len(model._forest) // max(K, 1)
    cat = category or ("Binomial" if spec.nclasses == 2 else "Multinomial" if spec.nclasses > 2 else "Regression")
    enc_info, enc_files = _encoding_kv(model, supervised)
    info = {"n_trees": ng, "n_trees_per_class": K, **enc_info}
    info.update(extra)
    ini, files = _header(model, algo_short, algo_full, cat, columns, len(x), spec.nclasses if supervised else 1,
                         domains, TREE_MOJO_VERSION, info, supervised=supervised)
    files.update(enc_files)
    z.write("model.ini", ini)
    for k, v in files.items():
        z.write(k, v)
    for t, tree in enumerate(model._forest.trees):
        k = model._forest.tclass[t]
        g = t // max(K, 1)
        lmk = leaf_maps(k, g)
        z.write("trees/t%02d_%03d.bin" % (k, g), _encode_tree(tree, lmk))
        z.write("trees/t%02d_%03d_aux.bin" % (k, g), _encode_aux(tree, lmk))


def _gbm(model, z):
    dist = model._dist
    fam = {"bernoulli": "bernoulli", "quasibinomial": "quasibinomial", "multinomial": "multinomial"}.get(
        dist.family, dist.family)
    K = model._n_tree_classes()
    init_f = list(model._init_f)
    extra = {"distribution": fam, "link_function": dist.link}
    if K > 1:
        # multinomial: the reference adds no init_f -- fold each class's
        # initial score into the leaves of that class's first tree
        extra["init_f"] = 0.0

        def leaf_maps(k, g):
            return (lambda v, c=init_f[k]: v + c) if g == 0 else None
    else:
        extra["init_f"] = float(init_f[0])

        def leaf_maps(k, g):
            return None
    _tree_model(model, z, "gbm", "Gradient Boosting Machine", extra, leaf_maps)


def _drf(model, z):
    spec = model._spec
    single = spec.nclasses == 2 and bool(model._binomial_single)
    extra = {"binomial_double_trees": spec.nclasses == 2 and not single}

    def leaf_maps(k, g):
        # the reference's single binomial DRF tree scores P(class 0)
        return (lambda v: 1.0 - v) if single else None
    _tree_model(model, z, "drf", "Distributed Random Forest", extra, leaf_maps)


# ---------------------------------------------------------------- XGBoost
_XGB_OBJ = {"bernoulli": "binary:logistic", "multinomial": "multi:softprob", "gaussian": "reg:squarederror",
            "poisson": "count:poisson", "gamma": "reg:gamma", "tweedie": "reg:tweedie"}
_XGB_MAX_NODES = 1 << 22


def _xgb_tree(tree, col_feat, cat_base, cat_card, leaf_add=0.0):
    """Our Tree -> XGBoost node / stat arrays over the one-hot feature space.

    Numeric splits map 1:1 (x < thr left, NA -> default direction).  A
    categorical split on column c (level mask going left, NA / unseen levels
    by na_left) becomes a chain of indicator tests over the smaller side S of
    the split: each chain node tests one level of S (hot = 1 >= 0.5 goes
    right, into a copy of S's subtree), the last chain node's left child is
    the other side's subtree.  Singleton sides (one-hot style splits) need no
    copies."""
    from .xgb_booster import nodes_from_lists, stats_from_lists
    parent, cleft, cright, feat, dleft, info = [], [], [], [], [], []
    loss, hess, bw = [], [], []

    def new(par, is_left, i):
        nid = len(cleft)
        if nid >= _XGB_MAX_NODES:
            raise NotImplementedError("categorical splits expand this tree beyond the XGBoost MOJO node limit")
        parent.append(-1 if par < 0 else (par | ((1 << 31) if is_left else 0)))
        cleft.append(-1); cright.append(-1); feat.append(0); dleft.append(0); info.append(0.0)
        loss.append(float(tree.gain[i]) if tree.left[i] >= 0 else 0.0)
        hess.append(float(tree.weight[i])); bw.append(float(tree.value[i]))
        return nid

    def emit(i, par, is_left):
        if tree.left[i] >= 0 and tree.is_cat[i]:
            card = cat_card[int(tree.feat[i])]
            m = np.asarray(tree.cat_left[i]).astype(bool)
            goes_left = np.array([bool(m[v]) if v < len(m) else bool(tree.na_left[i]) for v in range(card)] +
                                 [bool(tree.na_left[i])])
            lv, rv = np.flatnonzero(goes_left), np.flatnonzero(~goes_left)
            if len(lv) == 0 or len(rv) == 0:    # degenerate: every level on one side
                return emit(int(tree.left[i]) if len(rv) == 0 else int(tree.right[i]), par, is_left)
        nid = new(par, is_left, i)
        if tree.left[i] < 0:
            info[nid] = float(tree.value[i]) + leaf_add
            return nid
        f = int(tree.feat[i])
        l, r = int(tree.left[i]), int(tree.right[i])
        if not tree.is_cat[i]:
            feat[nid] = col_feat[f]
            dleft[nid] = 1 if tree.na_left[i] else 0
            info[nid] = float(np.float32(tree.thr[i]))
            cleft[nid] = emit(l, nid, True)
            cright[nid] = emit(r, nid, False)
            return nid
        s_levels, s_child, o_child = (lv, l, r) if len(lv) <= len(rv) else (rv, r, l)
        cur = nid
        for k, v in enumerate(s_levels):
            feat[cur] = cat_base[f] + int(v)
            dleft[cur] = 1
            info[cur] = 0.5
            cright[cur] = emit(s_child, cur, False)
            if k + 1 < len(s_levels):
                nxt = new(cur, True, i)
                cleft[cur] = nxt
                cur = nxt
            else:
                cleft[cur] = emit(o_child, cur, True)
        return nid

    emit(0, -1, True)
    return (nodes_from_lists(parent, cleft, cright, feat, dleft, info), stats_from_lists(loss, hess, bw))


def _xgboost(model, z):
    """XGBoostMojoWriter layout: model.ini (nums / cats / cat_offsets / sparse
    ...), feature_map and the native booster blob (mojo/xgb_booster.py).
    Columns are written categoricals first, as the reference's one-hot
    DataInfo orders them; each categorical contributes one indicator per
    level plus an NA indicator."""
    from .xgb_booster import Booster, margin_to_prob
    spec = model._spec
    x = list(spec.x)
    xd = getattr(model, "_x_domains", {}) or {}
    cats = [c for c in x if xd.get(c) is not None]
    nums = [c for c in x if xd.get(c) is None]
    offs = [0]
    for c in cats:
        offs.append(offs[-1] + len(xd[c]) + 1)
    col_feat, cat_base, cat_card = {}, {}, {}
    for j, c in enumerate(x):
        if c in xd and xd[c] is not None:
            ci = cats.index(c)
            cat_base[j], cat_card[j] = offs[ci], len(xd[c])
        else:
            col_feat[j] = offs[-1] + nums.index(c)
    obj = _XGB_OBJ.get(model._dist.family)
    if obj is None:
        raise NotImplementedError(f"XGBoost MOJO export: no XGBoost objective for distribution {model._dist.family}")
    K = model._n_tree_classes()
    init_f = [float(v) for v in model._init_f]
    b = Booster()
    b.name_obj, b.name_gbm = obj, "gbtree"
    b.num_feature = offs[-1] + len(nums)
    b.major_version, b.minor_version = 1, 6
    if K > 1:
        b.num_class, b.num_output_group = K, K
        b.base_score = 0.0                        # identity ProbToMargin; class offsets folded into tree 0
    else:
        b.num_class, b.num_output_group = 0, 1
        b.base_score = margin_to_prob(obj, init_f[0])
    for t, tree in enumerate(model._forest.trees):
        k = int(model._forest.tclass[t])
        add = init_f[k] if (K > 1 and t // K == 0) else 0.0
        b.trees.append(_xgb_tree(tree, col_feat, cat_base, cat_card, add))
        b.tree_info.append(k if K > 1 else 0)
    fmap = []
    for c in cats:
        for lev in xd[c]:
            fmap.append(f"{len(fmap)} {c}.{lev} i")
        fmap.append(f"{len(fmap)} {c}.missing(NA) i")
    for c in nums:
        fmap.append(f"{len(fmap)} {c} q")
    columns = cats + nums + [spec.y]
    domains = [list(xd[c]) for c in cats] + [None] * len(nums) + \
        [list(spec.response_domain) if spec.response_domain else None]
    cat = "Binomial" if spec.nclasses == 2 else "Multinomial" if spec.nclasses > 2 else "Regression"
    extra = {"nums": len(nums), "cats": len(cats), "cat_offsets": offs, "use_all_factor_levels": True,
             "sparse": False, "booster": "gbtree", "ntrees": len(model._forest) // max(K, 1),
             "use_java_scoring_by_default": True, "has_offset": False}
    ini, files = _header(model, "xgboost", "XGBoost", cat, columns, len(x), spec.nclasses, domains, "1.10", extra)
    z.write("model.ini", ini)
    for k_, v in files.items():
        z.write(k_, v)
    z.write("feature_map", "\n".join(fmap) + "\n")
    z.write("boosterBytes", b.to_bytes())


# ---------------------------------------------------------- TargetEncoder
def _targetencoder(model, z):
    """TargetEncoderMojoWriter layout: model.ini (blending parameters,
    non_predictors), feature_engineering/target_encoding/encoding_map.ini
    ([column] sections of `level = numerator denominator [target class]`, the
    last level being the NA level), the NA-presence map and the input ->
    encoded-column / input -> output-column maps."""
    spec = model._spec
    p = model._parms
    cols = list(model._cols)
    te_dir = "feature_engineering/target_encoding/"
    multi = spec.nclasses > 2
    enc_lines, na_lines, inenc, inout = [], [], [], []
    for c in cols:
        dom, per = model._tables[c]
        L = len(dom) + 1
        enc_lines.append(f"[{c}]")
        for lev in range(L):
            for ci, st in enumerate(per):
                num, den = float(st[0][lev]), float(st[1][lev])
                if multi:
                    enc_lines.append(f"{lev} = {num!r} {den!r} {ci + 1}")
                else:
                    enc_lines.append(f"{lev} = {num!r} {den!r}")
        has_na = any(float(st[1][L - 1]) > 0 for st in per)
        na_lines.append(f"{c} = {1 if has_na else 0}")
        inenc += ["[from]", c, "[to]", c]
        inout += ["[from]", c, "[to]"] + [f"{c}{sfx}_te" for sfx in model._suffix]
    x = [n for n in spec.x]
    columns = x + [spec.y]
    xd = {}
    for n in x:
        v = spec.frame.vec(n)
        xd[n] = list(v.domain) if v.domain is not None else None
    domains = [xd[n] for n in x] + [list(spec.response_domain) if spec.response_domain else None]
    nonpred = [c for c in (spec.weights_column, spec.offset_column, p.get("fold_column"), spec.y) if c]
    extra = {"keep_original_categorical_columns": bool(p.get("keep_original_categorical_columns", True)),
             "with_blending": bool(p.get("blending"))}
    if p.get("blending"):
        extra.update(inflection_point=float(p.get("inflection_point", 10.0)),
                     smoothing=float(p.get("smoothing", 20.0)))
    extra["non_predictors"] = ";".join(nonpred)
    cat = "Binomial" if spec.nclasses == 2 else "Multinomial" if spec.nclasses > 2 else "Regression"
    ini, files = _header(model, "targetencoder", "TargetEncoder", cat, columns, len(x), spec.nclasses, domains,
                         "1.00", extra)
    z.write("model.ini", ini)
    for k_, v in files.items():
        z.write(k_, v)
    z.write(te_dir + "encoding_map.ini", "\n".join(enc_lines) + "\n")
    z.write(te_dir + "te_column_name_to_missing_values_presence.ini", "\n".join(na_lines) + "\n")
    z.write(te_dir + "input_encoding_columns_map.ini", "\n".join(inenc) + "\n")
    z.write(te_dir + "input_output_columns_map.ini", "\n".join(inout) + "\n")


# ------------------------------------------------------------------ CoxPH
def _rect_blob(z, extra, title, a):
    """AbstractMojoWriter.writeRectangularDoubleArray: sizes in [info], a
    big-endian f64 blob."""
    a = np.asarray(a, dtype=np.float64)
    extra[title + "_size1"] = int(a.shape[0])
    extra[title + "_size2"] = int(a.shape[1]) if a.ndim > 1 else 0
    z.write(title, a.astype(">f8").tobytes())


def _coxph(model, z):
    """CoxPHMojoWriter layout: coef over [expanded cats | nums], per-stratum
    covariate means split into x_mean_cat / x_mean_num, strata keys as the
    strata columns' level codes; the strata columns lead the column list."""
    di = model._dinfo
    if getattr(di, "ia_recipe", None):
        raise NotImplementedError("CoxPH MOJO export with interaction columns is not implemented")
    spec = model._spec
    p = model._parms
    cats, nums = list(di.cat_cols), list(di.num_cols)
    sb = list(p.get("stratify_by") or [])
    sdom = getattr(model, "_strata_domains", {})
    offs = [0]
    for c in cats:
        offs.append(offs[-1] + (len(di.domains[c]) if di.use_all else len(di.domains[c]) - 1))
    beta = model._beta.detach().cpu().numpy().astype(np.float64)
    if len(beta) != offs[-1] + len(nums):
        raise NotImplementedError("CoxPH MOJO export: unexpected coefficient layout")
    keys = list(model._strata_keys)
    mc = np.stack([model._means[s].detach().cpu().numpy()[:offs[-1]] for s in keys])
    mn = np.stack([model._means[s].detach().cpu().numpy()[offs[-1]:] for s in keys])
    extra = {"coef": list(beta), "cats": len(cats), "cat_offsets": offs, "use_all_factor_levels": bool(di.use_all)}
    _rect_blob(z, extra, "x_mean_cat", mc)
    _rect_blob(z, extra, "x_mean_num", mn)
    extra["strata_count"] = len(keys) if sb else 0
    if sb:
        for i, k in enumerate(keys):
            codes = []
            k = int(k)
            for c in reversed(sb):
                base = len(sdom[c]) + 1 if c in sdom else 1_000_003
                codes.append(k % base - 1)
                k //= base
            extra[f"strata_{i}"] = [float(v) for v in reversed(codes)]
    columns = sb + cats + nums + [spec.y]
    domains = [list(sdom[c]) if c in sdom else None for c in sb] + [list(di.domains[c]) for c in cats] + \
        [None] * len(nums) + [list(spec.response_domain) if spec.response_domain else None]
    ini, files = _header(model, "coxph", "Cox Proportional Hazards", "CoxPH", columns, len(columns) - 1, 1,
                         domains, "1.00", extra)
    z.write("model.ini", ini)
    for k_, v in files.items():
        z.write(k_, v)


# -------------------------------------------------------------------- GLM
def _glm(model, z):
    di = model._dinfo
    if getattr(di, "ia_recipe", None):
        # GLMModel.haveMojo() is false for models with interactions
        # (GLMModel.java:1979): the reference exports none either
        raise NotImplementedError("reference-layout GLM MOJOs carry no interaction columns")
    spec = model._spec
    cats, nums = list(di.cat_cols), list(di.num_cols)
    columns = cats + nums + [spec.y]
    domains = [list(di.domains[c]) for c in cats] + [None] * len(nums) + \
        [list(spec.response_domain) if spec.response_domain else None]
    offs = [0]
    for c in cats:
        offs.append(offs[-1] + (len(di.domains[c]) if di.use_all else len(di.domains[c]) - 1))
    P = di.P
    multi = getattr(model, "_multi", None)
    extra = {"use_all_factor_levels": bool(di.use_all), "cats": len(cats), "cat_offsets": offs, "nums": len(nums),
             "mean_imputation": di.mvh == "meanimputation",
             "num_means": [float(v) for v in di.plug], "cat_modes": [int(di.cat_modes[c]) for c in cats]}
    if multi is None:
        b = np.asarray(model._beta_std, dtype=np.float64)
        beta, icpt = di.destandardize(b[:P], b[P] if b.size > P else b[-1])
        extra.update(beta=list(beta[:P]) + [icpt], family=model._fam.family, link=model._fam.link)
        if model._fam.link == "tweedie":
            extra["tweedie_link_power"] = float(model._fam.tlp)
        cat = "Binomial" if spec.nclasses == 2 else "Regression"
    elif multi["kind"] == "multinomial":
        B = multi["B"].cpu().numpy().astype(np.float64)
        b0 = multi["b0"].cpu().numpy().astype(np.float64)
        blocks = []
        for c in range(B.shape[1]):
            beta, icpt = di.destandardize(B[:P, c], b0[c])
            blocks += list(beta[:P]) + [icpt]
        extra.update(beta=blocks, family="multinomial", link="multinomial")
        cat = "Multinomial"
    elif multi["kind"] == "ordinal":
        bt = multi["beta"].cpu().numpy().astype(np.float64)
        th = multi["theta"].cpu().numpy().astype(np.float64)
        thc = np.cumsum(np.concatenate([th[:1], np.log1p(np.exp(th[1:]))]))
        blocks = []
        for c in range(spec.nclasses):
            if c < len(thc):
                beta, icpt = di.destandardize(-bt[:P], thc[c])
                blocks += list(beta[:P]) + [icpt]
            else:
                blocks += [0.0] * (P + 1)
        extra.update(beta=blocks, family="ordinal", link="ologit")
        cat = "Ordinal"
    else:
        raise NotImplementedError(f"GLM kind {multi['kind']}")
    ini, files = _header(model, "glm", "Generalized Linear Modeling", cat, columns, len(cats) + len(nums),
                         spec.nclasses, domains, GLM_MOJO_VERSION, extra)
    z.write("model.ini", ini)
    for k, v in files.items():
        z.write(k, v)


# ------------------------------------------------------------ isolation forests
def _isofor(model, z):
    """IsolationForestMojoModel: tree sums of path lengths, normalised by the
    integer min / max total path length of the training rows (the reference
    keeps them as ints: IsolationForestMojoModel.java:7)."""
    nt = max(1, len(model._forest))
    extra = {"min_path_length": int(round(model._min_len * nt)), "max_path_length": int(round(model._max_len * nt)),
             "output_anomaly_flag": model._threshold is not None}
    if model._threshold is not None:
        extra["default_threshold"] = float(model._threshold)
    _tree_model(model, z, "isolationforest", "Isolation Forest", extra, lambda k, g: None, supervised=False,
                category="AnomalyDetection")


def _eif(model, z):
    """ExtendedIsolationForestMojoModel: one blob per tree -- int32 vector size
    k, then heap-numbered records (int32 node number; 'N' + k normal f64 + k
    point f64, or 'L' + int32 rows)."""
    di = model._dinfo
    if di.cat_cols:
        raise NotImplementedError("reference-layout Extended Isolation Forest MOJOs score numeric columns only")
    x = list(di.num_cols)
    P = len(x)
    ini, files = _header(model, "extendedisolationforest", "Extended Isolation Forest", "AnomalyDetection", x, P, 1,
                         [None] * P, "1.00", {"ntrees": len(model._trees), "sample_size": int(model._psi)},
                         supervised=False)
    z.write("model.ini", ini)
    for k, v in files.items():
        z.write(k, v)
    for t, nodes in enumerate(model._trees):
        out = bytearray(struct.pack("<i", P))
        stack = [(0, 0)]                       # (our node index, heap number)
        recs = []
        while stack:
            i, num = stack.pop()
            nd = nodes[i]
            if nd[2] < 0:
                if len(nd) < 6:
                    raise NotImplementedError("this Extended Isolation Forest predates leaf row counts: retrain it")
                recs.append((num, b"L" + struct.pack("<i", int(nd[5]))))
            else:
                recs.append((num, b"N" + np.asarray(nd[0], dtype="<f8").tobytes() +
                             np.asarray(nd[1], dtype="<f8").tobytes()))
                stack.append((nd[3], 2 * num + 2))
                stack.append((nd[2], 2 * num + 1))
        for num, body in sorted(recs):
            out += struct.pack("<i", num) + body
        z.write("trees/t%02d.bin" % t, bytes(out))


# ------------------------------------------------------------------ K-Means
def _kmeans(model, z):
    """KMeansMojoModel: columns in the clustering order (categoricals first),
    per-column standardisation means / multipliers / modes (-1 = numeric) and
    the centers in that space -- a categorical center is its level index (the
    one-hot block of our clustering space holds the mode at 1/sqrt(2), so the
    mismatch distance is the reference's 0/1)."""
    di = model._dinfo
    cats, nums = list(di.cat_cols), list(di.num_cols)
    columns = cats + nums
    domains = [list(di.domains[c]) for c in cats] + [None] * len(nums)
    C = model._C_std[:, :di.P].detach().cpu().numpy().astype(np.float64)
    centers = []
    for r in range(C.shape[0]):
        row = []
        for c in cats:
            off, L = di.cat_offsets[c], len(di.domains[c])
            row.append(float(np.argmax(C[r, off:off + L])))
        row += [float(v) for v in C[r, di.n_cat_expanded:di.P]]
        centers.append(row)
    extra = {"standardize": bool(di.standardize), "center_num": len(centers)}
    if di.standardize:
        extra["standardize_means"] = [0.0] * len(cats) + [float(m) for m in di.means]
        extra["standardize_mults"] = [0.0] * len(cats) + [1.0 / float(s) for s in di.sigmas]
        extra["standardize_modes"] = [int(di.cat_modes[c]) for c in cats] + [-1] * len(nums)
    for i, row in enumerate(centers):
        extra[f"center_{i}"] = row
    ini, files = _header(model, "kmeans", "K-means", "Clustering", columns, len(columns), 1, domains, "1.00", extra,
                         supervised=False)
    z.write("model.ini", ini)
    for k, v in files.items():
        z.write(k, v)


# ------------------------------------------------------------ Deep Learning
_DL_ACT = {"tanh": "Tanh", "rectifier": "Rectifier", "maxout": "Maxout", "exprectifier": "ExpRectifier"}


def _deeplearning(model, z):
    """DeepLearningMojoModel: one-hot categoricals with a trailing missing
    bucket per variable (GenModel.setInput), standardised numerics
    (norm_mul = 1 / sigma, norm_sub = mean), the regression response scale,
    and row-major float weights per layer.  Our NA handling (categorical
    mode, numeric mean) is expressed exactly: the missing bucket's weights
    are the mode level's, a missing numeric standardises to 0."""
    if getattr(model, "_cat_slots", None) is not None:
        raise NotImplementedError("MOJO export of a DL model with hashed categoricals (max_categorical_features)")
    if model._ae:
        raise NotImplementedError("reference-layout MOJO export of deep learning autoencoders is not implemented")
    di = model._dinfo
    spec = model._spec
    cats, nums = list(di.cat_cols), list(di.num_cols)
    columns = cats + nums + [spec.y]
    domains = [list(di.domains[c]) for c in cats] + [None] * len(nums) + \
        [list(spec.response_domain) if spec.response_domain else None]
    # expanded input map: reference column -> our design column (or -1 = zero)
    offs, src = [0], []
    for c in cats:
        L = len(di.domains[c])
        lv = list(range(L)) if di.use_all else list(range(1, L))
        ours = [di.cat_offsets[c] + (l if di.use_all else l - 1) for l in lv]
        mode = int(di.cat_modes[c])
        na = di.cat_offsets[c] + (mode if di.use_all else mode - 1) if (di.use_all or mode > 0) else -1
        src += ours + [na]
        offs.append(offs[-1] + len(ours) + 1)
    src += [di.n_cat_expanded + j for j in range(len(nums))]
    src = np.asarray(src, dtype=np.int64)
    layers = model._layers
    act_name = str(model._parms.get("activation") or "Rectifier")
    units = [len(src)] + [L.fout for L in layers]
    extra = {"nums": len(nums), "cats": len(cats), "cat_offsets": offs, "use_all_factor_levels": bool(di.use_all),
             "activation": act_name, "distribution": model._dist.family if spec.nclasses <= 1 else
             ("bernoulli" if spec.nclasses == 2 else "multinomial"),
             "mean_imputation": True, "cat_modes": [int(di.cat_modes[c]) for c in cats], "mini_batch_size": 1,
             "neural_network_sizes": units,
             "hidden_dropout_ratios": [float(L.drop) for L in layers[:-1]]}
    enc_info, enc_files = _encoding_kv(model)
    extra.update(enc_info)
    if di.standardize and nums:
        extra["norm_mul"] = [1.0 / float(s) for s in di.sigmas]
        extra["norm_sub"] = [float(m) for m in di.means]
    if spec.nclasses <= 1:
        extra["norm_resp_mul"] = [1.0 / float(model._ysd)]
        extra["norm_resp_sub"] = [float(model._ymu)]
    for li, L in enumerate(layers):
        W = L.W.detach().cpu().numpy().astype(np.float64)
        b = L.b.detach().cpu().numpy().astype(np.float64)
        if li == 0:
            Wr = np.zeros((W.shape[0], len(src)))
            ok = src >= 0
            Wr[:, ok] = W[:, src[ok]]
            W = Wr
        if L.k > 1:
            # ours: row 2u + j; the reference: [unit][input][piece]
            W = W.reshape(L.fout, L.k, -1).transpose(0, 2, 1)
        extra[f"weight_layer{li}"] = [float(v) for v in np.asarray(W, dtype=np.float32).reshape(-1)]
        extra[f"bias_layer{li}"] = [float(v) for v in b]
    cat = "Binomial" if spec.nclasses == 2 else "Multinomial" if spec.nclasses > 2 else "Regression"
    ini, files = _header(model, "deeplearning", "Deep Learning", cat, columns, len(cats) + len(nums), spec.nclasses,
                         domains, "1.10", extra)
    files.update(enc_files)
    z.write("model.ini", ini)
    for k, v in files.items():
        z.write(k, v)


# ---------------------------------------------------------------------- PCA
def _pca(model, z):
    """PCAMojoReader layout: columns in DataInfo order (categoricals, then
    numerics; identity permutation), normSub / normMul of the numerics and
    the [P][k] eigenvectors as a big-endian double blob.  Our transform NONE
    centres the data; that is expressible only without categoricals."""
    di = model._dinfo
    cats, nums = list(di.cat_cols), list(di.num_cols)
    mean = model._mean.detach().cpu().numpy().astype(np.float64)[:di.P]
    if cats and np.any(mean[:di.n_cat_expanded] != 0):
        raise NotImplementedError("reference-layout PCA MOJOs cannot centre one-hot columns: "
                                  "use transform='STANDARDIZE' (or another scaling) with categoricals")
    base = di.n_cat_expanded
    if di.standardize:
        sub = [float(m) for m in di.means]
        mul = [1.0 / float(s) for s in di.sigmas]
    else:
        sub = [float(mean[base + j]) for j in range(len(nums))]
        mul = [1.0] * len(nums)
    offs = [0]
    for c in cats:
        L = len(di.domains[c])
        offs.append(offs[-1] + (L if di.use_all else L - 1))
    E = model._evecs.detach().cpu().numpy().astype(np.float64)[:di.P]
    extra = {"use_all_factor_levels": bool(di.use_all), "pca_methods": str(model._parms.get("pca_method", "GramSVD")),
             "pca_impl": str(model._parms.get("pca_impl", "mtj_evd_symmmatrix")), "k": int(E.shape[1]),
             "permutation": list(range(len(cats) + len(nums))), "ncats": len(cats), "nnums": len(nums),
             "normSub": sub, "normMul": mul, "catOffsets": offs, "eigenvector_size": int(E.shape[0])}
    columns = cats + nums
    domains = [list(di.domains[c]) for c in cats] + [None] * len(nums)
    ini, files = _header(model, "pca", "Principal Components Analysis", "DimReduction", columns, len(columns),
                         int(E.shape[1]), domains, "1.00", extra, supervised=False)
    z.write("model.ini", ini)
    for k, v in files.items():
        z.write(k, v)
    z.write("eigenvectors_raw", E.astype(">f8").tobytes())


# ----------------------------------------------------------------- Word2Vec
def _word2vec(model, z):
    """Word2VecMojoModel: `vocabulary` (one word per line, newlines escaped)
    and `vectors` (big-endian float32, vocab x vec_size)."""
    V = model._vecs.detach().cpu().numpy().astype(">f4")
    ini, files = _header(model, "word2vec", "Word2Vec", "WordEmbedding", ["C1"], 1, 1, [None], "1.00",
                         {"vec_size": int(V.shape[1]), "vocab_size": int(V.shape[0])}, supervised=False)
    z.write("model.ini", ini)
    z.write("vocabulary", "\n".join(w.replace("\n", "\\n") for w in model._vocab) + "\n")
    z.write("vectors", V.tobytes())


# ---------------------------------------------------------- Stacked Ensemble
def _stackedensemble(model, z):
    """StackedEnsembleMojoModel: every base model and the metalearner as a
    nested reference-layout MOJO under models/<algo>/<key>/, the base models'
    inputs remapped by column name from the ensemble's columns."""
    spec = model._spec
    x = list(spec.x)
    for bm in model._base:
        for c in bm._spec.x:
            if c not in x:
                x.append(c)
    columns = x + [spec.y]
    xd = {}
    for bm in model._base:
        xd.update(getattr(bm, "_x_domains", None) or (bm._dinfo.domains if hasattr(bm, "_dinfo") else {}))
    domains = [xd.get(c) for c in x] + [list(spec.response_domain) if spec.response_domain else None]
    subs = list(model._base) + [model._meta]
    extra = {"submodel_count": len(subs), "base_models_num": len(model._base), "metalearner": model._meta.model_id,
             "metalearner_transform": "Logit" if str(model._parms.get("metalearner_transform") or "NONE").lower()
             == "logit" else "NONE"}
    for i, m in enumerate(subs):
        d = f"models/{m.algo}/{m.model_id}/"
        extra[f"submodel_key_{i}"] = m.model_id
        extra[f"submodel_dir_{i}"] = d
        _write_algo(m, z.nested(d))
    for i, m in enumerate(model._base):
        extra[f"base_model{i}"] = m.model_id
    cat = "Binomial" if spec.nclasses == 2 else "Multinomial" if spec.nclasses > 2 else "Regression"
    ini, files = _header(model, "stackedensemble", "StackedEnsemble", cat, columns, len(x), spec.nclasses, domains,
                         "1.01", extra)
    z.write("model.ini", ini)
    for k, v in files.items():
        z.write(k, v)


# ------------------------------------------------------------------ RuleFit
def _rulefit(model, z):
    """RuleFitMojoModel (hex/genmodel/algos/rulefit): the rule ensemble as
    per-(model, tree) lists of leaf rules with their conditions, and the
    linear model as a nested GLM MOJO whose rule columns are categoricals
    M<i>T<j> (level = the row's leaf rule, a never-matched first level keeps
    every rule's beta explicit) next to the linear terms.  Multinomial:
    one categorical M<i>T<j>C<k> per class tree, the rules of a (model,
    tree) written class by class (RuleFitMojoWriter.java:64-100,
    RuleEnsemble.createGLMTrainFrame) and a multinomial nested GLM whose
    class-c block holds every column's class-c betas."""
    spec = model._spec
    K = spec.nclasses
    classes = list(spec.response_domain) if K > 2 else None
    x = list(spec.x)
    xd = {}
    for tm in model._trees:
        xd.update(getattr(tm, "_x_domains", None) or {})
    mt = {"LINEAR": 0, "RULES_AND_LINEAR": 1, "RULES": 2}[model._mtype]
    rules = model._rules()
    if classes:
        tabs = model._glm._output["coefficients_table_multinomials"]
        coefs = [dict(tabs[c]) for c in classes]
    else:
        coefs = [model._glm.coef()]
    depth = len(model._trees)
    ntrees = len(model._trees[0]._forest.trees) // (model._trees[0]._n_tree_classes() if classes else 1) \
        if model._trees else 0
    extra = {"model_type": mt, "depth": depth, "ntrees": ntrees}
    groups = {}
    for r in rules:
        groups.setdefault((r[0], r[1], r[8]), []).append(r)
    cat_cols, cat_doms, cat_betas = [], [], []
    for i in range(depth):
        for j in range(ntrees):
            rs_all = []
            for k in (range(K) if classes else [None]):
                rs = groups.get((i, j, k), [])
                rs_all += rs
                cat_cols.append(f"M{i}T{j}C{k}" if classes else f"M{i}T{j}")
                cat_doms.append(["__no_rule__"] + [r[5] for r in rs])
                cat_betas.append([[0.0] + [float(cf.get(r[5], 0.0)) for r in rs] for cf in coefs])
            extra[f"num_rules_M{i}T{j}"] = len(rs_all)
            for k, r in enumerate(rs_all):
                rid = f"{i}_{j}_{k}"
                extra[f"num_conditions_rule_id_{rid}"] = len(r[6])
                extra[f"prediction_value_rule_id_{rid}"] = 0.0
                extra[f"language_rule_rule_id_{rid}"] = r[3]
                extra[f"coefficient_rule_id_{rid}"] = float(coefs[r[8] or 0].get(r[5], 0.0))
                extra[f"var_name_rule_id_{rid}"] = r[5]
                for c, (f, op, v, na) in enumerate(r[6]):
                    cid = f"{c}_{rid}"
                    extra[f"feature_index_{cid}"] = x.index(f)
                    extra[f"feature_name_{cid}"] = f
                    extra[f"nas_included_{cid}"] = bool(na)
                    if op == "in":
                        dom = xd.get(f, [])
                        extra[f"type_{cid}"] = 0
                        extra[f"operator_{cid}"] = 2
                        extra[f"language_cat_treshold_length_{cid}"] = len(v)
                        extra[f"cat_treshold_length_{cid}"] = len(v)
                        for t, lv in enumerate(v):
                            extra[f"language_cat_treshold_{t}_{cid}"] = str(dom[lv]) if lv < len(dom) else str(lv)
                            extra[f"cat_treshold_length_{t}_{cid}"] = int(lv)
                        extra[f"language_condition{cid}"] = f"({f} in {{...}})"
                    else:
                        extra[f"type_{cid}"] = 1
                        extra[f"operator_{cid}"] = 0 if op == "<" else 1
                        extra[f"num_treshold{cid}"] = float(v)
                        extra[f"language_condition{cid}"] = f"({f} {op} {float(v):.6g})"
    lin_cats = [c for c in x if c in xd and mt != 2]
    lin_nums = [c for c in x if c not in xd and mt != 2]
    gcols_cat = (cat_cols if mt != 0 else []) + [f"linear.{c}" for c in lin_cats]
    gdoms = (cat_doms if mt != 0 else []) + [list(xd[c]) for c in lin_cats]
    gnums = [f"linear.{c}" for c in lin_nums]
    beta = []
    for ci, cf in enumerate(coefs):
        bl = [cb[ci] for cb in cat_betas] if mt != 0 else []
        bl += [[float(cf.get(f"linear.{c}.{lv}", 0.0)) for lv in xd[c]] for c in lin_cats]
        beta += [b for blk in bl for b in blk] + [float(cf.get(n, 0.0)) for n in gnums] + \
            [float(cf.get("Intercept", 0.0))]
    offs = [0]
    for d in gdoms:
        offs.append(offs[-1] + len(d))
    key = f"{model.model_id}_linear"
    gdi = model._glm._dinfo
    plug = dict(zip(gdi.num_cols, gdi.plug))
    modes = [0] * (len(cat_cols) if mt != 0 else 0) + [int(gdi.cat_modes.get(f"linear.{c}", 0)) for c in lin_cats]
    fam, link = ("multinomial", "multinomial") if classes else (model._glm._fam.family, model._glm._fam.link)
    gextra = {"use_all_factor_levels": True, "cats": len(gcols_cat), "cat_offsets": offs, "nums": len(gnums),
              "mean_imputation": True, "num_means": [float(plug.get(n, 0.0)) for n in gnums], "cat_modes": modes,
              "beta": beta, "family": fam, "link": link}
    cat = "Multinomial" if classes else "Binomial" if K == 2 else "Regression"
    resp_dom = [list(spec.response_domain) if spec.response_domain else None]
    gini, gfiles = _header(model._glm, "glm", "Generalized Linear Modeling", cat, gcols_cat + gnums + [spec.y],
                           len(gcols_cat) + len(gnums), K, gdoms + [None] * len(gnums) + resp_dom,
                           GLM_MOJO_VERSION, gextra)
    sub = z.nested(f"models/glm/{key}/")
    sub.write("model.ini", gini)
    for k_, v_ in gfiles.items():
        sub.write(k_, v_)
    linear_names = (cat_cols if mt != 0 else []) + ([f"linear.{c}" for c in x] if mt != 2 else [])
    extra.update({"submodel_count": 1, "submodel_key_0": key, "submodel_dir_0": f"models/glm/{key}/",
                  "linear_model": key, "data_from_rules_codes_len": len(cat_cols) if mt != 0 else 0,
                  "weights_column": model._parms.get("weights_column") or "null",
                  "linear_names_len": len(linear_names)})
    for i, n in enumerate(cat_cols if mt != 0 else []):
        extra[f"data_from_rules_codes_{i}"] = n
    for i, n in enumerate(linear_names):
        extra[f"linear_names_{i}"] = n
    columns = x + [spec.y]
    domains = [xd.get(c) for c in x] + resp_dom
    ini, files = _header(model, "rulefit", "rulefit", cat, columns, len(x), K, domains, "1.00", extra)
    z.write("model.ini", ini)
    for k_, v_ in files.items():
        z.write(k_, v_)


def _glrm(model, z):
    """GlrmMojoWriter layout (mojo 1.10): the DataInfo permutation puts the
    categorical columns first; norm_sub / norm_mul express the numeric
    transform; `losses` holds one GlrmLoss name per (permuted) column;
    `archetypes` is Y [k][ncolY] in the permuted one-hot layout, as a
    big-endian double blob (java.nio.ByteBuffer order)."""
    p = model._parms
    cols = list(model._cols)
    blocks = model._blocks
    cats = [i for i, (kind, _, _) in enumerate(blocks) if kind == "cat"]
    nums = [i for i, (kind, _, _) in enumerate(blocks) if kind == "num"]
    perm = cats + nums
    starts, j = [], 0
    for _, _, w in blocks:
        starts.append(j)
        j += w
    Y = model._Y.detach().cpu().numpy().astype(np.float64)
    order = [c for i in perm for c in range(starts[i], starts[i] + blocks[i][2])]
    Yp = Y[:, order]
    num_levels = [blocks[i][2] for i in cats]
    offs = [0]
    for L in num_levels:
        offs.append(offs[-1] + L)
    tr = str(p.get("transform") or "NONE").upper()
    sub, mul = [], []
    for i in nums:
        mu, sd, lo, hi = model._stats[blocks[i][1]]
        s_, m_ = {"STANDARDIZE": (mu, 1.0 / sd), "NORMALIZE": (lo, 1.0 / max(hi - lo, 1e-12)),
                  "DEMEAN": (mu, 1.0), "DESCALE": (0.0, 1.0 / sd)}.get(tr, (0.0, 1.0))
        sub.append(float(s_))
        mul.append(float(m_))
    losses = [model._multi_loss()] * len(cats)
    for i in nums:
        nm = model._col_loss(blocks[i][1])
        nm = {k.lower(): k for k in ("Quadratic", "Absolute", "Huber", "Poisson", "Periodic", "Logistic",
                                     "Hinge")}.get(str(nm).lower(), nm)
        losses.append(f"Periodic({int(p.get('period', 1))})" if nm == "Periodic" else nm)
    regs = {k.lower(): k for k in ("None", "Quadratic", "L2", "L1", "NonNegative", "OneSparse", "UnitOneSparse",
                                   "Simplex")}
    inits = {k.lower(): k for k in ("Random", "SVD", "PlusPlus", "User", "Power")}
    seed = p.get("seed", -1)
    extra = {"initialization": inits.get(str(p.get("init") or "PlusPlus").lower(), "PlusPlus"),
             "regularizationX": regs.get(str(p.get("regularization_x") or "None").lower(), "None"),
             "regularizationY": regs.get(str(p.get("regularization_y") or "None").lower(), "None"),
             "gammaX": float(p.get("gamma_x", 0.0)), "gammaY": float(p.get("gamma_y", 0.0)),
             "ncolX": int(Y.shape[0]), "seed": int(seed) if seed not in (None, -1) else 12345,
             "reverse_transform": bool(p.get("impute_original")), "cols_permutation": perm,
             "num_categories": len(cats), "num_numeric": len(nums), "norm_sub": sub, "norm_mul": mul,
             "transposed": False, "ncolA": len(blocks), "ncolY": int(Y.shape[1]), "nrowY": int(Y.shape[0]),
             "num_levels_per_category": num_levels, "catOffsets": offs}
    domains = [list(model._doms[c]) if c in model._doms else None for c in cols]
    ini, files = _header(model, "glrm", "Generalized Low Rank Modeling", "DimReduction", cols, len(cols),
                         1, domains, "1.10", extra, supervised=False)
    z.write("model.ini", ini)
    for k_, v_ in files.items():
        z.write(k_, v_)
    z.write("losses", "\n".join(losses) + "\n")
    z.write("archetypes", Yp.astype(">f8").tobytes())


def _be_f8(rows):
    """java.nio.ByteBuffer putDouble order (big endian), rows flattened."""
    flat = [float(v) for r in rows for v in np.asarray(r, dtype=np.float64).reshape(-1)]
    return np.asarray(flat, dtype=">f8").tobytes()


def _gam(model, z):
    """GAMMojoWriter layout (mojo 1.00): the GLM part (cats first, then the
    plain numerics, then the centred smoother columns in bs-sorted order --
    cubic regression, I-spline, thin plate -- and the intercept) with
    beta_center for scoring and beta (uncentred smoother coefficients Z b);
    per smoother the knots, zTranspose (Z'), the cubic-spline B^-1 D
    (_binvD), the thin-plate zCS', polynomial exponent lists, raw means and
    inverse standard deviations.  Text files hold the column-name lists."""
    if any(b == 3 for b in model._bs):
        raise NotImplementedError("the reference GAM MOJO scorer has no M-spline (bs=3) smoothers")
    from ..models.glm.gam import _SUFFIX, _cr_matrices, _gname
    di = model._dinfo
    spec = model._spec
    gcols = list(model._gam_cols)
    rank = {0: 0, 2: 1, 1: 2}
    order = sorted(range(len(gcols)), key=lambda g: (rank[model._bs[g]], g))
    cen_names, nc_names, gam_set = {}, {}, set()
    for g in range(len(gcols)):
        nm, suf = _gname(gcols[g]), _SUFFIX[model._bs[g]]
        Z = np.asarray(model._Z[g])
        cen_names[g] = [f"{nm}_{suf}_{i}" for i in range(Z.shape[1])]
        nc_names[g] = [f"{nm}_{suf}_nc_{i}" for i in range(Z.shape[0])]
        gam_set.update(cen_names[g])
    cats = list(di.cat_cols)
    plain = [c for c in di.num_cols if c not in gam_set]
    gam_cols_sorted = [n for g in order for n in cen_names[g]]
    nums = plain + gam_cols_sorted
    pos = {c: j for j, c in enumerate(di.num_cols)}
    P = di.P
    base = di.n_cat_expanded
    offs = [0]
    for c in cats:
        offs.append(offs[-1] + (len(di.domains[c]) if di.use_all else len(di.domains[c]) - 1))
    plug = list(di.plug)
    # a missing smoother input: the model scores the basis at the column mean,
    # so the centred columns' fill values are that basis row
    fills = {}
    for g in range(len(gcols)):
        cc_ = gcols[g] if isinstance(gcols[g], tuple) else (gcols[g],)
        import pandas as pd
        from ..core.frame import H2OFrame
        one = H2OFrame(pd.DataFrame({c: [model._col_means[c]] for c in cc_}))
        Xg, _ = model._basis(one, gcols[g], model._bs[g], model._knots[g], model._orders[g], g)
        row = (Xg @ __import__("torch").as_tensor(model._Z[g], dtype=Xg.dtype)).cpu().numpy()[0]
        fills.update(dict(zip(cen_names[g], row.tolist())))
    num_fill = [float(plug[pos[c]]) if c in plain else float(fills[c]) for c in nums]

    def beta_blocks(b_std, icpt_std):
        beta, icpt = di.destandardize(np.asarray(b_std, dtype=np.float64)[:P], icpt_std)
        center = list(beta[:base]) + [float(beta[base + pos[c]]) for c in nums] + [icpt]
        nc = list(beta[:base]) + [float(beta[base + pos[c]]) for c in plain]
        for g in order:
            bc = np.asarray([beta[base + pos[c]] for c in cen_names[g]])
            nc += list(np.asarray(model._Z[g]) @ bc)
        return center, nc + [icpt]

    multi = getattr(model, "_multi", None)
    fam = model._fam.family if multi is None else multi["kind"]
    if multi is None:
        b = np.asarray(model._beta_std, dtype=np.float64)
        bc, bnc = beta_blocks(b[:P], b[P] if b.size > P else b[-1])
        beta_kv = {"beta": bnc, "beta length per class": len(bnc), "beta_center": bc,
                   "beta center length per class": len(bc)}
        blobs = {}
        cat = "Binomial" if spec.nclasses == 2 else "Regression"
    elif multi["kind"] == "multinomial":
        B = multi["B"].cpu().numpy().astype(np.float64)
        b0 = multi["b0"].cpu().numpy().astype(np.float64)
        rows_c, rows_nc = [], []
        for c in range(B.shape[1]):
            bc, bnc = beta_blocks(B[:P, c], b0[c])
            rows_c.append(bc)
            rows_nc.append(bnc)
        beta_kv = {"beta length per class": len(rows_nc[0]), "beta center length per class": len(rows_c[0])}
        blobs = {"beta_multinomial": _be_f8(rows_nc), "beta_multinomial_centering": _be_f8(rows_c)}
        cat = "Multinomial"
    else:
        raise NotImplementedError(f"reference-layout GAM MOJO for {multi['kind']} models")
    family = {"binomial": "bernoulli"}.get(fam, fam)
    link = "multinomial" if multi is not None else model._fam.link
    gs = [gcols[g] for g in order]
    as_list = lambda c: list(c) if isinstance(c, tuple) else [c]          # noqa: E731
    tp = [g for g in order if model._bs[g] == 1]
    iss = [g for g in order if model._bs[g] == 2]
    csg = [g for g in order if model._bs[g] == 0]
    nk = [len(model._knots[g]) for g in range(len(gcols))]
    extra = {"use_all_factor_levels": bool(di.use_all), "cats": len(cats), "cat_offsets": offs,
             "numsCenter": len(nums), "num": len(nums) + len(gcols),
             "mean_imputation": di.mvh == "meanimputation"}
    if extra["mean_imputation"]:
        extra["numNAFillsCenter"] = num_fill
        extra["catNAFills"] = [int(di.cat_modes[c]) for c in cats]
    extra.update(family=family, link=link)
    if fam == "tweedie":
        extra["tweedie_link_power"] = float(model._fam.tlp)
    extra.update({"num_knots": nk, "num_knots_sorted": [nk[g] for g in order],
                  "gam_column_dim": [len(as_list(c)) for c in gcols],
                  "gam_column_dim_sorted": [len(as_list(c)) for c in gs],
                  "num_expanded_gam_columns": sum(len(nc_names[g]) for g in order),
                  "num_expanded_gam_columns_center": len(gam_cols_sorted)})
    names_nc = cats + plain + [n for g in order for n in nc_names[g]]
    extra.update({"total feature size": len(names_nc), "gamColName_dim": [len(nc_names[g]) for g in order]})
    extra.update(beta_kv)
    extra.update({"bs": list(model._bs), "bs_sorted": [model._bs[g] for g in order],
                  "_d": [len(as_list(c)) for c in gs], "num_CS_col": len(csg), "num_IS_col": len(iss)})
    if iss:
        extra["spline_orders_sorted"] = [int(model._orders[g]) for g in order]
        extra["spline_orders"] = [int(o) for o in model._orders]
    if tp:
        extra.update({"_M": [int(model._tp[g]["M"]) for g in tp], "_m": [int(model._tp[g]["m"]) for g in tp],
                      "num_knots_TP": [nk[g] for g in tp],
                      # the scorer's thin-plate standardisation flag
                      "standardize": any(bool(model._tp[g]["standardize"]) for g in tp), "num_TP_col": len(tp)})
    else:
        extra["num_TP_col"] = 0
    columns = cats + nums + [spec.y]
    domains = [list(di.domains[c]) for c in cats] + [None] * len(nums) + \
        [list(spec.response_domain) if spec.response_domain else None]
    ini, files = _header(model, "gam", "Generalized Additive Model", cat, columns, len(cats) + len(nums),
                         spec.nclasses, domains, "1.00", extra)
    z.write("model.ini", ini)
    for k_, v_ in files.items():
        z.write(k_, v_)
    txt = lambda rows: "\n".join(str(r) for r in rows) + "\n"                 # noqa: E731
    z.write("gam_columns", txt([c for col in gcols for c in as_list(col)]))
    z.write("gam_columns_sorted", txt([c for col in gs for c in as_list(col)]))
    z.write("_names_no_centering", txt(names_nc))
    z.write("gamColNames", txt([n for g in order for n in nc_names[g]]))
    z.write("gamColNamesCenter", txt(gam_cols_sorted))
    for k_, v_ in blobs.items():
        z.write(k_, v_)
    knot_rows, zt_rows = [], []
    for g in order:
        kn = np.asarray(model._knots[g], dtype=np.float64)
        kn = kn.reshape(len(kn), -1)
        knot_rows += [kn[:, j] for j in range(kn.shape[1])]
        Z = np.asarray(model._Z[g], dtype=np.float64)
        if model._bs[g] == 2:                       # I-splines are not centred: the reader skips this block
            zt_rows += [np.zeros(nk[g])] * Z.shape[1]
        else:
            zt_rows += list(Z.T)
    z.write("knots", _be_f8(knot_rows))
    z.write("zTranspose", _be_f8(zt_rows))
    if csg:
        z.write("_binvD", _be_f8([r for g in csg for r in _cr_matrices(np.asarray(model._knots[g]))[0][1:-1]]))
    if tp:
        ints = [int(e) for g in tp for term in model._tp[g]["terms"] for e in term]
        z.write("polynomialBasisList", np.asarray(ints, dtype=">i4").tobytes())
        z.write("zTransposeCS", _be_f8([r for g in tp for r in np.asarray(model._tp[g]["zCS"]).T]))
        z.write("gamColMeansRaw", _be_f8([model._tp[g]["means"] for g in tp]))
        z.write("gamColStdRaw", _be_f8([model._tp[g]["ostd"] for g in tp]))


_WRITERS = {"rulefit": _rulefit, "gbm": _gbm, "drf": _drf, "glm": _glm, "kmeans": _kmeans, "isolationforest": _isofor,
            "extendedisolationforest": _eif, "deeplearning": _deeplearning, "word2vec": _word2vec,
            "stackedensemble": _stackedensemble, "pca": _pca, "xgboost": _xgboost,
            "coxph": _coxph, "targetencoder": _targetencoder, "glrm": _glrm, "gam": _gam}


def _write_algo(model, z):
    if model.algo == "glm" and getattr(model, "_hglm", None) is not None:
        raise NotImplementedError("HGLM models have no MOJO (as in the reference)")
    w = _WRITERS.get(model.algo)
    if w is None:
        raise NotImplementedError(f"reference-layout MOJO export is not implemented for {model.algo} "
                                  f"(supported: {', '.join(sorted(_WRITERS))})")
    w(model, z)


def build_h2o_mojo(model) -> bytes:
    """MOJO zip bytes in the reference's layout (GBM, DRF, XGBoost, GLM,
    CoxPH, K-Means, Isolation Forest, Extended Isolation Forest, Deep Learning,
    Word2Vec, Stacked Ensemble, PCA)."""
    z = _Zip()
    _write_algo(model, z)
    write_model_details(model, z)
    return z.close()


def model_details_json(model) -> str:
    """The model's ModelSchemaV3 JSON (output: metrics, variable importances,
    model summary, scoring history; parameters) as the reference writes it to
    experimental/modelDetails.json (ModelMojoWriter.writeModelDetails,
    hex/ModelMojoWriter.java:96) and ModelJsonReader reads it back."""
    import json
    from ..server import schemas as S
    try:
        d = S.model_v3(model.model_id, model)
    except Exception as e:  # noqa: BLE001 - details are informational; the MOJO stays valid
        d = {"model_id": S.key(model.model_id, "Model"), "algo": model.algo, "output": None,
             "details_error": repr(e)}
    return json.dumps(S.jsonable(d))


def write_model_details(model, z):
    z.write("experimental/modelDetails.json", model_details_json(model))
    z.write("experimental/README.md", "Outputting model information in JSON is an experimental feature and we "
            "appreciate any feedback.\nThe contents of this folder may change with another version of H2O.\n")


def build_mojo_pipeline(models, mapping, main_alias) -> bytes:
    """MojoPipelineBuilder / MojoPipelineWriter: one zip holding every
    sub-model under models/<alias>/ and a model.ini whose columns are the
    sub-models' inputs followed by the main model's non-generated columns
    (its response included); mapping = {generated column: "alias:prediction
    index"} feeds the main model's inputs from the other models' scores.
    models: {alias: MOJO zip path or bytes}."""
    from .h2o_mojo import H2OMojoModel
    loaded, blobs = {}, {}
    for alias, src in models.items():
        data = src if isinstance(src, (bytes, bytearray)) else open(src, "rb").read()
        blobs[alias] = bytes(data)
        loaded[alias] = H2OMojoModel(bytes(data))
    if main_alias not in loaded:
        raise ValueError(f"Main model is missing. There is no model with alias '{main_alias}'.")
    final = loaded[main_alias]
    schema = {}
    for alias, m in loaded.items():
        if alias == main_alias:
            continue
        for c, d in zip(m.features, m.domains[:len(m.features)]):
            if c in schema and schema[c] != d:
                raise ValueError(f"Domains of column '{c}' differ.")
            schema.setdefault(c, d)
    for c, d in zip(final.columns, final.domains):
        if c not in mapping:
            schema[c] = d
    columns = list(schema)
    domains = [schema[c] for c in columns]
    extra = {"submodel_count": len(loaded)}
    for i, alias in enumerate(loaded):
        extra[f"submodel_key_{i}"] = alias
        extra[f"submodel_dir_{i}"] = f"models/{alias}/"
    extra["generated_column_count"] = len(mapping)
    for i, (col, spec) in enumerate(mapping.items()):
        alias, idx = spec.rsplit(":", 1)
        extra[f"generated_column_name_{i}"] = col
        extra[f"generated_column_model_{i}"] = alias
        extra[f"generated_column_index_{i}"] = int(idx)
    extra["main_model"] = main_alias

    class _M:                                  # header fields of the pipeline's own descriptor
        model_id = f"pipeline_{main_alias}"
        _training_metrics = None
        _validation_metrics = None
    nf = len(columns) - (1 if final.supervised else 0)
    ini, files = _header(_M, "pipeline", "MOJO Pipeline", final.category, columns, nf, final.nclasses, domains,
                         "1.00", extra, supervised=final.supervised)
    z = _Zip()
    z.write("model.ini", ini)
    for k_, v_ in files.items():
        z.write(k_, v_)
    for alias, data in blobs.items():
        src = zipfile.ZipFile(io.BytesIO(data))
        for name in src.namelist():
            z.write(f"models/{alias}/{name}", src.read(name))
    return z.close()
