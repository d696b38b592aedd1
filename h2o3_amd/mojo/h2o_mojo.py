"""Reader + numpy scorer for MOJOs in the reference's (h2o-genmodel) layout.

The reference's MOJO zip holds `model.ini` ([info] key = value pairs, the
[columns] list, the [domains] map), `domains/dNNN.txt` level files and
per-algorithm payloads -- compressed tree byte streams `trees/tCC_GGG.bin`
(+ `_aux.bin` node statistics) for GBM / DRF, `beta` / `cat_offsets` / means
in model.ini for GLM, `center_i` for K-Means, nested sub-MOJOs under
`models/<algo>/<key>/` for Stacked Ensembles.  This module reads that layout
(zip file or unpacked directory) and scores pandas frames with vectorised
numpy, so MOJOs exported by the reference import into this platform
(`H2OGenericEstimator.from_file` / `h2o.import_mojo`).

Parity references (behaviour studied, not translated):
  hex/genmodel/ModelMojoReader.java            (ini / domain parsing)
  hex/genmodel/algos/tree/SharedTreeMojoReader.java, SharedTreeMojoModel.java:129
                                               (tree byte format, scoreTree v1.0 / 1.1 / >= 1.2)
  hex/genmodel/utils/GenmodelBitSet.java       (categorical split bitsets)
  hex/genmodel/algos/gbm/GbmMojoModel.java     (unifyPreds: init_f, link, multinomial rescale)
  hex/genmodel/algos/drf/DrfMojoModel.java     (tree averaging, binomial class-0 trees)
  hex/genmodel/algos/glm/Glm*MojoModel.java    (cat offsets, mean imputation, ordinal / multinomial)
  hex/genmodel/algos/kmeans/KMeansMojoModel.java, GenModel.KMeans_distance
  hex/genmodel/algos/ensemble/StackedEnsembleMojoModel.java (base model remap, logit transform)
  hex/genmodel/algos/coxph/CoxPHMojoModel.java, svm/SvmMojoModel.java
  h2o-genmodel-extensions/xgboost XGBoostJavaMojoModel.java, OneHotEncoderFactory.java
                                               (native booster blob: mojo/xgb_booster.py)

Instead of walking one row at a time through the byte stream (the
reference's scoreTree), every tree is decoded ONCE into flat node arrays and
all rows descend level by level together.
"""
from __future__ import annotations

import io
import math
import os
import struct
import zipfile

import numpy as np

# NaSplitDir (hex/genmodel/algos/tree/NaSplitDir.java)
_NSD_NA_VS_REST, _NSD_NA_LEFT, _NSD_LEFT = 1, 2, 4


_ALGO_BY_NAME = {
    "Distributed Random Forest": "drf", "Gradient Boosting Method": "gbm", "Gradient Boosting Machine": "gbm",
    "Generalized Low Rank Modeling": "glrm", "Generalized Low Rank Model": "glrm",
    "Generalized Linear Modeling": "glm", "Generalized Linear Model": "glm", "Generalized Additive Model": "gam",
    "Word2Vec": "word2vec", "TargetEncoder": "targetencoder", "Isolation Forest": "isolationforest",
    "Extended Isolation Forest": "extendedisolationforest", "K-means": "kmeans", "Deep Learning": "deeplearning",
    "deep learning": "deeplearning", "Support Vector Machine (*Spark*)": "svm", "StackedEnsemble": "stackedensemble",
    "Stacked Ensemble": "stackedensemble", "k-LIME": "klime", "MOJO Pipeline": "pipeline",
    "Principal Components Analysis": "pca", "Principal Component Analysis": "pca", "Cox Proportional Hazards": "coxph", "RuleFit": "rulefit",
}


# ----------------------------------------------------------------- backends
class _Backend:
    """Zip archive or directory, optionally rooted at a nested prefix (the
    Stacked Ensemble's submodel_dir_i)."""

    def __init__(self, src, prefix=""):
        self.prefix = prefix
        if isinstance(src, (_ZipSrc, _DirSrc)):
            self.src = src
        elif isinstance(src, (bytes, bytearray)):
            self.src = _ZipSrc(zipfile.ZipFile(io.BytesIO(bytes(src))))
        elif os.path.isdir(src):
            self.src = _DirSrc(src)
        else:
            self.src = _ZipSrc(zipfile.ZipFile(src))

    def nested(self, sub):
        return _Backend(self.src, self.prefix + sub)

    def exists(self, name):
        return self.src.exists(self.prefix + name)

    def read(self, name) -> bytes:
        return self.src.read(self.prefix + name)

    def text(self, name) -> list:
        return self.read(name).decode("utf-8").splitlines()


class _ZipSrc:
    def __init__(self, z):
        self.z = z
        self.names = set(z.namelist())

    def exists(self, n):
        return n in self.names

    def read(self, n):
        return self.z.read(n)


class _DirSrc:
    def __init__(self, d):
        self.d = d

    def exists(self, n):
        return os.path.exists(os.path.join(self.d, n))

    def read(self, n):
        with open(os.path.join(self.d, n), "rb") as f:
            return f.read()


def _parse_val(s: str):
    """[info] value -> python (ParseUtils.tryParse: null, booleans, numbers,
    [a, b, ...] arrays, else the raw string)."""
    s = s.strip()
    if s == "null":
        return None
    if s in ("true", "false"):
        return s == "true"
    if s.startswith("[") and s.endswith("]"):
        body = s[1:-1].strip()
        if not body:
            return []
        out = []
        for t in body.split(","):
            v = _parse_val(t)
            out.append(v)
        return out
    try:
        if s.lstrip("-").isdigit():
            return int(s)
        return float(s)          # also NaN / Infinity
    except ValueError:
        return s


def is_h2o_layout(src) -> bool:
    """True when src (path / bytes) is a reference-layout MOJO: model.ini
    without this platform's model.json."""
    try:
        b = _Backend(src)
    except Exception:
        return False
    return b.exists("model.ini") and not b.exists("model.json")


# --------------------------------------------------------------- tree decode
# AuxInfo record of trees/tXX_YYY_aux.bin (SharedTreeMojoModel.AuxInfo: 10 x 4 bytes)
_AUX_DT = np.dtype([("nid", "<i4"), ("res", "<i4"), ("wl", "<f4"), ("wr", "<f4"), ("pl", "<f4"), ("pr", "<f4"),
                    ("sel", "<f4"), ("ser", "<f4"), ("l", "<i4"), ("r", "<i4")])


class _Tree:
    """One compressed tree decoded into flat node arrays.  Children are node
    indices (>= 0) or leaves encoded as -(leaf_index + 1)."""

    __slots__ = ("col", "kind", "split", "na_left", "bs_off", "bs_n", "bs_pos", "left", "right", "leaf", "raw",
                 "root_leaf", "_nid")

    def __init__(self, buf: bytes, version: float):
        self.raw = np.frombuffer(buf, dtype=np.uint8)
        col, kind, split, na_left, bs_off, bs_n, bs_pos, left, right = ([] for _ in range(9))
        leaf = []
        self.root_leaf = None
        b = buf

        def f32(p):
            return struct.unpack_from("<f", b, p)[0]

        def u16(p):
            return struct.unpack_from("<H", b, p)[0]

        def u32(p):
            return struct.unpack_from("<i", b, p)[0]

        # explicit stack: (position, parent node index, is_right)
        if u16(1) == 65535:
            self.root_leaf = f32(3)
        else:
            stack = [(0, -1, False)]
            while stack:
                pos, parent, is_right = stack.pop()
                node_type = b[pos]
                c = u16(pos + 1)
                nsd = b[pos + 3]
                p = pos + 4
                na_vs_rest = nsd == _NSD_NA_VS_REST
                equal = node_type & 12
                k, sv, bo, bn, bp = 0, 0.0, 0, 0, 0
                if na_vs_rest:
                    k = 2
                elif equal == 0:
                    sv = f32(p)
                    p += 4
                elif equal == 8:                     # 32-bit inline bitset, offset 0
                    k, bo, bn, bp = 1, 0, 32, p
                    p += 4
                else:                                # general bitset
                    k = 1
                    bo = u16(p)
                    if version >= 1.2:
                        bn = u32(p + 2)
                        bp = p + 6
                        p = bp + ((bn - 1) >> 3) + 1
                    else:
                        nbytes = u16(p + 2)
                        bn = nbytes << 3
                        bp = p + 4
                        p = bp + nbytes
                idx = len(col)
                col.append(c)
                kind.append(k)
                split.append(sv)
                na_left.append(nsd in (_NSD_NA_LEFT, _NSD_LEFT))
                bs_off.append(bo)
                bs_n.append(bn)
                bs_pos.append(bp)
                left.append(0)
                right.append(0)
                if parent >= 0:
                    (right if is_right else left)[parent] = idx
                lmask = node_type & 51
                rmask = (node_type & 0xC0) >> 2
                # left subtree: size field of lmask+1 bytes unless it is a leaf
                if lmask & 16:
                    left[idx] = -(len(leaf) + 1)
                    leaf.append(f32(p))
                    rpos = p + 4
                else:
                    nsz = lmask + 1
                    size = int.from_bytes(b[p:p + nsz], "little")
                    lpos = p + nsz
                    rpos = lpos + size
                    stack.append((lpos, idx, False))
                if rmask & 16:
                    right[idx] = -(len(leaf) + 1)
                    leaf.append(f32(rpos))
                else:
                    stack.append((rpos, idx, True))
        self.col = np.asarray(col, dtype=np.int64)
        self.kind = np.asarray(kind, dtype=np.int8)
        self.split = np.asarray(split, dtype=np.float32).astype(np.float64)
        self.na_left = np.asarray(na_left, dtype=bool)
        self.bs_off = np.asarray(bs_off, dtype=np.int64)
        self.bs_n = np.asarray(bs_n, dtype=np.int64)
        self.bs_pos = np.asarray(bs_pos, dtype=np.int64)
        self.left = np.asarray(left, dtype=np.int64)
        self.right = np.asarray(right, dtype=np.int64)
        self.leaf = np.asarray(leaf, dtype=np.float32).astype(np.float64)

    def node_right(self, j, X, dom_len, version):
        """The scoring rule of score() for one split node j over every row."""
        c = self.col[j]
        d = X[:, c]
        nan = np.isnan(d)
        di = np.where(nan, 0, d).astype(np.int64)
        kind = self.kind[j]
        right = np.zeros(d.shape[0], dtype=bool)
        if kind == 0:
            right = d >= self.split[j]
        elif kind == 1:
            rel = di - self.bs_off[j]
            inr = (rel >= 0) & (rel < self.bs_n[j])
            relc = np.clip(rel, 0, None)
            byte = self.raw[np.minimum(self.bs_pos[j] + (relc >> 3), self.raw.size - 1)]
            right = ((byte >> (relc & 7)) & 1).astype(bool) & inr
            if version >= 1.1:
                nan = nan | ~inr
        if version >= 1.2 and dom_len is not None:
            dl = dom_len[c]
            nan = nan | ((dl > 0) & (di >= dl) & ~np.isnan(d))
        return np.where(nan, ~self.na_left[j], right)

    def shap_graph(self, aux: bytes):
        """Flat node arrays for TreeSHAP: split nodes keep their ids, leaf i
        becomes node I + i; covers from the tree's _aux.bin records (AuxInfo:
        nid, child weights, child node ids -- SharedTreeMojoModel.AuxInfo;
        the root is node id 0, children are found by the records' nidL / nidR
        as SharedTreeMojoModel.computeTreeGraph does)."""
        I, L = len(self.col), len(self.leaf)
        lt = lambda a: np.where(a >= 0, a, I + (-a - 1))   # noqa: E731
        left = np.full(I + L, -1, dtype=np.int64)
        right = np.full(I + L, -1, dtype=np.int64)
        left[:I], right[:I] = lt(self.left), lt(self.right)
        value = np.zeros(I + L)
        value[I:] = self.leaf
        feat = np.zeros(I + L, dtype=np.int64)
        feat[:I] = self.col
        cover = np.zeros(I + L)
        nid = np.zeros(I + L, dtype=np.int64)
        rec = np.frombuffer(aux, dtype=_AUX_DT) if aux else np.zeros(0, dtype=_AUX_DT)
        by_nid = {int(r["nid"]): r for r in rec}
        if I:
            r0 = by_nid[0]
            cover[0] = float(r0["wl"]) + float(r0["wr"])
            stack = [(0, 0)]
            while stack:
                j, nd = stack.pop()
                nid[j] = nd
                r = by_nid[nd]
                cover[left[j]] = float(r["wl"])
                cover[right[j]] = float(r["wr"])
                nid[left[j]], nid[right[j]] = int(r["l"]), int(r["r"])
                if self.left[j] >= 0:
                    stack.append((int(self.left[j]), int(r["l"])))
                if self.right[j] >= 0:
                    stack.append((int(self.right[j]), int(r["r"])))
        self._nid = nid
        return left, right, cover, value, feat

    def score(self, X: np.ndarray, dom_len: np.ndarray | None, version: float, paths: list | None = None) -> np.ndarray:
        """Leaf value per row of X [n, ncols] (category indices for enums).
        paths: optional list of n strings, extended in place with the row's
        'L'/'R' decisions (leaf assignment, SharedTreeMojoModel.getDecisionPath)."""
        n = X.shape[0]
        if self.root_leaf is not None:
            return np.full(n, self.root_leaf)
        out = np.empty(n)
        rows = np.arange(n)
        node = np.zeros(n, dtype=np.int64)
        while rows.size:
            c = self.col[node]
            d = X[rows, c]
            kind = self.kind[node]
            nan = np.isnan(d)
            di = np.where(nan, 0, d).astype(np.int64)
            right = np.zeros(rows.size, dtype=bool)
            num = kind == 0
            right[num] = d[num] >= self.split[node[num]]
            bsm = kind == 1
            if bsm.any():
                nb = node[bsm]
                rel = di[bsm] - self.bs_off[nb]
                inr = (rel >= 0) & (rel < self.bs_n[nb])
                relc = np.clip(rel, 0, None)
                byte = self.raw[np.minimum(self.bs_pos[nb] + (relc >> 3), self.raw.size - 1)]
                contains = ((byte >> (relc & 7)) & 1).astype(bool) & inr
                right[bsm] = contains
                if version >= 1.1:
                    tmp = nan[bsm] | ~inr
                    nan[bsm] = tmp
            if version >= 1.2 and dom_len is not None:
                dl = dom_len[c]
                nan |= (dl > 0) & (di >= dl) & ~np.isnan(d)
            go_right = np.where(nan, ~self.na_left[node], right)
            if paths is not None:
                for r, gr in zip(rows.tolist(), go_right.tolist()):
                    paths[r] += "R" if gr else "L"
            nxt = np.where(go_right, self.right[node], self.left[node])
            done = nxt < 0
            if done.any():
                out[rows[done]] = self.leaf[-nxt[done] - 1]
            keep = ~done
            rows, node = rows[keep], nxt[keep]
        return out


# ------------------------------------------------------------- native walk
_FOREST = [False, None]


def _forest_lib():
    """libmojo_forest.so (h2o3_amd/native/mojo_forest.cpp, built with the
    other native libraries) via ctypes, or None (numpy walk)."""
    if _FOREST[0]:
        return _FOREST[1]
    _FOREST[0] = True
    if os.environ.get("H2O3_MOJO_NATIVE", "1") != "1":
        return None
    import ctypes
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ops", "lib", "libmojo_forest.so")
    if not os.path.exists(p):
        return None
    try:
        lib = ctypes.CDLL(p)
    except OSError:
        return None
    cv = ctypes.c_void_p
    lib.h2o_mojo_forest_score.argtypes = [ctypes.c_longlong, ctypes.c_int, cv, ctypes.c_int] + [cv] * 18 + \
        [ctypes.c_int, cv, ctypes.c_double, cv, ctypes.c_int]
    _FOREST[1] = lib
    return lib


def _pack_forest(trees):
    """[(output column, _Tree)] -> contiguous arrays of the native walk."""
    cat = lambda xs, dt: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(0), dtype=dt)  # noqa: E731
    ts = [t for _, t in trees]
    nn = [0 if t.root_leaf is not None else len(t.col) for t in ts]
    nl = [0 if t.root_leaf is not None else len(t.leaf) for t in ts]
    nr = [t.raw.size for t in ts]
    off = lambda v: np.ascontiguousarray(np.concatenate([[0], np.cumsum(v)]), dtype=np.int64)  # noqa: E731
    live = [t for t in ts if t.root_leaf is None]
    pk = {
        "ntrees": len(ts),
        "node_off": off(nn), "leaf_off": off(nl), "raw_off": off(nr),
        "raw_len": np.ascontiguousarray(nr, dtype=np.int64),
        "col": cat([t.col for t in live], np.int32), "kind": cat([t.kind for t in live], np.int8),
        "split": cat([t.split for t in live], np.float64), "na_left": cat([t.na_left for t in live], np.uint8),
        "bs_off": cat([t.bs_off for t in live], np.int64), "bs_n": cat([t.bs_n for t in live], np.int64),
        "bs_pos": cat([t.bs_pos for t in live], np.int64), "left": cat([t.left for t in live], np.int64),
        "right": cat([t.right for t in live], np.int64), "leaf": cat([t.leaf for t in live], np.float64),
        "raw": cat([t.raw for t in ts], np.uint8),
        "root_leaf": np.ascontiguousarray([t.root_leaf if t.root_leaf is not None else 0.0 for t in ts],
                                          dtype=np.float64),
        "has_root": np.ascontiguousarray([t.root_leaf is not None for t in ts], dtype=np.uint8),
        "tree_out": np.ascontiguousarray([o for o, _ in trees], dtype=np.int32),
    }
    return pk


def _forest_score(lib, pk, X, preds, version, dom_len):
    import ctypes
    Xc = np.ascontiguousarray(X, dtype=np.float64)
    dl = None if dom_len is None else np.ascontiguousarray(dom_len, dtype=np.int32)
    P = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert preds.flags.c_contiguous and preds.dtype == np.float64
    rc = lib.h2o_mojo_forest_score(
        Xc.shape[0], Xc.shape[1], P(Xc), pk["ntrees"], P(pk["node_off"]), P(pk["leaf_off"]), P(pk["raw_off"]),
        P(pk["raw_len"]), P(pk["col"]), P(pk["kind"]), P(pk["split"]), P(pk["na_left"]), P(pk["bs_off"]),
        P(pk["bs_n"]), P(pk["bs_pos"]), P(pk["left"]), P(pk["right"]), P(pk["leaf"]), P(pk["raw"]),
        P(pk["root_leaf"]), P(pk["has_root"]), P(pk["tree_out"]), preds.shape[1], P(preds), float(version), P(dl),
        int(os.environ.get("H2O3_MOJO_THREADS", "0")))
    if rc != 0:
        raise RuntimeError(f"h2o_mojo_forest_score failed: {rc}")


# ------------------------------------------------------------------- models
class H2OMojoModel:
    """A reference-layout MOJO.  predict(df) returns the reference's output
    columns (predict, p0, p1, ... / cluster / predict); predict_raw(df)
    returns the class-probability (or value) matrix used by Generic metrics."""

    def __init__(self, src, backend: _Backend | None = None):
        self.be = backend if backend is not None else _Backend(src)
        self.info, self.columns, dom_files = self._parse_ini()
        # ModelMojoFactory dispatches on the long "algorithm" name; "algo" is
        # missing from some early MOJOs
        self.algo = _ALGO_BY_NAME.get(str(self.info.get("algorithm")), str(self.info.get("algo")))
        self.version = float(self.info.get("mojo_version", 1.0))
        self.nclasses = int(self.info.get("n_classes", 1) or 1)
        self.nfeatures = int(self.info.get("n_features", len(self.columns)))
        self.supervised = bool(self.info.get("supervised", False))
        self.category = str(self.info.get("category", ""))
        self.default_threshold = float(self.info.get("default_threshold", 0.5) or 0.5)
        self.domains = [None] * len(self.columns)
        esc = bool(self.info.get("escape_domain_values", False))
        for ci, (cnt, fname) in dom_files.items():
            if ci >= len(self.columns):
                continue
            lines = self.be.text("domains/" + fname)
            if esc:
                lines = [ln.replace("\\n", "\n") for ln in lines]
            if len(lines) < cnt:
                raise ValueError(f"domain file {fname}: {len(lines)} levels, expected {cnt}")
            self.domains[ci] = lines[:cnt]
        self.response = self.columns[-1] if self.supervised else None
        self.features = self.columns[:self.nfeatures]
        self.response_domain = self.domains[-1] if self.supervised else None
        self.dom_len = np.array([len(d) if d is not None else 0 for d in self.domains], dtype=np.int64)
        self.meta = {"algo": self.algo, "x": list(self.features), "response": self.response,
                     "nclasses": self.nclasses, "response_domain": self.response_domain, "format": "h2o"}
        loader = getattr(self, f"_load_{self.algo}", None)
        if loader is None:
            raise NotImplementedError(f"reference MOJO algo '{self.algo}' is not supported by this reader")
        loader()
        # the original model's ModelSchemaV3 JSON (ModelMojoWriter.writeModelDetails;
        # read by hex.genmodel.attributes.ModelJsonReader)
        self.details = None
        if self.be.exists("experimental/modelDetails.json"):
            import json
            self.details = json.loads(self.be.read("experimental/modelDetails.json").decode("utf-8"))

    # ------------------------------------------------------------ ini parse
    def _parse_ini(self):
        info, cols, doms = {}, [], {}
        sec = None
        for line in self.be.text("model.ini"):
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            if line in ("[info]", "[columns]", "[domains]"):
                sec = line
                continue
            if sec == "[info]":
                k, _, v = line.partition("=")
                k = k.strip()
                info[k] = v.strip() if k == "uuid" else _parse_val(v)
            elif sec == "[columns]":
                cols.append(line)
            elif sec == "[domains]":
                ci, _, rest = line.partition(":")
                cnt, _, fname = rest.strip().partition(" ")
                doms[int(ci)] = (int(cnt), fname.strip())
        return info, cols, doms

    def kv(self, k, default=None):
        v = self.info.get(k, default)
        return default if v is None else v

    # -------------------------------------------------------------- loaders
    def _load_trees(self):
        tpc = self.info.get("n_trees_per_class")
        if tpc is None:
            bdt = self.info.get("binomial_double_trees")
            tpc = 1 if (self.nclasses == 2 and not bdt) else self.nclasses
        self.ntree_groups = int(self.kv("n_trees", 0))
        self.ntrees_per_group = int(tpc)
        self.trees = [[None] * self.ntree_groups for _ in range(self.ntrees_per_group)]
        for j in range(self.ntree_groups):
            for i in range(self.ntrees_per_group):
                name = "trees/t%02d_%03d.bin" % (i, j)
                if self.be.exists(name):
                    self.trees[i][j] = _Tree(self.be.read(name), self.version)
        self.calib_beta = None
        if self.info.get("calib_method") is not None:
            if self.info["calib_method"] != "platt":
                raise ValueError(f"unknown calibration method {self.info['calib_method']}")
            self.calib_beta = list(self.kv("calib_glm_beta", []))
        enc = str(self.kv("_genmodel_encoding", "AUTO")) if self.version >= 1.40 else "AUTO"
        self.catenc = self._orig_encoding(enc)

    def _load_gbm(self):
        self._load_trees()
        self.family = str(self.kv("distribution"))
        self.init_f = float(self.kv("init_f", 0.0))
        link = self.info.get("link_function")
        if link is None:
            link = {"bernoulli": "logit", "fractionalbinomial": "logit", "quasibinomial": "logit",
                    "modified_huber": "logit", "ordinal": "logit", "multinomial": "log", "poisson": "log",
                    "gamma": "log", "tweedie": "log"}.get(self.family, "identity")
        self.link = str(link)

    def _load_drf(self):
        self._load_trees()
        self.binomial_double_trees = bool(self.kv("binomial_double_trees", False))

    def _load_glm(self):
        self.use_all_levels = bool(self.kv("use_all_factor_levels", False))
        self.cats = int(self.kv("cats", -1))
        self.cat_modes = list(self.kv("cat_modes", []))
        self.cat_offsets = list(self.kv("cat_offsets", [0]))
        self.nums = int(self.kv("nums", -1))
        self.num_means = list(self.kv("num_means", []))
        self.mean_imputation = bool(self.kv("mean_imputation", False))
        self.beta = np.asarray(self.kv("beta"), dtype=np.float64)
        self.family = str(self.kv("family"))
        self.glm_link = str(self.kv("link", "identity"))
        self.tweedie_link_power = float(self.kv("tweedie_link_power", 0.0))

    def _load_kmeans(self):
        self.standardize = bool(self.kv("standardize", False))
        if self.standardize:
            self.km_means = np.asarray(self.kv("standardize_means"), dtype=np.float64)
            mults = self.info.get("standardize_mults")
            self.km_mults = None if mults is None else np.asarray(mults, dtype=np.float64)
            self.km_modes = np.asarray(self.kv("standardize_modes"), dtype=np.int64)
        k = int(self.kv("center_num"))
        self.centers = np.asarray([self.kv(f"center_{i}") for i in range(k)], dtype=np.float64)

    def _load_rulefit(self):
        """RuleFitMojoReader: the linear model (a nested GLM MOJO), the rule
        ensemble per (depth, tree) and the linear-name mapping."""
        key = str(self.kv("linear_model"))
        d = None
        for i in range(int(self.kv("submodel_count", 0))):
            if str(self.kv(f"submodel_key_{i}")) == key:
                d = str(self.kv(f"submodel_dir_{i}"))
        self.rf_linear = H2OMojoModel(None, backend=self.be.nested(d))
        self.rf_type = int(self.kv("model_type"))
        self.rf_depth, self.rf_ntrees = int(self.kv("depth")), int(self.kv("ntrees"))
        self.rf_rules = {}
        if self.rf_type != 0:
            for i in range(self.rf_depth):
                for j in range(self.rf_ntrees):
                    rules = []
                    for k in range(int(self.kv(f"num_rules_M{i}T{j}"))):
                        rid = f"{i}_{j}_{k}"
                        conds = []
                        for c in range(int(self.kv(f"num_conditions_rule_id_{rid}"))):
                            cid = f"{c}_{rid}"
                            typ, op = int(self.kv(f"type_{cid}")), int(self.kv(f"operator_{cid}"))
                            if typ == 0:
                                thr = [int(self.kv(f"cat_treshold_length_{t}_{cid}"))
                                       for t in range(int(self.kv(f"cat_treshold_length_{cid}")))]
                            else:
                                thr = float(self.kv(f"num_treshold{cid}"))
                            conds.append((int(self.kv(f"feature_index_{cid}")), typ, op, thr,
                                          bool(self.kv(f"nas_included_{cid}"))))
                        rules.append((str(self.kv(f"var_name_rule_id_{rid}")), conds))
                    self.rf_rules[(i, j)] = rules
        self.rf_linear_names = [str(self.kv(f"linear_names_{i}")) for i in range(int(self.kv("linear_names_len")))]

    def _load_glrm(self):
        """GlrmMojoReader (mojo 1.10): permutation / normalisation, one
        GlrmLoss per permuted column, archetypes [nrowY][ncolY] big-endian."""
        self.gl_ncolA, self.gl_ncolY = int(self.kv("ncolA")), int(self.kv("ncolY"))
        self.gl_nrowY, self.gl_ncolX = int(self.kv("nrowY")), int(self.kv("ncolX"))
        self.gl_regx = str(self.kv("regularizationX", "None"))
        self.gl_gammax = float(self.kv("gammaX", 0.0))
        self.gl_ncats, self.gl_nnums = int(self.kv("num_categories")), int(self.kv("num_numeric"))
        self.gl_sub = np.asarray(self.kv("norm_sub", []) or [], dtype=np.float64)
        self.gl_mul = np.asarray(self.kv("norm_mul", []) or [], dtype=np.float64)
        self.gl_perm = [int(v) for v in self.kv("cols_permutation")]
        self.gl_losses = [ln.strip() for ln in self.be.text("losses") if ln.strip()][:self.gl_ncolA]
        self.gl_levels = [int(v) for v in (self.kv("num_levels_per_category", []) or [])]
        raw = self.be.read("archetypes")
        self.gl_Y = np.frombuffer(raw, dtype=">f8", count=self.gl_nrowY * self.gl_ncolY).astype(np.float64) \
            .reshape(self.gl_nrowY, self.gl_ncolY)
        self.gl_seed = int(self.kv("seed", 0))
        self.gl_reverse = bool(self.kv("reverse_transform", True))
        self.gl_rcnt = 0                      # GlrmMojoModel._rcnt: row counter added to the seed

    def _glrm_obj_grad(self, x, A, want_grad):
        """GlrmMojoModel.objective / gradientL for every row at once."""
        n = x.shape[0]
        Y = self.gl_Y
        obj = np.zeros(n)
        grad = np.zeros_like(x) if want_grad else None
        off = 0
        for j in range(self.gl_ncats):
            L = self.gl_levels[j]
            a = A[:, j]
            ok = ~np.isnan(a)
            ai = np.where(ok, a, 0).astype(np.int64)
            u = x @ Y[:, off:off + L]
            r = np.arange(n)
            if self.gl_losses[j] == "Ordinal":
                ar = np.arange(L).reshape(1, -1)
                below = (ar < ai.reshape(-1, 1)) & (ar < L - 1)
                lo = np.where(below, np.maximum(1 - u, 0), np.where(ar < L - 1, 1.0, 0.0)).sum(1)
                gl = np.where(below & (1 - u > 0), -1.0, 0.0)
            else:
                ua = u[r, ai]
                lo = np.maximum(1 + u, 0).sum(1) + np.maximum(1 - ua, 0) - np.maximum(1 + ua, 0)
                gl = (1 + u > 0).astype(np.float64)
                gl[r, ai] = np.where(1 - ua > 0, -1.0, 0.0)
            obj += np.where(ok, lo, 0.0)
            if want_grad:
                grad += np.where(ok[:, None], gl @ Y[:, off:off + L].T, 0.0)
            off += L
        for j in range(self.gl_ncats, self.gl_ncolA):
            js = j - self.gl_ncats
            a = (A[:, j] - self.gl_sub[js]) * self.gl_mul[js]
            ok = ~np.isnan(a)
            a0 = np.where(ok, a, 0.0)
            u = x @ Y[:, off + js]
            lo, gl = _glrm_loss(self.gl_losses[j], u, a0)
            obj += np.where(ok, lo, 0.0)
            if want_grad:
                grad += np.where(ok, gl, 0.0)[:, None] * Y[:, off + js][None, :]
        obj += self.gl_gammax * _glrm_regularize(self.gl_regx, x)
        return obj, grad

    def _score_glrm(self, X):
        """GlrmMojoModel.score0: x from N(0, 1) draws of java.util.Random(seed
        + row counter), projected by the X regulariser, then up to 100
        proximal-gradient steps, each trying the 10 step sizes 0.5^i (scaled
        by 1/obj when obj > 10) and keeping the best; a row stops once its
        relative improvement is negative or below 1e-10."""
        n = X.shape[0]
        k = self.gl_ncolX
        A = self.glrm_row_data(X)
        seeds = self.gl_seed + self.gl_rcnt + np.arange(n, dtype=np.int64)
        self.gl_rcnt += n
        x = _JavaRandom(seeds).gaussians(k)
        x = _glrm_prox(self.gl_regx, x, 1.0, project=True)
        alphas = 0.5 ** np.arange(1, 11)
        old, _ = self._glrm_obj_grad(x, A, False)
        live = np.ones(n, dtype=bool)
        for _ in range(100):
            if not live.any():
                break
            _, g = self._glrm_obj_grad(x, A, True)
            scale = np.where(old > 10, 1.0 / np.where(old == 0, 1.0, old), 1.0)
            best = np.full(n, np.finfo(np.float64).max)
            bestx = np.zeros_like(x)
            hit0 = np.zeros(n, dtype=bool)
            for al in alphas:
                a_ = (al * scale)[:, None]
                xn = _glrm_prox(self.gl_regx, x - a_ * g, a_[:, 0] * self.gl_gammax)
                on, _ = self._glrm_obj_grad(xn, A, False)
                take = (best > on) & ~hit0
                bestx[take] = xn[take]
                best = np.where(take, on, best)
                hit0 |= on == 0
            zero = old == 0                                     # applyBestAlpha: already at zero loss
            obj = np.where(zero, 0.0, best)
            upd = live & ~zero & (best < old)
            x[upd] = bestx[upd]
            with np.errstate(divide="ignore", invalid="ignore"):
                imp = 1 - obj / old
            live &= ~((imp < 0) | (imp < 1e-10))
            old = np.where(live | upd, obj, old)
        self.glrm_x = x
        return x

    def glrm_row_data(self, X):
        """GlrmMojoModel.getRowData: the permuted row (categoricals first),
        unseen categorical levels as NA."""
        A = np.empty((X.shape[0], self.gl_ncolA))
        for i in range(self.gl_ncats):
            v = X[:, self.gl_perm[i]]
            A[:, i] = np.where(v >= self.gl_levels[i], np.nan, v)
        for i in range(self.gl_ncats, self.gl_ncolA):
            A[:, i] = X[:, self.gl_perm[i]]
        return A

    def glrm_impute(self, x):
        """GlrmMojoModel.impute_data: the reconstructed row (categorical level
        indices and numerics, back-transformed when reverse_transform)."""
        n = x.shape[0]
        out = np.zeros((n, self.gl_ncolA))
        Y = self.gl_Y
        off = 0
        for d in range(self.gl_ncats):
            L = self.gl_levels[d]
            u = x @ Y[:, off:off + L]
            if self.gl_losses[d] == "Ordinal" and L > 1:
                loss = np.concatenate([np.zeros((n, 1)), -np.cumsum(np.minimum(u[:, :L - 1], 1.0), 1)], 1)
                lv = np.zeros(n, dtype=np.int64)
                bl = loss[:, 0].copy()
                for a in range(1, L):
                    b = loss[:, a] < bl
                    lv[b] = a
                    bl[b] = loss[b, a]
            else:
                lv = u.argmax(1)
            out[:, self.gl_perm[d]] = lv
            off += L
        for d in range(self.gl_ncats, self.gl_ncolA):
            ds = d - self.gl_ncats
            v = _glrm_loss_impute(self.gl_losses[d], x @ Y[:, off + ds])
            if self.gl_reverse:
                v = v / self.gl_mul[ds] + self.gl_sub[ds]
            out[:, self.gl_perm[d]] = v
        return out

    def _load_gam(self):
        """GamMojoReader: the GLM part (scored by the GLM scorer on
        beta_center) and per smoother (bs-sorted: cubic regression, I-spline,
        thin plate) the knots, Z', B^-1 D, zCS', polynomial exponents and raw
        means / inverse standard deviations."""
        fam = str(self.kv("family"))
        self.family = {"bernoulli": "binomial"}.get(fam, fam)
        self.glm_link = str(self.kv("link", "identity"))
        self.tweedie_link_power = float(self.kv("tweedie_link_power", 0.0))
        self.use_all_levels = bool(self.kv("use_all_factor_levels", False))
        self.cats = int(self.kv("cats", -1))
        self.cat_offsets = list(self.kv("cat_offsets", [0]))
        self.nums = int(self.kv("numsCenter"))
        self.mean_imputation = bool(self.kv("mean_imputation", False))
        self.cat_modes = list(self.kv("catNAFills", []) or [])
        self.num_means = list(self.kv("numNAFillsCenter", []) or [])
        K = self.nclasses
        if self.family in ("multinomial", "ordinal"):
            L = int(self.kv("beta center length per class"))
            self.beta = np.frombuffer(self.be.read("beta_multinomial_centering"), dtype=">f8",
                                      count=K * L).astype(np.float64)
        else:
            self.beta = np.asarray(self.kv("beta_center"), dtype=np.float64)
        nk = [int(v) for v in self.kv("num_knots_sorted")]
        bs = [int(v) for v in self.kv("bs_sorted")]
        dims = [int(v) for v in self.kv("_d")]
        cols = self.be.text("gam_columns_sorted")
        ng = len(nk)
        self.gm_cols, p = [], 0
        for g in range(ng):
            self.gm_cols.append(cols[p:p + dims[g]])
            p += dims[g]
        orders = [int(v) for v in (self.kv("spline_orders_sorted", []) or [])]
        ntp = int(self.kv("num_TP_col", 0))
        Ms = [int(v) for v in (self.kv("_M", []) or [])]
        kb = io.BytesIO(self.be.read("knots"))
        zb = io.BytesIO(self.be.read("zTranspose"))
        rd = lambda b, r, c: np.frombuffer(b.read(8 * r * c), dtype=">f8").astype(np.float64).reshape(r, c)  # noqa
        self.gm = []
        ti = 0
        binv = io.BytesIO(self.be.read("_binvD")) if self.be.exists("_binvD") else None
        if ntp:
            zcs = io.BytesIO(self.be.read("zTransposeCS"))
            poly = io.BytesIO(self.be.read("polynomialBasisList"))
            mraw = io.BytesIO(self.be.read("gamColMeansRaw"))
            sraw = io.BytesIO(self.be.read("gamColStdRaw"))
        std = bool(self.kv("standardize", False))
        for g in range(ng):
            k = nk[g]
            knots = rd(kb, dims[g], k)
            nb = k + orders[g] - 2 if bs[g] == 2 else k - 1
            zt = rd(zb, nb, k)
            e = {"bs": bs[g], "knots": knots, "zt": zt, "ncen": nb}
            if bs[g] == 0:
                e["binvD"] = rd(binv, k - 2, k)
            elif bs[g] == 2:
                e["order"] = orders[g]
            elif bs[g] == 1:
                M = Ms[ti]
                d = dims[g]
                e["zcsT"] = rd(zcs, k - M, k)
                e["terms"] = np.frombuffer(poly.read(4 * M * d), dtype=">i4").astype(np.int64).reshape(M, d)
                e["means"] = rd(mraw, 1, d)[0]
                e["ostd"] = rd(sraw, 1, d)[0]
                e["standardize"] = std
                ti += 1
            else:
                raise NotImplementedError(f"GAM spline type {bs[g]}")
            self.gm.append(e)
        self.gm_start = self.nfeatures - int(self.kv("num_expanded_gam_columns_center"))

    def _gamify(self, df, X):
        """GamMojoModelBase.addExpandGamCols: when the centred smoother columns
        are absent, evaluate every smoother from its raw input column(s) (a
        missing input leaves its columns NA for mean imputation)."""
        from .gam_np import ispline_basis, tp_constant
        if not np.all(np.isnan(X[:, self.gm_start:self.nfeatures])):
            return
        j = self.gm_start
        n = X.shape[0]
        for gi, e in enumerate(self.gm):
            cols = []
            for c in self.gm_cols[gi]:
                cols.append(np.asarray(pd_numeric(df[c]) if c in df else np.full(n, np.nan), dtype=np.float64))
            V = np.stack(cols, 1)
            ok = ~np.isnan(V).any(1)
            Vz = np.where(np.isnan(V), 0.0, V)
            if e["bs"] == 0:
                kn = e["knots"][0]
                x = Vz[:, 0]
                k = kn.size
                h = np.diff(kn)
                b = np.clip(np.searchsorted(kn, x, side="right") - 1, 0, k - 2)
                cm = ((kn[b + 1] - x) ** 3 / h[b] - h[b] * (kn[b + 1] - x)) / 6
                cp = ((x - kn[b]) ** 3 / h[b] - h[b] * (x - kn[b])) / 6
                Fp = np.vstack([np.zeros(k), e["binvD"], np.zeros(k)])
                B = cm[:, None] * Fp[b] + cp[:, None] * Fp[b + 1]
                r = np.arange(n)
                B[r, b] += (kn[b + 1] - x) / h[b]
                B[r, b + 1] += (x - kn[b]) / h[b]
                out = B @ e["zt"].T
            elif e["bs"] == 2:
                out = ispline_basis(Vz[:, 0], e["knots"][0], e["order"])
            else:
                kn = e["knots"].T                                   # [k, d]
                d = kn.shape[1]
                m = (d + 1) // 2 + 1
                diff = Vz[:, None, :] - kn[None, :, :]
                if e["standardize"]:
                    diff = diff * e["ostd"]
                dist = np.sqrt((diff * diff).sum(-1)) ** (2 * m - d)
                E = tp_constant(m, d) * dist
                if d % 2 == 0:
                    E = np.where(dist != 0, E * np.log(np.where(dist != 0, dist, 1.0)), E)
                Vp = Vz - e["means"] * e["ostd"] if e["standardize"] else Vz
                P = np.stack([np.prod(Vp ** t, 1) for t in e["terms"].astype(np.float64)], 1)
                out = np.concatenate([E @ e["zcsT"].T, P], 1) @ e["zt"].T
            X[:, j:j + e["ncen"]] = np.where(ok[:, None], out, np.nan)
            j += e["ncen"]

    def _score_gam(self, X):
        return self._score_glm(X)

    def _load_pipeline(self):
        """MojoPipelineReader: sub-models under models/<alias>/, the main
        model's generated input columns (generated_column_name_i <- prediction
        generated_column_index_i of sub-model generated_column_model_i), the
        other main-model inputs taken from the pipeline row by name."""
        subs = {}
        for i in range(int(self.kv("submodel_count", 0))):
            subs[str(self.kv(f"submodel_key_{i}"))] = H2OMojoModel(
                None, backend=self.be.nested(str(self.kv(f"submodel_dir_{i}"))))
        main_alias = str(self.kv("main_model"))
        self.pl_main = subs[main_alias]
        gen = []
        for i in range(int(self.kv("generated_column_count", 0))):
            gen.append((str(self.kv(f"generated_column_name_{i}")), str(self.kv(f"generated_column_model_{i}")),
                        int(self.kv(f"generated_column_index_{i}", 0))))
        names = list(self.columns)
        gen_names = {g[0] for g in gen}
        mf = self.pl_main.features
        self.pl_direct = [(mf.index(c), names.index(c)) for c in mf if c not in gen_names]
        self.pl_subs = []
        for alias, m in subs.items():
            if alias == main_alias:
                continue
            inp = [names.index(c) for c in m.features]
            outs = [(mf.index(g[0]), g[2]) for g in gen if g[1] == alias]
            self.pl_subs.append((m, np.asarray(inp, dtype=np.int64), outs))
        self.nclasses = self.pl_main.nclasses
        self.category = self.pl_main.category
        self.response_domain = self.pl_main.response_domain
        self.default_threshold = self.pl_main.default_threshold

    def _score_pipeline(self, X):
        """MojoPipeline.score0: sub-model predictions fill the generated
        columns of the main model's input row, then the main model scores."""
        n = X.shape[0]
        row = np.full((n, len(self.pl_main.columns)), np.nan)
        for t, s_ in self.pl_direct:
            row[:, t] = X[:, s_]
        for m, inp, outs in self.pl_subs:
            sub = np.full((n, len(m.columns)), np.nan)
            sub[:, :inp.size] = X[:, inp]
            preds = m.score0(sub)
            for t, j in outs:
                row[:, t] = preds[:, j]
        return self.pl_main.score0(row)

    def _load_stackedensemble(self):
        subs = {}
        for i in range(int(self.kv("submodel_count", 0))):
            key = str(self.kv(f"submodel_key_{i}"))
            subs[key] = H2OMojoModel(None, backend=self.be.nested(str(self.kv(f"submodel_dir_{i}"))))
        tr = str(self.kv("metalearner_transform", "NONE"))
        if tr not in ("NONE", "Logit"):
            raise NotImplementedError(f"metalearner transform {tr}")
        self.logit_transform = tr == "Logit"
        self.metalearner = subs[str(self.kv("metalearner"))]
        self.base = []
        for i in range(int(self.kv("base_models_num", 0))):
            key = self.info.get(f"base_model{i}")
            if key is None:
                self.base.append(None)
                continue
            m = subs[str(key)]
            mapping = []
            for f in m.features:
                if f not in self.columns:
                    raise ValueError(f"model {key} needs input column {f} missing from the ensemble")
                mapping.append(self.columns.index(f))
            self.base.append((m, np.asarray(mapping, dtype=np.int64)))

    def _load_isolationforest(self):
        self._load_trees()
        self.min_path_length = int(self.kv("min_path_length", 0))
        self.max_path_length = int(self.kv("max_path_length", 0))
        self.output_anomaly_flag = bool(self.kv("output_anomaly_flag", False))

    def _load_extendedisolationforest(self):
        self.eif_ntrees = int(self.kv("ntrees", 0))
        self.eif_sample_size = int(self.kv("sample_size", 0))
        self.eif_trees = [self._eif_decode(self.be.read("trees/t%02d.bin" % t)) for t in range(self.eif_ntrees)]

    @staticmethod
    def _eif_decode(buf):
        """ExtendedIsolationForestMojoModel tree blob (little endian): int32 branching-array size
        k, then records (int32 node number, 'N' + k normal f64 + k point f64 |
        'L' + int32 rows), node numbers heap-ordered (children 2i+1, 2i+2)."""
        k = struct.unpack_from("<i", buf, 0)[0]
        p = 4
        nodes = {}
        while p + 5 <= len(buf):
            num = struct.unpack_from("<i", buf, p)[0]
            typ = buf[p + 4]
            p += 5
            if typ == ord("N"):
                v = np.frombuffer(buf, dtype="<f8", count=2 * k, offset=p).astype(np.float64)
                nodes[num] = ("N", v[:k], v[k:])
                p += 16 * k
            elif typ == ord("L"):
                nodes[num] = ("L", struct.unpack_from("<i", buf, p)[0])
                p += 4
            else:
                break      # zero padding after the last record (the blob is a fixed-size buffer)
        return nodes

    def _load_word2vec(self):
        vocab = int(self.kv("vocab_size", -1))
        vec = int(self.kv("vec_size", -1))
        raw = self.be.read("vectors")
        if len(raw) != vocab * vec * 4:
            raise ValueError(f"corrupted word2vec vectors: {len(raw)} bytes")
        V = np.frombuffer(raw, dtype=">f4").astype(np.float32).reshape(vocab, vec)
        words = [w.strip().replace("\\n", "\n") for w in self.be.text("vocabulary")]
        if len(words) != vocab:
            raise ValueError("corrupted word2vec vocabulary")
        self.vec_size = vec
        self.embeddings = {w: V[i] for i, w in enumerate(words)}

    def _load_pca(self):
        """PCAMojoReader: k components, categorical offsets, normSub / normMul
        of the numerics, the eigenvectors as a BIG-endian double blob
        (java.nio.ByteBuffer default order), [eigenvector_size][k]."""
        self.pca_k = int(self.kv("k"))
        self.pca_use_all = bool(self.kv("use_all_factor_levels", False))
        self.pca_perm = list(self.kv("permutation", []))
        self.pca_ncats = int(self.kv("ncats", 0))
        self.pca_nnums = int(self.kv("nnums", 0))
        self.pca_norm_sub = list(self.kv("normSub", [])) if self.pca_nnums else []
        self.pca_norm_mul = list(self.kv("normMul", [])) if self.pca_nnums else []
        self.pca_cat_offsets = list(self.kv("catOffsets", [0]))
        size = int(self.kv("eigenvector_size"))
        raw = self.be.read("eigenvectors_raw")
        self.pca_evecs = np.frombuffer(raw, dtype=">f8", count=size * self.pca_k).astype(np.float64) \
            .reshape(size, self.pca_k)

    def _load_xgboost(self):
        """XGBoostMojoReader.java:14: one-hot layout keys + the native booster
        blob (mojo/xgb_booster.py); cats come first in the column order."""
        from .xgb_booster import Booster
        self.xgb_nums = int(self.kv("nums", 0))
        self.xgb_cats = int(self.kv("cats", 0))
        self.xgb_cat_offsets = np.asarray(self.kv("cat_offsets", [0]), dtype=np.int64)
        self.xgb_use_all = bool(self.kv("use_all_factor_levels", True))
        self.xgb_sparse = bool(self.kv("sparse", False))
        if bool(self.kv("has_offset", False)):
            raise NotImplementedError("XGBoost MOJOs trained with an offset column are not supported")
        self.booster = Booster.parse(self.be.read("boosterBytes"))
        if self.be.exists("auxNodeWeights"):
            self._xgb_aux_weights(self.be.read("auxNodeWeights"))
        self.calib_beta = None
        if self.info.get("calib_method") is not None:
            if self.info["calib_method"] != "platt":
                raise ValueError(f"unknown calibration method {self.info['calib_method']}")
            self.calib_beta = list(self.kv("calib_glm_beta", []))

    def _xgb_aux_weights(self, raw):
        """AuxNodeWeightsHelper.java: int32 tree count, then per tree an int32
        node count and that many f64 node weights (big endian), replacing the
        booster's hessian sums (weighted training)."""
        p = 0
        nt = struct.unpack_from("<i", raw, p)[0]
        p += 4
        for t in range(nt):
            nn = struct.unpack_from("<i", raw, p)[0]
            p += 4
            w = np.frombuffer(raw, dtype="<f8", count=nn, offset=p)
            p += 8 * nn
            if t < len(self.booster.trees):
                self.booster.trees[t][1]["sum_hess"][:nn] = w

    def _load_targetencoder(self):
        """TargetEncoderMojoReader.java: per-column encoding maps (level ->
        numerator, denominator[, target class]; the last level is NA), the NA
        presence map, blending parameters and the input -> output column
        maps (legacy MOJOs without maps encode every mapped column to
        <col>_te / <col>_<k>_te)."""
        d = "feature_engineering/target_encoding/"
        self.te_blend = bool(self.kv("with_blending", False))
        self.te_k = float(self.kv("inflection_point", 0.0) or 0.0)
        self.te_f = float(self.kv("smoothing", 0.0) or 0.0)
        self.te_maps = {}
        sec = None
        for line in self.be.text(d + "encoding_map.ini"):
            line = line.strip()
            if not line:
                continue
            if line.startswith("[") and line.endswith("]"):
                sec = line[1:-1]
                self.te_maps[sec] = {}
                continue
            lev, _, rest = line.partition("=")
            vals = [float(t) for t in rest.split()]
            tc = int(vals[2]) if len(vals) > 2 else -1
            self.te_maps[sec].setdefault(int(lev.strip()), {})[tc] = (vals[0], vals[1])
        self.te_has_na = {}
        if self.be.exists(d + "te_column_name_to_missing_values_presence.ini"):
            for line in self.be.text(d + "te_column_name_to_missing_values_presence.ini"):
                if "=" in line:
                    k, _, v = line.partition("=")
                    self.te_has_na[k.strip()] = int(v.strip()) == 1

        def maps(name):
            out, cur, key = [], None, None
            if not self.be.exists(d + name):
                return out
            for line in self.be.text(d + name):
                if line in ("[from]", "[to]", "[to_domain]"):
                    if line == "[from]":
                        cur = {"from": [], "to": [], "to_domain": []}
                        out.append(cur)
                    key = line[1:-1]
                    continue
                if cur is not None and line:
                    cur[key].append(line)
            return out
        self.te_inenc = maps("input_encoding_columns_map.ini")
        self.te_inout = maps("input_output_columns_map.ini")
        nout = self.nclasses - 1 if self.nclasses > 1 else 1
        if not self.te_inenc:
            for c in self.te_maps:
                self.te_inenc.append({"from": [c], "to": [c], "to_domain": []})
                outs = [f"{c}_{i + 1}_te" for i in range(nout)] if nout > 1 else [f"{c}_te"]
                self.te_inout.append({"from": [c], "to": outs, "to_domain": []})
        for m in self.te_inenc:
            if len(m["from"]) > 1:
                raise NotImplementedError("target-encoding MOJOs over column interactions are not supported")
        self.te_out_names = [n for m in self.te_inout for n in m["to"]]

    def _te_prior(self, enc, tc):
        num = sum(v[tc][0] for v in enc.values())
        den = sum(v[tc][1] for v in enc.values())
        return num / den

    def _score_targetencoder(self, X):
        """TargetEncoderMojoModel.score0: posterior mean num / den of the
        row's level (blended with the prior by lambda = 1 / (1 + exp((k - n)
        / f)) when blending); missing / unseen levels use the NA level if the
        column had NAs in training, else the prior."""
        cols = {c: i for i, c in enumerate(self.columns)}
        tcs = list(range(1, self.nclasses)) if self.nclasses > 2 else [-1]
        outs = []
        for m in self.te_inenc:
            c, te = m["from"][0], m["to"][0]
            enc = self.te_maps[te]
            v = X[:, cols[c]]
            na_cat = len(enc) - 1
            for tc in tcs:
                prior = self._te_prior(enc, tc)
                num = np.array([enc[k][tc][0] for k in range(len(enc))])
                den = np.array([enc[k][tc][1] for k in range(len(enc))])
                miss = np.isnan(v) | (np.nan_to_num(v, nan=-1) >= na_cat) | (np.nan_to_num(v, nan=-1) < 0)
                lev = np.where(miss, na_cat, np.nan_to_num(v, nan=0)).astype(np.int64)
                with np.errstate(divide="ignore", invalid="ignore"):
                    post = num[lev] / den[lev]
                    if self.te_blend:
                        lam = 1.0 / (1.0 + np.exp((self.te_k - np.floor(den[lev])) / self.te_f))
                        post = lam * post + (1 - lam) * prior
                if not self.te_has_na.get(te, False):
                    post = np.where(miss, prior, post)
                outs.append(post)
        return np.stack(outs, 1) if outs else np.zeros((X.shape[0], 0))

    def _load_svm(self):
        """SvmMojoReader.java (Sparkling Water's linear SVM): weights over the
        raw feature values, intercept, label threshold, optional mean
        imputation."""
        self.svm_mean_imp = bool(self.kv("meanImputation", False))
        self.svm_means = np.asarray(self.kv("means", []), dtype=np.float64) if self.svm_mean_imp else None
        self.svm_w = np.asarray(self.kv("weights", []), dtype=np.float64)
        self.svm_b = float(self.kv("interceptor", 0.0))
        self.svm_default_thr = float(self.kv("defaultThreshold", 0.0))
        self.svm_thr = float(self.kv("threshold", 0.0))

    def _score_svm(self, X):
        """SvmMojoModel.score0: margin = b + w.x; binomial label = margin >
        threshold, p1 = the margin clamped to the default threshold's side."""
        P = len(self.svm_w)
        V = X[:, :P]
        if self.svm_mean_imp:
            V = np.where(np.isnan(V), self.svm_means[:P], V)
        pred = self.svm_b + V @ self.svm_w
        if self.nclasses == 1:
            return pred.reshape(-1, 1)
        out = np.zeros((X.shape[0], 3))
        pos = pred > self.svm_thr
        dt = self.svm_default_thr
        out[:, 2] = np.where(pos, np.where(pred < dt, dt, pred), np.where(pred >= dt, dt - 1, pred))
        out[:, 1] = np.where(pos, out[:, 2] - 1, out[:, 2] + 1)
        out[:, 0] = pos.astype(np.float64)
        return out

    def _rect(self, title):
        """ModelMojoReader.readRectangularDoubleArray: <title>_size1/_size2 in
        model.ini, a big-endian f64 blob."""
        s1, s2 = int(self.kv(title + "_size1", 0)), int(self.kv(title + "_size2", 0))
        if s1 * s2 == 0:
            return np.zeros((s1, s2))
        return np.frombuffer(self.be.read(title), dtype=">f8", count=s1 * s2).astype(np.float64).reshape(s1, s2)

    def _load_coxph(self):
        """CoxPHMojoReader.java: coefficients over [expanded cats | nums],
        per-stratum covariate means (the linear predictor is centred by the
        row's stratum), strata keys = the strata columns' values, which lead
        the column order."""
        self.cox_coef = np.asarray(self.kv("coef", []), dtype=np.float64)
        self.cox_cats = int(self.kv("cats", 0))
        self.cox_cat_offsets = np.asarray(self.kv("cat_offsets", [0]), dtype=np.int64)
        self.cox_use_all = bool(self.kv("use_all_factor_levels", False))
        mc, mn = self._rect("x_mean_cat"), self._rect("x_mean_num")
        nstrata = int(self.kv("strata_count", 0))
        self.cox_strata = {}
        for i in range(nstrata):
            key = tuple(int(v) for v in self.kv(f"strata_{i}"))
            self.cox_strata[key] = i
        self.cox_strata_len = len(next(iter(self.cox_strata))) if self.cox_strata else 0
        ns = mc.shape[1] if mc.shape[0] else 0
        self.cox_lp_base = np.array([mc[s] @ self.cox_coef[:mc.shape[1]] + mn[s] @ self.cox_coef[ns:ns + mn.shape[1]]
                                     for s in range(max(nstrata, 1))]) if max(mc.shape[0], mn.shape[0]) else np.zeros(1)
        self.cox_ia = None
        if self.info.get("interaction_targets") is not None:
            self.cox_ia = (list(self.kv("interactions_1")), list(self.kv("interactions_2")),
                           list(self.kv("interaction_targets")))

    def _score_coxph(self, X):
        """CoxPHMojoModel.score0: categorical coefficients + numeric dot
        product - the stratum's centring term."""
        n = X.shape[0]
        if self.cox_ia is not None:
            for a, b, t in zip(*self.cox_ia):
                miss = np.isnan(X[:, t])
                X[miss, t] = X[miss, a] * X[miss, b]
        sl = self.cox_strata_len
        F = X[:, sl:]
        lp = np.zeros(n)
        offs = self.cox_cat_offsets
        low = 0 if self.cox_use_all else 1
        for c in range(self.cox_cats):
            v = F[:, c]
            idx = np.where(np.isnan(v), -1, v).astype(np.int64) - low
            x = idx + offs[c]
            ok = (idx >= 0) & (x < offs[c + 1])
            lp += np.where(ok, self.cox_coef[np.clip(x, 0, len(self.cox_coef) - 1)], 0.0)
            lp[np.isnan(v)] = np.nan
        diff = int(offs[self.cox_cats]) - self.cox_cats
        nnum = len(self.cox_coef) - int(offs[self.cox_cats])
        if nnum > 0:
            lp += F[:, self.cox_cats:self.cox_cats + nnum] @ self.cox_coef[diff + self.cox_cats:]
        if self.cox_strata:
            keys = X[:, :sl]
            s = np.array([self.cox_strata.get(tuple(int(v) for v in r), -1) if not np.isnan(r).any() else -1
                          for r in keys])
            base = np.where(s >= 0, self.cox_lp_base[np.maximum(s, 0)], np.nan)
        else:
            base = self.cox_lp_base[0]
        return (lp - base).reshape(n, 1)

    def xgb_features(self, X: np.ndarray) -> np.ndarray:
        """Rows in MOJO column order -> the booster's f32 feature matrix
        (OneHotEncoderFactory.java: one indicator per level plus an NA level
        per categorical, then the numerics; sparse models treat 0 and
        not-hot as missing)."""
        n = X.shape[0]
        offs = self.xgb_cat_offsets
        ncat_feat = int(offs[self.xgb_cats]) if self.xgb_cats else 0
        not_hot = np.float32(np.nan) if self.xgb_sparse else np.float32(0.0)
        F = np.full((n, ncat_feat + self.xgb_nums), not_hot, dtype=np.float32)
        rows = np.arange(n)
        for c in range(self.xgb_cats):
            v = X[:, c]
            hi = offs[c + 1] - 1
            nan = np.isnan(v)
            iv = np.where(nan, 0, v).astype(np.int64)
            if self.xgb_use_all:
                hot = iv + offs[c]
            else:
                hot = np.where(iv != 0, iv - 1 + offs[c], -1)
            hot = np.where(hot >= offs[c + 1], hi, hot)
            hot = np.where(nan, hi, hot)
            ok = hot >= 0
            F[rows[ok], hot[ok]] = 1.0
        num = X[:, self.xgb_cats:self.xgb_cats + self.xgb_nums].astype(np.float32)
        if self.xgb_sparse:
            num = np.where(num == 0, np.float32(np.nan), num)
        F[:, ncat_feat:] = num
        return F

    def transform(self, word):
        """Word2Vec embedding of one word (None if out of vocabulary)."""
        v = self.embeddings.get(word)
        return None if v is None else v.copy()

    def _load_deeplearning(self):
        self.dl_nums = int(self.kv("nums"))
        self.dl_cats = int(self.kv("cats"))
        self.dl_cat_offsets = list(self.kv("cat_offsets", [0]))
        self.dl_norm_mul = self.info.get("norm_mul") or []
        self.dl_norm_sub = self.info.get("norm_sub") or []
        self.dl_resp_mul = self.info.get("norm_resp_mul")
        self.dl_resp_sub = self.info.get("norm_resp_sub")
        self.dl_use_all = bool(self.kv("use_all_factor_levels", False))
        self.dl_activation = str(self.kv("activation"))
        self.dl_family = str(self.kv("distribution"))
        self.dl_units = list(self.kv("neural_network_sizes", []))
        self.dl_dropout = list(self.kv("hidden_dropout_ratios", []))
        self.dl_layers = []
        for li in range(len(self.dl_units) - 1):
            b = np.asarray(self.kv(f"bias_layer{li}", []), dtype=np.float64)
            w = np.asarray(self.kv(f"weight_layer{li}", []), dtype=np.float32).astype(np.float64)
            self.dl_layers.append((w, b))
        enc = str(self.kv("_genmodel_encoding", "AUTO")) if self.version >= 1.10 else "AUTO"
        self.catenc = self._orig_encoding(enc)
        nl = len(self.dl_units) - 1
        out_act = self.dl_activation if self.category == "AutoEncoder" else (
            "Softmax" if self.nclasses > 1 else "Linear")
        self.dl_acts = [self.dl_activation] * (nl - 1) + [out_act]

    def _orig_encoding(self, enc):
        """A non-AUTO categorical_encoding (hex.genmodel.CategoricalEncoding):
        the original columns / domains (_orig_names, _orig_domain_values_i,
        _orig_projection_array) turned into the encoding record that
        mojo/genmodel.encode_df replays before the model columns are read
        (OneHotEncoder, BinaryEncoder, LabelEncoder, EnumLimitedEncoder,
        EigenEncoder of h2o-genmodel's easy package)."""
        if enc in ("AUTO", "Enum", "SortByResponse", "OneHotInternal"):
            return None
        if enc not in ("OneHotExplicit", "Binary", "LabelEncoder", "EnumLimited", "Eigen"):
            raise NotImplementedError(f"MOJO categorical encoding {enc} is not supported")
        n = int(self.kv("_n_orig_names", 0) or 0)
        names = self.be.text("_orig_names")[:n] if n else []
        nd = int(self.kv("_n_orig_domain_values", 0) or 0)
        doms = []
        for i in range(nd):
            m = int(self.kv(f"_m_orig_domain_values_{i}", 0) or 0)
            doms.append([x.replace("\\n", "\n") for x in self.be.text(f"_orig_domain_values_{i}")[:m]]
                        if m > 0 else None)
        resp = self.response
        x_in = [c for c in names if c != resp]
        proj = list(self.kv("_orig_projection_array", []) or [])
        cols, pos = {}, 0
        for i, c in enumerate(names):
            d = doms[i] if i < len(doms) else None
            if c == resp or d is None:
                continue
            st = {"domain": list(d)}
            if enc == "EnumLimited":
                mc = next((cc for cc in self.columns if cc.startswith(c + ".top_") and cc.endswith("_levels")), c)
                nd_ = list(self.domains[self.columns.index(mc)] or []) if mc in self.columns else []
                st["limited"] = mc != c
                if st["limited"]:
                    other = nd_.index("other") if "other" in nd_ else -1
                    idx = {v: j for j, v in enumerate(nd_)}
                    st["lut"] = [idx.get(v, other) for v in d] + [idx.get("NA", other)]
                    st["new_domain"], st["name"] = nd_, mc
            elif enc == "Eigen":
                st["proj"] = proj[pos:pos + len(d)]
                pos += len(d)
            cols[c] = st
        return {"scheme": enc, "max_levels": 10, "x_in": x_in, "cols": cols}

    # --------------------------------------------------------------- inputs
    def row_matrix(self, df) -> np.ndarray:
        """DataFrame (or dict of columns) -> [n, ncolumns] doubles in the MOJO's
        column order: enum levels -> domain index (unseen / missing -> NaN,
        like EasyPredictModelWrapper with convertUnknownCategoricalLevelsToNa),
        numbers parsed from numerics or strings."""
        import pandas as pd
        if isinstance(df, dict):
            multi = any(isinstance(v, (list, tuple, np.ndarray, pd.Series)) for v in df.values())
            df = pd.DataFrame(df) if multi else pd.DataFrame([df])
        if getattr(self, "catenc", None) and not getattr(df, "_catenc_done", False):
            from .genmodel import encode_df
            df = encode_df(df, self.catenc)
        n = len(df)
        X = np.full((n, len(self.columns)), np.nan)
        for j, c in enumerate(self.columns):
            if c not in df:
                continue
            vals = df[c].values
            dom = self.domains[j]
            if dom is not None:
                idx = {d: i for i, d in enumerate(dom)}
                for r, v in enumerate(vals):
                    if v is None or (isinstance(v, float) and math.isnan(v)):
                        continue
                    if isinstance(v, str):
                        k = idx.get(v)
                    else:
                        fv = float(v)
                        k = idx.get(str(int(fv)) if fv.is_integer() else str(v), idx.get(str(v)))
                    if k is not None:
                        X[r, j] = k
            else:
                try:
                    X[:, j] = np.asarray(pd.to_numeric(pd.Series(vals), errors="coerce"), dtype=np.float64)
                except Exception:
                    pass
        if self.algo == "gam":
            self._gamify(df, X)
        return X

    # -------------------------------------------------------------- scoring
    def score0(self, X: np.ndarray) -> np.ndarray:
        """Rows [n, ncolumns] -> preds [n, 1 + K] exactly like MojoModel.score0
        (preds[:, 0] = label index / value / cluster)."""
        return getattr(self, f"_score_{self.algo}")(np.array(X, dtype=np.float64, copy=True))

    def _tree_sums(self, X):
        K = self.nclasses
        preds = np.zeros((X.shape[0], 1 + K if K > 1 else 1))
        off = 0 if K == 1 else 1
        dl = self.dom_len if self.version >= 1.2 else None
        lib = _forest_lib()
        if lib is not None and X.shape[0] >= 64:
            # native per-row walk of every tree (native/mojo_forest.cpp); the
            # numpy level-by-level walk below is the fallback and the spec
            pk = self.__dict__.get("_forest_pack")
            if pk is None:
                pk = self._forest_pack = _pack_forest(
                    [(off + ci, t) for ci in range(self.ntrees_per_group) for t in self.trees[ci] if t is not None])
            _forest_score(lib, pk, X, preds, self.version, dl)
            return preds
        for ci in range(self.ntrees_per_group):
            acc = preds[:, off + ci]
            for t in self.trees[ci]:
                if t is not None:
                    acc += t.score(X, dl, self.version)
        return preds

    def _label(self, preds):
        if preds.shape[1] == 3:
            preds[:, 0] = (preds[:, 2] >= self.default_threshold).astype(np.float64)
        else:
            preds[:, 0] = np.argmax(preds[:, 1:], axis=1)
        return preds

    def _calibrate(self, preds):
        if self.calib_beta is None or preds.shape[1] != 3:
            return preds
        b = self.calib_beta
        # PlattScalingMojoHelper: p1 = logitInv(p0 * beta[0] + beta[1])
        p1 = 1.0 / (np.exp(-(preds[:, 1] * b[0] + b[1])) + 1.0)
        self.calibrated = np.stack([1 - p1, p1], 1)
        return preds

    @staticmethod
    def _link_inv(link, f):
        if link == "log":
            return np.minimum(1e19, np.exp(f))
        if link in ("logit", "ologit"):
            return 1.0 / (1.0 + np.exp(-f))
        if link == "ologlog":
            return 1.0 - np.exp(-np.exp(f))
        if link == "inverse":
            xx = np.where(f < 0, np.minimum(-1e-5, f), np.maximum(-1e-5, f))
            return 1.0 / xx
        return f

    def _score_gbm(self, X):
        preds = self._tree_sums(X)
        fam = self.family
        if fam in ("bernoulli", "quasibinomial", "modified_huber"):
            f = preds[:, 1] + self.init_f
            preds[:, 2] = self._link_inv(self.link, f)
            preds[:, 1] = 1.0 - preds[:, 2]
        elif fam == "multinomial":
            if self.nclasses == 2:
                preds[:, 1] += self.init_f
                preds[:, 2] = -preds[:, 1]
            z = preds[:, 1:]
            z = np.exp(z - z.max(1, keepdims=True))
            preds[:, 1:] = z / z.sum(1, keepdims=True)
        else:
            preds[:, 0] = self._link_inv(self.link, preds[:, 0] + self.init_f)
            return preds
        return self._calibrate(self._label(preds))

    def _score_xgboost(self, X):
        """XGBoostMojoModel.toPreds: binomial p1 = booster output, p0 = 1 - p1;
        multinomial class probabilities; regression the transformed margin."""
        out = self.booster.predict(self.xgb_features(X))
        K = self.nclasses
        if K > 2:
            preds = np.zeros((X.shape[0], 1 + K))
            preds[:, 1:] = out[:, :K]
        elif K == 2:
            preds = np.zeros((X.shape[0], 3))
            preds[:, 2] = out[:, 0]
            preds[:, 1] = 1.0 - out[:, 0]
        else:
            return out[:, :1].astype(np.float64)
        return self._calibrate(self._label(preds))

    def _score_drf(self, X):
        preds = self._tree_sums(X)
        if self.nclasses == 1:
            preds[:, 0] /= self.ntree_groups
            return preds
        if self.nclasses == 2 and not self.binomial_double_trees:
            preds[:, 1] /= self.ntree_groups
            preds[:, 2] = 1.0 - preds[:, 1]
        else:
            s = preds[:, 1:].sum(1, keepdims=True)
            preds[:, 1:] = np.where(s > 0, preds[:, 1:] / np.where(s > 0, s, 1.0), preds[:, 1:])
        return self._calibrate(self._label(preds))

    def _glm_impute(self, X):
        if not self.mean_imputation:
            return
        nc = max(self.cats, 0)
        for i in range(nc):
            m = np.isnan(X[:, i])
            X[m, i] = self.cat_modes[i]
        for i in range(max(self.nums, 0)):
            m = np.isnan(X[:, nc + i])
            X[m, nc + i] = self.num_means[i]

    def _glm_eta(self, X, beta, P):
        """Linear predictor for one class block of beta (length P)."""
        n = X.shape[0]
        eta = np.zeros(n)
        offs = self.cat_offsets
        for i in range(len(offs) - 1):
            v = X[:, i]
            ok = ~np.isnan(v)
            iv = np.where(ok, v, 0).astype(np.int64)
            if not self.use_all_levels:
                ok &= iv != 0
                iv = iv - 1
            iv = iv + offs[i]
            ok &= iv < offs[i + 1]
            eta += np.where(ok, beta[np.clip(iv, 0, P - 1)], 0.0)
        nc = max(self.cats, 0)
        noff = offs[nc] if nc < len(offs) else 0
        nn = self.nums if self.nums >= 0 else P - 1 - noff
        # sequential accumulation in the reference's order (cats, nums,
        # intercept): bit-identical etas keep threshold ties (mu == the stored
        # default_threshold) on the same side as the reference scorer
        for i in range(nn):
            eta += beta[noff + i] * X[:, nc + i]
        return eta + beta[P - 1]

    def _score_glm(self, X):
        self._glm_impute(X)
        n = X.shape[0]
        fam = self.family
        if fam in ("multinomial", "ordinal"):
            K = self.nclasses
            P = self.beta.size // K
            etas = np.stack([self._glm_eta(X, self.beta[c * P:(c + 1) * P], P) for c in range(K)], 1)
            preds = np.zeros((n, 1 + K))
            if fam == "multinomial":
                # the reference clamps the row max at >= 0 before exponentiating
                mx = np.maximum(etas.max(1, keepdims=True), 0.0)
                e = np.exp(etas - mx)
                preds[:, 1:] = e / e.sum(1, keepdims=True)
            else:
                cdf_prev = np.zeros(n)
                for c in range(K - 1):
                    cdf = 1.0 / (1.0 + np.exp(-etas[:, c]))
                    preds[:, c + 1] = cdf - cdf_prev
                    cdf_prev = cdf
                preds[:, K] = 1.0 - cdf_prev
            preds[:, 0] = np.argmax(preds[:, 1:], axis=1)
            return preds
        eta = self._glm_eta(X, self.beta, self.beta.size)
        link = self.glm_link
        if link == "tweedie":
            p = self.tweedie_link_power
            mu = np.maximum(2e-16, np.exp(eta)) if p == 0 else np.power(eta, 1.0 / p)
        elif link == "inverse":
            xx = np.where(eta < 0, np.minimum(-1e-5, eta), np.maximum(1e-5, eta))
            mu = 1.0 / xx
        else:
            mu = self._link_inv(link, eta)
        if fam in ("binomial", "fractionalbinomial", "quasibinomial"):
            preds = np.zeros((n, 3))
            preds[:, 0] = (mu >= self.default_threshold).astype(np.float64)
            preds[:, 1] = 1.0 - mu
            preds[:, 2] = mu
            return preds
        return mu.reshape(n, 1)

    def _score_kmeans(self, X):
        X = X[:, :self.centers.shape[1]]
        if self.standardize:
            for i in range(X.shape[1]):
                m = np.isnan(X[:, i])
                if self.km_modes[i] == -1:
                    X[m, i] = self.km_means[i]
                    if self.km_mults is not None:
                        X[:, i] = (X[:, i] - self.km_means[i]) * self.km_mults[i]
                else:
                    X[m, i] = self.km_modes[i]
        cat = np.array([d is not None for d in self.domains[:X.shape[1]]])
        nan = np.isnan(X)
        pts = (~nan).sum(1).astype(np.float64)
        dist = np.zeros((X.shape[0], self.centers.shape[0]))
        for k, c in enumerate(self.centers):
            dd = np.where(cat, (X != c).astype(np.float64), (X - c) ** 2)
            dd = np.where(nan, 0.0, dd)
            s = dd.sum(1)
            scale = np.where((pts > 0) & (pts < X.shape[1]), X.shape[1] / np.maximum(pts, 1), 1.0)
            dist[:, k] = s * scale
        self.last_distances = dist
        return np.argmin(dist, axis=1).reshape(-1, 1).astype(np.float64)

    def _score_pca(self, X):
        """PCAMojoModel.score0: categorical level rows of the eigenvectors
        (missing / unseen levels skipped), numerics (x - sub) * mul."""
        n = X.shape[0]
        E = self.pca_evecs
        offs = self.pca_cat_offsets
        perm = self.pca_perm or list(range(self.pca_ncats + self.pca_nnums))
        out = np.zeros((n, self.pca_k))
        for j in range(self.pca_ncats):
            v = X[:, perm[j]]
            ok = ~np.isnan(v)
            lvl = np.where(ok, v, 0).astype(np.int64) - (0 if self.pca_use_all else 1)
            last = offs[j + 1] - offs[j] - 1
            ok &= (lvl >= 0) & (lvl <= last)
            out += np.where(ok[:, None], E[np.clip(offs[j] + lvl, 0, E.shape[0] - 1)], 0.0)
        base = offs[self.pca_ncats]
        for j in range(self.pca_nnums):
            x = (X[:, perm[self.pca_ncats + j]] - self.pca_norm_sub[j]) * self.pca_norm_mul[j]
            out += x[:, None] * E[base + j][None, :]
        return out

    def _score_rulefit(self, X):
        """RuleFitMojoModel.score0: per (depth, tree) the last rule whose
        conditions all hold gives the level of categorical M<i>T<j>
        (MojoRuleEnsemble.decode), then the rows are mapped by name onto the
        linear model's columns (map()) and scored by it."""
        n = X.shape[0]
        lin = self.rf_linear
        test = []
        rdom = self.domains[self.columns.index(self.response)] if self.response in self.columns else None
        classes = list(rdom) if rdom is not None and len(rdom) > 2 else None
        if self.rf_type != 0:
            for i in range(self.rf_depth):
                for j in range(self.rf_ntrees):
                    rules = self.rf_rules[(i, j)]
                    for k in range(len(classes) if classes else 1):
                        # multinomial (MojoRuleEnsemble.transformRow): the
                        # rules of class k decode into column M<i>T<j>C<k>
                        name = f"M{i}T{j}C{k}" if classes else f"M{i}T{j}"
                        rs = [r for r in rules if r[0].endswith(classes[k])] if classes else rules
                        test.append(self._rulefit_decode(X, rs, lin.domains[lin.columns.index(name)]))
        if self.rf_type != 2:
            test += [X[:, c] for c in range(X.shape[1]) if c < len(self.features)]
        Xl = np.full((n, len(lin.columns)), np.nan)
        for i, nm in enumerate(self.rf_linear_names):
            Xl[:, lin.columns.index(nm)] = test[i]
        return lin.score0(Xl)

    @staticmethod
    def _rulefit_decode(X, rules, dom):
        """MojoRuleEnsemble.decode: the level of the last rule that holds."""
        n = X.shape[0]
        val = np.full(n, np.nan)
        for var, conds in rules:
            ok = np.ones(n, dtype=bool)
            for fi, typ, op, thr, nas in conds:
                col = X[:, fi]
                isna = np.isnan(col)
                if typ == 0:
                    hit = np.isin(col, np.asarray(thr, dtype=np.float64))
                elif op == 0:
                    hit = col < thr
                else:
                    hit = col >= thr
                ok &= np.where(isna, nas, hit & ~isna)
            val = np.where(ok, float(dom.index(var)) if var in dom else np.nan, val)
        return val

    def _score_stackedensemble(self, X):
        n = X.shape[0]
        K = self.nclasses
        nb = len(self.base)
        # one slot per base model (per class for multinomial); unused models
        # (pruned by the metalearner) keep their slots at 0, as in the reference
        B = np.zeros((n, nb * K if K > 2 else nb))
        for i, b in enumerate(self.base):
            if b is None:
                continue
            m, mapping = b
            p = m.score0(X[:, mapping])
            if K > 2:
                B[:, i * K:(i + 1) * K] = p[:, 1:1 + K]
            elif K == 2:
                B[:, i] = p[:, 2]
            else:
                B[:, i] = p[:, 0]
        if self.logit_transform and K >= 2:
            q = np.clip(B, 1e-9, 1 - 1e-9)
            x = q / (1 - q)
            B = np.where(x == 0, -19.0, np.maximum(-19.0, np.log(np.where(x > 0, x, 1.0))))
        # the metalearner's columns are the base predictions (+ its response)
        Xm = np.full((n, len(self.metalearner.columns)), np.nan)
        Xm[:, :B.shape[1]] = B
        return self.metalearner.score0(Xm)

    def _score_isolationforest(self, X):
        preds = self._tree_sums(X)
        tot = preds[:, 0]
        n = X.shape[0]
        mean_len = tot / self.ntree_groups if self.ntree_groups >= 1 else np.zeros(n)
        lo, hi = self.min_path_length, self.max_path_length
        score = (hi - tot) / (hi - lo) if hi > lo else np.ones(n)
        if self.output_anomaly_flag:
            return np.stack([(score > self.default_threshold).astype(np.float64), score, mean_len], 1)
        return np.stack([score, mean_len], 1)

    @staticmethod
    def _avg_path_unsuccessful(nrows):
        n = np.asarray(nrows, dtype=np.float64)
        h = np.log(np.maximum(n - 1, 1)) + 0.5772156649
        return np.where(n < 2, 0.0, np.where(n == 2, 1.0, 2 * h - 2.0 * (n - 1.0) / np.maximum(n, 1)))

    def _score_extendedisolationforest(self, X):
        n = X.shape[0]
        tot = np.zeros(n)
        for nodes in self.eif_trees:
            num = np.zeros(n, dtype=np.int64)
            height = np.zeros(n)
            out = np.full(n, -1.0)
            active = np.arange(n)
            while active.size:
                nxt_active = []
                for nd in np.unique(num[active]).tolist():
                    sel = active[num[active] == nd]
                    rec = nodes.get(nd)
                    if rec is None:
                        continue
                    if rec[0] == "L":
                        out[sel] = height[sel] + float(self._avg_path_unsuccessful(rec[1]))
                        continue
                    _, nv, pv = rec
                    mul = ((X[np.ix_(sel, np.arange(nv.size))] - pv) * nv).sum(1)
                    height[sel] += 1
                    num[sel] = np.where(mul <= 0, 2 * nd + 1, 2 * nd + 2)
                    nxt_active.append(sel)
                active = np.concatenate(nxt_active) if nxt_active else np.zeros(0, dtype=np.int64)
            tot += out
        path = tot / max(self.eif_ntrees, 1)
        score = np.power(2.0, -path / float(self._avg_path_unsuccessful(self.eif_sample_size)))
        return np.stack([score, path], 1)

    def _dl_input(self, X):
        """GenModel.setInput: one-hot categoricals (NA / unseen -> the extra
        last level of the variable), standardised numerics, missing -> 0."""
        n = X.shape[0]
        offs = self.dl_cat_offsets
        nc, nn = self.dl_cats, self.dl_nums
        width = offs[nc] + nn
        A = np.zeros((n, width))
        for i in range(nc):
            v = X[:, i]
            nan = np.isnan(v)
            c = np.where(nan, 0, v).astype(np.int64)
            if self.dl_use_all:
                t = c + offs[i]
            else:
                t = np.where(c != 0, c - 1 + offs[i], -1)
            t = np.where(nan, offs[i + 1] - 1, t)
            t = np.where(t >= offs[i + 1], offs[i + 1] - 1, t)
            ok = t >= 0
            A[np.nonzero(ok)[0], t[ok]] = 1.0
        for j in range(nn):
            d = X[:, nc + j]
            if len(self.dl_norm_mul):
                d = (d - self.dl_norm_sub[j]) * self.dl_norm_mul[j]
            A[:, offs[nc] + j] = np.where(np.isnan(d), 0.0, d)
        return A

    @staticmethod
    def _dl_affine(x, w, b, out_size):
        """NeuralNetwork.formNNInputs in the reference's summation order (8
        partial sums over column blocks, then the tail, then the bias)."""
        n, cols = x.shape
        W = w.reshape(out_size, cols)
        res = np.zeros((n, out_size))
        multiple = (cols // 8) * 8 - 1
        extra = cols - cols % 8
        ps = [np.zeros((n, out_size)) for _ in range(8)]
        col = 0
        while col < multiple:
            for k in range(8):
                ps[k] += x[:, col + k:col + k + 1] * W[:, col + k][None, :]
            col += 8
        res += ps[0] + ps[1] + ps[2] + ps[3]
        res += ps[4] + ps[5] + ps[6] + ps[7]
        for c in range(extra, cols):
            res += x[:, c:c + 1] * W[:, c][None, :]
        return res + b[None, :out_size]

    def _score_deeplearning(self, X):
        h = self._dl_input(X)
        for li, (w, b) in enumerate(self.dl_layers):
            act = self.dl_acts[li]
            out = self.dl_units[li + 1]
            drop = self.dl_dropout[li] if li < len(self.dl_dropout) else 0.0
            if act.startswith("Maxout"):
                k = b.size // out
                W = w.reshape(out, h.shape[1], k)
                z = np.einsum("ni,oik->nok", h, W) + b.reshape(out, k)[None]
                h = z.max(2)
            else:
                z = self._dl_affine(h, w, b, out)
                if act == "Softmax":
                    e = np.exp(z - z.max(1, keepdims=True))
                    h = e / e.sum(1, keepdims=True)
                elif act == "Linear":
                    h = z
                elif act.startswith("ExpRectifier"):
                    h = np.where(z >= 0, z, np.exp(z) - 1)
                elif act.startswith("Rectifier"):
                    h = 0.5 * (z + np.abs(z))
                elif act.startswith("Tanh"):
                    h = 1.0 - 2.0 / (1.0 + np.exp(2.0 * z))
                else:
                    raise NotImplementedError(f"activation {act}")
            if act.endswith("WithDropout") and drop > 0:
                h = h * (1.0 - drop)
        n = X.shape[0]
        if self.category == "AutoEncoder":
            out = h.copy()
            if len(self.dl_norm_mul):
                k0 = out.shape[1] - self.dl_nums
                out[:, k0:] = out[:, k0:] / np.asarray(self.dl_norm_mul) + np.asarray(self.dl_norm_sub)
            return out
        if self.nclasses > 1:
            preds = np.zeros((n, 1 + self.nclasses))
            preds[:, 1:] = h
            return self._label(preds)
        v = h[:, 0]
        if self.dl_resp_mul is not None:
            v = v / self.dl_resp_mul[0] + self.dl_resp_sub[0]
        fam = self.dl_family
        if fam in ("bernoulli", "quasibinomial", "modified_huber", "ordinal"):
            v = 1.0 / (1.0 + np.minimum(1e19, np.exp(-v)))
        elif fam in ("multinomial", "poisson", "gamma", "tweedie"):
            v = np.minimum(1e19, np.exp(v))
        return v.reshape(n, 1)

    def decision_paths(self, df):
        """Leaf assignment per (row, tree) as 'L'/'R' strings (tree models)."""
        X = self.row_matrix(df)
        dl = self.dom_len if self.version >= 1.2 else None
        out = []
        for ci in range(self.ntrees_per_group):
            for t in self.trees[ci]:
                paths = [""] * X.shape[0]
                if t is not None:
                    t.score(X, dl, self.version, paths)
                out.append(paths)
        return [list(r) for r in zip(*out)]

    # ------------------------------------------------------------- outputs
    def predict_contributions(self, df, output_format="Original", top_n=None, bottom_n=None, compare_abs=False):
        """TreeSHAP contributions of a reference-layout GBM / DRF MOJO
        (h2o-genmodel TreeSHAP.java over the trees + _aux.bin node weights;
        GbmMojoModel adds init_f to the bias, DrfMojoModel's
        ContributionsPredictorDRF divides by the number of trees -- binomial:
        1/(F+1) - contribution to the P(class 0) trees)."""
        from .treeshap_np import contributions_frame, tree_shap
        if self.algo not in ("gbm", "drf"):
            raise ValueError(f"contributions are not available for a {self.algo} MOJO")
        if self.nclasses > 2:
            raise ValueError("Calculating contributions is currently not supported for multinomial models.")
        X = self.row_matrix(df)
        n, F = X.shape[0], self.nfeatures
        phi = np.zeros((n, F + 1))
        dl = self.dom_len if self.version >= 1.2 else None
        for g, t in enumerate(self.trees[0]):
            if t is None:
                continue
            if t.root_leaf is not None:
                phi[:, -1] += t.root_leaf
                continue
            name = "trees/t%02d_%03d_aux.bin" % (0, g)
            if not self.be.exists(name):
                raise ValueError("this MOJO has no auxiliary tree info (node weights) for contributions")
            left, right, cover, value, feat = t.shap_graph(self.be.read(name))
            I = len(t.col)
            tree_shap(left, right, cover, value, feat, lambda j, t=t, I=I: ~t.node_right(j, X, dl, self.version) if
                      j < I else np.ones(n, dtype=bool), n, phi)
        if self.algo == "gbm":
            phi[:, -1] += self.init_f
        else:
            ng = max(1, sum(1 for t in self.trees[0] if t is not None))
            if self.nclasses == 2 and not self.binomial_double_trees:
                phi = 1.0 / (F + 1) - phi / ng
            else:
                phi = phi / ng
        return contributions_frame(phi, list(self.features), top_n=top_n, bottom_n=bottom_n, compare_abs=compare_abs)

    def predict_raw(self, df) -> np.ndarray:
        """[n, K] class probabilities (classification) or [n, 1] values /
        cluster ids (Generic model metrics)."""
        preds = self.score0(self.row_matrix(df))
        if self.nclasses > 1 and preds.shape[1] > 1:
            return preds[:, 1:]
        return preds[:, :1]

    def predict(self, df):
        import pandas as pd
        preds = self.score0(self.row_matrix(df))
        if self.algo == "kmeans":
            return pd.DataFrame({"predict": preds[:, 0].astype(np.int64)})

        if self.algo == "isolationforest":
            cols = ["predict", "score", "mean_length"] if self.output_anomaly_flag else ["predict", "mean_length"]
            return pd.DataFrame(preds, columns=cols)
        if self.algo == "extendedisolationforest":
            return pd.DataFrame(preds, columns=["anomaly_score", "mean_length"])
        if self.algo == "pca":
            return pd.DataFrame(preds, columns=[f"PC{i + 1}" for i in range(preds.shape[1])])
        if self.algo == "glrm":
            rec = self.glrm_impute(preds)
            out = {}
            for j, c in enumerate(self.columns):
                dom = self.domains[j]
                out[f"reconstr_{c}"] = np.array(dom, dtype=object)[rec[:, j].astype(np.int64)] if dom else rec[:, j]
            return pd.DataFrame(out)
        if self.algo == "coxph":
            return pd.DataFrame({"lp": preds[:, 0]})
        if self.algo == "targetencoder":
            return pd.DataFrame(preds, columns=self.te_out_names)
        if self.category == "AutoEncoder":
            return pd.DataFrame(preds, columns=[f"reconstr_{i}" for i in range(preds.shape[1])])
        if self.nclasses > 1 and preds.shape[1] > 1:
            dom = self.response_domain or [str(i) for i in range(self.nclasses)]
            lab = np.array(dom, dtype=object)[preds[:, 0].astype(np.int64)]
            out = {"predict": lab}
            from .genmodel import scoring_names
            for k, d in enumerate(scoring_names(dom)[1:]):
                out[d] = preds[:, 1 + k]
            cal = getattr(self, "calibrated", None)
            if cal is not None and self.calib_beta is not None:
                out["cal_" + dom[0]] = cal[:, 0]
                out["cal_" + dom[1]] = cal[:, 1]
            return pd.DataFrame(out)
        return pd.DataFrame({"predict": preds[:, 0]})

    def predict_row(self, row: dict):
        return self.predict(row).iloc[0].to_dict()


class _JavaRandom:
    """java.util.Random, vectorised over one generator per row (48-bit LCG;
    uint64 products wrap mod 2^64, so the low 48 bits stay exact)."""
    _MUL, _ADD, _MASK = np.uint64(0x5DEECE66D), np.uint64(0xB), np.uint64((1 << 48) - 1)

    def __init__(self, seeds):
        s = np.asarray(seeds, dtype=np.int64).astype(np.uint64)
        self.s = (s ^ self._MUL) & self._MASK

    def _next(self, bits, rows):
        with np.errstate(over="ignore"):
            self.s[rows] = (self.s[rows] * self._MUL + self._ADD) & self._MASK
        return (self.s[rows] >> np.uint64(48 - bits)).astype(np.int64)

    def _double(self, rows):
        return ((self._next(26, rows) << 27) + self._next(27, rows)) * (1.0 / (1 << 53))

    def gaussians(self, k):
        """k successive nextGaussian() values per generator (polar method:
        pairs (v1 m, v2 m), the second one cached for the next call)."""
        n = self.s.shape[0]
        out = np.zeros((n, k))
        for t in range(0, k, 2):
            v1, v2, m = np.zeros(n), np.zeros(n), np.zeros(n)
            todo = np.arange(n)
            while todo.size:
                a = 2 * self._double(todo) - 1
                b = 2 * self._double(todo) - 1
                ss = a * a + b * b
                ok = (ss < 1) & (ss != 0)
                r = todo[ok]
                v1[r], v2[r] = a[ok], b[ok]
                m[r] = np.sqrt(-2 * np.log(ss[ok]) / ss[ok])
                todo = todo[~ok]
            out[:, t] = v1 * m
            if t + 1 < k:
                out[:, t + 1] = v2 * m
        return out


def _glrm_loss(name, u, a):
    """GlrmLoss loss / lgrad of a numeric column."""
    if name == "Quadratic":
        return (u - a) ** 2, 2 * (u - a)
    if name == "Absolute":
        return np.abs(u - a), np.sign(u - a)
    if name == "Huber":
        x = u - a
        return (np.where(x > 1, x - 0.5, np.where(x < -1, -x - 0.5, 0.5 * x * x)),
                np.where(x > 1, 1.0, np.where(x < -1, -1.0, x)))
    if name == "Poisson":
        with np.errstate(divide="ignore", invalid="ignore"):
            extra = np.where(a == 0, 0.0, -a * u + a * np.log(np.where(a > 0, a, 1.0)) - a)
        return np.exp(u) + extra, np.exp(u) - a
    if name == "Logistic":
        s = 1 - 2 * a
        return np.log1p(np.exp(s * u)), s / (1 + np.exp(-s * u))
    if name == "Hinge":
        s = 1 - 2 * a
        return np.maximum(1 + s * u, 0), np.where(1 + s * u > 0, s, 0.0)
    if name.startswith("Periodic"):
        f = 2 * math.pi / float(name[name.index("(") + 1:name.index(")")])
        return 1 - np.cos((u - a) * f), f * np.sin((u - a) * f)
    raise NotImplementedError(f"GLRM loss {name}")


def _glrm_loss_impute(name, u):
    if name == "Poisson":
        return np.exp(u)
    if name in ("Logistic", "Hinge"):
        return (u > 0).astype(np.float64)
    return u


def _glrm_regularize(name, x):
    """GlrmRegularizer.regularize per row (indicator regularisers are 0 inside
    their set, +inf outside)."""
    if name == "Quadratic":
        return (x * x).sum(1)
    if name == "L2":
        return np.sqrt((x * x).sum(1))
    if name == "L1":
        return np.abs(x).sum(1)
    if name == "NonNegative":
        return np.where((x < 0).any(1), np.inf, 0.0)
    if name == "OneSparse":
        return np.where(((x < 0).any(1)) | ((x > 0).sum(1) != 1), np.inf, 0.0)
    if name == "UnitOneSparse":
        ok = ((x == 1).sum(1) == 1) & ((x == 0).sum(1) == x.shape[1] - 1)
        return np.where(ok, 0.0, np.inf)
    if name == "Simplex":
        s = x.sum(1)
        ok = ~(x < 0).any(1) & (np.abs(s - 1) <= 1e-10 * np.maximum(1, np.abs(x).sum(1)) * x.shape[1])
        return np.where(ok, 0.0, np.inf)
    return np.zeros(x.shape[0])


def _glrm_prox(name, u, delta, project=False):
    """GlrmRegularizer.rproxgrad(u, delta) per row (delta = 0 returns u, as
    in the reference); project=True is GlrmRegularizer.project."""
    delta = np.broadcast_to(np.asarray(delta, dtype=np.float64), (u.shape[0],))
    if name in ("None",) or (project and name in ("Quadratic", "L2", "L1")):
        return u
    if project and name == "Simplex":
        inside = _glrm_regularize("Simplex", u) == 0
        out = _glrm_prox("Simplex", u, 1.0)
        return np.where(inside[:, None], u, out)
    keep = (delta == 0)[:, None]
    if name == "Quadratic":
        v = u / (1 + 2 * delta)[:, None]
    elif name == "L2":
        nr = np.sqrt((u * u).sum(1))
        with np.errstate(divide="ignore", invalid="ignore"):
            w = 1 - delta / nr
        v = np.where((w < 0)[:, None], 0.0, w[:, None] * u)
    elif name == "L1":
        d = delta[:, None]
        v = np.maximum(u - d, 0) + np.minimum(u + d, 0)
    elif name == "NonNegative":
        v = np.maximum(u, 0)
    elif name in ("OneSparse", "UnitOneSparse"):
        idx = u.argmax(1)
        r = np.arange(u.shape[0])
        v = np.zeros_like(u)
        v[r, idx] = (np.where(u[r, idx] > 0, u[r, idx], 1e-6)) if name == "OneSparse" else 1.0
    elif name == "Simplex":
        # Chen & Ye projection onto the simplex
        n = u.shape[1]
        srt = np.sort(u, 1)
        csum = np.cumsum(srt[:, ::-1], 1)[:, ::-1]            # csum[:, i] = sum_{j >= i} srt[:, j]
        t = (csum[:, 0] - 1) / n
        found = np.zeros(u.shape[0], dtype=bool)
        for i in range(n - 1, 0, -1):
            tmp = (csum[:, i] - 1) / (n - i)
            hit = ~found & (tmp >= srt[:, i - 1])
            t = np.where(hit, tmp, t)
            found |= hit
        v = np.maximum(u - t[:, None], 0)
    else:
        raise NotImplementedError(f"GLRM regularizer {name}")
    return np.where(keep, u, v)


def pd_numeric(col):
    import pandas as pd
    return pd.to_numeric(col, errors="coerce").values


def load(src) -> H2OMojoModel:
    return H2OMojoModel(src)
