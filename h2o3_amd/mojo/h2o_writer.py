"""MOJO export in the reference's h2o-genmodel layout.

`build_h2o_mojo(model)` writes GBM, DRF and GLM models as the reference's
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
"""
from __future__ import annotations

import io
import struct
import time
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

    def close(self) -> bytes:
        self.z.close()
        return self.buf.getvalue()


def _threshold(model):
    """The labelling threshold predict() uses: max-F1 of the validation (else
    training) metrics, 0.5 without metrics (base.py _pred_frame_from_raw)."""
    thr = 0.5
    for m in (getattr(model, "_training_metrics", None), getattr(model, "_validation_metrics", None)):
        if m is not None and m.get("max_f1_threshold") is not None:
            thr = float(m["max_f1_threshold"])
    return thr


def _header(model, algo_short, algo_full, category, columns, nfeatures, nclasses, domains, mojo_version, extra):
    info = {
        "h2o_version": "3.46.0.99999", "mojo_version": mojo_version, "license": "Apache License Version 2.0",
        "algo": algo_short, "algorithm": algo_full, "endianness": "LITTLE_ENDIAN", "category": category,
        "uuid": str(abs(hash(model.model_id)) % (1 << 62)), "supervised": True, "n_features": nfeatures,
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


def _encode_tree(tree, leaf_map=None):
    """Our Tree (x < thr goes left; cat_left = level mask going left) -> the
    reference's pre-order byte stream.  leaf_map(value) transforms leaf values
    (e.g. DRF binomial class-0 probabilities)."""
    lm = leaf_map or (lambda v: v)

    def is_leaf(i):
        return tree.left[i] < 0

    if is_leaf(0):
        return b"\x00" + struct.pack("<H", 65535) + _f32(lm(tree.value[0]))

    def enc(i):
        node_type = 0
        body = bytearray()
        f = int(tree.feat[i])
        if f >= 65535:
            raise ValueError("reference tree MOJOs address at most 65534 columns")
        if tree.is_cat[i]:
            mask = np.asarray(tree.cat_left[i]).astype(bool)
            right = ~mask                         # bitset bit set -> go right
            nbits = len(right)
            nsd = _NSD_NA_LEFT if tree.na_left[i] else _NSD_NA_RIGHT
            if nbits <= 32:
                node_type |= 8
                bits = np.zeros(32, dtype=bool)
                bits[:nbits] = right
                split = np.packbits(bits, bitorder="little").tobytes()
            else:
                node_type |= 12
                split = struct.pack("<Hi", 0, nbits) + np.packbits(right, bitorder="little").tobytes()
        elif not np.isfinite(tree.thr[i]) and tree.thr[i] > 0:
            nsd = _NSD_NA_VS_REST                 # every number left, NA right
            split = b""
        else:
            nsd = _NSD_NA_LEFT if tree.na_left[i] else _NSD_NA_RIGHT
            split = _f32(tree.thr[i])
        l, r = int(tree.left[i]), int(tree.right[i])
        if is_leaf(l):
            node_type |= 48
            left_bytes = _f32(lm(tree.value[l]))
        else:
            sub = enc(l)
            n = len(sub)
            width = 1 if n < (1 << 8) else 2 if n < (1 << 16) else 3 if n < (1 << 24) else 4
            node_type |= width - 1
            left_bytes = n.to_bytes(width, "little") + sub
        if is_leaf(r):
            node_type |= 0xC0
            right_bytes = _f32(lm(tree.value[r]))
        else:
            right_bytes = enc(r)
        body += bytes([node_type]) + struct.pack("<H", f) + bytes([nsd]) + split + left_bytes + right_bytes
        return bytes(body)

    return enc(0)


def _encode_aux(tree, leaf_map=None):
    """AuxInfo records (pre-order over split nodes): nid, #split nodes in the
    left subtree, child weights, child predictions, squared errors (0: not
    tracked), child node ids."""
    lm = leaf_map or (lambda v: v)
    out = bytearray()

    def n_splits(i):
        if tree.left[i] < 0:
            return 0
        return 1 + n_splits(tree.left[i]) + n_splits(tree.right[i])

    def walk(i):
        if tree.left[i] < 0:
            return
        l, r = int(tree.left[i]), int(tree.right[i])
        out.extend(struct.pack("<ii", i, n_splits(l)))
        out.extend(struct.pack("<ffff", tree.weight[l], tree.weight[r], lm(tree.value[l]), lm(tree.value[r])))
        out.extend(struct.pack("<ffii", 0.0, 0.0, l, r))
        walk(l)
        walk(r)

    walk(0)
    return bytes(out)


def _tree_model(model, z, algo_short, algo_full, extra, leaf_maps):
    spec = model._spec
    x = list(spec.x)
    xd = getattr(model, "_x_domains", {}) or {}
    columns = x + [spec.y]
    domains = [xd.get(c) for c in x] + [list(spec.response_domain) if spec.response_domain else None]
    K = model._n_tree_classes()
    ng = len(model._forest) // max(K, 1)
    cat = "Binomial" if spec.nclasses == 2 else "Multinomial" if spec.nclasses > 2 else "Regression"
    info = {"n_trees": ng, "n_trees_per_class": K, "_genmodel_encoding": "AUTO"}
    info.update(extra)
    ini, files = _header(model, algo_short, algo_full, cat, columns, len(x), spec.nclasses, domains,
                         TREE_MOJO_VERSION, info)
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


# -------------------------------------------------------------------- GLM
def _glm(model, z):
    di = model._dinfo
    if getattr(di, "ia_recipe", None):
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


def build_h2o_mojo(model) -> bytes:
    """MOJO zip bytes in the reference's layout (GBM, DRF, GLM)."""
    z = _Zip()
    if model.algo == "gbm":
        _gbm(model, z)
    elif model.algo == "drf":
        _drf(model, z)
    elif model.algo == "glm":
        if getattr(model, "_hglm", None) is not None:
            raise NotImplementedError("HGLM models have no MOJO (as in the reference)")
        _glm(model, z)
    else:
        raise NotImplementedError(f"reference-layout MOJO export is implemented for gbm, drf and glm, not {model.algo}")
    return z.close()
