"""MOJO export (Model ObJect, Optimized) — standalone scoring artifacts.

Reference: h2o-genmodel (hex/genmodel/AbstractMojoWriter.java writes a zip
with `model.ini` ([info]/[columns]/[domains]) plus algorithm blobs; every
algo has a *MojoWriter: SharedTreeMojoWriter, GLMMojoWriter,
KMeansMojoWriter, DeepLearningMojoWriter, PCAMojoWriter,
StackedEnsembleMojoWriter, ...).

Format here: zip containing
  model.ini    — [info] algorithm / category / n_features / n_classes /
                 mojo_version, [columns] feature + response names,
                 [domains] categorical domains (one file per domain under
                 domains/, like the reference)
  model.json   — algorithm parameters (small)
  arrays/*.npy — numeric blobs (numpy .npy, never pickled)
  models/<i>/  — nested MOJOs (stacked ensembles)
The matching reader (h2o3_amd.mojo.genmodel) needs only numpy.
"""
from __future__ import annotations

import io
import json
import os
import zipfile

import numpy as np
import torch

MOJO_VERSION = "1.00"


def _npy(arr):
    b = io.BytesIO()
    np.save(b, np.asarray(arr), allow_pickle=False)
    return b.getvalue()


class _Writer:
    def __init__(self):
        self.files = {}
        self.meta = {}
        self.arrays = {}

    def add_array(self, name, arr):
        self.arrays[name] = np.asarray(arr)

    def to_zip_bytes(self, info, columns, domains):
        b = io.BytesIO()
        # deflate level 1: forests of deep DRF models reach GBs of node arrays,
        # where level 6 costs minutes for a few % of size; nested model zips
        # (stacked ensembles, RuleFit) are stored, not deflated a second time
        with zipfile.ZipFile(b, "w", zipfile.ZIP_DEFLATED, compresslevel=1) as z:
            ini = ["[info]"] + [f"{k} = {v}" for k, v in info.items()] + ["", "[columns]"] + list(columns) + \
                  ["", "[domains]"]
            for i, (col, dom) in enumerate(domains):
                ini.append(f"{col}: {len(dom)} d{i:03d}.txt")
                z.writestr(f"domains/d{i:03d}.txt", "\n".join(dom))
            z.writestr("model.ini", "\n".join(ini) + "\n")
            z.writestr("model.json", json.dumps(self.meta, default=_json_default))
            for k, v in self.arrays.items():
                z.writestr(f"arrays/{k}.npy", _npy(v))
            for k, v in self.files.items():
                z.writestr(k, v, compress_type=zipfile.ZIP_STORED if k.endswith(".zip") else None)
        return b.getvalue()


def _json_default(o):
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        return float(o)
    if isinstance(o, np.ndarray):
        return o.tolist()
    if isinstance(o, torch.Tensor):
        return o.cpu().tolist()
    return str(o)


def _category(model):
    spec = model._spec
    if not model.supervised_learning:
        return {"kmeans": "Clustering", "pca": "DimReduction", "svd": "DimReduction", "glrm": "DimReduction",
                "isolationforest": "AnomalyDetection", "extendedisolationforest": "AnomalyDetection",
                "deeplearning": "AutoEncoder", "word2vec": "WordEmbedding",
                "targetencoder": "TargetEncoder"}.get(model.algo, "Unknown")
    if model.algo == "coxph":
        return "CoxPH"
    if model.algo == "upliftdrf":
        return "BinomialUplift"
    if spec.nclasses == 2:
        return "Binomial"
    if spec.nclasses > 2:
        return "Multinomial"
    return "Regression"


def _dinfo_meta(w, di, prefix="di"):
    w.meta[prefix] = {"cat_cols": di.cat_cols, "num_cols": di.num_cols, "domains": di.domains,
                      "cat_offsets": di.cat_offsets, "use_all": di.use_all, "standardize": di.standardize,
                      "means": di.means, "sigmas": di.sigmas, "plug": di.plug, "cat_modes": di.cat_modes,
                      "P": di.P, "mvh": di.mvh, "ia": getattr(di, "ia_recipe", None)}


def _forest_arrays(w, forest, names):
    P = forest.pack(torch.device("cpu"))
    for k in ("feat", "thr", "left", "right", "na_left", "cat_off", "cat_len", "cat_bits", "value", "roots", "tclass"):
        w.add_array(f"forest_{k}", P[k].cpu().numpy())
    # node training weights (covers), in the packed node order: the standalone
    # scorer's TreeSHAP background distribution (predict_contributions)
    w.add_array("forest_weight", np.concatenate([np.asarray(t.weight, dtype=np.float64) for t in forest.trees])
                if forest.trees else np.zeros(0))


def build_mojo(model) -> bytes:
    w = _Writer()
    algo = model.algo
    spec = model._spec
    w.meta["algo"] = algo
    w.meta["x"] = list(spec.x) if spec is not None else []
    w.meta["response"] = spec.y if spec is not None else None
    w.meta["response_domain"] = spec.response_domain if spec is not None else None
    w.meta["nclasses"] = spec.nclasses if spec is not None else 1
    w.meta["model_id"] = model.model_id
    if getattr(model, "_catenc", None) is not None:
        w.meta["catenc"] = model._catenc.to_dict()     # categorical_encoding, replayed by the scorer
    domains = []
    if algo in ("gbm", "drf", "xgboost", "isolationforest"):
        w.meta["x_domains"] = getattr(model, "_x_domains", {})
        _forest_arrays(w, model._forest, spec.x)
        w.meta["K"] = model._n_tree_classes()
        w.meta["ntrees"] = len(model._forest)
        if algo in ("gbm", "xgboost"):
            w.meta["init_f"] = list(model._init_f)
            w.meta["link"] = model._dist.link
            w.meta["family"] = model._dist.family
            w.meta["tweedie_power"] = getattr(model._dist, "tweedie_power", 1.5)
        if algo == "drf":
            w.meta["binomial_single"] = bool(model._binomial_single)
        if algo == "isolationforest":
            w.meta["min_len"] = model._min_len
            w.meta["max_len"] = model._max_len
            w.meta["threshold"] = model._threshold
    elif algo in ("glm", "gam"):
        if getattr(model, "_hglm", None) is not None:
            raise NotImplementedError("MOJO export of HGLM models is not supported (as in the reference)")
        _dinfo_meta(w, model._dinfo)
        if algo == "gam":
            w.meta["gam"] = {"cols": model._gam_cols, "bs": model._bs, "orders": model._orders,
                             "knots": [k.tolist() for k in model._knots], "means": model._col_means,
                             "keep": bool(model._parms.get("keep_gam_cols")),
                             "tp": {str(gi): {"terms": [list(e) for e in t["terms"]],
                                              "means": [float(v) for v in t["means"]],
                                              "ostd": [float(v) for v in t["ostd"]],
                                              "standardize": bool(t["standardize"])}
                                    for gi, t in getattr(model, "_tp", {}).items()}}
            for gi, Z in enumerate(model._Z):
                w.add_array(f"gamZ{gi}", np.asarray(Z))
            for gi, t in getattr(model, "_tp", {}).items():
                w.add_array(f"gamZcs{gi}", np.asarray(t["zCS"]))
        if getattr(model, "_multi", None) is not None:
            m = model._multi
            w.meta["multi"] = m["kind"]
            if m["kind"] == "multinomial":
                w.add_array("B", m["B"].cpu().numpy())
                w.add_array("b0", m["b0"].cpu().numpy())
            else:
                w.add_array("beta", m["beta"].cpu().numpy())
                w.add_array("theta", m["theta"].cpu().numpy())
        else:
            w.add_array("beta_std", np.asarray(model._beta_std))
            w.meta["family"] = model._fam.family
            w.meta["link"] = model._fam.link
            w.meta["tlp"] = model._fam.tlp
    elif algo == "glrm":
        p = model._parms
        lbc = {}
        if p.get("loss_by_col"):
            for name, i in zip(p["loss_by_col"], p.get("loss_by_col_idx") or []):
                lbc[model._cols[i] if isinstance(i, int) else i] = name
        w.meta["glrm"] = {"blocks": [list(b) for b in model._blocks], "doms": model._doms,
                          "stats": {c: list(v) for c, v in model._stats.items()},
                          "transform": str(p.get("transform") or "NONE").upper(),
                          "loss": p.get("loss") or "Quadratic", "loss_by_col": lbc,
                          "multi_loss": str(p.get("multi_loss") or "Categorical"), "period": float(p.get("period", 1)),
                          "regularization_x": p.get("regularization_x") or "None",
                          "gamma_x": float(p.get("gamma_x", 0.0)), "impute_original": bool(p.get("impute_original")),
                          "iters": int(model._score_iters())}
        w.meta["x_domains"] = model._doms
        w.add_array("Y", model._Y.detach().cpu().numpy().astype(np.float64))
    elif algo == "kmeans":
        _dinfo_meta(w, model._dinfo)
        # clustering space: one-hot categoricals at cat_scale (mismatch distance 1)
        w.meta["cat_scale"] = float(getattr(model, "_cat_scale", 1.0))
        w.add_array("centers_std", model._C_std[:, :model._dinfo.P].cpu().numpy())
    elif algo in ("pca",):
        _dinfo_meta(w, model._dinfo)
        w.add_array("evecs", model._evecs.cpu().numpy())
        w.add_array("mean", model._mean.cpu().numpy())
    elif algo == "deeplearning" and getattr(model, "_cat_slots", None) is not None:
        raise NotImplementedError("MOJO export of a DL model with hashed categoricals (max_categorical_features)")
    elif algo == "deeplearning":
        _dinfo_meta(w, model._dinfo)
        layers = []
        act_kind = {"tanh": "tanh", "rectifier": "relu", "exprectifier": "elu"}
        for i, L in enumerate(model._layers):
            w.add_array(f"W{i}", L.W.detach().cpu().numpy())
            w.add_array(f"b{i}", L.b.detach().cpu().numpy())
            if L.k > 1:
                layers.append(["maxout", i, L.k])
            else:
                layers.append(["linear", i])
                if L.act in act_kind:
                    layers.append([act_kind[L.act], i])
            if L.drop > 0:
                layers.append(["scale", i, 1.0 - L.drop])   # test-time dropout scaling
        w.meta["layers"] = layers
        w.meta["autoencoder"] = bool(model._ae)
        w.meta["K"] = model._K
        w.meta["ymu"] = getattr(model, "_ymu", 0.0)
        w.meta["ysd"] = getattr(model, "_ysd", 1.0)
    elif algo == "naivebayes":
        w.meta["nb"] = {}
        w.add_array("prior", model._prior.cpu().numpy())
        for i, (c, t) in enumerate(model._tables.items()):
            if t[0] == "cat":
                w.add_array(f"nb_{i}", t[1].cpu().numpy())
                w.meta["nb"][c] = ["cat", i, t[2]]
            else:
                w.add_array(f"nb_{i}_mean", t[1].cpu().numpy())
                w.add_array(f"nb_{i}_sd", t[2].cpu().numpy())
                w.meta["nb"][c] = ["num", i]
        w.meta["nb_params"] = {k: model._parms[k] for k in ("min_sdev", "eps_sdev", "min_prob", "eps_prob")}
    elif algo == "extendedisolationforest":
        _dinfo_meta(w, model._dinfo)
        for k in ("normal", "point", "left", "right", "value", "roots"):
            w.add_array(f"eif_{k}", model._packed[k].cpu().numpy())
        w.meta["psi"] = model._psi
        w.meta["height"] = model._height
        w.meta["ntrees"] = len(model._trees)
    elif algo == "isotonicregression":
        w.add_array("thresholds_x", np.asarray(model._tx))
        w.add_array("thresholds_y", np.asarray(model._ty))
        w.meta["out_of_bounds"] = str(model._parms.get("out_of_bounds", "NA"))
    elif algo == "coxph":
        _dinfo_meta(w, model._dinfo)
        w.add_array("beta", model._beta.cpu().numpy())
        keys = sorted(model._means)
        w.add_array("strata_keys", np.asarray(keys, dtype=np.int64))
        w.add_array("strata_means", np.stack([model._means[k].cpu().numpy() for k in keys]))
        w.meta["stratify_by"] = list(model._parms.get("stratify_by") or [])
        w.meta["strata_domains"] = getattr(model, "_strata_domains", {})
    elif algo == "upliftdrf":
        w.meta["x_domains"] = getattr(model, "_x_domains", {})
        _forest_arrays(w, model._forest, spec.x)
        w.meta["ntrees"] = len(model._forest) // 2
    elif algo == "word2vec":
        w.add_array("vectors", model._vecs.cpu().numpy())
        w.files["vocabulary.txt"] = "\n".join(model._vocab)
    elif algo == "targetencoder":
        te = {}
        for c, (dom, per) in model._tables.items():
            te[c] = {"domain": dom, "num": [st[0].cpu().tolist() for st in per], "den": [st[1].cpu().tolist() for st in per]}
        w.meta["te"] = te
        w.meta["suffix"] = model._suffix
        w.meta["prior"] = model._prior
        w.meta["te_params"] = {k: model._parms.get(k) for k in ("blending", "inflection_point", "smoothing",
                                                               "keep_original_categorical_columns")}
    elif algo == "rulefit":
        # nested tree MOJOs (leaf assignment) + ancestor tables -> rule columns,
        # then the nested GLM MOJO on [rule_i..., linear.<x>...]
        w.meta["rf_trees"] = []
        for mi, tm in enumerate(model._trees):
            w.files[f"models/tree_{mi}.zip"] = build_mojo(tm)
            nt = len(tm._forest.trees)
            w.meta["rf_trees"].append(nt)
            for ti in range(nt):
                w.add_array(f"anc_{mi}_{ti}", model._anc[(mi, ti)].cpu().numpy().astype(np.uint8))
        w.add_array("keep_cols", model._keep_cols.cpu().numpy().astype(np.int64))
        w.files["models/glm.zip"] = build_mojo(model._glm)
        w.meta["mtype"] = model._mtype
        w.meta["rule_names"] = model._rule_names
    elif algo == "stackedensemble":
        subs = []
        for i, bm in enumerate(model._base):
            w.files[f"models/{i}.zip"] = build_mojo(bm)
            subs.append(bm.model_id)
        w.files["models/meta.zip"] = build_mojo(model._meta)
        w.meta["base"] = subs
        w.meta["level1_names"] = model._names
        w.meta["metalearner_transform"] = str(model._parms.get("metalearner_transform") or "NONE")
    else:
        raise NotImplementedError(f"MOJO export not supported for {algo}")
    cols = (list(spec.x) + ([spec.y] if spec is not None and spec.y else [])) if spec is not None else []
    xd = getattr(model, "_x_domains", None) or (model._dinfo.domains if hasattr(model, "_dinfo") else {})
    for c in cols:
        if c in xd:
            domains.append((c, xd[c]))
    if spec is not None and spec.response_domain:
        domains.append((spec.y, spec.response_domain))
    info = {"algorithm": algo, "category": _category(model), "mojo_version": MOJO_VERSION,
            "n_features": len(spec.x) if spec else 0, "n_classes": spec.nclasses if spec else 1,
            "supervised": str(model.supervised_learning).lower(), "uuid": model.model_id,
            "h2o_version": "h2o3_amd-0.1.0"}
    try:
        from .h2o_writer import model_details_json
        w.files["experimental/modelDetails.json"] = model_details_json(model)
    except Exception:  # noqa: BLE001 - informational only
        pass
    return w.to_zip_bytes(info, cols, domains)


def write_mojo(model, path="."):
    data = build_mojo(model)
    if os.path.isdir(path) or not path.endswith(".zip"):
        os.makedirs(path, exist_ok=True)
        path = os.path.join(path, f"{model.model_id}.zip")
    with open(path, "wb") as f:
        f.write(data)
    return path
