"""Binary model save / load (h2o.save_model / h2o.load_model).

Reference: hex/Model.exportBinaryModel / importBinaryModel (Java
serialization of the whole model).  Here a saved model is a directory-free
zip: the full estimator state (models/state_io.py: plain containers +
tensors, read back with torch.load(weights_only=True)), the MOJO when the
algorithm has one, params.json and metrics.json -- no pickle, so loading
never executes code from the file.  A loaded model is the same estimator:
it scores, keeps its outputs and metrics, and can be a checkpoint.
"""
from __future__ import annotations

import io
import json
import os
import zipfile

import numpy as np


def _metrics_dict(m):
    if m is None:
        return None
    out = {"kind": m.kind}
    for k, v in m._m.items():
        if isinstance(v, (int, float, str, bool)) or v is None:
            out[k] = v
        elif k == "cm":
            out[k] = {kk: (vv if not isinstance(vv, np.ndarray) else vv.tolist()) for kk, vv in v.items()}
    return out


def save_model(model, path="", force=False, filename=None):
    from ..core.persist import exists, is_remote, upload
    if is_remote(path):
        # object store: write locally, then upload (PersistManager.create);
        # an existing object is only replaced with force=True, as on disk
        import tempfile
        dest = path.rstrip("/") + "/" + (filename or model.model_id)
        if not force and exists(dest):
            raise FileExistsError(dest)
        from ..parallel import cloud
        with tempfile.TemporaryDirectory() as td:
            local = save_model(model, td, force=True, filename=filename)
            if cloud.rank() == 0:
                upload(local, dest)
        cloud.barrier()
        return dest
    from ..mojo.writer import build_mojo
    from ..parallel import cloud
    from ..parallel import collectives as coll
    os.makedirs(path or ".", exist_ok=True)
    fn = os.path.join(path or ".", filename or model.model_id)
    # rank 0 checks and writes (the model is replicated); every rank agrees
    if coll.broadcast_object(os.path.exists(fn)) and not force:
        raise FileExistsError(fn)
    from .state_io import dumps
    # every rank packs (row-sharded state -- CV holdout predictions, GLRM X,
    # SVD U frames -- is all-gathered so the archive holds every row)
    state = dumps(model, gather=cloud.world() > 1)
    err = None
    if cloud.rank() == 0:
        try:
            params = {k: _jsonable(v) for k, v in model._parms.items()
                      if isinstance(v, (int, float, str, bool, list, type(None)))}
            try:
                mojo = build_mojo(model)
            except NotImplementedError:
                mojo = None          # no MOJO for this algorithm: the state archive carries it
            with zipfile.ZipFile(fn, "w", zipfile.ZIP_DEFLATED) as z:
                z.writestr("state.pt", state)
                if mojo is not None:
                    z.writestr("mojo.zip", mojo)
                z.writestr("params.json", json.dumps({"algo": model.algo, "model_id": model.model_id,
                                                      "params": params}))
                z.writestr("metrics.json", json.dumps({"training": _metrics_dict(model._training_metrics),
                                                       "validation": _metrics_dict(model._validation_metrics),
                                                       "xval": _metrics_dict(model._cross_validation_metrics),
                                                       "output": {k: v for k, v in model._output.items()
                                                                  if isinstance(v, (dict, list, float, int, str))}},
                                                      default=str))
        except Exception as e:          # noqa: BLE001 -- re-raised on every rank below
            err = f"{type(e).__name__}: {e}"
    # a failure on rank 0 is raised on every rank (no rank left waiting in a
    # barrier that the writer's next collective would pair with)
    err = coll.broadcast_object(err)
    if err is not None:
        raise RuntimeError(f"save_model failed on rank 0: {err}")
    return fn


def _jsonable(v):
    if isinstance(v, list):
        return [_jsonable(x) for x in v]
    if isinstance(v, (int, float, str, bool, type(None))):
        return v
    return getattr(v, "model_id", None) or getattr(v, "frame_id", None) or type(v).__name__


def load_model(path):
    from ..core.persist import is_remote, resolve
    if is_remote(path):
        # the saved model IS a zip: download it as is (no archive unpacking)
        path = resolve(path, raw=True)
    from . import metrics as mm
    from .generic import H2OGenericEstimator
    from ..core import dkv
    with zipfile.ZipFile(path) as z:
        names = set(z.namelist())
        if "state.pt" in names:
            from .state_io import loads
            est = loads(z.read("state.pt"))
            dkv.put(est.model_id, est)
            return est
        mojo = z.read("mojo.zip")
        meta = json.loads(z.read("params.json"))
        mets = json.loads(z.read("metrics.json"))
    tmp = path + ".mojo.zip"
    with open(tmp, "wb") as f:
        f.write(mojo)
    est = H2OGenericEstimator.from_file(tmp, model_id=meta["model_id"])
    est.algo = meta["algo"]
    est._parms.update(meta["params"])
    kinds = {"binomial": mm.ModelMetricsBinomial, "multinomial": mm.ModelMetricsMultinomial,
             "regression": mm.ModelMetricsRegression, "clustering": mm.ModelMetricsClustering}
    for attr, key in (("_training_metrics", "training"), ("_validation_metrics", "validation"),
                      ("_cross_validation_metrics", "xval")):
        d = mets.get(key)
        if d:
            cls = kinds.get(d.pop("kind", ""), mm.ModelMetrics)
            setattr(est, attr, cls(**d))
    est._output.update(mets.get("output") or {})
    dkv.put(est.model_id, est)
    return est
