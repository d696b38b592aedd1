"""REST API (subset of the reference's /3 endpoints).

Reference: water/api/RequestServer.java + the schema handlers under
water/api/ (CloudHandler, ImportFilesHandler, ParseHandler, FramesHandler,
ModelBuilderHandler, ModelsHandler, ModelMetricsHandler (predictions),
JobsHandler, DKVHandler, TimelineHandler, MetadataHandler).  JSON shapes
follow the reference's field names where clients read them (frame_id /
model_id as {"name": ...}, job {"key", "status", "progress", "dest"}).

Model builds run synchronously inside the request on the serving process
(the compute itself runs on the GPU through the same estimators the
Python API uses).  Multi-rank clouds are driven SPMD from Python; the
REST server serves a single-process (world size 1) cloud.
"""
from __future__ import annotations

import math

from fastapi import Body, FastAPI, HTTPException

import importlib

api = importlib.import_module("h2o3_amd.api")  # the module (the package re-exports a function named api)
from ..core import dkv
from ..core.frame import H2OFrame
from ..parallel import cloud


def _algo_cls(algo):
    from .. import estimators as E
    table = {"gbm": E.H2OGradientBoostingEstimator, "glm": E.H2OGeneralizedLinearEstimator,
             "drf": E.H2ORandomForestEstimator, "xgboost": E.H2OXGBoostEstimator,
             "deeplearning": E.H2ODeepLearningEstimator, "kmeans": E.H2OKMeansEstimator,
             "pca": E.H2OPrincipalComponentAnalysisEstimator, "svd": E.H2OSingularValueDecompositionEstimator,
             "naivebayes": E.H2ONaiveBayesEstimator, "isolationforest": E.H2OIsolationForestEstimator,
             "extendedisolationforest": E.H2OExtendedIsolationForestEstimator, "glrm": E.H2OGeneralizedLowRankEstimator,
             "coxph": E.H2OCoxProportionalHazardsEstimator, "gam": E.H2OGeneralizedAdditiveEstimator,
             "rulefit": E.H2ORuleFitEstimator, "isotonicregression": E.H2OIsotonicRegressionEstimator,
             "upliftdrf": E.H2OUpliftRandomForestEstimator, "psvm": E.H2OSupportVectorMachineEstimator,
             "word2vec": E.H2OWord2vecEstimator, "targetencoder": E.H2OTargetEncoderEstimator,
             "aggregator": E.H2OAggregatorEstimator, "anovaglm": E.H2OANOVAGLMEstimator,
             "modelselection": E.H2OModelSelectionEstimator, "stackedensemble": E.H2OStackedEnsembleEstimator}
    if algo not in table:
        raise HTTPException(404, f"unknown algo {algo}")
    return table[algo]


def _jsonable(v):
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return None
    if isinstance(v, (int, float, str, bool)) or v is None:
        return v
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    try:
        import numpy as np
        if isinstance(v, np.generic):
            return _jsonable(v.item())
        if isinstance(v, np.ndarray):
            return _jsonable(v.tolist())
    except ImportError:
        pass
    return str(v)


def _frame_json(fid, fr: H2OFrame, rows=10):
    cols = []
    for n in fr.names:
        v = fr.vec(n)
        c = {"label": n, "type": v.type, "domain": v.domain}
        if v.is_numeric:
            r = v.rollups()
            c.update(min=r.get("min"), max=r.get("max"), mean=r.get("mean"), sigma=r.get("sigma"),
                     missing_count=r.get("nas"))
        cols.append(c)
    head = fr.head(rows).as_data_frame() if fr.nrow else None
    return _jsonable({"frame_id": {"name": fid}, "rows": fr.nrow, "column_count": fr.ncol, "columns": cols,
                      "data": head.to_dict(orient="list") if head is not None else {}})


def _model_json(mid, m):
    out = {"model_id": {"name": mid}, "algo": m.algo, "parameters": {k: _jsonable(v) for k, v in m._parms.items()
                                                                    if not hasattr(v, "as_data_frame")},
           "output": {"model_category": m.type if hasattr(m, "type") else None}}
    tm = m._training_metrics
    if tm is not None:
        out["output"]["training_metrics"] = {k: _jsonable(v) for k, v in tm._m.items()
                                             if isinstance(v, (int, float, str)) or v is None}
    return _jsonable(out)


def create_app() -> FastAPI:
    app = FastAPI(title="h2o3_amd REST API", version="3")

    @app.get("/3/Cloud")
    def cloud_status():
        i = cloud.info()
        return _jsonable({"cloud_name": i.get("name"), "cloud_size": i.get("world"), "cloud_healthy": True,
                          "consensus": True, "locked": False, "version": "h2o3_amd-0.1.0",
                          "nodes": [{"h2o": f"rank{r}", "healthy": True} for r in range(i.get("world", 1))],
                          "backend": i.get("backend"), "device": str(i.get("device"))})

    @app.post("/3/ImportFiles")
    def import_files(path: str, destination_frame: str | None = None):
        fr = api.import_file(path, destination_frame=destination_frame)
        fid = destination_frame or fr.frame_id
        dkv.put(fid, fr)
        return {"destination_frames": [fid], "files": [path], "fails": []}

    @app.post("/3/PostFile")
    def post_file(body: dict = Body(...)):
        import pandas as pd
        df = pd.DataFrame(body["data"])
        fr = H2OFrame(df)
        fid = body.get("destination_frame") or fr.frame_id
        dkv.put(fid, fr)
        return {"destination_frame": fid}

    @app.get("/3/Frames")
    def frames():
        return {"frames": [{"frame_id": {"name": k}, "rows": dkv.get(k).nrow, "columns": dkv.get(k).ncol}
                           for k in dkv.keys() if isinstance(dkv.get(k), H2OFrame)]}

    @app.get("/3/Frames/{fid}")
    def frame(fid: str, row_count: int = 10):
        fr = dkv.get(fid)
        if not isinstance(fr, H2OFrame):
            raise HTTPException(404, f"frame {fid} not found")
        return {"frames": [_frame_json(fid, fr, row_count)]}

    @app.get("/3/Frames/{fid}/summary")
    def frame_summary(fid: str):
        return frame(fid, 0)

    @app.post("/3/ModelBuilders/{algo}")
    def build(algo: str, params: dict = Body(...)):
        cls = _algo_cls(algo)
        p = dict(params)
        tf = dkv.get(p.pop("training_frame", None))
        if not isinstance(tf, H2OFrame):
            raise HTTPException(400, "training_frame not found")
        vf = p.pop("validation_frame", None)
        vf = dkv.get(vf) if vf else None
        y = p.pop("response_column", None)
        x = p.pop("x", None)
        ignored = p.pop("ignored_columns", None) or []
        if x is None:
            x = [c for c in tf.names if c != y and c not in ignored]
        m = cls(**p)
        try:
            if m.supervised_learning:
                m.train(x=x, y=y, training_frame=tf, validation_frame=vf)
            else:
                m.train(x=x, training_frame=tf)
        except Exception as e:  # noqa: BLE001 - reported to the client as a failed job
            raise HTTPException(400, f"model build failed: {e}")
        j = m._job
        return {"job": {"key": {"name": j.key}, "status": j.status, "progress": j.progress,
                        "dest": {"name": m.model_id}}, "messages": []}

    @app.get("/3/Models")
    def models():
        from ..models.base import H2OEstimator
        return {"models": [_model_json(k, dkv.get(k)) for k in dkv.keys() if isinstance(dkv.get(k), H2OEstimator)]}

    @app.get("/3/Models/{mid}")
    def model(mid: str):
        m = dkv.get(mid)
        if m is None:
            raise HTTPException(404, f"model {mid} not found")
        return {"models": [_model_json(mid, m)]}

    @app.post("/3/Predictions/models/{mid}/frames/{fid}")
    def predict(mid: str, fid: str, predictions_frame: str | None = None):
        m, fr = dkv.get(mid), dkv.get(fid)
        if m is None or not isinstance(fr, H2OFrame):
            raise HTTPException(404, "model or frame not found")
        pr = m.predict(fr)
        key = predictions_frame or f"prediction_{mid}_on_{fid}"
        dkv.put(key, pr)
        perf = None
        try:
            if m._spec is not None and m._spec.y in fr.names:
                mm_ = m.model_performance(fr)
                perf = {k: _jsonable(v) for k, v in mm_._m.items() if isinstance(v, (int, float, str))}
        except Exception:  # noqa: BLE001 - metrics are optional for scoring
            perf = None
        return {"predictions_frame": {"name": key}, "model_metrics": [perf] if perf else []}

    @app.get("/3/Jobs")
    def jobs():
        return {"jobs": [{"key": {"name": j.key}, "description": j.description, "status": j.status,
                          "progress": j.progress, "dest": {"name": j.dest}, "msec": int(j.run_time * 1000),
                          "exception": j.exception} for j in api.jobs()]}

    @app.get("/3/Jobs/{jid}")
    def job(jid: str):
        for j in api.jobs():
            if j.key == jid:
                return {"jobs": [{"key": {"name": j.key}, "status": j.status, "progress": j.progress,
                                  "dest": {"name": j.dest}}]}
        raise HTTPException(404, f"job {jid} not found")

    @app.delete("/3/DKV/{key}")
    def delete(key: str):
        dkv.remove(key)
        return {"key": key}

    @app.delete("/3/DKV")
    def delete_all():
        dkv.remove_all()
        return {}

    @app.get("/3/Timeline")
    def timeline():
        return {"events": api.timeline()}

    @app.post("/99/Rapids")
    def rapids_exec(body: dict = Body(...)):
        """Rapids expression evaluation (water/api/RapidsHandler.java): frame
        results are stored under their key and described; scalars/lists/strings
        come back inline."""
        from ..core.rapids import RapidsError, rapids
        try:
            res = rapids(body.get("ast", ""))
        except (RapidsError, KeyError, ValueError, TypeError) as e:
            raise HTTPException(400, f"Rapids error: {e}")
        if isinstance(res, H2OFrame):
            dkv.put(res.frame_id, res)
            return {"key": {"name": res.frame_id}, "num_rows": res.nrows, "num_cols": res.ncols}
        if isinstance(res, str):
            return {"string": res}
        if isinstance(res, (list, tuple)):
            return {"scalar": None, "ns": [_jsonable(x) for x in res]}
        return {"scalar": _jsonable(res)}

    @app.get("/3/Metadata/endpoints")
    def endpoints():
        return {"routes": [{"url_pattern": r.path, "http_method": sorted(r.methods)[0]} for r in app.routes
                           if hasattr(r, "methods")]}

    return app


def start(ip="127.0.0.1", port=54321, log_level="warning"):
    """Serve the REST API (blocking) on rank 0 of a single-process cloud."""
    import uvicorn
    api.init()
    uvicorn.run(create_app(), host=ip, port=port, log_level=log_level)
