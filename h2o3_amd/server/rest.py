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

    @app.post("/3/ParseSetup")
    def parse_setup(body: dict = Body(...)):
        """ParseSetupHandler: guessed separator / header for the source files."""
        src = body.get("source_frames") or body.get("paths") or []
        src = [s["name"] if isinstance(s, dict) else s for s in (src if isinstance(src, list) else [src])]
        if not src:
            raise HTTPException(400, "source_frames required")
        from ..core import parse as P
        st = P.parse_setup(src[0] if len(src) == 1 else src)
        return _jsonable({"source_frames": [{"name": s} for s in src], "separator": ord(st["separator"]),
                          "check_header": st.get("header", 0), "destination_frame": body.get("destination_frame")})

    @app.post("/3/Parse")
    def parse(body: dict = Body(...)):
        src = [s["name"] if isinstance(s, dict) else s for s in body.get("source_frames", [])]
        sep = body.get("separator")
        fr = api.import_file(src if len(src) > 1 else src[0], destination_frame=body.get("destination_frame"),
                             sep=chr(sep) if isinstance(sep, int) else sep, header=body.get("check_header", 0),
                             col_names=body.get("column_names"), col_types=body.get("column_types"))
        fid = body.get("destination_frame") or fr.frame_id
        dkv.put(fid, fr)
        return {"job": {"key": {"name": f"parse_{fid}"}, "status": "DONE", "progress": 1.0,
                        "dest": {"name": fid}}, "destination_frame": {"name": fid}}

    @app.get("/3/DownloadDataset")
    def download_dataset(frame_id: str):
        from fastapi.responses import PlainTextResponse
        fr = dkv.get(frame_id)
        if not isinstance(fr, H2OFrame):
            raise HTTPException(404, f"frame {frame_id} not found")
        return PlainTextResponse(fr.as_data_frame().to_csv(index=False), media_type="text/csv")

    @app.get("/3/Models/{mid}/mojo")
    def model_mojo(mid: str):
        from fastapi.responses import Response
        from ..mojo.writer import build_mojo
        m = dkv.get(mid)
        if m is None:
            raise HTTPException(404, f"model {mid} not found")
        try:
            data = build_mojo(m)
        except NotImplementedError as e:
            raise HTTPException(400, str(e))
        return Response(content=data, media_type="application/zip",
                        headers={"Content-Disposition": f'attachment; filename="{mid}.zip"'})

    @app.get("/3/Models.java/{mid}")
    def model_pojo(mid: str):
        from fastapi.responses import PlainTextResponse
        from ..mojo.pojo import to_java
        m = dkv.get(mid)
        if m is None:
            raise HTTPException(404, f"model {mid} not found")
        try:
            return PlainTextResponse(to_java(m), media_type="text/plain")
        except NotImplementedError as e:
            raise HTTPException(400, str(e))

    @app.post("/3/ModelMetrics/models/{mid}/frames/{fid}")
    def model_metrics(mid: str, fid: str):
        m, fr = dkv.get(mid), dkv.get(fid)
        if m is None or not isinstance(fr, H2OFrame):
            raise HTTPException(404, "model or frame not found")
        mm_ = m.model_performance(fr)
        return {"model_metrics": [{k: _jsonable(v) for k, v in mm_._m.items() if isinstance(v, (int, float, str))}]}

    @app.post("/99/Grid/{algo}")
    def grid(algo: str, body: dict = Body(...)):
        """GridSearchHandler: hyper_parameters + search_criteria over one algo."""
        from ..grid import H2OGridSearch
        cls = _algo_cls(algo)
        p = dict(body)
        tf = dkv.get(p.pop("training_frame", None))
        if not isinstance(tf, H2OFrame):
            raise HTTPException(400, "training_frame not found")
        vf = p.pop("validation_frame", None)
        hyper = p.pop("hyper_parameters", {})
        crit = p.pop("search_criteria", None)
        gid = p.pop("grid_id", None)
        y = p.pop("response_column", None)
        g = H2OGridSearch(cls(**p), hyper, grid_id=gid, search_criteria=crit)
        g.train(y=y, training_frame=tf, validation_frame=dkv.get(vf) if vf else None)
        return {"job": {"key": {"name": f"grid_{g.grid_id}"}, "status": "DONE", "progress": 1.0,
                        "dest": {"name": g.grid_id}}}

    @app.get("/99/Grids/{gid}")
    def grid_get(gid: str):
        g = dkv.get(gid)
        if g is None or not hasattr(g, "model_ids"):
            raise HTTPException(404, f"grid {gid} not found")
        tab = g.get_grid().sorted_metric_table()
        return _jsonable({"grid_id": {"name": gid}, "model_ids": [{"name": m} for m in g.model_ids],
                          "failure_details": [e for _, e in g.failed_params],
                          "summary_table": tab.to_dict(orient="list")})

    @app.post("/99/AutoMLBuilder")
    def automl(body: dict = Body(...)):
        """AutoMLBuilderHandler: build_control / input_spec / build_models."""
        from ..automl import H2OAutoML
        bc, ispec, bm = body.get("build_control", {}), body.get("input_spec", {}), body.get("build_models", {})
        tf = dkv.get(ispec.get("training_frame"))
        if not isinstance(tf, H2OFrame):
            raise HTTPException(400, "input_spec.training_frame not found")
        sc = bc.get("stopping_criteria", {})
        aml = H2OAutoML(project_name=bc.get("project_name"), nfolds=bc.get("nfolds", -1),
                        max_models=sc.get("max_models"), max_runtime_secs=sc.get("max_runtime_secs"),
                        seed=sc.get("seed"), exclude_algos=bm.get("exclude_algos"),
                        include_algos=bm.get("include_algos"), sort_metric=ispec.get("sort_metric", "AUTO"))
        aml.train(y=ispec.get("response_column"), training_frame=tf,
                  validation_frame=dkv.get(ispec["validation_frame"]) if ispec.get("validation_frame") else None,
                  leaderboard_frame=dkv.get(ispec["leaderboard_frame"]) if ispec.get("leaderboard_frame") else None)
        return {"job": {"key": {"name": f"automl_{aml.project_name}"}, "status": "DONE", "progress": 1.0,
                        "dest": {"name": aml.project_name}}}

    @app.get("/99/Leaderboards/{project}")
    def leaderboard(project: str):
        aml = dkv.get(project)
        if aml is None or not hasattr(aml, "leaderboard"):
            raise HTTPException(404, f"AutoML project {project} not found")
        lb = aml.leaderboard.as_data_frame()
        return _jsonable({"project_name": project, "models": [{"name": m} for m in lb["model_id"]],
                          "table": lb.to_dict(orient="list")})

    @app.get("/3/About")
    def about():
        i = cloud.info()
        return {"entries": [{"name": "Build project version", "value": "h2o3_amd-0.1.0"},
                            {"name": "Device", "value": str(i.get("device"))},
                            {"name": "Cloud size", "value": str(i.get("world"))}]}

    @app.get("/3/Capabilities")
    def capabilities():
        return {"capabilities": [{"name": n} for n in ("Algos", "AutoML", "Grid", "MOJO", "POJO", "Rapids",
                                                      "HIP-gfx950", "RCCL")]}

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
