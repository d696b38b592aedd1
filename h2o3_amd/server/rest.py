"""REST API speaking the reference's /3 protocol.

Reference: water/api/RequestServer.java and the handlers under water/api/
(CloudHandler, MetadataHandler, SessionsHandler (/4/sessions), PostFile,
ParseSetupHandler, ParseHandler, FramesHandler, DownloadDataHandler,
ModelBuilderHandler, ModelsHandler, ModelMetricsHandler, JobsHandler,
DKVHandler, RapidsHandler, GridSearchHandler, AutoMLBuilderHandler,
TimelineHandler, AboutHandler).

Requests are accepted the way the reference clients send them -- form
fields (x-www-form-urlencoded or multipart) in H2O's list syntax, query
strings for GETs -- and also as JSON bodies.  Responses carry the schema
``__meta`` blocks the clients dispatch on (see schemas.py), so the
reference's own Python client (h2o-py: h2o.connect / H2OFrame / estimators
/ predict / model_performance / Rapids frame munging) runs against this
server; tests/test_rest_wire.py drives it end to end.

One REST endpoint drives the whole multi-GPU cloud (spmd.py): rank 0
serves HTTP, every request that touches frames, models or collectives is
replayed as a command on every rank by rank 0's executor thread (ranks
1..N-1 run `spmd.worker_loop`), and model / grid / AutoML builds answer with
the RUNNING job at once and keep training on the executor, so `/3/Jobs`
polls see live progress and `/3/Jobs/{id}/cancel` stops a build at its next
tree / iteration.  Launch a cloud with
`torchrun --nproc-per-node N -m h2o3_amd.server`.
"""
from __future__ import annotations

import asyncio
import json as _json
import os
import sys
import tempfile
import time
import uuid

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, Response

import importlib

api = importlib.import_module("h2o3_amd.api")  # the module (the package re-exports a function named api)
from ..core import dkv
from ..core.frame import H2OFrame
from ..parallel import cloud
from . import schemas as S
from . import spmd

# requests served straight from rank 0's state on the HTTP thread (no
# collective, no command replay): clients poll / cancel jobs and read the
# cloud status while a build holds the executor
# GETs served on the HTTP thread while a build runs (collectives refused:
# collectives.forbid; a read that needs one is queued as usual)
# GET routes served on the HTTP thread while a build runs (exact route
# templates, no prefixes): pure reads of finished DKV objects and listings.
# Export / download / binary-model / scoring routes are NOT here -- they write
# files, serialise whole models or score, so they queue behind the build.
_READ_ROUTES = frozenset((
    "/3/Frames", "/3/Frames/{fid}", "/3/Frames/{fid}/light", "/3/Frames/{fid}/summary",
    "/3/Frames/{fid}/columns", "/3/Frames/{fid}/columns/{col}", "/3/Frames/{fid}/columns/{col}/domain",
    "/3/Frames/{fid}/columns/{col}/summary",
    "/3/Models", "/3/Models/{mid}", "/99/Models/{mid}", "/99/Models/{mid}/json",
    "/3/ModelBuilders", "/3/ModelBuilders/{algo}",
    "/99/Leaderboards", "/99/Leaderboards/{project}", "/99/AutoML/{project}",
    "/99/Grids", "/99/Grids/{gid}",
    "/3/ModelMetrics", "/3/ModelMetrics/models/{mid}", "/3/ModelMetrics/frames/{fid}",
    "/99/Rapids/help"))
# builds accepted while another build runs: CREATED job at once, run later
_BUILD_ROUTES = {"/3/ModelBuilders/{algo}": "model", "/99/Grid/{algo}": "grid", "/99/AutoMLBuilder": "automl"}

_LOCAL_PREFIXES = ("/3/Cloud", "/3/Metadata", "/4/sessions", "/3/InitID", "/3/Capabilities", "/3/About",
                   "/3/Jobs", "/3/NodePersistentStorage", "/3/Ping", "/3/Logs", "/3/JStack", "/3/WaterMeter",
                   "/3/SteamMetrics", "/3/Profiler", "/3/SessionProperties", "/3/Typeahead", "/3/LogAndEcho")

_ALGOS = {"gbm": "H2OGradientBoostingEstimator", "glm": "H2OGeneralizedLinearEstimator",
          "drf": "H2ORandomForestEstimator", "xgboost": "H2OXGBoostEstimator",
          "deeplearning": "H2ODeepLearningEstimator", "kmeans": "H2OKMeansEstimator",
          "pca": "H2OPrincipalComponentAnalysisEstimator", "svd": "H2OSingularValueDecompositionEstimator",
          "naivebayes": "H2ONaiveBayesEstimator", "isolationforest": "H2OIsolationForestEstimator",
          "extendedisolationforest": "H2OExtendedIsolationForestEstimator", "glrm": "H2OGeneralizedLowRankEstimator",
          "coxph": "H2OCoxProportionalHazardsEstimator", "gam": "H2OGeneralizedAdditiveEstimator",
          "rulefit": "H2ORuleFitEstimator", "isotonicregression": "H2OIsotonicRegressionEstimator",
          "upliftdrf": "H2OUpliftRandomForestEstimator", "psvm": "H2OSupportVectorMachineEstimator",
          "word2vec": "H2OWord2vecEstimator", "targetencoder": "H2OTargetEncoderEstimator",
          "aggregator": "H2OAggregatorEstimator", "anovaglm": "H2OANOVAGLMEstimator",
          "modelselection": "H2OModelSelectionEstimator", "stackedensemble": "H2OStackedEnsembleEstimator",
          "infogram": "H2OInfogram", "hglm": "H2OGeneralizedLinearEstimator"}

# parameters naming frames / models that are resolved from the key store
_FRAME_PARAMS = {"training_frame", "validation_frame", "calibration_frame", "blending_frame", "user_points",
                 "beta_constraints", "plug_values", "linear_constraints", "pre_trained", "user_x", "user_y",
                 "leaderboard_frame", "loading_frame", "offset_frame"}
_MODEL_PARAMS = {"checkpoint", "pretrained_autoencoder", "metalearner_model"}
# client-side bookkeeping the estimators do not take
_DROP_PARAMS = {"_rest_version", "ignored_columns", "response_column", "training_frame", "validation_frame", "x",
                "interactions_only"}

_TYPE_NAMES = {"real": "Numeric", "int": "Numeric", "enum": "Enum", "string": "String", "time": "Time",
               "uuid": "UUID", "bad": "BAD"}
_TYPE_IN = {"numeric": "numeric", "real": "real", "int": "int", "enum": "enum", "categorical": "enum",
            "factor": "enum", "string": "string", "time": "time", "uuid": "uuid", "bad": "numeric"}


class _HTTPError(Exception):
    def __init__(self, status, msg, exc=None, builder=False):
        super().__init__(msg)
        self.status, self.msg, self.exc, self.builder = status, msg, exc, builder


def _algo_cls(algo):
    from .. import estimators as E
    name = _ALGOS.get(algo.lower())
    cls = getattr(E, name, None) if name else None
    if cls is None:
        raise _HTTPError(404, f"Unknown algo: {algo}")
    return cls


_NUMERIC_STR = None


def _coerce_params(cls, p):
    """Model parameters arriving as strings in JSON bodies (Flow sends
    "ntrees": "100", "learn_rate": "0.01") are parsed into the parameter's
    type, as the reference's schema layer does (water/api/Schema.java
    parse): by the type of the builder's default, numbers for numeric text
    when the default is None (keys, columns and frames are left alone)."""
    import re
    global _NUMERIC_STR
    if _NUMERIC_STR is None:
        _NUMERIC_STR = re.compile(r"[-+]?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?")
    try:
        defaults = cls()._parms
    except Exception:  # noqa: BLE001 - no coercion when the defaults are unavailable
        return p
    out = {}
    for k, v in p.items():
        d = defaults.get(k)
        if isinstance(v, str) and not isinstance(d, str) and k not in _FRAME_PARAMS | _MODEL_PARAMS and \
                not k.endswith(("_id", "_column", "_columns", "_frame")):
            t = v.strip()
            if len(t) > 1 and t[-1] in "fFdDlL" and _NUMERIC_STR.fullmatch(t[:-1]):
                t = t[:-1]                             # Java literals: Float.parseFloat("1.0f")
            if isinstance(d, bool):
                v = t.lower() in ("true", "1")
            elif _NUMERIC_STR.fullmatch(t):
                f = float(t)
                v = float(t) if isinstance(d, float) else (int(f) if f.is_integer() and "." not in t
                                                          and "e" not in t.lower() else f)
            elif isinstance(d, (list, dict)) and t[:1] in "[{":
                try:
                    v = _json.loads(t)
                except ValueError:
                    pass
        out[k] = v
    return out


def _multipart(body: bytes, ctype: str) -> list[tuple[str, str | None, bytes]]:
    """multipart/form-data body -> [(field name, filename or None, bytes)]
    (stdlib email parser; python-multipart is not available here)."""
    from email.parser import BytesParser
    from email.policy import HTTP
    msg = BytesParser(policy=HTTP).parsebytes(b"Content-Type: " + ctype.encode() + b"\r\n\r\n" + body)
    out = []
    for part in msg.iter_parts():
        name = part.get_param("name", header="content-disposition")
        out.append((name, part.get_filename(), part.get_payload(decode=True) or b""))
    return out


async def _params(request: Request) -> dict:
    """Query + form (urlencoded / multipart, files excluded) + JSON body,
    decoded from the client's encoding (schemas.parse_value)."""
    from urllib.parse import parse_qsl
    raw = dict(request.query_params)
    ctype = request.headers.get("content-type", "")
    if ctype.startswith("application/json"):
        body = await request.body()
        if body:
            j = _json.loads(body)
            if isinstance(j, dict):
                return {**S.parse_params(raw), **j}
    elif ctype.startswith("application/x-www-form-urlencoded"):
        raw.update(parse_qsl((await request.body()).decode("utf-8"), keep_blank_values=True))
    elif ctype.startswith("multipart/form-data"):
        for name, fname, data in _multipart(await request.body(), ctype):
            if fname is None and name:
                raw[name] = data.decode("utf-8", "replace")
    return S.parse_params(raw)


def _frame(fid, what="frame") -> H2OFrame:
    fr = dkv.get(fid) if fid is not None else None
    if not isinstance(fr, H2OFrame):
        raise _HTTPError(404, f"Object '{fid}' not found for argument: {what}")
    return fr


def _model(mid):
    from ..models.base import H2OEstimator
    m = dkv.get(mid) if mid is not None else None
    if not isinstance(m, H2OEstimator):
        raise _HTTPError(404, f"Object '{mid}' not found for argument: key")
    return m


def _put_frame(fr: H2OFrame, fid=None) -> str:
    fid = fid or fr.frame_id
    if fr.frame_id != fid:
        try:
            fr.frame_id = fid
        except AttributeError:
            pass
    dkv.put(fid, fr)
    # row counts and rollups now, on every rank (this runs replayed on the
    # executor): later frame reads are served from these caches without
    # collectives, also while a build runs (the reference's parse ends with
    # the rollups too, water/parser/ParseDataset.java)
    if cloud.is_distributed():
        for v in fr._vecs:
            v.nrow()
            if v.is_numeric and not v.on_host:
                try:
                    v.rollups()
                except Exception:  # noqa: BLE001 - a column without rollups is read through the executor
                    pass
    return fid


class _Uploads:
    """Raw uploaded files (the reference's raw ByteVec keys from PostFile /
    ImportFiles): key -> local path, plus the parse-setup guess per key."""

    def __init__(self):
        self.dir = tempfile.mkdtemp(prefix="h2o3_amd_upload_")
        self.paths: dict[str, list[str]] = {}
        self.setups: dict[str, tuple] = {}

    def add_bytes(self, data: bytes, name: str | None = None) -> str:
        import re
        k = name or f"upload_{spmd.rand_hex(16)}"
        # the key names the file inside the upload directory: no separators, no dot-files
        p = os.path.join(self.dir, re.sub(r"[^A-Za-z0-9._-]", "_", k).lstrip(".") or "upload")
        with open(p, "wb") as f:
            f.write(data)
        self.paths[k] = [p]
        return k

    def resolve(self, keys) -> list[str]:
        out = []
        for k in keys:
            out += self.paths.get(k, [k])
        return out


def create_app(flow_dir: str | None = None, serve: bool = True) -> FastAPI:
    """The REST app.  serve=False (ranks 1..N-1 of a multi-rank cloud): the
    same handler table, replayed from rank 0's commands by
    spmd.worker_loop(app.state.run_command); no HTTP."""
    app = FastAPI(title="h2o3_amd REST API", version="3")
    table = {}                        # (method, path) -> handler(p, r, **path)
    uploads = _Uploads()
    sessions: dict[str, float] = {}
    t_start = time.time()

    @app.exception_handler(_HTTPError)
    async def _err(request: Request, e: _HTTPError):
        return JSONResponse(S.error_v3(e.msg, e.status, e.exc, builder=e.builder, url=str(request.url.path)),
                            status_code=e.status)

    import re as _re
    from urllib.parse import unquote as _unquote
    app.state.flow_routes = []      # (method, path regex, handler, jsonify): flow.LocalTransport

    def _jsonify(out):
        if isinstance(out, Response):
            return out.body.decode("utf-8", "replace")
        return S.jsonable(out)

    def _to_response(out):
        if isinstance(out, Response):
            return out
        return JSONResponse(S.jsonable(out))

    def run_command(cmd, loop):
        """Execute one replayed command on this rank (spmd.execute)."""
        if cmd["kind"] == "flow":
            res = flow_runner.run_cell(cmd["input"], cmd["type"])
            return JSONResponse({"ok": True, "result": S.jsonable(res)})
        fn = table[(cmd["method"], cmd["path"])]
        req = spmd.Req(**cmd["req"])
        try:
            out = fn(cmd["p"], req, **cmd["kw"])
            if hasattr(out, "__await__"):
                out = loop.run_until_complete(out)
        except _HTTPError:
            raise
        except (KeyError, ValueError, TypeError, RuntimeError, AssertionError, IndexError,
                NotImplementedError) as e:
            raise _HTTPError(400 if not isinstance(e, KeyError) else 404, str(e), e)
        if isinstance(out, spmd.Deferred):
            out.response = _to_response(out.response)
            return out
        return _to_response(out)

    app.state.run_command = run_command
    executor = spmd.Executor(run_command) if serve else None
    app.state.executor = executor

    def _queue_build(kind, cmd, path_params):
        """A build that arrives while another one runs: fix its job key and
        destination now (hints broadcast with the command, so every rank uses
        them), answer with the CREATED job, and let the executor run it in
        turn (ModelBuilderHandler / GridSearchHandler / AutoMLBuilderHandler
        return the job without waiting, water/api/ModelBuilderHandler.java:51)."""
        from ..core import job as jobmod
        import secrets
        q = secrets.token_hex(6)
        p = dict(cmd["p"])
        algo = path_params.get("algo", "automl")
        if kind == "model":
            dest = p.get("model_id") or f"{algo}_model_q{q}"
            p["model_id"] = dest
            desc, dk = f"{algo} Model Build", "Model"
        elif kind == "grid":
            dest = p.get("grid_id") or f"Grid_{algo}_q{q}"
            p["grid_id"] = dest
            desc, dk = "GridSearch", "Grid"
        else:
            bc = dict(p.get("build_control") or {})
            dest = bc.get("project_name") or f"automl_q{q}"
            bc["project_name"] = dest
            p["build_control"] = bc
            desc, dk = "AutoML", "AutoML"
        key = f"job_q{q}"
        job = jobmod.Job(desc, dest=dest, key=key, dest_kind=dk)        # CREATED, rank 0's job table
        cmd = dict(cmd, p=p, hints={"job_key": key})

        def _done(f):
            e = f.exception()
            if e is not None and job.status == "CREATED":
                job.fail(e)
        executor.submit(cmd).add_done_callback(_done)
        if kind == "model":
            return JSONResponse(S.jsonable({"__meta": S.meta(f"{algo.capitalize()}V3", "ModelBuilder"), "algo": algo,
                                            "job": S.job_v3(job, dest=dest, dest_kind="Model"), "messages": [],
                                            "error_count": 0, "parameters": None}))
        if kind == "grid":
            return JSONResponse(S.jsonable({"__meta": S.meta("GridSearchSchemaV99", "Grid", 99),
                                            "grid_id": S.key(dest, "Grid"), "job": S.job_v3(job),
                                            "total_models": 0}))
        return JSONResponse(S.jsonable({"__meta": S.meta("AutoMLBuildSpecV99", "AutoMLBuildSpec", 99),
                                        "job": S.job_v3(job), "build_control": {"project_name": dest}}))

    def route(method, path):
        """Register an async handler taking (params, request, **path)."""
        rx = _re.compile(_re.sub(r"\{(\w+)\}", r"(?P<\1>[^/]+)", _re.escape(path).replace(r"\{", "{")
                                 .replace(r"\}", "}")))

        def local(fn):
            return lambda p, r, **kw: fn(p, r, **{k: _unquote(v) for k, v in kw.items()})

        is_local = path.startswith(_LOCAL_PREFIXES)

        def deco(fn):
            app.state.flow_routes.append((method, rx, local(fn), _jsonify))
            table[(method, path)] = fn

            async def h(request: Request):
                p = await _params(request)
                if is_local:
                    try:
                        out = fn(p, request, **request.path_params)
                        if hasattr(out, "__await__"):
                            out = await out
                    except _HTTPError:
                        raise
                    except (KeyError, ValueError, TypeError, RuntimeError, AssertionError, IndexError,
                            NotImplementedError) as e:
                        raise _HTTPError(400 if not isinstance(e, KeyError) else 404, str(e), e)
                    return _to_response(out)
                if method == "GET" and path in _READ_ROUTES and executor is not None and \
                        cloud.is_distributed() and executor.busy():
                    # a read while a build runs: on this thread, no collectives
                    from ..parallel import collectives as _coll
                    try:
                        with _coll.forbid():
                            out = fn(p, request, **request.path_params)
                            if hasattr(out, "__await__"):
                                out = await out
                        return _to_response(out)
                    except _HTTPError:
                        raise
                    except _coll.CollectiveForbidden as e:
                        if os.environ.get("H2O3_REST_DEBUG"):
                            import traceback as _tb
                            print(f"read {path} needs a collective ({e}):", "".join(_tb.format_exception(type(e), e, e.__traceback__)[-8:]),
                                  file=sys.stderr, flush=True)
                        # needs the cloud: queue it below
                    except (KeyError, ValueError, TypeError, AssertionError, IndexError, NotImplementedError) as e:
                        raise _HTTPError(400 if not isinstance(e, KeyError) else 404, str(e), e)
                    except RuntimeError as e:
                        if os.environ.get("H2O3_REST_DEBUG"):
                            import traceback as _tb
                            print(f"read {path} failed off the executor: {e!r}", _tb.format_exc(), file=sys.stderr,
                                  flush=True)
                        # e.g. a dict the build is mutating: queue it
                # replayed on every rank by the executor (spmd.py)
                req = {"method": request.method, "path": request.url.path, "headers": dict(request.headers),
                       "body": await request.body(), "query": dict(request.query_params)}
                cmd = {"kind": "route", "method": method, "path": path, "p": p, "kw": dict(request.path_params),
                       "req": req, "defer": True}
                kind = _BUILD_ROUTES.get(path) if method == "POST" else None
                if kind is not None and executor is not None and executor.busy():
                    return _queue_build(kind, cmd, request.path_params)
                try:
                    return await asyncio.wrap_future(executor.submit(cmd))
                except _HTTPError:
                    raise
                except RuntimeError as e:
                    raise _HTTPError(503 if not cloud.healthy() else 400, str(e), e)
            h.__name__ = fn.__name__
            app.add_api_route(path, h, methods=[method], name=f"{method} {path}")
            return fn
        return deco

    # ------------------------------------------------------------- Flow UI
    def _flow_page():
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "static", "flow.html"),
                  encoding="utf-8") as f:
            return f.read()

    from fastapi.responses import HTMLResponse, RedirectResponse

    @app.get("/", include_in_schema=False)
    async def root():
        return RedirectResponse("/flow/index.html")

    @app.get("/flow/index.html", include_in_schema=False)
    async def flow():
        """Flow notebook (h2o-web): cells run through POST /flow/cell (flow.py)."""
        return HTMLResponse(_flow_page())

    # ------------------------------------------------------------ cloud
    @route("GET", "/3/Cloud")
    def cloud_status(p, r):
        return S.cloud_v3(cloud.info(), t_start)

    @route("HEAD", "/3/Cloud")
    def cloud_head(p, r):
        return Response(status_code=200)

    @route("GET", "/3/Metadata/schemas/{name}")
    def schema_meta(p, r, name):
        m = S.schema_metadata(name)
        if m is None:
            raise _HTTPError(404, f"Schema {name} not found")
        return m

    @route("GET", "/3/Metadata/endpoints")
    def endpoints(p, r):
        routes = [{"__meta": S.meta("RouteV3", "Iced"), "url_pattern": rt.path,
                   "http_method": sorted(rt.methods)[0], "summary": rt.name, "input_schema": None,
                   "output_schema": None} for rt in app.routes if hasattr(rt, "methods")]
        return {"__meta": S.meta("MetadataV3", "Iced"), "routes": routes, "schemas": []}

    @route("POST", "/4/sessions")
    def session_open(p, r):
        sid = f"_sid_{uuid.uuid4().hex[:8]}"
        sessions[sid] = time.time()
        return {"__meta": S.meta("SessionIdV4", "Iced", 4), "session_key": sid}

    @route("DELETE", "/4/sessions/{sid}")
    def session_close(p, r, sid):
        sessions.pop(sid, None)
        return {"__meta": S.meta("SessionIdV4", "Iced", 4), "session_key": sid}

    @route("GET", "/3/InitID")
    def init_id(p, r):
        sid = f"_sid_{uuid.uuid4().hex[:8]}"
        sessions[sid] = time.time()
        return {"__meta": S.meta("InitIDV3", "Iced"), "session_key": sid, "session_properties_allowed": False}

    app.add_api_route("/3/InitID", app.routes[-1].endpoint, methods=["POST"], name="POST /3/InitID")

    @route("POST", "/3/LogAndEcho")
    def log_and_echo(p, r):
        """LogAndEchoHandler (h2o-r writes its session markers here)."""
        from ..utils import log as _log
        msg = str(p.get("message", ""))
        try:
            _log.info(msg)
        except Exception:  # noqa: BLE001 - logging never fails a request
            pass
        return {"__meta": S.meta("LogAndEchoV3", "Iced"), "message": msg}

    @route("GET", "/3/Capabilities/Core")
    def capabilities_core(p, r):
        return {"capabilities": [{"name": "Core"}, {"name": "Rapids"}, {"name": "MOJO"}]}

    @route("POST", "/3/Shutdown")
    def shutdown(p, r):
        """ShutdownHandler: a served cloud (rest.start) stops HTTP after the
        answer and then every rank (the executor's stop command ends the
        workers' loops); an embedded app just acknowledges."""
        srv = getattr(app.state, "uvicorn", None)
        if srv is not None:
            import threading as _th
            _th.Timer(0.5, lambda: setattr(srv, "should_exit", True)).start()
        return {"__meta": S.meta("ShutdownV3", "Iced")}

    @route("GET", "/3/About")
    def about(p, r):
        i = cloud.info()
        ent = [("Build project version", S.VERSION), ("Built by", "h2o3_amd"), ("Device", str(i.get("device"))),
               ("Cloud size", str(i.get("cloud_size")))]
        return {"__meta": S.meta("AboutV3", "Iced"),
                "entries": [{"__meta": S.meta("AboutEntryV3", "Iced"), "name": a, "value": b} for a, b in ent]}

    @route("GET", "/3/Capabilities")
    def capabilities(p, r):
        return {"capabilities": [{"name": n} for n in ("Algos", "AutoML", "Grid", "MOJO", "POJO", "Rapids",
                                                      "HIP-gfx950", "RCCL")]}

    @route("GET", "/3/Capabilities/API")
    def capabilities_api(p, r):
        return {"capabilities": [{"name": "/3"}, {"name": "/4"}, {"name": "/99"}]}

    @route("GET", "/3/Timeline")
    def timeline(p, r):
        return {"__meta": S.meta("TimelineV3", "Timeline"), "events": api.timeline()}

    @route("POST", "/3/GarbageCollect")
    def gc(p, r):
        import gc as _gc
        _gc.collect()
        return {}

    @route("GET", "/3/Logs/nodes/{node}/files/{name}")
    def logs(p, r, node, name):
        return {"__meta": S.meta("LogsV3", "Iced"), "nodeidx": node, "name": name, "log": ""}

    # ----------------------------------------------------------- import
    @route("POST", "/3/PostFile")
    async def post_file(p, r):
        ctype = r.headers.get("content-type", "")
        if ctype.startswith("application/json"):
            # JSON upload of columns (h2o3_amd extension): {"data": {col: [...]}, "destination_frame": ...}
            import pandas as pd
            fr = H2OFrame(pd.DataFrame(p["data"]))
            fid = _put_frame(fr, p.get("destination_frame"))
            return {"destination_frame": fid, "total_bytes": 0}
        if ctype.startswith("multipart/form-data"):
            files = [d for _, fname, d in _multipart(await r.body(), ctype) if fname is not None]
            if not files:
                raise _HTTPError(400, "PostFile: no file part")
            data = files[0]
            name = p.get("destination_frame") or None
        else:
            data = await r.body()
            name = p.get("destination_frame") or None
        k = uploads.add_bytes(data, name)
        return {"__meta": S.meta("PostFileV3", "Iced"), "destination_frame": k, "total_bytes": len(data)}

    app.add_api_route("/3/PostFile.bin", app.routes[-1].endpoint, methods=["POST"], name="POST /3/PostFile.bin")

    @route("GET", "/3/ImportFiles")
    def import_files(p, r):
        from ..core.parse import _files
        path = p.get("path")
        if not path:
            raise _HTTPError(400, "ImportFiles: path is required")
        fs = _files(path, p.get("pattern"))
        keys = []
        for f in fs:
            k = f if "://" not in f else os.path.basename(f)
            uploads.paths[k] = [f]
            keys.append(k)
        return {"__meta": S.meta("ImportFilesV3", "Iced"), "path": path, "pattern": p.get("pattern"),
                "files": fs, "destination_frames": keys, "fails": [], "dels": []}

    app.add_api_route("/3/ImportFiles", app.routes[-1].endpoint, methods=["POST"], name="POST /3/ImportFiles")

    def _guess(srcs, header, sep):
        """Parse (cached) with the guessed setup -> (frame, separator)."""
        from ..core import parse as P
        key_ = (tuple(srcs), header, sep)
        hit = uploads.setups.get(key_)
        if hit is not None:
            return hit
        files = uploads.resolve(srcs)
        st = P.parse_setup(files if len(files) > 1 else files[0], sep=sep)
        s = sep or st["separator"]
        fr = P.import_file(files if len(files) > 1 else files[0], sep=s, header=header)
        uploads.setups[key_] = (fr, s)
        return fr, s

    def _src_keys(v):
        if v is None:
            return []
        v = v if isinstance(v, list) else [v]
        return [s["name"] if isinstance(s, dict) else str(s) for s in v]

    def _header(v):
        return 1 if v in (1, True, "1") else (-1 if v in (-1, "-1") else 0)

    @route("POST", "/3/ParseSetup")
    def parse_setup(p, r):
        srcs = _src_keys(p.get("source_frames") or p.get("paths"))
        if not srcs:
            raise _HTTPError(400, "source_frames required")
        sep = p.get("separator")
        sep = (chr(sep) if 0 < sep < 128 else None) if isinstance(sep, int) else sep   # -1: guess
        hdr = _header(p.get("check_header", 0))
        fr, s = _guess(srcs, hdr, sep)
        base = os.path.splitext(os.path.basename(uploads.resolve(srcs)[0]))[0]
        dest = p.get("destination_frame") or (base.replace("-", "_").replace(".", "_") + ".hex")
        preview = fr.head(min(10, fr.nrow)).as_data_frame() if fr.nrow else None
        data = [] if preview is None else [[None if v != v else str(v) for v in row] for row in preview.values.tolist()]
        return {"__meta": S.meta("ParseSetupV3", "ParseSetup"),
                "source_frames": [S.key(k) for k in srcs], "parse_type": "CSV", "separator": ord(s),
                "single_quotes": False, "check_header": hdr if hdr != 0 else 1, "column_names": list(fr.names),
                "column_types": [_TYPE_NAMES.get(fr.vec(n).type, "Numeric") for n in fr.names],
                "na_strings": None, "column_name_filter": None, "column_offset": 0, "column_count": fr.ncol,
                "destination_frame": dest, "header_lines": 1 if hdr != -1 else 0, "number_columns": fr.ncol,
                "data": data, "chunk_size": 4194304, "total_filtered_column_count": fr.ncol,
                "custom_non_data_line_markers": None, "partition_by": None, "escapechar": 0,
                "quotechar": None, "skipped_columns": None, "force_col_types": False,
                "tz_adjust_to_local": False, "warnings": []}

    @route("POST", "/3/Parse")
    def parse(p, r):
        from ..core import parse as P
        srcs = _src_keys(p.get("source_frames"))
        if not srcs:
            raise _HTTPError(400, "source_frames required")
        sep = p.get("separator")
        sep = (chr(sep) if 0 < sep < 128 else None) if isinstance(sep, int) else sep   # -1: guess
        hdr = _header(p.get("check_header", 0))
        dest = p.get("destination_frame") or (os.path.basename(srcs[0]) + ".hex")
        names = p.get("column_names")
        types = p.get("column_types")
        skipped = p.get("skipped_columns")
        fr, s = _guess(srcs, hdr, sep)
        guessed = [_TYPE_NAMES.get(fr.vec(n).type, "Numeric") for n in fr.names]
        want = [str(t) for t in types] if types else guessed
        if (types and [t.lower() for t in want] != [t.lower() for t in guessed]) or skipped or \
                p.get("na_strings"):
            files = uploads.resolve(srcs)
            ct = [_TYPE_IN.get(str(t).lower(), "numeric") for t in want] if types else None
            fr = P.import_file(files if len(files) > 1 else files[0], sep=s, header=hdr, col_types=ct,
                               skipped_columns=skipped, na_strings=p.get("na_strings") or None)
        else:
            fr = fr.deep_copy()
        if names:
            names = [str(n) for n in names]
            if len(names) == fr.ncol and names != list(fr.names):
                fr.names = names
        fid = _put_frame(fr, dest)
        if p.get("delete_on_done", True):
            # the raw upload is consumed by the parse (ParseHandler delete_on_done)
            for k in srcs:
                uploads.setups = {kk: v for kk, v in uploads.setups.items() if k not in kk[0]}
                for f in uploads.paths.get(k, []):
                    if os.path.dirname(f) == uploads.dir:
                        try:
                            os.remove(f)
                        except OSError:
                            pass
                        uploads.paths.pop(k, None)
        return {"__meta": S.meta("ParseV3", "Parse"), "destination_frame": S.key(fid),
                "job": S.job_v3(key_name=f"parse_{fid}", dest=fid, description="Parse"), "rows": fr.nrow}

    # ----------------------------------------------------------- frames
    @route("GET", "/3/Frames")
    def frames(p, r):
        from ..parallel import collectives as _coll
        fs = [(k, dkv.get(k)) for k in list(dkv.keys())]
        out = []
        for k, f in fs:
            if not isinstance(f, H2OFrame):
                continue
            try:
                out.append(S.frame_base_v3(k, f))
            except _coll.CollectiveForbidden:
                # a frame whose row count was never reduced, listed while a build
                # runs: its key only (h2o.ls() reads the keys)
                out.append({"__meta": S.meta("FrameBaseV3", "Frame"), "frame_id": S.key(k), "byte_size": -1,
                            "is_text": False, "rows": -1, "columns": f.ncol})
        return {"__meta": S.meta("FramesListV3", "Frames"), "frames": out}

    def _frame_get(p, fid, rollups=True, percentiles=False):
        fr = _frame(fid)
        rc = p.get("row_count", 10)
        return {"__meta": S.meta("FramesV3", "Frames"), "frame_id": S.key(fid),
                "frames": [S.frame_v3(fid, fr, int(p.get("row_offset", 0) or 0), -1 if rc is None else int(rc),
                                      int(p.get("column_offset", 0) or 0), int(p.get("column_count", -1)),
                                      int(p.get("full_column_count", -1)), rollups=rollups,
                                      percentiles=percentiles)]}

    @route("GET", "/3/Frames/{fid}")
    def frame(p, r, fid):
        return _frame_get(p, fid)

    @route("GET", "/3/Frames/{fid}/light")
    def frame_light(p, r, fid):
        return _frame_get(p, fid, rollups=False)

    @route("GET", "/3/Frames/{fid}/summary")
    def frame_summary(p, r, fid):
        return _frame_get({"row_count": p.get("row_count", 0)}, fid, percentiles=True)

    @route("GET", "/3/Frames/{fid}/columns/{col}/summary")
    def column_summary(p, r, fid, col):
        fr = _frame(fid)
        return _frame_get({"row_count": 0}, _put_frame(fr[[col]], f"{fid}_{col}_summary"), percentiles=True)

    @route("DELETE", "/3/Frames/{fid}")
    def frame_delete(p, r, fid):
        dkv.remove(fid)
        return {"__meta": S.meta("FramesV3", "Frames"), "frame_id": S.key(fid)}

    @route("DELETE", "/3/Frames")
    def frames_delete(p, r):
        for k in list(dkv.keys()):
            if isinstance(dkv.get(k), H2OFrame):
                dkv.remove(k)
        return {}

    @route("GET", "/3/DownloadDataset")
    def download_dataset(p, r):
        fr = _frame(p.get("frame_id"), "frame_id")
        df = fr.as_data_frame()
        return PlainTextResponse(df.to_csv(index=False, na_rep=""), media_type="text/csv")

    app.add_api_route("/3/DownloadDataset.bin", app.routes[-1].endpoint, methods=["GET"],
                      name="GET /3/DownloadDataset.bin")

    @route("POST", "/3/SplitFrame")
    def split_frame(p, r):
        fr = _frame(p.get("dataset"), "dataset")
        ratios = [float(x) for x in (p.get("ratios") or [0.75])]
        dests = p.get("destination_frames")
        parts = fr.split_frame(ratios=ratios, destination_frames=dests, seed=p.get("seed"))
        keys = [_put_frame(f, (dests[i] if dests and i < len(dests) else None)) for i, f in enumerate(parts)]
        return {"__meta": S.meta("SplitFrameV3", "SplitFrame"), "key": S.key(keys[0]),
                "job": S.job_v3(key_name=f"split_{keys[0]}", dest=keys[0], description="SplitFrame"),
                "destination_frames": [S.key(k) for k in keys]}

    @route("POST", "/3/CreateFrame")
    def create_frame(p, r):
        kw = {k: v for k, v in p.items() if k not in ("dest", "_exclude_fields")}
        fr = api.create_frame(**{("frame_id" if k == "destination_frame" else k): v for k, v in kw.items()})
        fid = _put_frame(fr, p.get("dest") or p.get("destination_frame"))
        return {"__meta": S.meta("CreateFrameV3", "CreateFrame"), "destination_frame": S.key(fid),
                "job": S.job_v3(key_name=f"create_{fid}", dest=fid, description="CreateFrame")}

    # ----------------------------------------------------------- models
    def _resolve_params(p):
        out = {}
        for k, v in p.items():
            if k in _FRAME_PARAMS and isinstance(v, str):
                out[k] = _frame(v, k)
            elif k in _MODEL_PARAMS and isinstance(v, str) and v:
                out[k] = dkv.get(v) or v
            else:
                out[k] = v
        return out

    def _build(algo, p, defer=False):
        """ModelBuilderHandler: validate + create the builder now; train now
        (defer=False: Flow cells, sync callers) or return (model, job, work)
        for the executor to run after answering with the RUNNING job."""
        from ..core import job as jobmod
        cls = _algo_cls(algo)
        p = _resolve_params(_coerce_params(cls, p))
        tf = p.get("training_frame")
        if not isinstance(tf, H2OFrame) and algo != "stackedensemble":
            raise _HTTPError(400, "ERRR on field: _train: Missing training frame", builder=True)
        vf = p.get("validation_frame")
        y = p.get("response_column")
        ignored = set(p.get("ignored_columns") or [])
        special = {y, p.get("weights_column"), p.get("offset_column"), p.get("fold_column"),
                   p.get("treatment_column")}
        x = p.get("x")
        if x is None and isinstance(tf, H2OFrame):
            x = [c for c in tf.names if c not in special and c not in ignored]
        kw = {k: v for k, v in p.items() if k not in _DROP_PARAMS and v is not None}
        if algo == "hglm":
            kw["HGLM"] = True
        try:
            m = cls(**kw)
        except (ValueError, TypeError) as e:      # parameter validation (ModelBuilder.init error(...))
            raise _HTTPError(412, f"Illegal argument(s) for {algo} model: {e}", e, builder=True)
        job = jobmod.Job(f"{algo} Model Build", dest=m.model_id, key=spmd.hint("job_key")).start()
        job.spmd = cloud.is_distributed()

        def work():
            jobmod.set_pending(job)
            try:
                if m.supervised_learning:
                    m.train(x=x, y=y, training_frame=tf, validation_frame=vf)
                else:
                    m.train(x=x, training_frame=tf, validation_frame=vf) if vf is not None else \
                        m.train(x=x, training_frame=tf)
            finally:
                jobmod.take_pending()
            dkv.put(m.model_id, m)
            for cm in getattr(m, "_cv_models", None) or []:   # cross_validation_models are fetched by key
                dkv.put(cm.model_id, cm)
            if algo == "stackedensemble" and getattr(m, "_meta", None) is not None:
                dkv.put(m._meta.model_id, m._meta)                # output.metalearner is fetched by key

        if defer:
            return m, job, work
        try:
            work()
        except _HTTPError:
            raise
        except jobmod.JobCancelled as e:
            raise _HTTPError(400, f"{algo} model build cancelled", e, builder=True)
        except Exception as e:  # noqa: BLE001 - reported to the client as an H2OModelBuilderError
            raise _HTTPError(400, f"Illegal argument(s) for {algo} model: {e}", e, builder=True)
        if job.is_running:
            job.done()
        return m

    @route("POST", "/3/ModelBuilders/{algo}")
    def build(p, r, algo):
        defer = spmd.defer_allowed()
        out = _build(algo, p, defer=defer)
        m, job, work = out if defer else (out, getattr(out, "_job", None), None)
        resp = {"__meta": S.meta(f"{algo.capitalize()}V3", "ModelBuilder"), "algo": algo,
                "job": S.job_v3(job, dest=m.model_id, dest_kind="Model") if job is not None else
                S.job_v3(key_name=f"job_{m.model_id}", dest=m.model_id, dest_kind="Model",
                         description=f"{algo} Model Build"),
                "messages": [], "error_count": 0, "parameters": None}
        return spmd.Deferred(resp, work, job) if defer else resp

    app.add_api_route("/99/ModelBuilders/{algo}", app.routes[-1].endpoint, methods=["POST"],
                      name="POST /99/ModelBuilders/{algo}")

    @route("POST", "/3/ModelBuilders/{algo}/parameters")
    def validate_params(p, r, algo):
        _algo_cls(algo)
        return {"__meta": S.meta("ModelParametersSchemaV3", "ModelBuilder"), "algo": algo, "messages": [],
                "error_count": 0, "parameters": None}

    @route("GET", "/3/ModelBuilders/{algo}")
    def builder_info(p, r, algo):
        cls = _algo_cls(algo)
        est = cls()
        from ..models.param_meta import META
        from ..models.param_tables import PARAMS
        names = PARAMS.get(cls.__name__) or list(est._parms)
        pm = META.get(cls.__name__, {})
        params = [S._param_entry(k, est._parms.get(k), est._parms.get(k), pm.get(k, {})) for k in names]
        return {"__meta": S.meta("ModelBuildersV3", "Iced"),
                "model_builders": {algo: {"algo": algo, "algo_full_name": cls.__name__, "parameters": params,
                                          "can_build": ["Binomial", "Multinomial", "Regression"],
                                          "visibility": "Stable", "supervised": cls.supervised_learning}}}

    @route("GET", "/3/Models")
    def models(p, r):
        from ..models.base import H2OEstimator
        ms = [(k, dkv.get(k)) for k in dkv.keys()]
        return {"__meta": S.meta("ModelsV3", "Models"),
                "models": [S.model_v3(k, m) for k, m in ms if isinstance(m, H2OEstimator)]}

    @route("GET", "/3/Models/{mid}")
    def model(p, r, mid):
        return {"__meta": S.meta("ModelsV3", "Models"), "models": [S.model_v3(mid, _model(mid))]}

    @route("GET", "/99/Models/{mid}")
    def model99(p, r, mid):
        return model(p, r, mid)

    @route("DELETE", "/3/Models/{mid}")
    def model_delete(p, r, mid):
        dkv.remove(mid)
        return {"__meta": S.meta("ModelsV3", "Models"), "models": []}

    @route("GET", "/3/Models/{mid}/mojo")
    def model_mojo(p, r, mid):
        from ..mojo.writer import build_mojo
        data = build_mojo(_model(mid))
        return Response(content=data, media_type="application/zip",
                        headers={"Content-Disposition": f'attachment; filename="{mid}.zip"'})

    @route("GET", "/3/Models.java/{mid}")
    def model_pojo(p, r, mid):
        from ..mojo.pojo import to_java
        return PlainTextResponse(to_java(_model(mid)), media_type="text/plain",
                                 headers={"Content-Disposition": f'attachment; filename="{mid}.java"'})

    def _predict(p, mid, fid, v4=False):
        m, fr = _model(mid), _frame(fid)
        dest = p.get("predictions_frame")
        if p.get("leaf_node_assignment"):
            pr = m.predict_leaf_node_assignment(fr, type=p.get("leaf_node_assignment_type") or "Path")
        elif p.get("predict_contributions"):
            pr = m.predict_contributions(fr)
        elif p.get("reconstruction_error"):
            pr = m.anomaly(fr)
        elif p.get("deep_features_hidden_layer") is not None and int(p["deep_features_hidden_layer"]) >= 0:
            pr = m.deepfeatures(fr, int(p["deep_features_hidden_layer"]))
        elif p.get("predict_staged_proba"):
            pr = m.staged_predict_proba(fr)
        elif p.get("exemplar_index") is not None and int(p["exemplar_index"]) >= 0:
            pr = m.aggregated_frame
        else:
            pr = m.predict(fr)
        key_ = _put_frame(pr, dest or f"prediction_{mid}_on_{fid}")
        mm = None
        spec = getattr(m, "_spec", None)
        if spec is not None and spec.y and spec.y in fr.names:
            try:
                mm = S.metrics_v3(m.model_performance(fr), m, fid, S.model_category(m))
            except Exception:  # noqa: BLE001 - metrics are optional for scoring
                mm = None
        if mm is None:
            # prediction-only result (anomaly / leaf assignment / contributions...): the
            # reference still returns a metrics record carrying the predictions frame
            mm = {"__meta": S.meta("ModelMetricsBaseV3", "ModelMetricsBase"), "model": S.key(mid, "Model"),
                  "frame": S.key(fid), "predictions": S.frame_base_v3(key_, pr)}
        else:
            mm["predictions"] = S.frame_base_v3(key_, pr)
        if v4:
            return {"__meta": S.meta("JobV4", "Job", 4),
                    "key": S.key(f"predict_{key_}", "Job"), "dest": S.key(key_), "status": "DONE",
                    "job": S.job_v3(key_name=f"predict_{key_}", dest=key_, description="Prediction"),
                    "predictions_frame": S.key(key_)}
        return {"__meta": S.meta("ModelMetricsListSchemaV3", "ModelMetricsList"), "model": S.key(mid, "Model"),
                "frame": S.key(fid), "predictions_frame": S.key(key_), "model_metrics": [mm] if mm else []}

    @route("POST", "/3/Predictions/models/{mid}/frames/{fid}")
    def predict(p, r, mid, fid):
        return _predict(p, mid, fid)

    @route("POST", "/4/Predictions/models/{mid}/frames/{fid}")
    def predict4(p, r, mid, fid):
        return _predict(p, mid, fid, v4=True)

    @route("POST", "/3/ModelMetrics/models/{mid}/frames/{fid}")
    def model_metrics(p, r, mid, fid):
        m, fr = _model(mid), _frame(fid)
        mm = S.metrics_v3(m.model_performance(fr), m, fid, S.model_category(m))
        return {"__meta": S.meta("ModelMetricsListSchemaV3", "ModelMetricsList"), "model": S.key(mid, "Model"),
                "frame": S.key(fid), "model_metrics": [mm]}

    @route("GET", "/3/ModelMetrics/models/{mid}/frames/{fid}")
    def model_metrics_get(p, r, mid, fid):
        return model_metrics(p, r, mid, fid)

    # ------------------------------------------------ persistence / misc
    def _models_list(mid):
        return {"__meta": S.meta("ModelsV3", "Models"), "models": [S.model_v3(mid, _model(mid))]}

    @route("GET", "/99/Models.bin/{mid}")
    def model_save(p, r, mid):
        """ModelsHandler.exportModel: write the model binary under `dir` on the server."""
        m = _model(mid)
        path = str(p.get("dir") or "")
        out = api.save_model(m, os.path.dirname(path) or ".", force=bool(p.get("force", False)),
                             filename=os.path.basename(path) or None)
        return {"__meta": S.meta("ModelExportV3", "Iced"), "model_id": S.key(mid, "Model"), "dir": out}

    @route("POST", "/99/Models.bin/{mid}")
    def model_load(p, r, mid=""):
        """ModelsHandler.importModel: load a binary model from `dir` on the server."""
        m = api.load_model(str(p.get("dir")))
        dkv.put(m.model_id, m)
        return _models_list(m.model_id)

    app.add_api_route("/99/Models.bin/", app.routes[-1].endpoint, methods=["POST"], name="POST /99/Models.bin/")

    @route("POST", "/99/Models.upload.bin/{mid}")
    def model_upload(p, r, mid=""):
        """Load a model binary that was sent with PostFile (its raw key in `dir`)."""
        src = uploads.resolve([str(p.get("dir"))])[0]
        m = api.load_model(src)
        dkv.put(m.model_id, m)
        return _models_list(m.model_id)

    app.add_api_route("/99/Models.upload.bin/", app.routes[-1].endpoint, methods=["POST"],
                      name="POST /99/Models.upload.bin/")

    @route("GET", "/3/Models.fetch.bin/{mid}")
    def model_fetch(p, r, mid):
        """The model binary as a download (h2o.download_model)."""
        m = _model(mid)
        d = tempfile.mkdtemp(prefix="h2o3_amd_fetch_")
        path = api.save_model(m, d, force=True)
        with open(path, "rb") as f:
            data = f.read()
        return Response(content=data, media_type="application/octet-stream",
                        headers={"Content-Disposition": f'attachment; filename="{mid}"'})

    @route("GET", "/99/Models.mojo/{mid}")
    def model_save_mojo(p, r, mid):
        from ..mojo.writer import build_mojo
        path = str(p.get("dir"))
        if os.path.exists(path) and not p.get("force", False):
            raise _HTTPError(400, f"File {path} already exists")
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "wb") as f:
            f.write(build_mojo(_model(mid)))
        return {"__meta": S.meta("ModelExportV3", "Iced"), "model_id": S.key(mid, "Model"), "dir": path}

    @route("POST", "/3/Frames/{fid}/export")
    def frame_export(p, r, fid):
        fr = _frame(fid)
        sep = p.get("separator", 44)
        api.export_file(fr, str(p.get("path")), force=bool(p.get("force", False)),
                        sep=chr(sep) if isinstance(sep, int) else str(sep), header=bool(p.get("header", True)),
                        format=str(p.get("format") or "csv"))
        return {"__meta": S.meta("FramesV3", "Frames"),
                "job": S.job_v3(key_name=f"export_{fid}", dest=fid, description="Export File")}

    @route("POST", "/3/ModelMetrics/predictions_frame/{pf}/actuals_frame/{af}")
    def make_metrics(p, r, pf, af):
        pred, act = _frame(pf, "predictions_frame"), _frame(af, "actuals_frame")
        w = _frame(p["weights_frame"]) if p.get("weights_frame") else None
        mm = api.make_metrics(pred, act, domain=p.get("domain"), distribution=p.get("distribution"), weights=w,
                              auc_type=p.get("auc_type") or "NONE")
        return {"__meta": S.meta("ModelMetricsMakerSchemaV3", "Iced"), "model_metrics": S.metrics_v3(mm)}

    @route("POST", "/3/MissingInserter")
    def missing_inserter(p, r):
        fid = p.get("dataset")
        fr = _frame(fid, "dataset")
        fr.insert_missing_values(fraction=float(p.get("fraction", 0.1)), seed=p.get("seed"))
        return S.job_v3(key_name=f"missing_{fid}", dest=fid, description="Insert Missing Values")

    @route("POST", "/3/Interaction")
    def interaction(p, r):
        fr = _frame(p.get("source_frame"), "source_frame")
        facs = p.get("factor_columns") or []
        facs = [fr.names[int(f)] if isinstance(f, int) else str(f) for f in facs]
        out = api.interaction(fr, facs, bool(p.get("pairwise", False)), int(p.get("max_factors", 100)),
                              int(p.get("min_occurrence", 1)))
        fid = _put_frame(out, p.get("dest"))
        return S.job_v3(key_name=f"interaction_{fid}", dest=fid, description="Interactions")

    @route("POST", "/3/ImportFilesMulti")
    def import_files_multi(p, r):
        from ..core.parse import _files
        keys, files = [], []
        for path in p.get("paths") or []:
            for f in _files(path, p.get("pattern")):
                uploads.paths[f] = [f]
                keys.append(f)
                files.append(f)
        return {"__meta": S.meta("ImportFilesMultiV3", "Iced"), "paths": p.get("paths"), "files": files,
                "destination_frames": keys, "fails": [], "dels": []}

    @route("POST", "/99/ImportSQLTable")
    def import_sql(p, r):
        if p.get("select_query"):
            fr = api.import_sql_select(p["connection_url"], p["select_query"], p.get("username"), p.get("password"))
        else:
            cols = p.get("columns")
            cols = [c.strip() for c in cols.split(",")] if isinstance(cols, str) else cols
            fr = api.import_sql_table(p["connection_url"], p["table"], p.get("username"), p.get("password"),
                                      columns=cols)
        fid = _put_frame(fr)
        return S.job_v3(key_name=f"sql_{fid}", dest=fid, description="Import SQL Table")

    @route("POST", "/3/PartialDependence/")
    def partial_dependence(p, r):
        """PartialDependenceHandler: 1-D partial dependence tables per column
        (per target class when `targets` is given), kept under destination_key."""
        m, fr = _model(p.get("model_id")), _frame(p.get("frame_id"))
        cols = p.get("cols") or [c for c in (m._spec.x if m._spec is not None else [])]
        w = p.get("weight_column_index")
        wname = fr.names[int(w)] if isinstance(w, int) and w >= 0 else None
        row = p.get("row_index")
        tabs = m.partial_plot(fr, cols=list(cols), nbins=int(p.get("nbins", 20)), weight_column=wname,
                              include_na=bool(p.get("add_missing_na", False)), targets=p.get("targets"),
                              row_index=None if row is None or int(row) < 0 else int(row))
        dest = p.get("destination_key") or f"pdp_{spmd.rand_hex(8)}"
        pdp[dest] = {"model_id": m.model_id, "frame_id": fr.frame_id, "tables": tabs}
        return S.job_v3(key_name=f"pdp_{dest}", dest=dest, description="PartialDependencePlot")

    pdp: dict = {}

    @route("GET", "/3/PartialDependence/{dest}")
    def partial_dependence_get(p, r, dest):
        rec = pdp.get(dest)
        if rec is None:
            raise _HTTPError(404, f"partial dependence {dest} not found")
        tabs = []
        for t in rec["tables"]:
            df = t if hasattr(t, "columns") else t.as_data_frame()
            tabs.append(S.twodim_from_df(f"PartialDependence for {df.columns[0]}", df))
        return {"__meta": S.meta("PartialDependenceV3", "PartialDependence"), "model_id": S.key(rec["model_id"], "Model"),
                "frame_id": S.key(rec["frame_id"]), "destination_key": S.key(dest), "partial_dependence_data": tabs}

    @route("GET", "/3/GetGLMRegPath")
    def glm_reg_path(p, r):
        """GetGLMRegPathHandler: the lambda path of a GLM (coefficient rows in
        coefficient_names order)."""
        m = _model(p.get("model"))
        rp = (m._output or {}).get("regularization_path")
        if rp is None:
            raise _HTTPError(400, f"model {m.model_id} has no regularization path")
        names = list(rp["coefficients"][0].keys()) if rp["coefficients"] else []
        out = {"__meta": S.meta("GLMRegularizationPathV3", "Iced"), "model": S.key(m.model_id, "Model"),
               "lambdas": rp["lambdas"], "alphas": rp.get("alphas"),
               "explained_deviance_train": rp.get("explained_deviance_train"),
               "explained_deviance_valid": rp.get("explained_deviance_valid"), "coefficient_names": names,
               "coefficients": [[c.get(n) for n in names] for c in rp["coefficients"]],
               "coefficients_std": [[c.get(n) for n in names] for c in rp["coefficients_std"]]
               if rp.get("coefficients_std") else None}
        return out

    @route("GET", "/3/NetworkTest")
    def network_test(p, r):
        return {"__meta": S.meta("NetworkTestV3", "Iced"), "table": S.twodim("Network Test", {"bandwidth": [0.0]})}

    # -------------------------------------------------------------- jobs
    @route("GET", "/3/Jobs")
    def jobs(p, r):
        return {"__meta": S.meta("JobsV3", "Jobs"),
                "jobs": [S.job_v3(j, dest_kind="Model") for j in api.jobs()]}

    @route("GET", "/3/Jobs/{jid}")
    def job(p, r, jid):
        for j in api.jobs():
            if j.key == jid:
                return {"__meta": S.meta("JobsV3", "Jobs"), "job_id": S.key(jid, "Job"),
                        "jobs": [S.job_v3(j, dest_kind="Model")]}
        # synthetic jobs of synchronous requests (parse, split, predictions) are finished by construction
        return {"__meta": S.meta("JobsV3", "Jobs"), "job_id": S.key(jid, "Job"),
                "jobs": [S.job_v3(key_name=jid, dest=jid.split("_", 1)[-1], description=jid.split("_", 1)[0])]}

    @route("POST", "/3/Jobs/{jid}/cancel")
    def job_cancel(p, r, jid):
        for j in api.jobs():
            if j.key == jid:
                j.cancel()
        return {}

    # --------------------------------------------------------------- DKV
    @route("DELETE", "/3/DKV/{key_}")
    def delete(p, r, key_):
        dkv.remove(key_)
        return {"__meta": S.meta("RemoveV3", "Iced"), "key": S.key(key_)}

    @route("DELETE", "/3/DKV")
    def delete_all(p, r):
        retained = set(p.get("retained_keys") or [])
        for k in list(dkv.keys()):
            if k not in retained:
                dkv.remove(k)
        return {"__meta": S.meta("RemoveAllV3", "Iced")}

    # ------------------------------------------------------------ Rapids
    @route("POST", "/99/Rapids")
    def rapids_exec(p, r):
        """Rapids expression evaluation (water/api/RapidsHandler.java): frame
        results are stored under their key and described; scalars/lists/strings
        come back inline (RapidsFrameV3 / RapidsNumberV3 / RapidsStringV3...)."""
        from ..core.rapids import RapidsError, rapids
        try:
            res = rapids(p.get("ast", ""))
        except (RapidsError, KeyError, ValueError, TypeError, IndexError) as e:
            raise _HTTPError(400, f"Rapids error: {e}", e)
        if isinstance(res, H2OFrame):
            if dkv.get(res.frame_id) is not res:
                dkv.put(res.frame_id, res)
            return {"__meta": S.meta("RapidsFrameV3", "Iced", 99), "key": S.key(res.frame_id),
                    "num_rows": res.nrows, "num_cols": res.ncols}
        if isinstance(res, str):
            return {"__meta": S.meta("RapidsStringV3", "Iced", 99), "string": res}
        if isinstance(res, (list, tuple)):
            if res and all(isinstance(x, str) for x in res):
                return {"__meta": S.meta("RapidsStringsV3", "Iced", 99), "string": list(res)}
            return {"__meta": S.meta("RapidsNumbersV3", "Iced", 99), "scalar": [S.num(x) for x in res]}
        if res is None:
            return {"__meta": S.meta("RapidsNoneV3", "Iced", 99)}
        return {"__meta": S.meta("RapidsNumberV3", "Iced", 99), "scalar": S.num(res)}

    # --------------------------------------------------------- grid / automl
    @route("POST", "/99/Grid/{algo}")
    def grid(p, r, algo):
        """GridSearchHandler: hyper_parameters + search_criteria over one algo."""
        from ..grid import H2OGridSearch
        cls = _algo_cls(algo)
        p = _resolve_params(_coerce_params(cls, p))
        hyper = p.pop("hyper_parameters", {}) or {}
        if isinstance(hyper, str):
            hyper = _json.loads(hyper)
        crit = p.pop("search_criteria", None)
        if isinstance(crit, str):
            crit = _json.loads(crit)
        gid = p.pop("grid_id", None)
        p.pop("parallelism", None)              # GridSearchHandler-level (models build one at a time here)
        recovery_dir = p.pop("recovery_dir", None)
        tf, vf = p.pop("training_frame", None), p.pop("validation_frame", None)
        y = p.pop("response_column", None)
        ignored = set(p.pop("ignored_columns", None) or [])
        x = [c for c in tf.names if c != y and c not in ignored] if isinstance(tf, H2OFrame) else None
        p.pop("_rest_version", None)
        from ..core import job as jobmod
        g = H2OGridSearch(cls(**{k: v for k, v in p.items() if v is not None}), hyper, grid_id=gid,
                          search_criteria=crit, **({"recovery_dir": recovery_dir} if recovery_dir else {}))
        job = jobmod.Job("GridSearch", dest=g.grid_id, dest_kind="Grid", key=spmd.hint("job_key")).start()
        job.spmd = cloud.is_distributed()
        dkv.put(g.grid_id, g)           # visible (and growing) while the search runs

        def work():
            try:
                g.train(x=x, y=y, training_frame=tf, validation_frame=vf)
            finally:
                dkv.put(g.grid_id, g)
                for mid in g.model_ids:
                    mm = g.get_model(mid) if hasattr(g, "get_model") else dkv.get(mid)
                    if mm is not None:
                        dkv.put(mid, mm)

        resp = {"__meta": S.meta("GridSearchSchemaV99", "Grid", 99), "grid_id": S.key(g.grid_id, "Grid"),
                "job": None, "total_models": 0}
        if spmd.defer_allowed():
            resp["job"] = S.job_v3(job)
            return spmd.Deferred(resp, work, job)
        spmd.Deferred(resp, work, job).run()
        resp["job"] = S.job_v3(job)
        resp["total_models"] = len(g.model_ids)
        return resp

    def _metric_of(mid, name):
        """Sort key of a grid model (hex/grid/Grid.java sorting): the metric of
        the cross-validation, else validation, else training metrics."""
        m = dkv.get(mid)
        if m is None:
            return float("nan")
        mm = m._cross_validation_metrics or m._validation_metrics or m._training_metrics
        if mm is None:
            return float("nan")
        n = name.lower()
        alias = {"auc": "AUC", "mse": "MSE", "rmse": "RMSE", "aucpr": "pr_auc", "pr_auc": "pr_auc",
                 "gini": "Gini", "aic": "AIC"}
        v = mm.get(alias.get(n, n))
        if v is None and mm.get("thresholds_and_metric_scores") is not None:
            col = mm["thresholds_and_metric_scores"].get(n)
            v = max(col) if col is not None and len(col) else None
        try:
            return float(v)
        except (TypeError, ValueError):
            return float("nan")

    @route("GET", "/99/Grids/{gid}")
    def grid_get(p, r, gid):
        g = dkv.get(gid)
        if g is None or not hasattr(g, "model_ids"):
            raise _HTTPError(404, f"grid {gid} not found")
        tab = g.get_grid().sorted_metric_table()
        ids = list(g.model_ids)
        if p.get("sort_by"):
            import math
            vals = {mid: _metric_of(mid, str(p["sort_by"])) for mid in ids}
            dec = bool(p.get("decreasing"))
            ids.sort(key=lambda k: (math.isnan(vals[k]), -vals[k] if dec else vals[k]))
        return {"__meta": S.meta("GridSchemaV99", "Grid", 99), "grid_id": S.key(gid, "Grid"),
                "model_ids": [S.key(m, "Model") for m in ids],
                "failed_params": [], "failure_details": list(g.failure_details),
                "failure_stack_traces": [], "failed_raw_params": [],
                "hyper_names": list(getattr(g, "hyper_params", {}) or {}),
                "summary_table": S.twodim_from_df("Hyper-Parameter Search Summary", tab),
                "scoring_history": None, "warning_details": [], "export_checkpoints_dir": None,
                "training_metrics": [], "validation_metrics": [], "cross_validation_metrics": [],
                "cross_validation_metrics_summary": []}

    @route("GET", "/99/Grids")
    def grids(p, r):
        gs = [k for k in dkv.keys() if hasattr(dkv.get(k), "model_ids") and not hasattr(type(dkv.get(k)), "leaderboard")]
        return {"__meta": S.meta("GridsV99", "Grids", 99), "grids": [grid_get({}, r, k) for k in gs]}

    @route("POST", "/99/AutoMLBuilder")
    def automl(p, r):
        """AutoMLBuilderHandler: build_control / input_spec / build_models."""
        from ..automl import H2OAutoML
        bc, ispec, bm = p.get("build_control", {}), p.get("input_spec", {}), p.get("build_models", {})
        tf = _frame(ispec.get("training_frame"), "training_frame")
        sc = bc.get("stopping_criteria", {})
        aml = H2OAutoML(project_name=bc.get("project_name"), nfolds=bc.get("nfolds", -1),
                        max_models=sc.get("max_models"), max_runtime_secs=sc.get("max_runtime_secs"),
                        seed=sc.get("seed"), exclude_algos=bm.get("exclude_algos"),
                        include_algos=bm.get("include_algos"), sort_metric=ispec.get("sort_metric", "AUTO"))
        from ..core import job as jobmod
        y = ispec.get("response_column")
        ign = set(ispec.get("ignored_columns") or [])
        x = [c for c in tf.names if c != y and c not in ign]
        job = jobmod.Job("AutoML", dest=aml.project_name, dest_kind="AutoML",
                         key=spmd.hint("job_key") or f"automl_{aml.project_name}_{dkv.make_key('amljob')}").start()
        job.spmd = cloud.is_distributed()

        def work():
            try:
                aml.train(x=x, y=y, training_frame=tf,
                          validation_frame=dkv.get(ispec["validation_frame"]) if ispec.get("validation_frame")
                          else None,
                          leaderboard_frame=dkv.get(ispec["leaderboard_frame"]) if ispec.get("leaderboard_frame")
                          else None)
            finally:
                dkv.put(aml.project_name, aml)

        resp = {"__meta": S.meta("AutoMLBuildSpecV99", "AutoMLBuildSpec", 99), "job": None,
                "build_control": {"project_name": aml.project_name}}
        if spmd.defer_allowed():
            resp["job"] = S.job_v3(job)
            return spmd.Deferred(resp, work, job)
        spmd.Deferred(resp, work, job).run()
        resp["job"] = S.job_v3(job)
        return resp

    def _lb_table(aml):
        lbo = getattr(aml, "_leaderboard", None)
        lb = lbo.as_pandas() if hasattr(lbo, "as_pandas") else aml.leaderboard.as_data_frame()
        cols = {c: lb[c].tolist() for c in lb.columns}
        return lb, S.twodim("Leaderboard", cols, "models sorted by the leaderboard metric",
                            row_headers=[str(i) for i in range(len(lb))])

    @route("GET", "/99/Leaderboards/{project}")
    def leaderboard(p, r, project):
        aml = dkv.get(project)
        if aml is None or not hasattr(type(aml), "leaderboard"):
            raise _HTTPError(404, f"AutoML project {project} not found")
        lb, tab = _lb_table(aml)
        return {"__meta": S.meta("LeaderboardV99", "Leaderboard", 99), "project_name": project,
                "models": [S.key(m, "Model") for m in lb["model_id"]], "table": tab,
                "sort_metric": lb.columns[1] if lb.shape[1] > 1 else None}

    @route("GET", "/99/AutoML/{project}")
    def automl_get(p, r, project):
        """AutoMLHandler: project state (leaderboard + event log tables)."""
        lbj = leaderboard(p, r, project)
        aml = dkv.get(project)
        rows = list(getattr(aml, "event_log_rows", []) or [])
        info = getattr(aml, "training_info", None) or {}
        ev = {k: [str(e.get(k, "")) for e in rows] + [""] * len(info)
              for k in ("timestamp", "level", "stage", "message")}
        ev["name"] = [""] * len(rows) + [str(k) for k in info]
        ev["value"] = [""] * len(rows) + [str(v) for v in info.values()]
        n = len(rows) + len(info)
        return {"__meta": S.meta("AutoMLV99", "AutoML", 99),
                "automl_id": {"__meta": S.meta("AutoMLKeyV3", "Key<AutoML>"), "name": project},
                "project_name": project, "leaderboard": lbj, "leaderboard_table": lbj["table"],
                "event_log": {"events": rows},
                "event_log_table": S.twodim("Event Log", ev, "AutoML events", row_headers=[str(i) for i in range(n)]),
                "modeling_steps": [{"name": a, "steps": []} for a in
                                   sorted({str(m).split("_")[0] for m in lbj["table"]["data"][1]})]}

    # ---------------------------------------------- Flow notebooks / NPS
    from .flow import ROUTINES, FlowError, FlowRunner, FlowSyntaxError, LocalTransport
    flow_runner = FlowRunner(LocalTransport(app))

    @app.post("/flow/cell", include_in_schema=False)
    async def flow_cell(request: Request):
        """Run one notebook cell server-side (flow.py); variables persist
        across cells like Flow's notebook sandbox."""
        body = await request.json()
        cmd = {"kind": "flow", "input": body.get("input", ""), "type": body.get("type", "cs"), "defer": False}
        try:
            return await asyncio.wrap_future(executor.submit(cmd))
        except (FlowError, FlowSyntaxError) as e:
            return JSONResponse({"ok": False, "error": str(e)}, status_code=400)

    @app.get("/flow/routines", include_in_schema=False)
    async def flow_routines():
        return JSONResponse({"routines": sorted(ROUTINES)})

    nps_dir = flow_dir if flow_dir is not None else os.environ.get(
        "H2O3_FLOW_DIR", os.path.join(os.path.expanduser("~"), "h2oflows"))
    _nps_cat = _re.compile(r"[-a-zA-Z0-9]+")
    _nps_name = _re.compile(r"[-a-zA-Z0-9_ ()]+")

    def _nps_path(category, name=None):
        """water/init/NodePersistentStorage.java: validated category / key
        names, one file per entry under <flow_dir>/<category>/."""
        if not nps_dir:
            raise _HTTPError(400, "NodePersistentStorage directory not specified (try setting -flow_dir)")
        if not category or not _nps_cat.fullmatch(category):
            raise _HTTPError(400, f"NodePersistentStorage illegal category ({category})")
        if name is None:
            return os.path.join(nps_dir, category)
        if not _nps_name.fullmatch(name):
            raise _HTTPError(400, f"NodePersistentStorage illegal name ({name})")
        return os.path.join(nps_dir, category, name)

    def _nps(**kw):
        return {"__meta": S.meta("NodePersistentStorageV3", "Iced"), "category": None, "name": None,
                "value": None, "configured": bool(nps_dir), "exists": False, **kw}

    @route("GET", "/3/NodePersistentStorage/configured")
    def nps_configured(p, r):
        return _nps()

    @route("GET", "/3/NodePersistentStorage/categories/{category}/names/{name}/exists")
    def nps_exists_name(p, r, category, name):
        return _nps(category=category, name=name, exists=os.path.exists(_nps_path(category, name)))

    @route("GET", "/3/NodePersistentStorage/categories/{category}/exists")
    def nps_exists(p, r, category):
        return _nps(category=category, exists=os.path.isdir(_nps_path(category)))

    def _nps_put(category, name, value):
        path = _nps_path(category, name)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = os.path.join(nps_dir, "_tmp")
        os.makedirs(tmp, exist_ok=True)
        fd, tpath = tempfile.mkstemp(dir=tmp)
        with os.fdopen(fd, "w", encoding="utf-8") as f:
            f.write(value if isinstance(value, str) else _json.dumps(value))
        os.replace(tpath, path)                     # write to _tmp, then rename (reference put)
        return _nps(category=category, name=name)

    @route("POST", "/3/NodePersistentStorage/{category}/{name}")
    def nps_put_name(p, r, category, name):
        return _nps_put(category, name, p.get("value", ""))

    @route("POST", "/3/NodePersistentStorage/{category}")
    def nps_put(p, r, category):
        return _nps_put(category, str(uuid.uuid4()), p.get("value", ""))

    @route("GET", "/3/NodePersistentStorage/{category}/{name}")
    def nps_get(p, r, category, name):
        path = _nps_path(category, name)
        if not os.path.exists(path):
            raise _HTTPError(404, f"NodePersistentStorage: {category}/{name} not found")
        with open(path, encoding="utf-8") as f:
            return _nps(category=category, name=name, value=f.read())

    @route("GET", "/3/NodePersistentStorage/{category}")
    def nps_list(p, r, category):
        d = _nps_path(category)
        names = sorted(os.listdir(d)) if os.path.isdir(d) else []
        entries = [{"__meta": S.meta("NodePersistentStorageEntryV3", "Iced"), "category": category, "name": n,
                    "size": os.path.getsize(os.path.join(d, n)),
                    "timestamp_millis": int(os.path.getmtime(os.path.join(d, n)) * 1000)} for n in names]
        return {**_nps(category=category), "entries": entries}

    @route("DELETE", "/3/NodePersistentStorage/{category}/{name}")
    def nps_delete(p, r, category, name):
        path = _nps_path(category, name)
        if os.path.exists(path):
            os.remove(path)
        return _nps(category=category, name=name)

    from . import rest_more
    rest_more.register(app, route, {"api": api, "uploads": uploads,
                                    "uptime_ms": lambda: (time.time() - t_start) * 1000})
    return app


def create_server_app(login_conf=None, realm="h2o", flow_dir=None):
    """The REST app, behind HTTP Basic authentication when a HashLoginService
    realm file is given (auth.py)."""
    app = create_app(flow_dir)
    if login_conf:
        from .auth import basic_auth_middleware, load_realm
        return basic_auth_middleware(app, load_realm(login_conf), realm)
    return app


def start(ip="127.0.0.1", port=54321, log_level="warning", login_conf=None, ssl_certfile=None, ssl_keyfile=None,
          flow_dir=None):
    """Serve the REST API (blocking).  In a multi-rank cloud (torchrun
    --nproc-per-node N -m h2o3_amd.server) rank 0 serves HTTP and replays
    every command on ranks 1..N-1, which run spmd.worker_loop until rank 0
    shuts the cloud down; login_conf enables Basic auth (the reference's
    -hash_login), the PEM pair enables HTTPS."""
    import uvicorn
    api.init()
    if cloud.rank() != 0:
        app = create_app(flow_dir, serve=False)
        spmd.worker_loop(app.state.run_command)
        return
    inner = create_app(flow_dir)
    outer = inner
    if login_conf:
        from .auth import basic_auth_middleware, load_realm
        outer = basic_auth_middleware(inner, load_realm(login_conf), "h2o")
    server = uvicorn.Server(uvicorn.Config(outer, host=ip, port=port, log_level=log_level,
                                           ssl_certfile=ssl_certfile, ssl_keyfile=ssl_keyfile))
    inner.state.uvicorn = server
    try:
        server.run()
    finally:
        ex = inner.state.executor
        if ex is not None and not ex.stopped and cloud.healthy():
            ex.submit({"kind": "stop"}).result(timeout=600)
