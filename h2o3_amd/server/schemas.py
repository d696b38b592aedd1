"""JSON schemas of the reference REST protocol (water/api/schemas3/*).

The reference clients (h2o-py's H2OConnection, h2o-r's .h2o.doSafeREST) talk
to the server with form-encoded parameters in H2O's own list syntax and read
responses whose objects carry a ``__meta`` block naming their schema
(``schema_name`` / ``schema_type`` / ``schema_version``); h2o-py dispatches on
that name (backend/connection.py H2OResponse: CloudV3, H2OErrorV3,
TwoDimTableV3, ModelMetrics*V3).  This module renders h2o3_amd objects
(frames, jobs, models, metrics, tables) into those shapes and parses the
client's parameter encoding (h2o-py utils/shared_utils.py stringify_list /
_quoted; water/api/Schema.java parse for the server side).

Only the fields the reference clients read are filled; numbers that are NaN
or infinite go out as the strings "NaN" / "Infinity" like the reference's
JSON writer (water/api/SchemaServer + water/util/JSONUtils).
"""
from __future__ import annotations

import math
import time

import numpy as np

VERSION = "3.46.0.99"   # reported as the cluster version (client version checks are opt-in)


# ------------------------------------------------------------------ basics
def meta(name: str, typ: str | None = None, version: int = 3) -> dict:
    if typ is None:
        typ = name[:-2] if name[-2:] in ("V3", "V4", "V99") else name
        if name.endswith("V99"):
            typ = name[:-3]
    return {"schema_version": version, "schema_name": name, "schema_type": typ}


def key(name, kind: str = "Frame") -> dict | None:
    if name is None:
        return None
    route = {"Frame": "Frames", "Model": "Models", "Job": "Jobs", "Grid": "Grids"}.get(kind, kind + "s")
    return {"__meta": meta(f"{kind}KeyV3", f"Key<{kind}>"), "name": str(name), "type": f"Key<{kind}>",
            "URL": f"/3/{route}/{name}"}


def num(v):
    """A JSON-safe number (the reference writes non-finite doubles as strings)."""
    if v is None:
        return None
    if isinstance(v, (bool, np.bool_)):
        return bool(v)
    if isinstance(v, (int, np.integer)):
        return int(v)
    try:
        f = float(v)
    except (TypeError, ValueError):
        return v
    if math.isnan(f):
        return "NaN"
    if math.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    return f


def jsonable(v):
    if isinstance(v, dict):
        return {str(k): jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [jsonable(x) for x in v]
    if isinstance(v, np.ndarray):
        return [jsonable(x) for x in v.tolist()]
    if isinstance(v, (float, int, np.floating, np.integer, bool, np.bool_)):
        return num(v)
    if v is None or isinstance(v, str):
        return v
    if hasattr(v, "frame_id") and hasattr(v, "names"):
        return key(v.frame_id)
    return str(v)


# ------------------------------------------------- parameter decoding
def _split_top(s: str) -> list[str]:
    """Split on commas outside quotes / brackets / braces."""
    out, depth, q, cur = [], 0, None, []
    for ch in s:
        if q:
            cur.append(ch)
            if ch == q:
                q = None
            continue
        if ch in "\"'":
            q = ch
        elif ch in "[{(":
            depth += 1
        elif ch in "]})":
            depth -= 1
        elif ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
            continue
        cur.append(ch)
    if cur or out:
        out.append("".join(cur))
    return out


def _unquote(s: str) -> str:
    s = s.strip()
    if len(s) >= 2 and s[0] == s[-1] and s[0] in "\"'":
        return s[1:-1]
    return s


# parameters whose values are names / ids even when they look numeric
_STRING_PARAMS = {"model_id", "response_column", "training_frame", "validation_frame", "weights_column",
                  "offset_column", "fold_column", "destination_frame", "frame_id", "project_name", "grid_id",
                  "checkpoint", "blending_frame", "leaderboard_frame", "treatment_column", "path", "pattern",
                  "predictions_frame", "deviances_frame", "model", "frame", "session_id", "ast", "id"}


def parse_value(s, name: str | None = None):
    """One form value in the reference client's encoding -> Python value:
    "[a,b]" lists (items possibly quoted), True/False, numbers, quoted or bare
    strings, "{'key': k, 'value': v}" pairs as (k, v) dict entries."""
    if not isinstance(s, str):
        return s
    t = s.strip()
    if t.startswith("[") and t.endswith("]"):
        inner = t[1:-1].strip()
        if not inner:
            return []
        items = [parse_value(x, None if name in _STRING_PARAMS else "__item") for x in _split_top(inner)]
        if items and all(isinstance(i, dict) and set(i) == {"key", "value"} for i in items):
            return {i["key"]: i["value"] for i in items}
        return items
    if t.startswith("{") and t.endswith("}") and ":" in t:
        d = {}
        for part in _split_top(t[1:-1]):
            if ":" not in part:
                continue
            k, v = part.split(":", 1)
            d[_unquote(k)] = parse_value(v.strip())
        return d
    if name in _STRING_PARAMS:
        return _unquote(t)
    if len(t) >= 2 and t[0] == t[-1] and t[0] in "\"'":
        return t[1:-1]
    low = t.lower()
    if low in ("true", "false"):
        return low == "true"
    if low in ("null", "none"):
        return None
    try:
        if t.lstrip("+-").isdigit():
            return int(t)
        return float(t)
    except ValueError:
        return t


def parse_params(raw: dict) -> dict:
    return {k: parse_value(v, k) for k, v in raw.items()}


# ---------------------------------------------------------- tables
def _coltype(vals) -> str:
    kinds = set()
    for v in vals:
        if v is None:
            continue
        if isinstance(v, (bool, np.bool_)):
            kinds.add("string")
        elif isinstance(v, (int, np.integer)):
            kinds.add("long")
        elif isinstance(v, (float, np.floating)):
            kinds.add("double")
        else:
            kinds.add("string")
    if not kinds:
        return "double"
    if kinds <= {"long"}:
        return "long"
    if kinds <= {"long", "double"}:
        return "double"
    return "string"


def twodim(name: str, columns: dict, description: str = "", row_headers=None, row_header_name: str = "") -> dict:
    """TwoDimTableV3 from an ordered {column name: values} dict, column-major
    data; a leading string column carries the row headers when the table has
    them (water/api/schemas3/TwoDimTableV3.java fillFromImpl)."""
    names = list(columns)
    nrow = len(next(iter(columns.values()))) if columns else (len(row_headers) if row_headers is not None else 0)
    cols, data = [], []
    if row_headers is not None:
        cols.append({"__meta": meta("ColumnSpecsBase", "Iced", -1), "name": row_header_name, "type": "string",
                     "format": "%s", "description": row_header_name})
        data.append([None if x is None else str(x) for x in row_headers])
    for n in names:
        vals = list(columns[n])
        t = _coltype(vals)
        fmt = {"long": "%d", "double": "%.5f", "string": "%s"}[t]
        cols.append({"__meta": meta("ColumnSpecsBase", "Iced", -1), "name": str(n), "type": t, "format": fmt,
                     "description": str(n)})
        if t == "string":
            data.append([None if v is None else str(v) for v in vals])
        else:
            data.append([num(v) for v in vals])
    return {"__meta": meta("TwoDimTableV3", "TwoDimTable"), "name": name, "description": description,
            "columns": cols, "rowcount": nrow, "data": data}


def twodim_from_df(name: str, df, description: str = "") -> dict | None:
    if df is None:
        return None
    import pandas as pd
    if isinstance(df, dict):
        try:
            df = pd.DataFrame(df)
        except ValueError:
            df = pd.DataFrame([df])
    elif isinstance(df, list):
        df = pd.DataFrame(df)
    if not isinstance(df, pd.DataFrame):
        return None
    cols = {}
    for c in df.columns:
        s = df[c]
        cols[str(c)] = [None if (isinstance(v, float) and math.isnan(v) and s.dtype == object) else
                        (v.item() if hasattr(v, "item") else v) for v in s.tolist()]
    return twodim(name, cols, description)


# ------------------------------------------------------------ cloud
CLOUD_FIELDS = ["skip_ticks", "version", "branch_name", "last_commit_hash", "describe", "compiled_by", "compiled_on",
                "build_number", "build_age", "build_too_old", "node_idx", "cloud_name", "cloud_size",
                "cloud_uptime_millis", "cloud_internal_timezone", "datafile_parser_timezone", "cloud_healthy",
                "bad_nodes", "consensus", "locked", "is_client", "nodes", "internal_security_enabled", "leader_idx"]
ERROR_FIELDS = ["timestamp", "error_url", "msg", "dev_msg", "http_status", "values", "exception_type",
                "exception_msg", "stacktrace"]
BUILDER_ERROR_FIELDS = ERROR_FIELDS + ["parameters", "messages", "error_count"]
SCHEMA_FIELDS = {"CloudV3": CLOUD_FIELDS, "H2OErrorV3": ERROR_FIELDS,
                 "H2OModelBuilderErrorV3": BUILDER_ERROR_FIELDS}


def schema_metadata(name: str) -> dict | None:
    """MetadataV3 for /3/Metadata/schemas/{name} (field names + help)."""
    fields = SCHEMA_FIELDS.get(name)
    if fields is None:
        return None
    return {"__meta": meta("MetadataV3", "Iced"),
            "schemas": [{"__meta": meta("SchemaMetadataV3", "SchemaMetadata"), "name": name, "version": 3,
                         "type": name[:-2], "fields": [{"__meta": meta("FieldMetadataV3", "FieldMetadata"),
                                                         "name": f, "help": f, "is_schema": f == "nodes"}
                                                        for f in fields]}],
            "routes": []}


def cloud_v3(info: dict, start_time: float) -> dict:
    import os
    import psutil
    vm = psutil.virtual_memory()
    world = int(info.get("cloud_size") or 1)
    gpu = info.get("gpu") or {}
    gmem = int((gpu.get("total_memory_gb") or 0) * 2 ** 30)
    nodes = []
    for r in range(world):
        nodes.append({"__meta": meta("NodeV3", "Iced"), "h2o": f"{info.get('host', 'localhost')}/rank{r}",
                      "ip_port": f"127.0.0.1:{54321 + 2 * r}", "healthy": True,
                      "last_ping": int(time.time() * 1000), "pid": os.getpid(), "num_cpus": os.cpu_count() or 1,
                      "cpus_allowed": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1,
                      "nthreads": os.cpu_count() or 1, "sys_load": float(os.getloadavg()[0]) if hasattr(os, "getloadavg")
                      else 0.0, "my_cpu_pct": -1, "sys_cpu_pct": -1, "mem_value_size": 0, "pojo_mem": 0,
                      "free_mem": int(vm.available), "max_mem": int(vm.total), "swap_mem": 0, "num_keys": 0,
                      "free_disk": 0, "max_disk": 0, "rpcs_active": 0, "fjthrds": [], "fjqueue": [],
                      "tcps_active": 0, "open_fds": 0, "gflops": 0.0, "mem_bw": 0.0,
                      "gpu_name": gpu.get("name"), "gpu_mem": gmem})
    from ..core import timeops
    return {"__meta": meta("CloudV3", "Iced"), "skip_ticks": False, "version": VERSION,
            "branch_name": "h2o3_amd", "last_commit_hash": "", "describe": "h2o3_amd (MI355X)",
            "compiled_by": "h2o3_amd", "compiled_on": "", "build_number": "99", "build_age": "0 days",
            "build_too_old": False, "node_idx": int(info.get("rank") or 0),
            "cloud_name": info.get("cloud_name") or "h2o3_amd", "cloud_size": world,
            "cloud_uptime_millis": int((time.time() - start_time) * 1000),
            "cloud_internal_timezone": timeops.get_timezone(), "datafile_parser_timezone": timeops.get_timezone(),
            "cloud_healthy": True, "bad_nodes": 0, "consensus": True, "locked": True, "is_client": False,
            "nodes": nodes, "internal_security_enabled": False, "leader_idx": 0,
            "backend": info.get("backend"), "device": info.get("device")}


def error_v3(msg: str, status: int, exc: BaseException | None = None, builder: bool = False, **extra) -> dict:
    import traceback
    name = "H2OModelBuilderErrorV3" if builder else "H2OErrorV3"
    out = {"__meta": meta(name, "H2OError" if not builder else "H2OModelBuilderError"),
           "timestamp": int(time.time() * 1000), "error_url": extra.pop("url", None), "msg": msg, "dev_msg": msg,
           "http_status": status, "values": {}, "exception_type": type(exc).__name__ if exc else None,
           "exception_msg": str(exc) if exc else msg,
           "stacktrace": traceback.format_exception(type(exc), exc, exc.__traceback__) if exc else []}
    if builder:
        out.update(parameters=None, messages=extra.pop("messages", []), error_count=1)
    out.update(extra)
    return out


# ------------------------------------------------------------- jobs
def job_v3(job=None, *, key_name=None, dest=None, dest_kind="Frame", description="", status="DONE",
           exception=None) -> dict:
    """JobV3; `job` is an h2o3_amd Job record or None (synthetic finished job)."""
    msg, stack, warns = None, None, None
    if job is not None:
        key_name = job.key
        dest = job.dest
        dest_kind = getattr(job, "dest_kind", None) or dest_kind
        description = job.description or description
        status = job.status
        exception = job.exception
        start = int((job.start_time or time.time()) * 1000)
        msec = int(1000 * ((job.end_time or time.time()) - (job.start_time or time.time())))
        progress = float(job.progress)
        msg = getattr(job, "progress_msg", None) or None
        stack = getattr(job, "stacktrace", None)
        warns = list(getattr(job, "warnings", None) or []) or None
    else:
        start, msec, progress = int(time.time() * 1000), 0, 1.0 if status == "DONE" else 0.0
    status = {"CREATED": "CREATED", "RUNNING": "RUNNING", "DONE": "DONE", "CANCELLED": "CANCELLED",
              "FAILED": "FAILED"}.get(str(status).upper(), str(status).upper())
    dk = key(dest, dest_kind) if dest is not None else None
    return {"__meta": meta("JobV3", "Job"), "key": key(key_name, "Job"), "description": description,
            "status": status, "progress": progress if status != "DONE" else 1.0,
            "progress_msg": "Done." if status == "DONE" else (msg or status), "start_time": start, "msec": msec,
            "dest": dk, "warnings": warns, "exception": None if exception is None else str(exception),
            "stacktrace": stack, "auto_recoverable": False, "ready_for_view": status == "DONE"}


# ----------------------------------------------------------- frames
def _col_v3(name, v, row_offset, row_count, rollups=True):
    import torch
    t = v.type
    lo, hi = row_offset, row_offset + row_count
    c = {"__meta": meta("ColV3", "Vec"), "label": name, "type": t, "domain": v.domain,
         "domain_cardinality": len(v.domain) if v.domain else 0, "data": None, "string_data": None,
         "precision": -1, "histogram_bins": None, "histogram_base": None, "histogram_stride": None,
         "percentiles": None}
    n = len(v)
    if t in ("string", "uuid"):
        vals = v.to_numpy()[lo:hi] if hasattr(v, "to_numpy") else []
        c["string_data"] = [None if x is None or (isinstance(x, float) and math.isnan(x)) else str(x) for x in vals]
        nas = sum(1 for x in v.to_numpy() if x is None or (isinstance(x, float) and math.isnan(x)))
        c.update(missing_count=nas, zero_count=0, positive_infinity_count=0, negative_infinity_count=0,
                 mins=[], maxs=[], mean="NaN", sigma="NaN")
        return c
    data = v.data[lo:min(hi, n)]
    if t == "enum":
        d = data.to(torch.float64)
        d = torch.where(data < 0, torch.full_like(d, float("nan")), d) if data.dtype != torch.float32 else d
        c["data"] = [num(x) for x in d.cpu().tolist()]
    else:
        c["data"] = [num(x) for x in data.to(torch.float64).cpu().tolist()]
    if rollups:
        if t == "enum":
            codes = v.data
            nas = int((codes < 0).sum()) if codes.dtype != torch.float32 else int(torch.isnan(codes).sum())
            c.update(missing_count=nas, zero_count=0, positive_infinity_count=0, negative_infinity_count=0,
                     mins=[0.0], maxs=[float(max(0, len(v.domain or []) - 1))], mean="NaN", sigma="NaN")
        else:
            r = v.rollups()
            x = v.data.to(torch.float64)
            fin = x[torch.isfinite(x)]
            k = min(5, int(fin.numel()))
            mins = torch.topk(fin, k, largest=False).values.cpu().tolist() if k else []
            maxs = torch.topk(fin, k, largest=True).values.cpu().tolist() if k else []
            c.update(missing_count=int(r.get("nas") or 0), zero_count=int(r.get("zeros") or 0),
                     positive_infinity_count=int(r.get("pinfs") or 0),
                     negative_infinity_count=int(r.get("ninfs") or 0),
                     mins=[num(m) for m in mins], maxs=[num(m) for m in maxs], mean=num(r.get("mean")),
                     sigma=num(r.get("sigma")))
    return c


def frame_v3(fid, fr, row_offset=0, row_count=10, column_offset=0, column_count=-1, full_column_count=-1,
             rollups=True, percentiles=False) -> dict:
    names = list(fr.names)
    tot = len(names)
    row_count = fr.nrow if row_count is None or row_count < 0 else row_count
    row_count = max(0, min(row_count, fr.nrow - row_offset))
    cc = tot - column_offset if column_count is None or column_count < 0 else column_count
    sel = names[column_offset:column_offset + cc]
    cols = [_col_v3(n, fr.vec(n), row_offset, row_count, rollups) for n in sel]
    if percentiles:
        import torch
        ps = [0.001, 0.01, 0.1, 0.25, 0.333, 0.5, 0.667, 0.75, 0.9, 0.99, 0.999]
        for c, n in zip(cols, sel):
            v = fr.vec(n)
            if v.type in ("real", "int", "time"):
                x = v.data.to(torch.float64)
                x = x[~torch.isnan(x)]
                if x.numel():
                    q = torch.quantile(x.cpu(), torch.tensor(ps, dtype=torch.float64))
                    c["percentiles"] = [num(z) for z in q.tolist()]
    return {"__meta": meta("FrameV3", "Frame"), "frame_id": key(fid), "byte_size": int(fr.nrow * tot * 4),
            "is_text": False, "row_offset": row_offset, "row_count": row_count, "column_offset": column_offset,
            "column_count": len(sel), "full_column_count": tot if full_column_count is None or full_column_count < 0
            else full_column_count, "total_column_count": tot, "checksum": 0, "rows": fr.nrow,
            "num_columns": tot, "default_percentiles": [0.001, 0.01, 0.1, 0.25, 0.333, 0.5, 0.667, 0.75, 0.9,
                                                        0.99, 0.999],
            "columns": cols, "compatible_models": None,
            "chunk_summary": twodim("Chunk compression summary",
                                    {"chunk_type": ["HBM"], "chunk_name": ["device tensor"], "count": [tot],
                                     "count_percentage": [100.0], "size": [int(fr.nrow * tot * 4)],
                                     "size_percentage": [100.0]}),
            "distribution_summary": twodim("Frame distribution summary",
                                           {"size": [int(fr.nrow * tot * 4)], "number_of_rows": [fr.nrow],
                                            "number_of_chunks_per_column": [1], "number_of_chunks": [tot]},
                                           row_headers=["rank0"])}


def frame_base_v3(fid, fr) -> dict:
    return {"__meta": meta("FrameBaseV3", "Frame"), "frame_id": key(fid), "byte_size": int(fr.nrow * fr.ncol * 4),
            "is_text": False, "rows": fr.nrow, "columns": fr.ncol}


# ---------------------------------------------------------- metrics
_CATEGORY = {"ModelMetricsBinomial": "Binomial", "ModelMetricsMultinomial": "Multinomial",
             "ModelMetricsOrdinal": "Ordinal", "ModelMetricsRegression": "Regression",
             "ModelMetricsClustering": "Clustering", "ModelMetricsAnomaly": "AnomalyDetection",
             "ModelMetricsAutoEncoder": "AutoEncoder", "ModelMetricsDimReduction": "DimReduction",
             "ModelMetricsCoxPH": "CoxPH", "ModelMetricsUplift": "BinomialUplift"}
_METRICS_SCHEMA = {"Binomial": "ModelMetricsBinomialV3", "Multinomial": "ModelMetricsMultinomialV3",
                   "Ordinal": "ModelMetricsOrdinalV3", "Regression": "ModelMetricsRegressionV3",
                   "Clustering": "ModelMetricsClusteringV3", "AnomalyDetection": "ModelMetricsAnomalyV3",
                   "AutoEncoder": "ModelMetricsAutoEncoderV3", "DimReduction": "ModelMetricsPCAV3",
                   "CoxPH": "ModelMetricsRegressionCoxPHV3", "BinomialUplift": "ModelMetricsBinomialUpliftV3"}


def model_category(m) -> str:
    for mm in (m._training_metrics, m._validation_metrics, m._cross_validation_metrics):
        if mm is not None:
            return _CATEGORY.get(type(mm).__name__, "Unknown")
    algo = getattr(m, "algo", "")
    if algo == "word2vec":
        return "WordEmbedding"
    if algo == "targetencoder":
        return "TargetEncoder"
    if algo in ("pca", "svd", "glrm"):
        return "DimReduction"
    if algo in ("kmeans",):
        return "Clustering"
    if algo in ("isolationforest", "extendedisolationforest"):
        return "AnomalyDetection"
    spec = getattr(m, "_spec", None)
    if spec is not None and getattr(spec, "is_classification", False):
        return "Binomial" if getattr(spec, "nclasses", 0) == 2 else "Multinomial"
    return "Regression" if m.supervised_learning else "Unknown"


_MAX_CRIT = ["f1", "f2", "f0point5", "accuracy", "precision", "recall", "specificity", "absolute_mcc",
             "min_per_class_accuracy", "mean_per_class_accuracy", "tns", "fns", "fps", "tps", "tnr", "fnr", "fpr",
             "tpr"]


def _cm_table(cm: dict) -> dict:
    dom = [str(d) for d in cm["domain"]]
    mat = np.asarray(cm["matrix"], dtype=np.float64)
    K = len(dom)
    rows = mat.sum(1)
    cols = {d: list(mat[:, j]) + [float(mat[:, j].sum())] for j, d in enumerate(dom)}
    errs = [float(rows[i] - mat[i, i]) for i in range(K)]
    rate = [e / r if r > 0 else 0.0 for e, r in zip(errs, rows)]
    tot_e, tot = float(sum(errs)), float(rows.sum())
    cols["Error"] = rate + [tot_e / tot if tot > 0 else 0.0]
    cols["Rate"] = [f"{int(e)} / {int(r)}" for e, r in zip(errs, rows)] + [f"{int(tot_e)} / {int(tot)}"]
    thr = cm.get("threshold")
    desc = "" if thr is None else f"Confusion Matrix (Act/Pred) for max f1 @ threshold = {thr}"
    t = twodim("Confusion Matrix", cols, desc, row_headers=dom + ["Total"])
    return {"__meta": meta("ConfusionMatrixV3", "ConfusionMatrix"), "table": t}


def metrics_v3(mm, model=None, frame_id=None, category=None) -> dict | None:
    if mm is None:
        return None
    d = dict(mm._m)
    cat = category or _CATEGORY.get(type(mm).__name__, "Unknown")
    out = {"__meta": meta(_METRICS_SCHEMA.get(cat, "ModelMetricsBaseV3"),
                          type(mm).__name__ if cat in _METRICS_SCHEMA else "ModelMetricsBase"),
           "model": key(getattr(model, "model_id", None), "Model") if model is not None else None,
           "model_checksum": 0, "frame": key(frame_id) if frame_id else None, "frame_checksum": 0,
           "description": None, "model_category": cat, "scoring_time": int(time.time() * 1000),
           "predictions": None, "custom_metric_name": d.get("custom_metric_name"),
           "custom_metric_value": num(d.get("custom_metric_value", 0.0))}
    tables = {"thresholds_and_metric_scores", "gains_lift_table", "cm", "hit_ratio_table", "domain", "withinss",
              "size", "centroid_stats", "multinomial_auc_table", "multinomial_aucpr_table", "auuc_table",
              "aecu_table", "thresholds_and_metric_scores_uplift"}
    for k, v in d.items():
        if k in tables:
            continue
        if isinstance(v, (int, float, np.floating, np.integer, bool, str)) or v is None:
            out[k] = num(v) if not isinstance(v, str) else v
    if "domain" in d:
        out["domain"] = [str(x) for x in d["domain"]]
    tt = d.get("thresholds_and_metric_scores")
    if tt is not None:
        import pandas as pd
        df = pd.DataFrame(tt)
        if "idx" not in df.columns:
            df["idx"] = np.arange(len(df))
        out["thresholds_and_metric_scores"] = twodim_from_df("Metrics for Thresholds", df,
                                                             "Binomial metrics as a function of classification "
                                                             "thresholds")
        crit = {"threshold": [], "value": [], "idx": []}
        rh = []
        for c in _MAX_CRIT:
            if c in df.columns and len(df):
                i = int(np.nanargmax(df[c].to_numpy(dtype=np.float64)))
                rh.append("max " + c)
                crit["threshold"].append(float(df["threshold"].iloc[i]))
                crit["value"].append(float(df[c].iloc[i]))
                crit["idx"].append(i)
        out["max_criteria_and_metric_scores"] = twodim("Maximum Metrics", crit,
                                                       "Maximum metrics at their respective thresholds",
                                                       row_headers=rh, row_header_name="metric")
    if d.get("gains_lift_table") is not None:
        out["gains_lift_table"] = twodim_from_df("Gains/Lift Table", d["gains_lift_table"],
                                                 "Avg response rate: , Avg score: ")
    if isinstance(d.get("cm"), dict) and d["cm"].get("matrix") is not None:
        out["cm"] = _cm_table(d["cm"])
    if d.get("hit_ratio_table") is not None:
        out["hit_ratio_table"] = twodim_from_df("Top-K Hit Ratios", d["hit_ratio_table"])
    for tk, metric in (("multinomial_auc_table", "AUC"), ("multinomial_aucpr_table", "auc_pr")):
        rows = d.get(tk)
        if rows:
            # MultinomialAUC.getTable: row header "Type", then the two class domains and the value
            out[tk] = twodim(f"Multinomial {metric} values",
                             {"first_class_domain": [r["first_class_domain"] for r in rows],
                              "second_class_domain": [r["second_class_domain"] for r in rows],
                              metric: [r["value"] for r in rows]},
                             row_headers=[r["type"] for r in rows], row_header_name="Type")
    if cat == "Clustering":
        ws, sz = d.get("withinss"), d.get("size")
        if ws is not None:
            out["centroid_stats"] = twodim("Centroid Statistics",
                                           {"centroid": list(range(1, len(ws) + 1)),
                                            "size": [float(s) for s in (sz or [0] * len(ws))],
                                            "within_cluster_sum_of_squares": [float(w) for w in ws]})
    return jsonable(out)


# ------------------------------------------------------------ models
_CRITICAL = {"model_id", "training_frame", "validation_frame", "nfolds", "response_column", "ignored_columns",
             "ntrees", "max_depth", "learn_rate", "family", "solver", "alpha", "lambda_", "lambda_search", "k",
             "hidden", "epochs", "activation", "distribution", "gam_columns", "base_models", "metalearner_algorithm",
             "x", "y", "max_iterations", "transform", "pca_method", "loss", "init", "estimator", "treatment_column",
             "uplift_metric", "vec_size", "stop_column", "start_column"}
_EXPERT = ("checkpoint", "export_", "_dir", "custom_", "keep_cross_validation", "max_runtime_secs", "score_",
           "calibrat", "gainslift", "auc_type", "build_tree_one_node", "in_training", "max_confusion", "quiet_mode",
           "diagnostics", "verbose", "max_after_balance", "class_sampling", "pred_noise", "_eps", "epsilon",
           "single_node", "replicate", "shuffle", "reproducible", "sparse", "col_major", "elastic", "fast_mode",
           "force_load_balance", "initial_", "average_activation", "sparsity_beta", "max_categorical_features",
           "mini_batch", "use_all_factor_levels", "non_negative", "gradient_epsilon", "objective_epsilon",
           "beta_epsilon", "prior", "cold_start", "dispersion", "fix_", "generate_", "obj_reg", "max_active",
           "interaction_pairs", "plug_values", "rand_family", "rand_link", "startval", "theta")


def _ref_type(t, actual):
    """Reference client type string (h2o-py docstrings) -> the REST schema type name."""
    t = (t or "").replace(" ", "")
    if t.startswith("Literal["):
        return "enum"
    if "H2OFrame" in t:
        return "Key<Frame>"
    if "H2OEstimator" in t or "ModelBase" in t:
        return "Key<Model>"
    m = {"int": "int", "float": "double", "bool": "boolean", "str": "string", "List[str]": "string[]",
         "List[int]": "int[]", "List[float]": "double[]", "dict": "KeyValue[]", "List[List[str]]": "string[][]"}
    if t in m:
        return m[t]
    if t.startswith("List[") or t.startswith("Union[None,List"):
        return "string[]"
    return None


def _param_entry(name, actual, default, meta_=None):
    def enc(v):
        if hasattr(v, "frame_id") and hasattr(v, "names"):
            return key(v.frame_id)
        if hasattr(v, "model_id") and hasattr(v, "algo"):
            return key(v.model_id, "Model")
        if callable(v):
            return str(v)
        return jsonable(v)
    a, dv = enc(actual), enc(default)
    typ = ("boolean" if isinstance(actual, bool) else "int" if isinstance(actual, int) else
           "double" if isinstance(actual, float) else "string[]" if isinstance(actual, (list, tuple)) else
           "Key<Frame>" if isinstance(a, dict) and a.get("type") == "Key<Frame>" else "string")
    help_, values, level = name, [], "critical"
    if meta_ is not None:
        typ = _ref_type(meta_.get("type"), actual) or typ
        values = list(meta_.get("values") or [])
        help_ = meta_.get("help") or name
        level = "critical" if name in _CRITICAL else \
            "expert" if any(x in name for x in _EXPERT) else "secondary"
    return {"__meta": meta("ModelParameterSchemaV3", "Iced"), "name": name, "label": name, "help": help_,
            "required": name in ("training_frame",) and meta_ is not None, "type": typ, "default_value": dv,
            "actual_value": a, "input_value": a, "level": level, "values": values, "is_member_of_frames": [],
            "is_mutually_exclusive_with": [], "gridable": typ in ("int", "double", "enum", "boolean")}


def model_v3(mid, m) -> dict:
    cat = model_category(m)
    spec = getattr(m, "_spec", None)
    names = list(spec.x) + ([spec.y] if spec is not None and spec.y else []) if spec is not None else []
    frame = getattr(spec, "frame", None) if spec is not None else None
    domains, ctypes = [], []
    for n in names:
        v = frame.vec(n) if frame is not None and n in frame.names else None
        domains.append(v.domain if v is not None and v.domain else None)
        ctypes.append({"enum": "Enum", "string": "String", "time": "Time", "uuid": "UUID"}.get(
            v.type if v is not None else "real", "Numeric"))
    output = {"__meta": meta("ModelOutputSchemaV3", "ModelOutput"), "names": names, "original_names": None,
              "column_types": ctypes, "domains": domains, "cross_validation_models": None,
              "cross_validation_predictions": None, "cross_validation_holdout_predictions_frame_id": None,
              "cross_validation_fold_assignment_frame_id": None, "model_category": cat, "model_summary": None,
              "scoring_history": None, "cv_scoring_history": None, "reproducibility_information_table": None,
              "training_metrics": metrics_v3(m._training_metrics, m, getattr(frame, "frame_id", None), cat),
              "validation_metrics": metrics_v3(m._validation_metrics, m, None,
                                               "Binomial" if cat == "AnomalyDetection" and
                                               type(m._validation_metrics).__name__ == "ModelMetricsBinomial"
                                               else cat),
              "cross_validation_metrics": metrics_v3(m._cross_validation_metrics, m, None, cat),
              "cross_validation_metrics_summary": None, "status": "DONE",
              "start_time": int(m._start_time or 0), "end_time": int(m._end_time or 0),
              "run_time": int((m._run_time or 0) * 1000), "default_threshold": 0.5, "help": {},
              "variable_importances": None, "topology": None}
    if m._cv_models:
        output["cross_validation_models"] = [key(c.model_id, "Model") for c in m._cv_models]
    try:
        sh = m.scoring_history()
        if sh is not None and len(sh):
            output["scoring_history"] = twodim_from_df("Scoring History", sh)
    except Exception:   # noqa: BLE001 - some algos keep no history
        pass
    try:
        vi = m.varimp(use_pandas=True)
        if vi is not None and len(vi):
            output["variable_importances"] = twodim_from_df("Variable Importances", vi)
    except Exception:   # noqa: BLE001
        pass
    ms = m._output.get("model_summary") if isinstance(m._output, dict) else None
    if ms is not None:
        output["model_summary"] = twodim_from_df("Model Summary", ms if not isinstance(ms, dict) else [ms])
    cvs = m._output.get("cross_validation_metrics_summary") if isinstance(m._output, dict) else None
    if cvs is not None:
        output["cross_validation_metrics_summary"] = twodim_from_df("Cross-Validation Metrics Summary", cvs)
    if m._cv_predictions is not None:
        output["cross_validation_holdout_predictions_frame_id"] = key(m._cv_predictions.frame_id)
    if isinstance(m._output, dict):
        _algo_output(m, output)
    if cat == "Binomial" and m._training_metrics is not None:
        thr = m._training_metrics.get("max_f1_threshold")
        if m._validation_metrics is not None and m._validation_metrics.get("max_f1_threshold") is not None:
            thr = m._validation_metrics.get("max_f1_threshold")
        if thr is not None:
            output["default_threshold"] = float(thr)
    params = []
    for k, v in m.params.items():
        params.append(_param_entry(k, v["actual"], v["default"]))
    for k, v in (("response_column", getattr(spec, "y", None)), ("training_frame", frame)):
        if v is not None and k not in m.params:
            params.append(_param_entry(k, v, None))
    for e in params:
        if e["name"] == "response_column" and isinstance(e["actual_value"], str):
            # ColSpecifierV3, as the reference clients read it (actual_params: column_name)
            col = {"__meta": meta("ColSpecifierV3", "VecSpecifier"), "column_name": e["actual_value"],
                   "is_member_of_frames": None}
            e["actual_value"] = e["input_value"] = col
            e["type"] = "VecSpecifier"
    return jsonable({"__meta": meta("ModelSchemaV3", "Model"), "model_id": key(mid, "Model"), "algo": m.algo,
                     "algo_full_name": type(m).__name__.replace("H2O", "").replace("Estimator", ""),
                     "response_column_name": getattr(spec, "y", None),
                     "treatment_column_name": m._parms.get("treatment_column"),
                     "data_frame": key(getattr(frame, "frame_id", None)), "timestamp": int(m._end_time or 0),
                     "have_pojo": True, "have_mojo": True, "parameters": params, "output": output,
                     "compatible_frames": None, "checksum": 0})


def _algo_output(m, output):
    """Algorithm-specific output fields the reference clients read."""
    o = m._output
    if "coefficients" in o:
        coefs = o["coefficients"]
        std = o.get("standardized_coefficients") or {}
        if isinstance(coefs, dict) and coefs and not isinstance(next(iter(coefs.values())), dict):
            names = list(coefs)
            output["coefficients_table"] = twodim("Coefficients", {
                "names": names, "coefficients": [float(coefs[n]) for n in names],
                "standardized_coefficients": [float(std.get(n, coefs[n])) for n in names]}, "glm coefficients")
        for k in ("null_deviance", "residual_deviance", "null_degrees_of_freedom", "residual_degrees_of_freedom",
                  "lambda_best", "lambda_max", "alpha_best", "aic"):
            if k in o:
                output[k] = o[k]
    if "centers" in o:
        # categorical columns' centers are their level names (KMeansModel output centers table)
        c = np.asarray(o["centers"], dtype=object)
        names = o.get("coef_names") or [f"C{j + 1}" for j in range(c.shape[1] if c.ndim == 2 else 0)]

        def _cell(x):
            try:
                return float(x)
            except (TypeError, ValueError):
                return str(x)
        if c.ndim == 2:
            cols = {"centroid": list(range(1, c.shape[0] + 1))}
            for j, n in enumerate(names[:c.shape[1]]):
                cols[str(n)] = [_cell(x) for x in c[:, j]]
            output["centers"] = twodim("Cluster Means", cols)
            cs = o.get("centers_std")
            if cs is not None:
                cs = np.asarray(cs, dtype=object)
                cols = {"centroid": list(range(1, cs.shape[0] + 1))}
                for j, n in enumerate(names[:cs.shape[1]]):
                    cols[str(n)] = [_cell(x) for x in cs[:, j]]
                output["centers_std"] = twodim("Cluster Means (standardized)", cols)
    imp = o.get("importance")
    if isinstance(imp, dict) and imp:
        # PCA / SVD / GLRM importance of components: rows = statistics, columns pc1..pck
        rows = list(imp)
        kk = len(next(iter(imp.values())))
        tab = twodim("Importance of components", {f"pc{j + 1}": [float(imp[r][j]) for r in rows] for j in range(kk)},
                     row_headers=rows)
        output["importance"] = tab
        if o.get("model_summary") is imp:
            output["model_summary"] = tab
    meta_m = getattr(m, "_meta", None)
    if getattr(m, "algo", "") == "stackedensemble" and meta_m is not None:
        output["metalearner"] = key(meta_m.model_id, "Model")
        output["base_models"] = [key(b.model_id, "Model") for b in getattr(m, "_base", [])]
    if "ntrees" in o or hasattr(m, "_forest"):
        output["ntrees"] = o.get("ntrees", len(getattr(m, "_forest", []) or []))
