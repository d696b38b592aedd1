"""Module-level API mirroring `import h2o` (h2o-py/h2o/h2o.py).

`init()` joins the cloud (torch.distributed; RCCL on GPUs), everything else
operates in-process on HBM-resident frames — there is no REST round trip
unless the optional server (h2o3_amd.server) is started.
"""
from __future__ import annotations

import os

from .core import dkv
from .core.frame import H2OFrame
from .parallel import cloud

_progress = {"on": True}


def init(url=None, ip=None, port=None, name=None, nthreads=-1, max_mem_size=None, min_mem_size=None,
         strict_version_check=None, ignore_config=False, extra_classpath=None, jvm_custom_args=None,
         bind_to_localhost=True, device=None, backend=None, verbose=True, **kw):
    info = cloud.init(device=device, backend=backend, name=name)
    if verbose and cloud.rank() == 0:
        g = info.get("gpu") or {}
        print(f"h2o3_amd cloud '{info['cloud_name']}': {info['cloud_size']} rank(s), device {info['device']}"
              + (f" ({g.get('name')}, {g.get('total_memory_gb')} GB)" if g else ""))
    return info


def connect(*a, **k):
    return init(*a, **k)


def cluster():
    return Cluster()


class Cluster:
    def show_status(self, detailed=False):
        print(cloud.info())

    def shutdown(self, prompt=False):
        cloud.shutdown()

    @property
    def cloud_size(self):
        return cloud.world()

    def is_running(self):
        return cloud._state["initialized"]

    def timezone(self):
        from .core import timeops
        return timeops.get_timezone()

    def list_timezones(self):
        from .core import timeops
        return timeops.list_timezones()


def cluster_info():
    return cloud.info()


def shutdown(prompt=False):
    cloud.shutdown()


def no_progress():
    _progress["on"] = False


def show_progress():
    _progress["on"] = True


def import_file(path=None, destination_frame=None, parse=True, header=0, sep=None, col_names=None,
                col_types=None, na_strings=None, pattern=None, skipped_columns=None, custom_non_data_line_markers=None,
                partition_by=None, quotechar=None, escapechar=None):
    from .core import parse as P
    cloud.ensure()
    return P.import_file(path, destination_frame=destination_frame, header=header, sep=sep, col_names=col_names,
                         col_types=col_types, na_strings=na_strings, pattern=pattern,
                         skipped_columns=skipped_columns, quotechar=quotechar)


def upload_file(path, destination_frame=None, header=0, sep=None, col_names=None, col_types=None,
                na_strings=None, skipped_columns=None, quotechar=None, escapechar=None):
    return import_file(path, destination_frame, header=header, sep=sep, col_names=col_names,
                       col_types=col_types, na_strings=na_strings, skipped_columns=skipped_columns,
                       quotechar=quotechar)


def parse_setup(raw_frames, destination_frame=None, header=0, separator=None, column_names=None,
                column_types=None, na_strings=None, **kw):
    from .core import parse as P
    return P.parse_setup(raw_frames, header=header, sep=separator)


def import_sql_table(connection_url, table, username=None, password=None, columns=None, optimize=True,
                     fetch_mode=None, num_chunks_hint=None):
    """Import a whole SQL table (water/jdbc/SQLManager.java importSqlTable): SELECT of
    the listed columns (all by default) through the same DB-API path as
    import_sql_select.  fetch_mode / num_chunks_hint only steer the reference's
    per-node JDBC readers and are accepted for compatibility."""
    import re
    if not re.fullmatch(r"[A-Za-z_][A-Za-z0-9_.$]*", str(table)):
        raise ValueError(f"invalid SQL table name {table!r}")
    if columns:
        cols = [columns] if isinstance(columns, str) else list(columns)
        sel = ", ".join('"' + str(c).replace('"', '""') + '"' for c in cols)
    else:
        sel = "*"
    return import_sql_select(connection_url, f"SELECT {sel} FROM {table}", username=username, password=password,
                             optimize=optimize, fetch_mode=fetch_mode)


def export_file(frame, path, force=False, sep=",", compression=None, parts=1, header=True, quote_header=True,
                parallel=False, format="csv", write_checksum=True):
    from .core import parse as P
    return P.export_file(frame, path, force=force, sep=sep, header=header, format=format)


def get_frame(frame_id, **kw):
    return dkv.get(frame_id)


def get_model(model_id):
    return dkv.get(model_id)


def get_grid(grid_id):
    return dkv.get(grid_id)


def remove(x, cascade=True):
    for o in (x if isinstance(x, (list, tuple)) else [x]):
        key = o if isinstance(o, str) else getattr(o, "frame_id", None) or getattr(o, "model_id", None)
        if key:
            dkv.remove(key)


def remove_all(retained=None):
    dkv.remove_all(retained)


def ls():
    import pandas as pd
    return pd.DataFrame({"key": dkv.keys()})


def frames():
    return [k for k in dkv.keys() if isinstance(dkv.get(k), H2OFrame)]


def models():
    from .models.base import H2OEstimator
    return [k for k in dkv.keys() if isinstance(dkv.get(k), H2OEstimator)]


def deep_copy(data, xid):
    return data.deep_copy(xid)


def assign(data, xid):
    data.frame_id = xid
    dkv.put(xid, data, weak=True)
    return data


def create_frame(frame_id=None, rows=10000, cols=10, randomize=True, real_fraction=None, categorical_fraction=None,
                 integer_fraction=None, binary_fraction=None, time_fraction=None, string_fraction=None,
                 value=0, real_range=100, factors=100, integer_range=100, binary_ones_fraction=0.02,
                 missing_fraction=0.01, has_response=False, response_factors=2, positive_response=False,
                 seed=None, seed_for_column_types=None):
    from .core.munging import create_frame as cf
    return cf(frame_id=frame_id, rows=rows, cols=cols, randomize=randomize, real_fraction=real_fraction,
              categorical_fraction=categorical_fraction, integer_fraction=integer_fraction,
              binary_fraction=binary_fraction, time_fraction=time_fraction, string_fraction=string_fraction,
              value=value, real_range=real_range, factors=factors, integer_range=integer_range,
              binary_ones_fraction=binary_ones_fraction, missing_fraction=missing_fraction,
              has_response=has_response, response_factors=response_factors,
              positive_response=positive_response, seed=seed)


def interaction(data, factors, pairwise, max_factors, min_occurrence, destination_frame=None):
    from .core.munging import interaction as it
    return it(data, factors, pairwise, max_factors, min_occurrence)


def save_model(model, path="", force=False, export_cross_validation_predictions=False, filename=None):
    from .models import persist
    return persist.save_model(model, path, force=force, filename=filename)


def load_model(path):
    from .models import persist
    return persist.load_model(path)


def download_model(model, path="", export_cross_validation_predictions=False, filename=None):
    return save_model(model, path, filename=filename)


def upload_model(path):
    return load_model(path)


def import_mojo(mojo_path, model_id=None):
    from .models.generic import H2OGenericEstimator
    return H2OGenericEstimator.from_file(mojo_path, model_id=model_id)


upload_mojo = import_mojo


def print_mojo(mojo_path, format="json", tree_index=None):
    from .mojo import reader
    return reader.describe(mojo_path)


def make_metrics(predicted, actuals, domain=None, distribution=None, weights=None, auc_type="NONE", **kw):
    from .models.base import TrainSpec
    from .models import metrics as mm
    import torch
    y = actuals.vec(0)
    if y.type == "enum" or (domain is not None):
        dom = domain or y.domain
        if len(dom) == 2:
            p1 = predicted.vec(predicted.ncols - 1).as_float(torch.float64)
            yy = y.data.to(torch.float64) if y.type == "enum" else y.as_float(torch.float64)
            return mm.binomial_metrics(yy, p1, None if weights is None else weights.vec(0).as_float(), dom)
        probs = predicted.to_tensor(predicted.names[-len(dom):], dtype=torch.float64)
        return mm.multinomial_metrics(y.data.long(), probs, None, dom)
    from .models.distributions import get_distribution
    return mm.regression_metrics(y.as_float(torch.float64), predicted.vec(0).as_float(torch.float64),
                                 None if weights is None else weights.vec(0).as_float(),
                                 get_distribution(distribution or "gaussian"))


def flow():
    print("Flow UI is not available; use the Python API or h2o3_amd.server")


def log_and_echo(message=""):
    print(message)


def api(endpoint, data=None, json=None, filename=None, save_to=None):
    raise NotImplementedError("REST endpoints are served by h2o3_amd.server")


def version_check():
    return True


def list_timezones():
    from .core import timeops
    return timeops.list_timezones()


def set_timezone(tz):
    from .core import timeops
    return timeops.set_timezone(tz)


def get_timezone():
    from .core import timeops
    return timeops.get_timezone()


def __getattr__(name):
    # lazy access to estimators / automl / grid at package level
    if name in ("estimators",):
        from . import estimators
        return estimators
    if name == "automl":
        from . import automl
        return automl
    if name == "grid":
        from . import grid
        return grid
    raise AttributeError(name)


def explain(models, frame, columns=None, top_n_features=5, include_explanations="ALL", exclude_explanations=(),
            plot=False, render=None, **kw):
    """h2o.explain(): explanation tables per section, plus matplotlib
    figures under out["plots"] with plot=True (render=True is an alias)."""
    from .models.explain import explain as _ex
    if hasattr(models, "leaderboard") and not isinstance(models, (list, tuple)):
        models = list(models._models) if hasattr(models, "_models") else [models.leader]
    return _ex(models, frame, columns=columns, top_n_features=top_n_features,
               include_explanations=include_explanations, exclude_explanations=exclude_explanations,
               plot=bool(plot or render))


def explain_row(models, frame, row_index, columns=None, top_n_features=5, plot=False, render=None, **kw):
    from .models.explain import explain_row as _er
    if hasattr(models, "leader") and not isinstance(models, (list, tuple)):
        models = [models.leader]
    return _er(models, frame, row_index, columns=columns, top_n_features=top_n_features, plot=bool(plot or render))


def _xp(name):
    def f(*a, **k):
        from .models import explain_plots
        return getattr(explain_plots, name)(*a, **k)
    f.__name__ = name
    f.__doc__ = f"h2o.{name} (h2o-py/h2o/explanation/_explain.py); see models/explain_plots.py"
    return f


varimp_heatmap = _xp("varimp_heatmap")
model_correlation_heatmap = _xp("model_correlation_heatmap")
model_correlation = _xp("model_correlation")
pd_multi_plot = _xp("pd_multi_plot")
varimp = _xp("varimp")


def permutation_importance(model, frame, metric="AUTO", n_samples=10000, n_repeats=1, features=None, seed=-1,
                           use_pandas=True):
    return model.permutation_importance(frame, metric, n_samples, n_repeats, features, seed)


def connection():
    """The 'connection' of an in-process cloud is the cloud itself."""
    return cluster()


def cluster_status():
    cluster().show_status(True)


def network_test():
    """Collective bandwidth probe across the ranks (water/init/NetworkTest.java analogue):
    times an all-reduce of 1 KB .. 64 MB and reports GB/s per size."""
    import time
    import torch
    from .parallel import collectives as coll
    dev = cloud.device()
    rows = []
    for nbytes in (1 << 10, 1 << 16, 1 << 20, 1 << 24, 1 << 26):
        t = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
        coll.allreduce_(t)
        cloud.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            coll.allreduce_(t)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        rows.append({"bytes": nbytes, "seconds": dt, "GB/s": nbytes / max(dt, 1e-12) / 1e9})
    import pandas as pd
    return pd.DataFrame(rows)


def estimate_cluster_mem(ncols, nrows, num_cols=0, string_cols=0, cat_cols=0, time_cols=0, uuid_cols=0):
    """Estimated device memory (GB, rounded up) to hold a frame in this platform's
    layout: f32 numerics, int32 enum codes, f64 epoch-ms times; strings/UUIDs live in
    host memory and are counted at their average host size.  Same arguments and
    validation as h2o-py/h2o/h2o.py:2408, which prices the JVM's compressed chunks."""
    import math
    for nm, v in (("ncols", ncols), ("nrows", nrows), ("num_cols", num_cols), ("string_cols", string_cols),
                  ("cat_cols", cat_cols), ("time_cols", time_cols), ("uuid_cols", uuid_cols)):
        if v < 0:
            raise ValueError(f"{nm} can't be a negative number")
    known = num_cols + string_cols + uuid_cols + cat_cols + time_cols
    if known > ncols:
        raise ValueError("There can not be more specific columns then columns in total")
    unknown = ncols - known
    per_row = 4 * (unknown + num_cols) + 4 * cat_cols + 8 * time_cols + 64 * string_cols + 16 * uuid_cols
    # x2 headroom for model state (binned codes, gradients, histograms) + 256 MB runtime
    return math.ceil((per_row * nrows * 2 + (256 << 20)) / (1 << 30))


def as_list(data, use_pandas=True, header=True):
    """Python object from a frame (h2o-py/h2o/h2o.py:1895)."""
    return data.as_data_frame(use_pandas=use_pandas, header=header)


def frame(frame_id):
    """Metadata of a frame by id (columns, types, rows)."""
    fr = dkv.get(frame_id)
    if fr is None:
        raise KeyError(frame_id)
    return {"frame_id": frame_id, "rows": fr.nrows, "columns": [
        {"label": n, "type": t} for n, t in fr.types.items()]}


def import_frame(path=None, **kw):
    return import_file(path, **kw)


def lazy_import(path, pattern=None):
    """Resolve the files an import would read (no parse)."""
    from .core import parse as P
    if hasattr(P, "resolve_paths"):
        return P.resolve_paths(path, pattern)
    import glob as _g
    paths = path if isinstance(path, (list, tuple)) else [path]
    out = []
    for p in paths:
        if os.path.isdir(p):
            import re
            out += sorted(os.path.join(p, f) for f in os.listdir(p) if not pattern or re.search(pattern, f))
        else:
            out += sorted(_g.glob(p)) or [p]
    return out


def parse_raw(setup, id=None, first_line_is_header=0):
    """Parse the files of a parse_setup() result."""
    paths = setup.get("source_frames") or setup.get("paths") or setup.get("path")
    return import_file(paths, destination_frame=id or setup.get("destination_frame"),
                       header=first_line_is_header or setup.get("check_header", 0),
                       sep=setup.get("separator"), col_names=setup.get("column_names"),
                       col_types=setup.get("column_types"), na_strings=setup.get("na_strings"))


def parse(*a, **k):
    """Deprecated no-op in the reference client."""
    return None


def import_sql_select(connection_url, select_query, username=None, password=None, optimize=True, **kw):
    """SQL import through a DB-API connection: sqlite URLs (jdbc:sqlite:<path>) are
    served by Python's sqlite3; other JDBC drivers are not available here."""
    import sqlite3
    import pandas as pd
    url = connection_url
    if url.startswith("jdbc:sqlite:"):
        url = url[len("jdbc:sqlite:"):]
    elif url.startswith("jdbc:"):
        raise NotImplementedError("only jdbc:sqlite: URLs are supported (no JDBC drivers here)")
    con = sqlite3.connect(url)
    try:
        df = pd.read_sql_query(select_query, con)
    finally:
        con.close()
    return H2OFrame(df)


def download_csv(data, filename):
    data.as_data_frame().to_csv(filename, index=False)
    return filename


def download_pojo(model, path="", get_jar=True, jar_name=""):
    """Java scoring source for the model (hex/Model.toJava); see mojo/pojo.py."""
    from .mojo.pojo import download_pojo as _dp
    return _dp(model, path)


def save_frame(frame, path, force=True):
    return frame.save(path, force=force)


def load_frame(frame_id, path, force=True):
    from .core.frame_io import load_frame as _lf
    return _lf(frame_id, path, force)


def save_grid(grid_directory, grid_id, save_params_references=False, export_cross_validation_predictions=False):
    from .grid import save_grid as _sg
    return _sg(grid_directory, grid_id)


def load_grid(grid_file_path, load_params_references=False):
    from .grid import load_grid as _lg
    return _lg(grid_file_path)


def resume(recovery_dir=None):
    """Resume grids / AutoML runs interrupted while writing to `recovery_dir`
    (hex/faulttolerance/Recovery.java)."""
    from .grid import resume_all
    return resume_all(recovery_dir)


def upload_custom_metric(func, func_file="metrics.py", func_name=None, class_name=None, source_provider=None):
    from .core.udf import upload_custom_metric as _u
    return _u(func, func_file, func_name, class_name, source_provider)


def upload_custom_distribution(func, func_file="distributions.py", func_name=None, class_name=None,
                               source_provider=None):
    from .core.udf import upload_custom_distribution as _u
    return _u(func, func_file, func_name, class_name, source_provider)


def load_dataset(relative_path):
    """Small bundled datasets: "iris" (from scikit-learn's copy, with h2o's column
    names) and any CSV found under $H2O3_AMD_DATA."""
    name = relative_path[:-4] if relative_path.endswith(".csv") else relative_path
    roots = [p for p in os.environ.get("H2O3_AMD_DATA", "").split(os.pathsep) if p]
    for r in roots:
        for cand in (os.path.join(r, relative_path), os.path.join(r, name + ".csv")):
            if os.path.exists(cand):
                return upload_file(cand)
    if name == "iris":
        import pandas as pd
        from sklearn.datasets import load_iris
        d = load_iris()
        df = pd.DataFrame(d.data, columns=["sepal_len", "sepal_wid", "petal_len", "petal_wid"])
        df["class"] = pd.Categorical.from_codes(d.target, ["Iris-setosa", "Iris-versicolor", "Iris-virginica"])
        return H2OFrame(df)
    raise ValueError(f"Data file {relative_path} cannot be found")


def demo(funcname, interactive=False, echo=True, test=False):
    """Run a tiny end-to-end demo ("gbm", "glm" or "deeplearning") on iris."""
    from . import estimators as E
    fr = load_dataset("iris")
    cls = {"gbm": E.H2OGradientBoostingEstimator, "glm": E.H2OGeneralizedLinearEstimator,
           "deeplearning": E.H2ODeepLearningEstimator}[funcname]
    kw = {"family": "multinomial"} if funcname == "glm" else {}
    m = cls(**kw)
    m.train(y="class", training_frame=fr)
    if echo:
        print(m)
    return m


def rapids(expr):
    """Evaluate a Rapids expression string (water/rapids/Rapids.java) — see core/rapids.py."""
    from .core.rapids import rapids as _r
    return _r(expr)


def enable_expr_optimizations(flag):
    """Frames execute eagerly on the GPU; there is no lazy expression tree to optimise."""
    _progress["expr_opt"] = bool(flag)


def is_expr_optimizations_enabled():
    return _progress.get("expr_opt", True)


def import_hive_table(*a, **k):
    raise NotImplementedError("Hive import needs a Hive metastore/JDBC stack, not available here")


def download_all_logs(dirname=".", filename=None, container=None):
    """Write the cloud's log records + timeline to a zip (water/api/LogsHandler)."""
    import json
    import zipfile
    from .utils.log import timeline as _tl
    os.makedirs(dirname, exist_ok=True)
    path = os.path.join(dirname, filename or "h2o3_amd_logs.zip")
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("timeline.json", json.dumps(_tl(), default=str))
        z.writestr("jobs.json", json.dumps([getattr(j, "__dict__", str(j)) for j in jobs()], default=str))
    return path


def jobs():
    """All job records (water/Job.java list)."""
    from .core.job import jobs as _jobs
    return _jobs()


def timeline():
    """Cloud-wide event timeline (water/TimeLine.java)."""
    from .utils.log import timeline as _tl
    return _tl()


# ---- h2o.scoring / h2o.persist (reference h2o-py h2o/scoring.py, h2o/persist/persist.py)
def make_leaderboard(object, leaderboard_frame=None, sort_metric="AUTO", extra_columns=[], scoring_data="AUTO"):
    from .automl.leaderboard import make_leaderboard as _mk
    return _mk(object, leaderboard_frame, sort_metric, extra_columns, scoring_data)


def set_s3_credentials(secret_key_id, secret_access_key, session_token=None):
    from .core.persist import set_s3_credentials as _set
    _set(secret_key_id, secret_access_key, session_token)


def remove_s3_credentials():
    from .core.persist import remove_s3_credentials as _rm
    _rm()
