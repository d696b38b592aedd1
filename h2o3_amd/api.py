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


def import_sql_table(*a, **k):
    raise NotImplementedError("JDBC import is not available (no JDBC drivers in this environment)")


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
            **kw):
    """h2o.explain(): returns the explanation tables (no plotting stack here)."""
    from .models.explain import explain as _ex
    if hasattr(models, "leaderboard") and not isinstance(models, (list, tuple)):
        models = list(models._models) if hasattr(models, "_models") else [models.leader]
    return _ex(models, frame, columns=columns, top_n_features=top_n_features,
               include_explanations=include_explanations, exclude_explanations=exclude_explanations)


def explain_row(models, frame, row_index, columns=None, top_n_features=5, **kw):
    from .models.explain import explain_row as _er
    if hasattr(models, "leader") and not isinstance(models, (list, tuple)):
        models = [models.leader]
    return _er(models, frame, row_index, columns=columns, top_n_features=top_n_features)


def permutation_importance(model, frame, metric="AUTO", n_samples=10000, n_repeats=1, features=None, seed=-1,
                           use_pandas=True):
    return model.permutation_importance(frame, metric, n_samples, n_repeats, features, seed)


def jobs():
    """All job records (water/Job.java list)."""
    from .core.job import jobs as _jobs
    return _jobs()


def timeline():
    """Cloud-wide event timeline (water/TimeLine.java)."""
    from .utils.log import timeline as _tl
    return _tl()
