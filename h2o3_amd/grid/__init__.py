"""Hyper-parameter grid search.

Reference: hex/grid/GridSearch.java, HyperSpaceWalker.java
(CartesianWalker / RandomDiscreteValueWalker with max_models,
max_runtime_secs, early stopping on the grid's sort metric),
hex/grid/Grid.java, h2o-py/h2o/grid/grid_search.py (client API:
train / get_grid / sorted_metric_table / models / model_ids).
"""
from __future__ import annotations

import itertools
import math
import random
import time

import numpy as np

from ..core import dkv
from ..core import job as jobmod
from ..parallel import cloud


class H2OGridSearch:
    def __init__(self, model, hyper_params, grid_id=None, search_criteria=None, export_checkpoints_dir=None,
                 recovery_dir=None, parallelism=1):
        self.model = model
        self.hyper_params = dict(hyper_params)
        self.grid_id = grid_id or dkv.make_key("Grid")
        self.search_criteria = dict(search_criteria or {"strategy": "Cartesian"})
        self.models = []
        self._failures = []          # (combo, message, stack trace) per failed build
        self._sort_metric = None
        self.export_checkpoints_dir = export_checkpoints_dir
        self.recovery_dir = recovery_dir
        self.parallelism = parallelism
        self._job = None
        self._thread = None
        self._error = None
        self._train_args = None

    def _estimator_factory(self):
        m = self.model
        if isinstance(m, type):
            return lambda **kw: m(**kw)
        base = m._user_parms()
        cls = type(m)
        return lambda **kw: cls(**{**base, **kw})

    def _combos(self):
        keys = list(self.hyper_params)
        vals = [v if isinstance(v, (list, tuple)) else [v] for v in (self.hyper_params[k] for k in keys)]
        combos = [dict(zip(keys, c)) for c in itertools.product(*vals)]
        sc = self.search_criteria
        if (sc.get("strategy") or "Cartesian").lower() == "randomdiscrete":
            rng = random.Random(sc.get("seed", 1234) if sc.get("seed", -1) != -1 else 1234)
            rng.shuffle(combos)
        return combos

    def train(self, x=None, y=None, training_frame=None, offset_column=None, fold_column=None, weights_column=None,
              validation_frame=None, **params):
        sc = self.search_criteria
        max_models = int(sc.get("max_models") or 0)
        max_rt = float(sc.get("max_runtime_secs") or 0)
        stop_rounds = int(sc.get("stopping_rounds") or 0)
        t0 = time.time()
        make = self._estimator_factory()
        history = []
        self._train_args = dict(x=x, y=y, training_frame=training_frame, offset_column=offset_column,
                                fold_column=fold_column, weights_column=weights_column,
                                validation_frame=validation_frame, **params)
        done = self._recover()
        # combinations already built (a resumed / restarted grid) are skipped
        done |= {repr(sorted(m._grid_params.items())) for m in self.models if getattr(m, "_grid_params", None)}
        if self.recovery_dir:
            self._save_train_inputs(x, y, training_frame, validation_frame, weights_column, offset_column,
                                    fold_column, params)
        combos = self._combos()
        for combo in combos:
            key = repr(sorted(combo.items()))
            if key in done:
                continue
            if max_models and len(self.models) >= max_models:
                break
            timed = bool(max_rt and time.time() - t0 > max_rt)
            # rank 0's clock decides (SPMD), and a REST cancel of the grid job stops here
            j = jobmod.current()
            if j is not None:
                tot = min(max_models, len(combos)) if max_models else len(combos)
                timed = bool(j.tick(len(self.models) / max(tot, 1), extra=(timed,))[0])
            elif max_rt and cloud.is_distributed():
                timed = bool(cloud.agree([timed])[0])
            if timed:
                break
            kw = dict(params)
            kw.update(combo)
            kw["model_id"] = f"{self.grid_id}_model_{len(self.models) + 1}"
            try:
                est = make(**kw)
                est.train(x=x, y=y, training_frame=training_frame, offset_column=offset_column,
                          fold_column=fold_column, weights_column=weights_column, validation_frame=validation_frame)
                est._grid_params = combo
                self.models.append(est)
                self._checkpoint(est, combo)
                if stop_rounds:
                    history.append(self._metric_of(est))
                    if self._stop(history, sc):
                        break
            except Exception as e:  # reference keeps failures in the grid's failure list
                if isinstance(e, jobmod.JobCancelled):
                    raise
                import traceback
                self._failures.append((combo, repr(e), traceback.format_exc()[-4000:]))
        dkv.put(self.grid_id, self)
        return self

    # ------------------------------------------------------------ recovery
    # reference: hex/faulttolerance/Recovery.java + grid recovery_dir: every
    # finished model and the grid state are written as they complete, so a
    # restarted grid (same recovery_dir / grid_id) resumes where it stopped.
    def _state_path(self):
        import os
        return os.path.join(self.recovery_dir, f"{self.grid_id}.grid.json")

    def _save_train_inputs(self, x, y, training_frame, validation_frame, weights_column, offset_column,
                           fold_column, params):
        """Persist what a resumed grid needs to continue: the frames (native binary
        format) and the train() arguments."""
        import os
        from ..core.frame_io import save_frame
        os.makedirs(self.recovery_dir, exist_ok=True)
        fdir = f"{self.grid_id}.train_frame"
        from ..parallel import collectives as coll
        if not coll.broadcast_object(os.path.exists(os.path.join(self.recovery_dir, fdir, "frame.json"))):
            save_frame(training_frame, os.path.join(self.recovery_dir, fdir))
        vdir = None
        if validation_frame is not None:
            vdir = f"{self.grid_id}.valid_frame"
            if not coll.broadcast_object(os.path.exists(os.path.join(self.recovery_dir, vdir, "frame.json"))):
                save_frame(validation_frame, os.path.join(self.recovery_dir, vdir))
        self._train_rec = {"frame_dir": fdir, "valid_dir": vdir, "x": x, "y": y, "weights_column": weights_column,
                           "offset_column": offset_column, "fold_column": fold_column,
                           "params": _json_safe(params)}
        self._write_state()

    def _write_state(self):
        import json
        base = self.model if isinstance(self.model, type) else type(self.model)
        st = {"grid_id": self.grid_id, "hyper_params": {k: list(v) if isinstance(v, (list, tuple)) else v
                                                        for k, v in self.hyper_params.items()},
              "search_criteria": self.search_criteria,
              "estimator": f"{base.__module__}:{base.__qualname__}",
              "base_params": _json_safe(getattr(self.model, "_parms", {}) if not isinstance(self.model, type)
                                        else {}),
              "train": getattr(self, "_train_rec", None),
              "models": [{"model_id": m.model_id, "params": m._grid_params} for m in self.models]}
        with open(self._state_path(), "w") as f:
            json.dump(st, f, default=str)

    def _checkpoint(self, est, combo):
        import os
        from ..models.persist import save_model
        for d in (self.export_checkpoints_dir, self.recovery_dir):
            if d:
                os.makedirs(d, exist_ok=True)
                save_model(est, d, force=True)
        if self.recovery_dir:
            self._write_state()

    def _recover(self):
        import json
        import os
        from ..models.persist import load_model
        if not self.recovery_dir or not os.path.exists(self._state_path()):
            return set()
        st = json.load(open(self._state_path()))
        have = {m.model_id for m in self.models}
        for rec in st["models"]:
            if rec["model_id"] in have:
                continue
            m = load_model(os.path.join(self.recovery_dir, rec["model_id"]))
            m._grid_params = rec["params"]
            self.models.append(m)
        return {repr(sorted(r["params"].items())) for r in st["models"]}

    def _default_metric(self):
        if not self.models:
            return "mse"
        m = self.models[0]
        if m._spec is None or not m.supervised_learning:
            return "tot_withinss"
        if m._spec.nclasses == 2:
            return "auc"
        if m._spec.nclasses > 2:
            return "logloss"
        return "residual_deviance"

    def _metric_of(self, est, metric=None):
        metric = (metric or self.search_criteria.get("stopping_metric") or self._default_metric()).lower()
        mt = est._cross_validation_metrics or est._validation_metrics or est._training_metrics
        if mt is None:
            return float("nan")
        key = {"auc": "AUC", "logloss": "logloss", "rmse": "RMSE", "mse": "MSE", "mae": "mae", "r2": "r2",
               "residual_deviance": "mean_residual_deviance", "deviance": "mean_residual_deviance",
               "mean_per_class_error": "mean_per_class_error", "aucpr": "pr_auc", "tot_withinss": "tot_withinss",
               "rmsle": "rmsle"}.get(metric, metric)
        v = mt.get(key)
        return float("nan") if v is None else float(v)

    @staticmethod
    def _stop(history, sc):
        from ..models.base import ScoreKeeper
        k = int(sc.get("stopping_rounds") or 0)
        metric = (sc.get("stopping_metric") or "auto").lower()
        less = metric not in ("auc", "aucpr", "r2")
        best = []
        for v in history:
            if not best:
                best.append(v)
            else:
                best.append(min(best[-1], v) if less else max(best[-1], v))
        return ScoreKeeper.stop_early(best, k, float(sc.get("stopping_tolerance", 0.001)), less)

    def get_grid(self, sort_by=None, decreasing=None):
        metric = (sort_by or self._default_metric()).lower()
        if decreasing is None:
            decreasing = metric in ("auc", "aucpr", "r2", "accuracy")
        g = H2OGridSearch(self.model, self.hyper_params, self.grid_id, self.search_criteria)
        g.models = sorted(self.models, key=lambda m: self._metric_of(m, metric), reverse=decreasing)
        g._sort_metric = metric
        g._failures = self._failures
        g._train_args = self._train_args
        return g

    def sorted_metric_table(self):
        import pandas as pd
        metric = self._sort_metric or self._default_metric()
        rows = []
        for m in self.models:
            r = dict(m._grid_params)
            r["model_ids"] = m.model_id
            r[metric] = self._metric_of(m, metric)
            rows.append(r)
        return pd.DataFrame(rows)

    @property
    def model_ids(self):
        return [m.model_id for m in self.models]

    # ------------------------------------------------------------ grid state
    # reference: h2o-py/h2o/grid/grid_search.py:110-206 (properties read from the
    # grid's JSON); here they read the in-process grid
    @property
    def key(self):
        return self.grid_id

    @property
    def hyper_names(self):
        return list(self.hyper_params)

    @property
    def failed_params(self):
        return [dict(c) for c, _, _ in self._failures]

    @property
    def failure_details(self):
        return [m for _, m, _ in self._failures]

    @property
    def failure_stack_traces(self):
        return [t for _, _, t in self._failures]

    @property
    def failed_raw_params(self):
        return [[str(c.get(k)) for k in self.hyper_params] for c, _, _ in self._failures]

    def detach(self):
        self.grid_id = None

    # ------------------------------------------------------------ async build
    def start(self, x, y=None, training_frame=None, offset_column=None, fold_column=None, weights_column=None,
              validation_frame=None, **params):
        """Asynchronous grid build (grid_search.py:209): the models are built on a
        background thread under a Job; join() waits, cancel() stops it after the
        model in progress (the grid job's cancel reaches each build's tick)."""
        import threading
        job = jobmod.Job(f"Grid search {self.grid_id}", dest=self.grid_id, dest_kind="Grid")
        self._job, self._error = job, None

        def run():
            job.start()
            jobmod.push(job)
            try:
                self.train(x=x, y=y, training_frame=training_frame, offset_column=offset_column,
                           fold_column=fold_column, weights_column=weights_column,
                           validation_frame=validation_frame, **params)
                job.done()
            except BaseException as e:    # surfaced by join()
                job.fail(e)
                self._error = e
            finally:
                jobmod.pop(job)
                dkv.put(self.grid_id, self)

        self._thread = threading.Thread(target=run, name=f"grid-{self.grid_id}", daemon=True)
        self._thread.start()
        return self

    def join(self):
        """Wait until the grid finishes (grid_search.py:252)."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        job, self._job = self._job, None
        err, self._error = self._error, None
        if err is not None and not isinstance(err, jobmod.JobCancelled) and not (job and job.cancel_requested):
            raise err
        return self

    def cancel(self):
        """Cancel a running grid (grid_search.py:274)."""
        if self._job is None:
            raise ValueError("Grid is not running.")
        self._job.cancel()

    def resume(self, recovery_dir=None, **kwargs):
        """Continue a stopped grid (grid_search.py:358): the combinations not yet
        built are trained with the arguments of the last train() / start() (or
        the recovery state in recovery_dir); kwargs override search criteria."""
        detach = kwargs.pop("detach", False)
        if recovery_dir is not None:
            self.recovery_dir = recovery_dir
        for k in ("max_models", "max_runtime_secs", "stopping_rounds", "stopping_metric", "stopping_tolerance"):
            if k in kwargs:
                self.search_criteria[k] = kwargs.pop(k)
        args = dict(self._train_args or {})
        if not args and self.recovery_dir:
            import json
            import os
            from ..core.frame_io import load_frame
            st = json.load(open(self._state_path()))
            tr = st["train"]
            args = dict(x=tr.get("x"), y=tr.get("y"),
                        training_frame=load_frame(None, os.path.join(self.recovery_dir, tr["frame_dir"])),
                        validation_frame=load_frame(None, os.path.join(self.recovery_dir, tr["valid_dir"]))
                        if tr.get("valid_dir") else None, weights_column=tr.get("weights_column"),
                        offset_column=tr.get("offset_column"), fold_column=tr.get("fold_column"),
                        **tr.get("params", {}))
        if not args:
            raise ValueError("resume: this grid was never trained (no training arguments to resume with)")
        args.update(kwargs)
        return self.start(**args) if detach else self.train(**args)

    def build_model(self, algo_params):
        """(internal, grid_search.py:373) train with a parameter dict."""
        p = dict(algo_params)
        keys = ("x", "y", "training_frame", "offset_column", "fold_column", "weights_column", "validation_frame")
        return self.train(**{k: p.pop(k, None) for k in keys}, **p)

    # ------------------------------------------------------------ per-model passthroughs
    # every one returns {model_id: value} over the grid's models, as the
    # reference client does (grid_search.py:485-1353)
    def _each(self, fn):
        return {m.model_id: fn(m) for m in self.models}

    def predict(self, test_data):
        return self._each(lambda m: m.predict(test_data))

    def is_cross_validated(self):
        return self._each(lambda m: m.is_cross_validated())

    def xval_keys(self):
        return self._each(lambda m: m.xval_keys())

    def get_xval_models(self, key=None):
        def one(m):
            xs = m.get_xval_models()
            if key is None:
                return xs
            return next((x for x in (xs or []) if x.model_id == key), None)
        return self._each(one)

    def xvals(self):
        return self._each(lambda m: m.xvals)

    def deepfeatures(self, test_data, layer):
        return self._each(lambda m: m.deepfeatures(test_data, layer))

    def weights(self, matrix_id=0):
        return self._each(lambda m: m.weights(matrix_id))

    def biases(self, vector_id=0):
        return self._each(lambda m: m.biases(vector_id))

    def normmul(self):
        return self._each(lambda m: m.normmul())

    def normsub(self):
        return self._each(lambda m: m.normsub())

    def respmul(self):
        return self._each(lambda m: m.respmul())

    def respsub(self):
        return self._each(lambda m: m.respsub())

    def catoffsets(self):
        return self._each(lambda m: m.catoffsets())

    def model_performance(self, test_data=None, train=False, valid=False, xval=False):
        return self._each(lambda m: m.model_performance(test_data, train, valid, xval))

    def scoring_history(self):
        return self._each(lambda m: m.scoring_history())

    def varimp(self, use_pandas=False):
        return self._each(lambda m: m.varimp(use_pandas))

    def residual_deviance(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.residual_deviance(train, valid, xval))

    def residual_degrees_of_freedom(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.residual_degrees_of_freedom(train, valid, xval))

    def null_deviance(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.null_deviance(train, valid, xval))

    def null_degrees_of_freedom(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.null_degrees_of_freedom(train, valid, xval))

    def pprint_coef(self):
        for i, m in enumerate(self.models):
            print("Model", i)
            m.pprint_coef()
            print()

    def coef(self):
        return self._each(lambda m: m.coef())

    def coef_norm(self):
        return self._each(lambda m: m.coef_norm())

    def r2(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.r2(train, valid, xval))

    def mse(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.mse(train, valid, xval))

    def rmse(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.rmse(train, valid, xval))

    def mae(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.mae(train, valid, xval))

    def rmsle(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.rmsle(train, valid, xval))

    def logloss(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.logloss(train, valid, xval))

    def mean_residual_deviance(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.mean_residual_deviance(train, valid, xval))

    def auc(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.auc(train, valid, xval))

    def aic(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.aic(train, valid, xval))

    def gini(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.gini(train, valid, xval))

    def aucpr(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.aucpr(train, valid, xval))

    pr_auc = aucpr

    # ------------------------------------------------------------ summaries
    def get_summary(self):
        """One row per model: its model summary with the model id first
        (grid_search.py:852)."""
        import pandas as pd
        rows = []
        for m in self.models:
            s = m.get_summary() if hasattr(m, "get_summary") else None
            if s is None:
                r = {}
            elif isinstance(s, pd.DataFrame):
                r = s.iloc[0].to_dict() if len(s) else {}
            elif isinstance(s, dict):
                r = dict(s)
            else:
                r = {"summary": str(s)}
            r.pop("", None)
            rows.append({"Model Id": m.model_id, **r})
        return pd.DataFrame(rows)

    def show_summary(self):
        print(self.get_summary().to_string())

    def summary(self):
        """Deprecated alias of show_summary (grid_search.py:886)."""
        self.show_summary()

    def sort_by(self, metric, increasing=True):
        """Deprecated (grid_search.py:1540): the sorted metric table by `metric`."""
        return self.get_grid(sort_by=metric.split("(")[0], decreasing=not increasing).sorted_metric_table()

    def pareto_front(self, test_frame, x_metric=None, y_metric=None, **kwargs):
        """Pareto front of the grid's models on test_frame (grid_search.py:1554):
        leaderboard with every extra column, optimum corner from the metrics'
        directions, then h2o.explanation.pareto_front."""
        from ..automl.leaderboard import make_leaderboard
        from ..explanation import pareto_front
        lb = make_leaderboard(self, test_frame, extra_columns="ALL")
        x_metric = x_metric or "predict_time_per_row_ms"
        y_metric = y_metric or lb.columns[1]
        hib = ("auc", "aucpr")
        optimum = "{} {}".format("top" if y_metric.lower() in hib else "bottom",
                                 "right" if x_metric.lower() in hib else "left")
        kwargs.setdefault("title", f"Pareto Front for {self.grid_id}")
        return pareto_front(lb, x_metric, y_metric, optimum=optimum, **kwargs)

    def get_hyperparams(self, id, display=True):
        m = self.models[id] if isinstance(id, int) else next(mm for mm in self.models if mm.model_id == id)
        if display:
            print("Hyperparameters: [" + ", ".join(self.hyper_params) + "]")
        return [m._grid_params[k] for k in self.hyper_params]

    def get_hyperparams_dict(self, id, display=True):
        m = self.models[id] if isinstance(id, int) else next(mm for mm in self.models if mm.model_id == id)
        if display:
            print("Hyperparameters: [" + ", ".join(self.hyper_params) + "]")
        return dict(m._grid_params)

    def __getitem__(self, i):
        return self.models[i]

    def __len__(self):
        return len(self.models)

    def __iter__(self):
        return iter(self.models)

    def show(self, verbosity=None, fmt=None):
        print(self.sorted_metric_table())


# ---------------------------------------------------------------- save / load / resume
# reference: h2o.save_grid / h2o.load_grid (h2o-py/h2o/h2o.py:504-549,
# hex/grid/Grid.exportBinary): the grid object plus every model, in one folder.
def _json_safe(d):
    return {k: (list(v) if isinstance(v, tuple) else v) for k, v in d.items()
            if isinstance(v, (int, float, str, bool, list, tuple, dict, type(None)))}


def save_grid(grid_directory, grid_id):
    import json
    import os
    from ..models.persist import save_model
    g = grid_id if isinstance(grid_id, H2OGridSearch) else dkv.get(grid_id)
    if g is None:
        raise KeyError(f"grid {grid_id} not found")
    os.makedirs(grid_directory, exist_ok=True)
    for m in g.models:
        save_model(m, grid_directory, force=True)
    base = g.model if isinstance(g.model, type) else type(g.model)
    st = {"format": "h2o3_amd.grid.v1", "grid_id": g.grid_id,
          "estimator": f"{base.__module__}:{base.__qualname__}",
          "base_params": _json_safe(getattr(g.model, "_parms", {}) if not isinstance(g.model, type) else {}),
          "hyper_params": _json_safe(g.hyper_params), "search_criteria": _json_safe(g.search_criteria),
          "models": [{"model_id": m.model_id, "params": _json_safe(getattr(m, "_grid_params", {}))}
                     for m in g.models],
          "failed": [[_json_safe(c), e] for c, e, _ in g._failures]}
    path = os.path.join(grid_directory, g.grid_id)
    with open(path, "w") as f:
        json.dump(st, f, default=str)
    return path


def _estimator_class(spec):
    import importlib
    mod, _, qn = spec.partition(":")
    obj = importlib.import_module(mod)
    for part in qn.split("."):
        obj = getattr(obj, part)
    return obj


def load_grid(grid_file_path):
    import json
    import os
    from ..models.persist import load_model
    with open(grid_file_path) as f:
        st = json.load(f)
    if st.get("format") != "h2o3_amd.grid.v1":
        raise ValueError(f"{grid_file_path} is not a saved h2o3_amd grid")
    d = os.path.dirname(grid_file_path)
    cls = _estimator_class(st["estimator"])
    base = cls(**cls._accepted({k: v for k, v in st["base_params"].items() if k != "model_id"})) \
        if st["base_params"] else cls
    g = H2OGridSearch(base, st["hyper_params"], grid_id=st["grid_id"], search_criteria=st["search_criteria"])
    for rec in st["models"]:
        m = load_model(os.path.join(d, rec["model_id"]))
        m._grid_params = rec["params"]
        g.models.append(m)
    g._failures = [(x[0], x[1], "") for x in st.get("failed", [])]
    dkv.put(g.grid_id, g)
    return g


def resume_all(recovery_dir):
    """Resume every grid whose recovery state lives in `recovery_dir`: models
    already finished are reloaded and the remaining hyper-parameter combinations
    are trained (hex/faulttolerance/Recovery.autoRecover).  The training frame
    must be recoverable: grids store it in the recovery dir when they start."""
    import json
    import os
    from ..core.frame_io import load_frame
    out = []
    if not recovery_dir or not os.path.isdir(recovery_dir):
        return out
    for fn in sorted(os.listdir(recovery_dir)):
        if not fn.endswith(".grid.json"):
            continue
        with open(os.path.join(recovery_dir, fn)) as f:
            st = json.load(f)
        if "estimator" not in st or "train" not in st:
            continue
        cls = _estimator_class(st["estimator"])
        base = cls(**cls._accepted({k: v for k, v in st.get("base_params", {}).items() if k != "model_id"}))
        g = H2OGridSearch(base, st["hyper_params"], grid_id=st["grid_id"], search_criteria=st["search_criteria"],
                          recovery_dir=recovery_dir)
        tr = st["train"]
        fr = load_frame(None, os.path.join(recovery_dir, tr["frame_dir"]))
        vf = load_frame(None, os.path.join(recovery_dir, tr["valid_dir"])) if tr.get("valid_dir") else None
        g.train(x=tr.get("x"), y=tr.get("y"), training_frame=fr, validation_frame=vf,
                weights_column=tr.get("weights_column"), offset_column=tr.get("offset_column"),
                fold_column=tr.get("fold_column"), **tr.get("params", {}))
        out.append(g)
    from ..automl import resume_automl
    out += resume_automl(recovery_dir)
    return out
