"""ModelBuilder / Model base shared by every algorithm.

Reference: hex/ModelBuilder.java (parameter validation, CV driver
`computeCrossValidation`, fold assignment hex/FoldAssignment.java),
hex/Model.java (scoring, `adaptTestForTrain`, predict frame layout),
hex/ScoreKeeper.java (early stopping), and the client API
h2o-py/h2o/estimators/estimator_base.py + h2o/model/model_base.py.

An estimator instance is both the builder and (after `train`) the model,
exactly like h2o-py.  Algorithms subclass `H2OEstimator` and implement
`_fit(spec)` (train on a TrainSpec) and `_predict_raw(frame)` (device
tensor [n, K] of link-inverse predictions / class probabilities).
"""
from __future__ import annotations

import copy
import json
import math
import os
import time

import numpy as np
import torch

from ..core import dkv
from ..core.frame import H2OFrame, _local_slice
from ..core.vec import NUMERIC_TYPES, T_ENUM, T_INT, T_REAL, Vec
from ..parallel import cloud
from ..parallel import collectives as coll
from . import metrics as mm

COMMON_DEFAULTS = dict(model_id=None, training_frame=None, validation_frame=None, nfolds=0,
                       keep_cross_validation_models=True, keep_cross_validation_predictions=False,
                       keep_cross_validation_fold_assignment=False, fold_assignment="auto", fold_column=None,
                       response_column=None, ignored_columns=None, ignore_const_cols=True, offset_column=None,
                       weights_column=None, max_runtime_secs=0.0, seed=-1, stopping_rounds=0,
                       stopping_metric="auto", stopping_tolerance=0.001, custom_metric_func=None,
                       export_checkpoints_dir=None, auc_type="auto", gainslift_bins=-1,
                       score_each_iteration=False, distribution="auto")

_LESS_IS_BETTER = {"deviance", "logloss", "mse", "rmse", "mae", "rmsle", "mean_per_class_error",
                   "misclassification", "anomaly_score", "custom"}


class TrainSpec:
    """Resolved training inputs (reference: ModelBuilder.init + DataInfo setup)."""

    def __init__(self, frame: H2OFrame, x, y, weights=None, offset=None, fold=None, valid=None):
        self.frame = frame
        self.x = list(x)
        self.y = y
        self.weights_column = weights
        self.offset_column = offset
        self.fold_column = fold
        self.valid = valid
        self.response_domain = None
        self.nclasses = 1
        if y is not None:
            v = frame.vec(y)
            if v.type == T_ENUM:
                self.response_domain = list(v.domain)
                self.nclasses = len(v.domain)

    @property
    def is_classification(self):
        return self.nclasses > 1

    def yvec(self, frame=None):
        return (frame if frame is not None else self.frame).vec(self.y)

    def y_tensor(self, frame=None, dtype=torch.float32):
        v = self.yvec(frame)
        if v.type == T_ENUM:
            return v.data.to(torch.int64)
        return v.as_float(dtype)

    def w_tensor(self, frame=None):
        fr = frame if frame is not None else self.frame
        if self.weights_column and self.weights_column in fr.names:
            w = fr.vec(self.weights_column).as_float()
            return torch.nan_to_num(w, nan=0.0)
        return None

    def offset_tensor(self, frame=None):
        fr = frame if frame is not None else self.frame
        if self.offset_column and self.offset_column in fr.names:
            return torch.nan_to_num(fr.vec(self.offset_column).as_float(), nan=0.0)
        return None


def scoring_names(domain):
    from ..mojo.genmodel import scoring_names as _names     # hex/Model.java makeScoringNames
    return _names(domain)


class ScoreSchedule:
    """When an iterative tree builder scores (SharedTree.java:792
    doScoringAndSaveModel): every score_tree_interval trees when set, always
    with score_each_iteration and at the final tree; otherwise time-based --
    every iteration during the first initial_score_interval ms (4 s), then at
    most every score_interval ms (4 s) and only while scoring stays under a
    10% duty cycle -- with or without early stopping, as in the reference.
    Callers pass final=True at the last iteration and on a max_runtime_secs
    stop, so the history always ends at the returned model.
    time_based=False (not used by the tree builders) scores only at final."""

    def __init__(self, parms, time_based=True):
        self.interval = int(parms.get("score_tree_interval") or 0)
        self.each = bool(parms.get("score_each_iteration"))
        self.init_ms = float(parms.get("initial_score_interval") or 4000)
        self.score_ms = float(parms.get("score_interval") or 4000)
        self.time_based = time_based
        self.first = None
        self.last_start = 0.0
        self.last_end = 0.0

    def due(self, it, final=False):
        import time as _t
        now = _t.time() * 1000.0
        if self.first is None:
            self.first = now
        if self.each or final:
            return True
        if self.interval > 0:
            return it % self.interval == 0
        if not self.time_based:
            return False
        since = now - self.last_start
        return (now - self.first < self.init_ms) or \
            (since > self.score_ms and (self.last_end - self.last_start) / max(since, 1e-9) < 0.1)

    def clock_dependent(self):
        """True when due() reads the wall clock (ranks could disagree)."""
        return self.time_based and not self.each and self.interval <= 0

    def started(self):
        import time as _t
        self.last_start = _t.time() * 1000.0

    def ended(self):
        import time as _t
        self.last_end = _t.time() * 1000.0


class ScoreKeeper:
    """Early stopping on moving averages (hex/ScoreKeeper.java:278 stopEarly)."""

    # StoppingMetric(..., lowerBoundBy0, ...) (ScoreKeeper.java:133-147)
    _LOWER_BOUND_0 = frozenset(["logloss", "mse", "rmse", "mae", "rmsle", "auc", "aucpr", "misclassification",
                                "mean_per_class_error"])

    @staticmethod
    def stop_early(history, k, tol, less_is_better=True, metric=None):
        """k + 1 simple moving averages (window k) over the last 2k scoring
        events: the first is the reference, the other k the new ones.  Stop
        when the best new average improves on the reference by less than the
        relative tolerance (ratio >= 1 - tol, or <= 1 + tol for metrics where
        more is better).  Never stop on a NaN average, on averages of mixed
        sign (deviance / R^2 crossing 0) or when the best new average has
        another sign than the reference; always stop when a metric bounded
        below by 0 has a reference average of exactly 0.  `history` holds
        the scoring events after the model's initial (zero-iteration) event,
        which the reference skips."""
        n = len(history)
        if k <= 0 or n < 2 * k:
            return False
        vals = [float("nan") if v is None else float(v) for v in history]
        avgs = []
        for i in range(k + 1):
            s = n - 2 * k + i
            a = sum(vals[s:s + k]) / k
            if math.isnan(a):
                return False
            avgs.append(a)
        ref, new = avgs[0], avgs[1:]
        lo, hi = min(new), max(new)
        if metric is not None and str(metric).lower() in ScoreKeeper._LOWER_BOUND_0 and ref == 0.0:
            return True
        extreme = lo if less_is_better else hi
        if np.sign(max(avgs)) != np.sign(min(avgs)) or np.sign(extreme) != np.sign(ref):
            return False
        if ref == 0.0:
            return False                              # 0 / 0 in the reference: NaN ratio
        ratio = extreme / ref
        return ratio >= 1 - tol if less_is_better else ratio <= 1 + tol


def _encoding_wrapper(fn):
    """Route a frame-taking scoring method through the model's fitted
    categorical encoding (idempotent on already-encoded frames)."""
    import functools

    correct = fn.__name__ == "_predict_raw"

    @functools.wraps(fn)
    def w(self, frame, *a, **k):
        enc = self.__dict__.get("_catenc")
        if enc is not None and frame is not None and hasattr(frame, "_vecs"):
            frame = enc.transform(frame)
        out = fn(self, frame, *a, **k)
        prior = self.__dict__.get("_prior_class_dist")
        if correct and prior is not None and isinstance(out, torch.Tensor) and out.dim() == 2 and \
                out.shape[1] == len(prior):
            # balance_classes: back to the prior class distribution (GenModel.correctProbabilities)
            from .balance import correct_probabilities
            out = correct_probabilities(out, prior, self._model_class_dist)
        return out
    w._catenc_wrapped = True
    return w


class H2OEstimator:
    algo = "base"
    supervised_learning = True
    _defaults: dict = {}
    # methods that turn a scoring frame into model inputs: wrapped so a model
    # trained with a categorical_encoding sees encoded frames everywhere
    _ENCODED_METHODS = ("_predict_raw", "_score_matrix", "_design", "predict_leaf_node_assignment",
                        "staged_predict_proba", "predict_contributions", "_unsupervised_perf")

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        for name in cls._ENCODED_METHODS:
            fn = cls.__dict__.get(name)
            if fn is not None and callable(fn) and not getattr(fn, "_catenc_wrapped", False):
                setattr(cls, name, _encoding_wrapper(fn))

    # parameters this implementation accepts beyond the reference client's
    # table for the class (internal plumbing, aliases)
    _extra_params: tuple = ()

    @classmethod
    def _param_names(cls):
        """The estimator's parameter table: the reference client's names for
        this class (or the nearest ancestor that has one), plus _extra_params;
        None when the reference has no such estimator."""
        from .param_tables import PARAMS
        for k in cls.__mro__:
            t = PARAMS.get(k.__name__)
            if t is not None:
                return set(t) | set(cls._extra_params)
        return None

    @classmethod
    def _accepted(cls, parms):
        """`parms` without the names this estimator does not take (internal
        clones of a validated estimator carry every shared default)."""
        names = cls._param_names()
        return dict(parms) if names is None else {k: v for k, v in parms.items() if k in names}

    def _user_parms(self):
        return self._accepted(self._parms)

    def __init__(self, **kwargs):
        parms = dict(COMMON_DEFAULTS)
        parms.update(self._defaults)
        names = self._param_names()
        if names is not None:
            unknown = sorted(k for k in kwargs if k not in names)
            if unknown:
                # the reference client's estimators take no such keyword, and
                # ModelBuilder.init reports unknown fields as errors
                raise TypeError(f"{type(self).__name__}: unknown parameter(s) {unknown}")
        for k, v in kwargs.items():
            parms[k] = v
        self._parms = parms
        self._id = parms.get("model_id") or dkv.make_key(self.algo)
        self._output = {}
        self._training_metrics = None
        self._validation_metrics = None
        self._cross_validation_metrics = None
        self._cv_models = []
        self._cv_predictions = None
        self._cv_fold_assignment = None
        self._scoring_history = []
        self._spec = None
        self._run_time = 0.0
        self._start_time = 0
        self._end_time = 0

    # ------------------------------------------------------------ params
    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        p = self.__dict__.get("_parms")
        if p is not None and name in p:
            return p[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if not name.startswith("_") and "_parms" in self.__dict__ and name in self._parms:
            self._parms[name] = value
        else:
            object.__setattr__(self, name, value)

    @property
    def params(self):
        return {k: {"default": (COMMON_DEFAULTS.get(k, self._defaults.get(k))), "actual": v}
                for k, v in self._parms.items()}

    @property
    def parms(self):
        return self.params

    def get_params(self, deep=True):
        return dict(self._parms)

    def set_params(self, **p):
        self._parms.update(p)
        return self

    @property
    def model_id(self):
        return self._id

    @model_id.setter
    def model_id(self, v):
        self._id = v

    key = model_id

    @property
    def type(self):
        if not self.supervised_learning:
            return "unsupervised"
        return "classifier" if self._spec and self._spec.is_classification else "regressor"

    # ------------------------------------------------------------ training
    def _resolve_columns(self, x, y, training_frame):
        p = self._parms
        names = training_frame.names
        if y is None and self.supervised_learning:
            y = p.get("response_column")
        if isinstance(y, int):
            y = names[y]
        special = {y, p.get("weights_column"), p.get("offset_column"), p.get("fold_column")}
        ignored = set(p.get("ignored_columns") or [])
        if x is None:
            x = [n for n in names if n not in special and n not in ignored]
        else:
            x = [names[i] if isinstance(i, int) else i for i in (x if isinstance(x, (list, tuple)) else [x])]
            x = [n for n in x if n not in special]
        if p.get("ignore_const_cols", True):
            from ..ops import frame_ops
            frame_ops.rollups_many([training_frame.vec(n) for n in x])   # one batched pass on the GPU
            x = [n for n in x if not training_frame.vec(n).is_const()]
        # drop string/uuid columns (reference ignores them for most algos)
        x = [n for n in x if not training_frame.vec(n).on_host]
        return x, y

    def train(self, x=None, y=None, training_frame=None, offset_column=None, fold_column=None,
              weights_column=None, validation_frame=None, max_runtime_secs=None, ignored_columns=None,
              model_id=None, verbose=False, **kw):
        p = self._parms
        if training_frame is None:
            training_frame = p.get("training_frame")
        if isinstance(training_frame, str):
            training_frame = dkv.get(training_frame)
        if validation_frame is None:
            validation_frame = p.get("validation_frame")
        if offset_column is not None:
            p["offset_column"] = offset_column
        if fold_column is not None:
            p["fold_column"] = fold_column
        if weights_column is not None:
            p["weights_column"] = weights_column
        if max_runtime_secs is not None:
            p["max_runtime_secs"] = max_runtime_secs
        if ignored_columns is not None:
            p["ignored_columns"] = ignored_columns
        if model_id is not None:
            self._id = model_id
        x, y = self._resolve_columns(x, y, training_frame)
        p["response_column"] = y
        self._check_response(training_frame, y)
        if y is not None and self._wants_categorical_response() and training_frame.vec(y).type != T_ENUM:
            training_frame = training_frame[:, :]
            training_frame[y] = training_frame[y].asfactor()
            if validation_frame is not None and y in validation_frame.names:
                validation_frame = validation_frame[:, :]
                validation_frame[y] = validation_frame[y].asfactor()
        # balance_classes (ModelBuilder.init -> MRUtils.sampleFrameStratified)
        from . import balance as _balance
        self._prior_class_dist = self._model_class_dist = None
        if getattr(self, "_balance_hidden", False):
            # GLM.init hides the three balance parameters ("Not applicable since
            # class balancing is not required for GLM"): accepted and ignored
            pass
        else:
            if p.get("class_sampling_factors") is not None and not p.get("balance_classes"):
                raise ValueError("class_sampling_factors: class_sampling_factors requires balance_classes to be "
                                 "enabled.")
            training_frame = _balance.apply(self, training_frame, y)
        # categorical_encoding (hex/Model.java:355, FrameUtils.categoricalEncoder):
        # fitted on the training frame, kept on the model, applied to every
        # frame it scores (see _encode / __init_subclass__)
        from . import catenc as _catenc
        self._catenc = None
        enc = _catenc.for_estimator(self)
        if enc is not None:
            enc.fit(training_frame, x, y, p.get("weights_column"))
            training_frame = enc.transform(training_frame)
            if validation_frame is not None:
                validation_frame = enc.transform(validation_frame)
            x = list(enc.out_names)
            self._catenc = enc
        self._start_time = int(time.time() * 1000)
        t0 = time.time()
        from ..core import job as _jobmod
        from ..utils import log as _log
        pend = _jobmod.take_pending()
        self._job = (pend or _jobmod.Job(f"{self.algo} model build", dest=self._id,
                                         parent=_jobmod.current())).start()
        _jobmod.push(self._job)
        _log.event("model_build_start", algo=self.algo, model_id=self._id)
        spec = TrainSpec(training_frame, x, y, p.get("weights_column"), p.get("offset_column"),
                         p.get("fold_column"), validation_frame)
        self._spec = spec
        nfolds = int(p.get("nfolds") or 0)
        # max_runtime_secs bounds the WHOLE build, cross-validation included
        # (reference ModelBuilder: the CV models share the budget)
        max_rt = float(p.get("max_runtime_secs") or 0)
        self._deadline = t0 + max_rt if max_rt > 0 else None
        try:
            if nfolds > 1 or p.get("fold_column"):
                if self.supervised_learning:
                    self._cross_validate(spec)
                elif hasattr(self, "_cross_validate_unsup"):
                    # clustering CV (KMeans): holdout metrics without labels
                    self._cross_validate_unsup(spec)
            if self._deadline is not None:
                p["max_runtime_secs"] = max(1e-3, self._deadline - time.time())
            try:
                self._fit(spec)
            finally:
                if self._deadline is not None:
                    p["max_runtime_secs"] = max_rt
            self._score_all(spec)
        except Exception as e:
            self._job.fail(e)
            _log.event("model_build_failed", algo=self.algo, model_id=self._id, error=str(e))
            raise
        finally:
            _jobmod.pop(self._job)
        self._job.done()
        _log.event("model_build_done", algo=self.algo, model_id=self._id, secs=round(time.time() - t0, 3))
        self._run_time = time.time() - t0
        self._end_time = int(time.time() * 1000)
        dkv.put(self._id, self)
        if p.get("export_checkpoints_dir"):
            # ModelBuilder: every finished model is exported as a binary model into the directory
            import os as _os
            from .persist import save_model
            _os.makedirs(p["export_checkpoints_dir"], exist_ok=True)
            save_model(self, path=p["export_checkpoints_dir"], force=True)
        return self

    def _check_response(self, frame, y):
        pass

    def _tick(self, it, total, sched=None, final=False, t0=None, max_rt=0.0, msg=None, deadline=None):
        """Per-iteration control point of an iterative builder (trees, epochs,
        IRLS / Lloyd iterations): job progress + cancellation
        (water/Job.java:206 update, :isStopping), and the decisions that hang
        on one host's clock -- is a scoring round due (ScoreSchedule), has
        max_runtime_secs run out -- taken as rank 0 takes them, so every rank
        scores and stops at the same iteration and the collective sequence
        stays aligned.  Returns (score_now, timed_out)."""
        timed_out = bool(max_rt and max_rt > 0 and t0 is not None and time.time() - t0 > max_rt)
        if deadline is not None:
            timed_out = timed_out or time.time() > deadline
            max_rt = max_rt or 1.0
        score = sched.due(it, final=final or timed_out) if sched is not None else False
        job = getattr(self, "_job", None)
        dist_ = cloud.is_distributed()
        need = dist_ and (bool(max_rt and max_rt > 0) or (sched is not None and sched.clock_dependent()))
        if job is None:
            if need:
                score, timed_out = (bool(v) for v in cloud.agree([score, timed_out]))
            return score, timed_out
        vals = job.tick(it / max(total, 1), msg=msg, extra=(score, timed_out) if (need or
                                                                            (dist_ and job._spmd_any())) else ())
        if vals:
            score, timed_out = bool(vals[0]), bool(vals[1])
        return score, timed_out

    def _wants_categorical_response(self):
        """Family/distribution implies classification (reference converts the
        response to categorical, e.g. GLM binomial on a 0/1 column)."""
        fam = str(self._parms.get("family") or self._parms.get("distribution") or "").lower()
        return fam in ("binomial", "bernoulli", "multinomial", "ordinal", "quasibinomial_cls")

    def _fit(self, spec: TrainSpec):
        raise NotImplementedError

    def _predict_raw(self, frame: H2OFrame) -> torch.Tensor:
        raise NotImplementedError

    # ------------------------------------------------------------ CV
    def _fold_ids(self, spec):
        p = self._parms
        fr = spec.frame
        n_local = fr.nlocal
        if p.get("fold_column"):
            fv = fr.vec(p["fold_column"])
            f = fv.data.to(torch.int64) if fv.type == T_ENUM else fv.as_float().to(torch.int64)
            uniq = torch.unique(f)
            if cloud.is_distributed():
                uniq = torch.unique(coll.all_gather_var(uniq))
            remap = {int(u): i for i, u in enumerate(uniq.tolist())}
            f = torch.tensor([remap[int(v)] for v in f.tolist()], device=f.device) if remap else f
            return f, len(remap)
        k = int(p["nfolds"])
        fa = (p.get("fold_assignment") or "auto").lower()
        seed = p.get("seed", -1)
        seed = 42 if seed is None or seed == -1 else int(seed)
        off = fr.row_offset()
        gidx = torch.arange(off, off + n_local, device=cloud.device())
        if fa == "modulo":
            return gidx % k, k
        if fa == "stratified" and spec.is_classification:
            yv = spec.y_tensor()
            g = torch.Generator(device="cpu").manual_seed(seed)
            r = torch.rand(fr.nrows, generator=g)[off:off + n_local].to(yv.device)
            f = torch.empty(n_local, dtype=torch.int64, device=yv.device)
            for c in range(-1, spec.nclasses):
                m = yv == c
                idx = torch.nonzero(m).flatten()
                if idx.numel() == 0:
                    continue
                ordr = torch.argsort(r[idx])
                f[idx[ordr]] = torch.arange(idx.numel(), device=yv.device) % k
            return f, k
        g = torch.Generator(device="cpu").manual_seed(seed)
        r = torch.randint(0, k, (fr.nrows,), generator=g)[off:off + n_local]
        return r.to(cloud.device()), k

    def _cross_validate(self, spec):
        p = self._parms
        folds, k = self._fold_ids(spec)
        self._cv_fold_assignment = folds
        fr = spec.frame
        holdout = None
        cv_models = []
        for i in range(k):
            tr_mask = folds != i
            te_mask = folds == i
            sub = self._cv_sub(i, k)
            tr = fr[tr_mask]
            te = fr[te_mask]
            sspec = TrainSpec(tr, spec.x, spec.y, spec.weights_column, spec.offset_column, None, te)
            sspec.response_domain, sspec.nclasses = spec.response_domain, spec.nclasses
            sub._spec = sspec
            sub._fit(sspec)
            pr = sub._predict_raw(te)
            if holdout is None:
                holdout = torch.full((fr.nlocal, pr.shape[1]), float("nan"), dtype=pr.dtype, device=pr.device)
            holdout[te_mask] = pr
            sub._score_all(sspec)
            cv_models.append(sub)
        self._cv_models = cv_models if p.get("keep_cross_validation_models", True) else []
        self._cv_optimal_params(cv_models)
        self._cv_holdout = holdout
        self._cross_validation_metrics = self._metrics_from_raw(spec, fr, holdout)
        if p.get("keep_cross_validation_predictions"):
            self._cv_predictions = self._pred_frame_from_raw(holdout, spec)
        # cv summary table
        rows = {}
        for m in cv_models:
            mt = m._validation_metrics or m._training_metrics
            if mt is None:
                continue
            for kk, v in mt._m.items():
                if isinstance(v, (int, float)) and not isinstance(v, bool):
                    rows.setdefault(kk, []).append(v)
        self._output["cross_validation_metrics_summary"] = {
            kk: {"mean": float(np.mean(v)), "sd": float(np.std(v, ddof=1)) if len(v) > 1 else 0.0, "values": v}
            for kk, v in rows.items()}

    def _cv_sub(self, i, k):
        """Fold model i of k: a copy of this builder with its own id, output
        and scoring history, nfolds off, and an equal share of what is left of
        max_runtime_secs for the k - i folds and the main model."""
        sub = copy.copy(self)
        sub.__dict__ = dict(self.__dict__)
        sub._parms = dict(self._parms)
        sub._parms["nfolds"] = 0
        sub._parms["fold_column"] = None
        dl = getattr(self, "_deadline", None)
        if dl is not None:
            sub._parms["max_runtime_secs"] = max(1e-3, (dl - time.time()) / (k - i + 1))
        sub._id = f"{self._id}_cv_{i + 1}"
        sub._cv_models = []
        sub._scoring_history = []
        sub._output = {}
        return sub

    def _cv_optimal_params(self, cv_models):
        """Hook: adopt CV-derived parameters for the main model
        (reference: ModelBuilder.cv_computeAndSetOptimalParameters)."""

    # ------------------------------------------------------------ scoring
    def _metrics_from_raw(self, spec, frame, raw, w=None, auc_type=None):
        if raw is None:
            return None
        y = spec.y_tensor(frame) if spec.y and spec.y in frame.names else None
        if y is None:
            return None
        if w is None:
            w = spec.w_tensor(frame)
        dist = getattr(self, "_dist", None)
        if spec.nclasses == 2:
            yy = y.to(torch.float64)
            # NA responses (code -1) become NaN: binomial_metrics drops rows
            # with a NaN response or score itself (no boolean-mask compaction
            # and host sync per call)
            yy = torch.where(yy >= 0, yy, torch.full_like(yy, float("nan")))
            # scoring rounds (scoring history / early stopping) skip the
            # gains/lift table: only the final metrics carry it
            res = mm.binomial_metrics(yy, raw[:, -1], w, spec.response_domain,
                                      gainslift_bins=self._parms.get("gainslift_bins", -1),
                                      gainslift=not self.__dict__.get("_lite_metrics", False))
        elif spec.nclasses > 2:
            res = mm.multinomial_metrics(y, raw, w, spec.response_domain,
                                         auc_type=auc_type or self._parms.get("auc_type") or "AUTO",
                                         max_cm_size=self._parms.get("max_confusion_matrix_size"))
        else:
            res = mm.regression_metrics(y.to(torch.float64), raw[:, 0], w, dist)
        cm = self._parms.get("custom_metric_func")
        if cm is not None and res is not None:
            self._attach_custom_metric(cm, res, spec, frame, raw, y, w)
        return res

    def _attach_custom_metric(self, ref, res, spec, frame, raw, y, w):
        """custom_metric_func (water/udf/CMetricFunc): rows are [label, p0..pk-1]
        for classifiers and [prediction] for regression, like the reference."""
        from ..core.udf import custom_metric_value, metric_name
        if spec.nclasses >= 2:
            probs = raw.to(torch.float64)
            if spec.nclasses == 2:
                thr = res.find_threshold_by_max_metric("f1") if res.get("thresholds_and_metric_scores") else 0.5
                label = (probs[:, -1] >= thr).to(torch.float64)
                probs = torch.stack([1 - probs[:, -1], probs[:, -1]], 1) if probs.shape[1] == 1 else probs
            else:
                label = probs.argmax(1).to(torch.float64)
            pred = torch.cat([label.view(-1, 1), probs], 1)
            act = torch.where(y < 0, torch.full_like(y, float("nan"), dtype=torch.float64), y.to(torch.float64))
        else:
            pred = raw[:, :1].to(torch.float64)
            act = y.to(torch.float64)
        o = spec.offset_tensor(frame)
        res._m["custom_metric_name"] = metric_name(ref)
        res._m["custom_metric_value"] = custom_metric_value(ref, pred, act, w, o, self)

    def _score_all(self, spec):
        if not self.supervised_learning:
            self._score_unsupervised(spec)
            return
        raw = self._predict_raw(spec.frame)
        self._training_metrics = self._metrics_from_raw(spec, spec.frame, raw)
        if spec.valid is not None:
            vraw = self._predict_raw(spec.valid)
            self._validation_metrics = self._metrics_from_raw(spec, spec.valid, vraw)

    def _score_unsupervised(self, spec):
        pass

    def _label_threshold(self):
        """Binomial labelling threshold (Model.defaultThreshold): max-F1 of the
        validation metrics, else of the training metrics, else the output's
        default_threshold (0.5)."""
        vm, tm = self._validation_metrics, self._training_metrics
        if vm is not None and vm.get("max_f1_threshold") is not None:
            return float(vm["max_f1_threshold"])
        if tm is not None and tm.get("max_f1_threshold") is not None:
            return float(tm["max_f1_threshold"])
        return float(self._output.get("default_threshold", 0.5))

    def _pred_frame_from_raw(self, raw, spec=None, threshold=None):
        spec = spec or self._spec
        if spec.nclasses == 2:
            p1 = raw[:, -1]
            thr = threshold if threshold is not None else getattr(self, "_threshold_override", None)
            if thr is None:
                thr = self._label_threshold()
            lab = (p1 >= thr).to(torch.int32)
            lab = torch.where(torch.isnan(p1), torch.full_like(lab, -1), lab)
            vecs = [Vec(lab, T_ENUM, spec.response_domain), Vec((1 - p1).to(torch.float32), T_REAL),
                    Vec(p1.to(torch.float32), T_REAL)]
            return H2OFrame.from_vecs(vecs, scoring_names(spec.response_domain))
        if spec.nclasses > 2:
            lab = torch.argmax(raw, 1).to(torch.int32)
            vecs = [Vec(lab, T_ENUM, spec.response_domain)] + [Vec(raw[:, k].to(torch.float32).contiguous(), T_REAL)
                                                               for k in range(raw.shape[1])]
            return H2OFrame.from_vecs(vecs, scoring_names(spec.response_domain))
        return H2OFrame.from_vecs([Vec(raw[:, 0].to(torch.float32).contiguous(), T_REAL)], ["predict"])

    def predict(self, test_data, **kw):
        raw = self._predict_raw(test_data)
        fr = self._pred_frame_from_raw(raw)
        cal = getattr(self, "_calibrator", None)
        if cal is not None and self._spec is not None and self._spec.nclasses == 2:
            # reference CalibrationHelper: calibrated probabilities as extra columns
            p1 = cal(raw[:, 1]).to(torch.float32)
            fr = H2OFrame.from_vecs([fr.vec(n) for n in fr.names] + [Vec((1 - p1).contiguous(), T_REAL),
                                                                     Vec(p1.contiguous(), T_REAL)],
                                    list(fr.names) + ["cal_p0", "cal_p1"])
        return fr

    def predict_leaf_node_assignment(self, test_data, type="Path"):
        raise NotImplementedError(f"{self.algo} has no leaf node assignment")

    def model_performance(self, test_data=None, train=False, valid=False, xval=False, auc_type=None, **kw):
        if test_data is None:
            if valid:
                return self._validation_metrics
            if xval:
                return self._cross_validation_metrics
            return self._training_metrics
        if not self.supervised_learning:
            return self._unsupervised_perf(test_data)
        raw = self._predict_raw(test_data)
        return self._metrics_from_raw(self._spec, test_data, raw, auc_type=auc_type)

    def _unsupervised_perf(self, frame):
        return None

    def _pick(self, key, train, valid, xval):
        res = {}
        if not (train or valid or xval):
            train = True
        for flag, m, name in ((train, self._training_metrics, "train"), (valid, self._validation_metrics, "valid"),
                              (xval, self._cross_validation_metrics, "xval")):
            if flag:
                res[name] = None if m is None else (getattr(m, key)() if callable(getattr(m, key, None)) else m.get(key))
        return list(res.values())[0] if len(res) == 1 else res

    def auc(self, train=False, valid=False, xval=False): return self._pick("auc", train, valid, xval)
    def aucpr(self, train=False, valid=False, xval=False): return self._pick("aucpr", train, valid, xval)
    def multinomial_auc_table(self, train=False, valid=False, xval=False):
        return self._pick("multinomial_auc_table", train, valid, xval)
    def multinomial_aucpr_table(self, train=False, valid=False, xval=False):
        return self._pick("multinomial_aucpr_table", train, valid, xval)
    pr_auc = aucpr
    def logloss(self, train=False, valid=False, xval=False): return self._pick("logloss", train, valid, xval)
    def mse(self, train=False, valid=False, xval=False): return self._pick("mse", train, valid, xval)
    def rmse(self, train=False, valid=False, xval=False): return self._pick("rmse", train, valid, xval)
    def mae(self, train=False, valid=False, xval=False): return self._pick("mae", train, valid, xval)
    def rmsle(self, train=False, valid=False, xval=False): return self._pick("rmsle", train, valid, xval)
    def r2(self, train=False, valid=False, xval=False): return self._pick("r2", train, valid, xval)
    def gini(self, train=False, valid=False, xval=False): return self._pick("gini", train, valid, xval)
    def mean_per_class_error(self, train=False, valid=False, xval=False): return self._pick("mean_per_class_error", train, valid, xval)
    def mean_residual_deviance(self, train=False, valid=False, xval=False): return self._pick("mean_residual_deviance", train, valid, xval)

    # ---- ModelBase methods that only some algorithms answer (reference
    # h2o-py/h2o/model/model_base.py): the generic answer of the reference
    # client for the others -- None, a message, or the server's refusal
    def _dev_pick(self, key, train, valid, xval):
        if xval:
            raise ValueError("Cross-validation metrics are not available.")
        m = self._validation_metrics if (valid and not train) else self._training_metrics
        if m is None:
            return None
        f = getattr(m, key, None)
        return f() if callable(f) else (m.get(key) if hasattr(m, "get") else None)

    def residual_deviance(self, train=False, valid=False, xval=False):
        return self._dev_pick("residual_deviance", train, valid, xval)

    def residual_degrees_of_freedom(self, train=False, valid=False, xval=False):
        return self._dev_pick("residual_degrees_of_freedom", train, valid, xval)

    def null_deviance(self, train=False, valid=False, xval=False):
        return self._dev_pick("null_deviance", train, valid, xval)

    def null_degrees_of_freedom(self, train=False, valid=False, xval=False):
        return self._dev_pick("null_degrees_of_freedom", train, valid, xval)

    def aic(self, train=False, valid=False, xval=False):
        return self._pick("aic", train, valid, xval)

    def coef(self):
        """Coefficients (GLM family); None for models without a coefficients table."""
        return None

    def coef_norm(self):
        return None

    def coef_with_p_values(self):
        raise ValueError("p-values, z-values and std_error are only found in GLM.")

    def rotation(self):
        raise ValueError("This function is available for PCA models only")

    def deepfeatures(self, test_data, layer):
        raise ValueError(f"{self.algo}: deep features are only available for Deep Learning models")

    def weights(self, matrix_id=0):
        raise ValueError(f"{self.algo}: weight matrices are only available for Deep Learning models")

    def biases(self, vector_id=0):
        raise ValueError(f"{self.algo}: bias vectors are only available for Deep Learning models")

    def staged_predict_proba(self, test_data):
        raise ValueError(f"{self.algo}: staged predictions are only available for tree models")

    def predict_contributions(self, test_data, output_format="Original", top_n=None, bottom_n=None,
                              compare_abs=False, **kw):
        raise ValueError(f"{self.algo}: contributions (SHAP) are only available for tree models")

    def feature_frequencies(self, test_data):
        raise ValueError(f"{self.algo}: feature frequencies are only available for tree models")

    def ntrees_actual(self):
        print("No actual number of trees for this model")

    def feature_interaction(self, max_interaction_depth=100, max_tree_depth=100, max_deepening=-1, path=None):
        print("No calculation available for this model")

    def update_tree_weights(self, frame, weights_column):
        print("Only supervised tree-based models support tree-reweighting")

    def plot(self, timestep="AUTO", metric="AUTO", server=False, save_plot_path=None, **kwargs):
        """Scoring-history plot (binomial: the ROC curve with metric="roc"),
        model_base.py / models/binomial.py plot."""
        from .explain_plots import _plt
        plt = _plt()
        fig = plt.figure(figsize=(7, 5))
        if str(metric).lower() == "roc":
            roc = self.roc()
            fpr, tpr = (roc if isinstance(roc, (tuple, list)) and len(roc) == 2 else ([0, 1], [0, 1]))
            plt.plot(fpr, tpr)
            plt.xlabel("False Positive Rate")
            plt.ylabel("True Positive Rate")
            plt.title(f"ROC curve for {self.model_id}")
        else:
            sh = self.scoring_history()
            if sh is not None and len(sh):
                num = [c for c in sh.columns if c.startswith("training_") or c.startswith("validation_")]
                want = str(metric).lower()
                cols = [c for c in num if want == "auto" or want in c.lower()][:4]
                xcol = next((c for c in ("number_of_trees", "iterations", "epochs", "iteration") if c in sh.columns),
                            None)
                xs = sh[xcol] if xcol else range(len(sh))
                for c in cols:
                    plt.plot(xs, sh[c], label=c)
                plt.legend()
                plt.xlabel(xcol or "scoring event")
            plt.title(f"Scoring History for {self.model_id}")
        if save_plot_path is not None:
            fig.savefig(save_plot_path)
        return fig

    def gains_lift_plot(self, type="both", server=False, save_plot_path=None, **kwargs):
        """Cumulative gains / lift of a binomial model (models/binomial.py)."""
        from .explain_plots import _plt
        plt = _plt()
        gl = self.gains_lift()
        fig = plt.figure(figsize=(7, 5))
        if gl is not None:
            import pandas as pd
            t = gl if isinstance(gl, pd.DataFrame) else pd.DataFrame(gl)
            x = t["cumulative_data_fraction"] if "cumulative_data_fraction" in t else range(len(t))
            if type in ("both", "gains") and "cumulative_capture_rate" in t:
                plt.plot(x, t["cumulative_capture_rate"], label="cumulative gains")
            if type in ("both", "lift") and "cumulative_lift" in t:
                plt.plot(x, t["cumulative_lift"], label="cumulative lift")
            plt.legend()
            plt.xlabel("cumulative data fraction")
        plt.title(f"Gains / Lift for {self.model_id}")
        if save_plot_path is not None:
            fig.savefig(save_plot_path)
        return fig
    def confusion_matrix(self, train=False, valid=False, xval=False, **kw): return self._pick("confusion_matrix", train, valid, xval)

    # ---- threshold metrics of binomial models (h2o-py model/models/binomial.py);
    # several of train/valid/xval -> dict keyed by "train"/"valid"/"xval"
    def _thr_metric(self, name, thresholds=None, train=False, valid=False, xval=False, **kw):
        picks = [(k, getattr(self, a)) for k, a, f in (("train", "_training_metrics", train),
                                                        ("valid", "_validation_metrics", valid),
                                                        ("xval", "_cross_validation_metrics", xval)) if f]
        if not picks:
            picks = [("train", self._training_metrics)]
        out = {}
        for k, m in picks:
            fn = getattr(m, name, None) if m is not None else None
            out[k] = None if fn is None else (fn(thresholds, **kw) if thresholds is not None or kw else fn())
        return out[picks[0][0]] if len(out) == 1 else out

    def F1(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("F1", thresholds, train, valid, xval)
    def F2(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("F2", thresholds, train, valid, xval)
    def F0point5(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("F0point5", thresholds, train, valid, xval)
    def accuracy(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("accuracy", thresholds, train, valid, xval)
    def error(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("error", thresholds, train, valid, xval)
    def precision(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("precision", thresholds, train, valid, xval)
    def recall(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("recall", thresholds, train, valid, xval)
    def sensitivity(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("recall", thresholds, train, valid, xval)
    def tpr(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("tpr", thresholds, train, valid, xval)
    def tnr(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("tnr", thresholds, train, valid, xval)
    def fnr(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("fnr", thresholds, train, valid, xval)
    def fpr(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("fpr", thresholds, train, valid, xval)
    def fallout(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("fpr", thresholds, train, valid, xval)
    def missrate(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("fnr", thresholds, train, valid, xval)
    def specificity(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("specificity", thresholds, train, valid, xval)
    def mcc(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("mcc", thresholds, train, valid, xval)
    def max_per_class_error(self, thresholds=None, train=False, valid=False, xval=False): return self._thr_metric("max_per_class_error", thresholds, train, valid, xval)

    def metric(self, metric, thresholds=None, train=False, valid=False, xval=False):
        return self._pick_metrics(train, valid, xval).metric(metric, thresholds)

    def _pick_metrics(self, train=False, valid=False, xval=False):
        if xval:
            return self._cross_validation_metrics
        if valid:
            return self._validation_metrics
        return self._training_metrics

    def roc(self, train=False, valid=False, xval=False):
        return self._pick_metrics(train, valid, xval).roc()

    def gains_lift(self, train=False, valid=False, xval=False):
        return self._pick_metrics(train, valid, xval).gains_lift()

    def kolmogorov_smirnov(self):
        return self._training_metrics.kolmogorov_smirnov()

    def find_threshold_by_max_metric(self, metric, train=False, valid=False, xval=False):
        return self._pick_metrics(train, valid, xval).find_threshold_by_max_metric(metric)

    def find_idx_by_threshold(self, threshold, train=False, valid=False, xval=False):
        return self._pick_metrics(train, valid, xval).find_idx_by_threshold(threshold)

    def hit_ratio_table(self, train=False, valid=False, xval=False):
        return self._pick_metrics(train, valid, xval).hit_ratio_table()

    def training_model_metrics(self):
        return self._training_metrics.as_dict() if self._training_metrics is not None else None

    # ---- DataInfo normalization (model_base.py normmul/normsub/respmul/respsub/catoffsets)
    def _di(self):
        di = getattr(self, "_dinfo", None)
        if di is None:
            raise AttributeError("this model has no design-matrix normalization (no DataInfo)")
        return di

    def normmul(self):
        di = self._di()
        return [1.0 / s for s in di.sigmas] if di.standardize else None

    def normsub(self):
        di = self._di()
        return list(di.means) if di.standardize else None

    def respmul(self):
        sd = getattr(self, "_ysd", None)
        return None if sd is None else 1.0 / sd

    def respsub(self):
        return getattr(self, "_ymu", None)

    def catoffsets(self):
        di = self._di()
        offs, acc = [0], 0
        for c in di.cat_cols:
            acc += len(di.domains[c]) - (0 if di.use_all else 1)
            offs.append(acc)
        return offs

    def pprint_coef(self):
        coefs = getattr(self, "coef", None)
        if coefs is None:
            print("No coefficients for this model")
            return
        c = coefs()
        for k, v in sorted(c.items(), key=lambda kv: -abs(kv[1])):
            print(f"{k:>30s} {v: .6g}")

    def predicted_vs_actual_by_variable(self, frame, predicted, variable, use_pandas=False):
        """Per-level weighted means of prediction and actual for a categorical
        variable (water/rapids/prims/AstPredictedVsActualByVar.java); the last
        row is the NA level."""
        import pandas as pd
        if not self.supervised_learning:
            raise ValueError("Only supervised models are supported for calculating predicted v actual")
        if self._spec.nclasses > 2:
            raise ValueError("Multinomial classification models are not supported by predicted v actual")
        if frame.nrows != predicted.nrows:
            raise ValueError("Input frame and frame of predictions need to have same number of rows.")
        v = frame.vec(variable)
        if v.type != T_ENUM:
            raise ValueError(f"'{variable}' is not categorical")
        L = len(v.domain)
        level = torch.where(v.data < 0, torch.full_like(v.data, L), v.data).long()
        pv = predicted.vec(predicted.names[0])
        pr = pv.data.to(torch.float64) if pv.type == T_ENUM else pv.as_float(torch.float64)
        act = self._spec.y_tensor(frame).to(torch.float64)
        ok = act >= 0 if self._spec.is_classification else ~torch.isnan(act)
        w = self._spec.w_tensor(frame)
        w = torch.ones_like(act) if w is None else w.to(torch.float64)
        w = torch.where(ok, w, torch.zeros_like(w))
        from ..core.groupsum import group_sum
        st = group_sum(level, torch.stack([w * torch.where(ok, pr, torch.zeros_like(pr)),
                                           w * torch.where(ok, act, torch.zeros_like(act)), w], 1),
                       L + 1).T.contiguous()
        coll.allreduce_(st)
        den = torch.where(st[2] > 0, st[2], torch.ones_like(st[2]))
        res = (st[:2] / den).cpu().numpy()
        df = pd.DataFrame({variable: list(v.domain) + [None], predicted.names[0]: res[0], "actual": res[1]})
        return df.set_index(variable) if use_pandas else df

    # ---- explanation plots (h2o-py ModelBase.pd_plot / ice_plot / shap_* / ...)
    def pd_plot(self, frame, column, **kw):
        from .explain_plots import pd_plot
        return pd_plot(self, frame, column, **kw)

    def ice_plot(self, frame, column, **kw):
        from .explain_plots import ice_plot
        return ice_plot(self, frame, column, **kw)

    def shap_summary_plot(self, frame, **kw):
        from .explain_plots import shap_summary_plot
        return shap_summary_plot(self, frame, **kw)

    def shap_explain_row_plot(self, frame, row_index, **kw):
        from .explain_plots import shap_explain_row_plot
        return shap_explain_row_plot(self, frame, row_index, **kw)

    def residual_analysis_plot(self, frame, **kw):
        from .explain_plots import residual_analysis_plot
        return residual_analysis_plot(self, frame, **kw)

    def learning_curve_plot(self, metric="AUTO", **kw):
        from .explain_plots import learning_curve_plot
        return learning_curve_plot(self, metric, **kw)

    def explain(self, frame, **kw):
        from .explain import explain
        return explain([self], frame, **kw)

    def explain_row(self, frame, row_index, **kw):
        from .explain import explain_row
        return explain_row([self], frame, row_index, **kw)

    def _plot_or_data(self, kind, data, server=False):
        """Plots need matplotlib; without it (this image) the plot's data is
        returned so callers still get the numbers."""
        try:
            import matplotlib  # noqa: F401
        except ImportError:
            import warnings
            warnings.warn(f"matplotlib is not installed: {kind} returns its data instead of a figure")
            return data
        import matplotlib
        if server:
            matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        fig, ax = plt.subplots()
        names, vals = zip(*data) if data else ((), ())
        ax.barh(list(names)[::-1], list(vals)[::-1])
        ax.set_title(kind)
        if not server:
            plt.show()
        return fig

    def varimp_plot(self, num_of_features=None, server=False, save_plot_path=None):
        vi = self.varimp()
        if vi is None:
            return None
        rows = [(r[0], r[2]) for r in vi] if isinstance(vi, list) and vi and isinstance(vi[0], (tuple, list)) \
            else sorted(((k, v) for k, v in dict(vi).items()), key=lambda kv: -kv[1])
        return self._plot_or_data("Variable Importance", rows[:num_of_features or 10], server)

    def std_coef_plot(self, num_of_features=None, server=False, save_plot_path=None):
        cn = getattr(self, "coef_norm", None)
        if cn is None:
            raise AttributeError("std_coef_plot needs a model with standardized coefficients")
        rows = sorted(((k, abs(v)) for k, v in cn().items() if k != "Intercept"), key=lambda kv: -kv[1])
        return self._plot_or_data("Standardized Coef. Magnitudes", rows[:num_of_features or 10], server)

    def permutation_importance_plot(self, frame, metric="AUTO", n_samples=10000, n_repeats=1, features=None,
                                    seed=-1, num_of_features=10, server=False, save_plot_path=None):
        from .explain import permutation_importance
        pi = permutation_importance(self, frame, metric=metric, n_samples=n_samples, n_repeats=n_repeats,
                                    features=features, seed=seed)
        if hasattr(pi, "columns") and "Relative Importance" in pi.columns:
            rows = list(zip(pi["Variable"], pi["Relative Importance"]))
        else:
            rows = list(zip(pi.iloc[:, 0], pi.iloc[:, 1:].mean(1))) if hasattr(pi, "iloc") else list(pi)
        return self._plot_or_data("Permutation Variable Importance", rows[:num_of_features], server)

    # ---- model bookkeeping (h2o-py model_base.py)
    @property
    def start_time(self):
        return self._start_time

    @property
    def end_time(self):
        return self._end_time

    @property
    def run_time(self):
        return int(self._run_time * 1000)

    @property
    def full_parameters(self):
        return self.params

    @property
    def default_params(self):
        return {k: v["default"] for k, v in self.params.items()}

    @property
    def have_mojo(self):
        from ..mojo import writer
        try:
            writer.build_mojo(self)
            return True
        except Exception:
            return False

    @property
    def have_pojo(self):
        try:
            from ..mojo.pojo import to_java
            to_java(self)
            return True
        except Exception:
            return False

    def download_model(self, path="", filename=None, **kw):
        from .persist import save_model
        return save_model(self, path or ".", force=True, filename=filename)

    def score_history(self):
        return self.scoring_history()

    def xval_keys(self):
        return [m.model_id for m in self._cv_models]

    def xvals(self):
        return list(self._cv_models)

    def get_summary(self):
        return self._output.get("model_summary")

    def show_summary(self):
        print(self._output.get("model_summary"))

    def detach(self):
        dkv.remove(self.model_id)

    def scoring_history(self):
        import pandas as pd
        return pd.DataFrame(self._scoring_history)

    def varimp(self, use_pandas=False):
        vi = self._output.get("variable_importances")
        if vi is None:
            return None
        rows = sorted(vi.items(), key=lambda kv: -kv[1])
        top = rows[0][1] if rows and rows[0][1] > 0 else 1.0
        tot = sum(v for _, v in rows) or 1.0
        out = [(k, float(v), float(v / top), float(v / tot)) for k, v in rows]
        if use_pandas:
            import pandas as pd
            return pd.DataFrame(out, columns=["variable", "relative_importance", "scaled_importance", "percentage"])
        return out

    def summary(self):
        return self._output.get("model_summary")

    def cross_validation_models(self):
        return self._cv_models

    def cross_validation_predictions(self):
        return [m.predict(self._spec.frame) for m in self._cv_models]

    def cross_validation_holdout_predictions(self):
        return self._cv_predictions if self._cv_predictions is not None else (
            self._pred_frame_from_raw(self._cv_holdout) if getattr(self, "_cv_holdout", None) is not None else None)

    def cross_validation_fold_assignment(self):
        if not self._parms.get("keep_cross_validation_fold_assignment"):
            return None          # kept only when asked (ModelBuilder cv_computeAndSetOptimalParameters)
        f = self._cv_fold_assignment
        return None if f is None else H2OFrame.from_vecs([Vec(f.to(torch.float32), T_INT)], ["fold_assignment"])

    def cross_validation_metrics_summary(self):
        return self._output.get("cross_validation_metrics_summary")

    @property
    def actual_params(self):
        """Parameters the model was built with, auto values resolved
        (model_base.py actual_params: {name: actual value})."""
        return {k: v["actual"] for k, v in self.params.items()}

    @property
    def actual_params_(self):
        return dict(self._parms)

    def get_xval_models(self):
        return self._cv_models

    def is_cross_validated(self):
        return bool(self._cv_models)

    def show(self):
        print(repr(self))

    def __repr__(self):
        s = f"{type(self).__name__} model_id={self._id}"
        if self._training_metrics is not None:
            s += f"\n  training: {self._training_metrics!r}"
        if self._validation_metrics is not None:
            s += f"\n  validation: {self._validation_metrics!r}"
        if self._cross_validation_metrics is not None:
            s += f"\n  xval: {self._cross_validation_metrics!r}"
        return s

    # ------------------------------------------------------------ persistence
    def train_segments(self, x=None, y=None, training_frame=None, offset_column=None, weights_column=None,
                       validation_frame=None, max_runtime_secs=None, segments=None, segment_models_id=None,
                       parallelism=1, verbose=False):
        from .segments import train_segments
        kw = {}
        if weights_column is not None:
            kw["weights_column"] = weights_column
        if offset_column is not None:
            kw["offset_column"] = offset_column
        # `segments`: list of column names to group by, or an explicit
        # enumeration (frame / list of dicts) of the segments to build
        if isinstance(segments, str) or (isinstance(segments, (list, tuple)) and segments and
                                         all(isinstance(c, str) for c in segments)):
            seg_cols, enum = [segments] if isinstance(segments, str) else list(segments), None
        else:
            import pandas as pd
            from ..core.frame import H2OFrame as _F
            enum = segments.as_data_frame() if isinstance(segments, _F) else pd.DataFrame(segments)
            seg_cols = list(enum.columns)
        return train_segments(self, x=x, y=y, training_frame=training_frame, segment_columns=seg_cols,
                              segments=enum, segment_models_id=segment_models_id, parallelism=parallelism,
                              verbose=verbose, **kw)

    # ---------------------------------------------------------------- explain
    def partial_plot(self, data, cols=None, destination_key=None, nbins=20, weight_column=None, plot=False,
                     plot_stddev=True, figsize=None, server=False, include_na=False, user_splits=None,
                     col_pairs_2dpdp=None, save_to_file=None, row_index=None, targets=None, **kw):
        from .explain import partial_dependence
        return partial_dependence(self, data, cols or [], nbins=nbins, weight_column=weight_column,
                                  include_na=include_na, user_splits=user_splits, targets=targets,
                                  row_index=row_index)

    def permutation_importance(self, frame, metric="AUTO", n_samples=10000, n_repeats=1, features=None, seed=-1,
                               use_pandas=True):
        from .explain import permutation_importance
        return permutation_importance(self, frame, metric, n_samples, n_repeats, features, seed)

    def h(self, frame, variables):
        from .explain import h_statistic
        return h_statistic(self, frame, variables)

    def explain(self, frame, **kw):
        from .explain import explain
        return explain(self, frame, **kw)

    def explain_row(self, frame, row_index, **kw):
        from .explain import explain_row
        return explain_row(self, frame, row_index, **kw)

    def download_pojo(self, path="", get_genmodel_jar=False, genmodel_name=""):
        """Java POJO scoring source (mojo/pojo.py); prints it when path is ""."""
        from ..mojo.pojo import download_pojo
        return download_pojo(self, path)

    def download_mojo(self, path=".", get_genmodel_jar=False, genmodel_name="", format="native", **kw):
        """Write the model's MOJO zip.  format="native": this platform's layout
        (every algorithm, numpy scorer in mojo/genmodel.py); format="h2o": the
        reference's h2o-genmodel layout (GBM / DRF / GLM), readable by the
        reference's Java MojoModel and by mojo/h2o_mojo.py."""
        from ..mojo import writer
        if format == "h2o":
            import os as _os
            from ..mojo.h2o_writer import build_h2o_mojo
            data = build_h2o_mojo(self)
            if _os.path.isdir(path) or not path.endswith(".zip"):
                _os.makedirs(path, exist_ok=True)
                path = _os.path.join(path, f"{self.model_id}.zip")
            with open(path, "wb") as f:
                f.write(data)
            return path
        return writer.write_mojo(self, path)

    save_mojo = download_mojo

    def save_model_details(self, path=".", force=False, filename=None):
        fn = os.path.join(path, filename or f"{self._id}.json")
        with open(fn, "w") as f:
            json.dump({"model_id": self._id, "algo": self.algo, "params": {k: v for k, v in self._parms.items()
                                                                             if isinstance(v, (int, float, str, bool, list, type(None)))}},
                      f, indent=1, default=str)
        return fn

    # ------------------------------------------------------------ frame adaptation
    def _adapt_enum(self, frame_vec: Vec, train_domain):
        """Map a test categorical column onto the training domain (unseen -> NA)
        (reference: Model.adaptTestForTrain)."""
        if frame_vec.type == T_ENUM:
            if frame_vec.domain == train_domain:
                return frame_vec.data
            idx = {d: i for i, d in enumerate(train_domain)}
            remap = torch.tensor([idx.get(d, -1) for d in frame_vec.domain] or [-1], dtype=torch.int32,
                                 device=frame_vec.data.device)
            return torch.where(frame_vec.data < 0, frame_vec.data, remap[frame_vec.data.clamp(min=0).long()])
        if frame_vec.on_host:
            idx = {d: i for i, d in enumerate(train_domain)}
            return torch.tensor([idx.get(str(x), -1) if x is not None else -1 for x in frame_vec.data],
                                dtype=torch.int32, device=cloud.device())
        # numeric column where training saw a categorical: match by label
        x = frame_vec.as_float(torch.float64)
        idx = {}
        for i, d in enumerate(train_domain):
            try:
                idx[float(d)] = i
            except ValueError:
                pass
        keys = torch.tensor(sorted(idx), dtype=torch.float64, device=x.device) if idx else None
        if keys is None:
            return torch.full(x.shape, -1, dtype=torch.int32, device=x.device)
        vals = torch.tensor([idx[k] for k in sorted(idx)], dtype=torch.int32, device=x.device)
        pos = torch.searchsorted(keys, torch.nan_to_num(x, nan=-1e308)).clamp(max=keys.numel() - 1)
        hit = keys[pos] == x
        return torch.where(hit, vals[pos], torch.full_like(vals[pos], -1))
