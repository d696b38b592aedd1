"""AutoML.

Reference: h2o-automl (ai/h2o/automl/AutoML.java, ModelingPlans.java,
modeling/*StepsProvider.java, preprocessing/TargetEncoding.java,
leaderboard/*, events/EventLog.java, hex/faulttolerance/Recovery.java).

The run is a *modeling plan*: an ordered list of (algo, step) definitions,
each step is a default model ("def_N"), a random grid ("grid_N") or an
exploitation step on the best model so far ("lr_annealing" / "lr_search"),
followed by Stacked Ensembles ("best_of_family", "all").  The default plan is
the reference's ONE_LAYERED plan (ModelingPlans.java); a user plan uses the
same syntax as h2o-py (`["GBM", ("XGBoost", "defaults"), {"name": "DRF",
"steps": [{"id": "XRT"}]}]`, aliases "all" / "defaults" / "grids").

All models are cross-validated with shared Modulo folds (nfolds default 5),
so the SEs can blend their holdout predictions; with nfolds=0 and no
validation frame, 10% of the training rows are held out for early stopping
(AutoML.java `splitTrainingFrame`).  Budgets: max_models (base models),
max_runtime_secs (whole run), max_runtime_secs_per_model.  With recovery_dir
the frames, the plan position and every finished model are written as the run
progresses, so `h2o.resume(recovery_dir)` continues an interrupted run.
"""
from __future__ import annotations

import json
import math
import os
import time
import zlib

import numpy as np

from ..core import dkv
from ..core.frame import H2OFrame
from .leaderboard import Leaderboard

_ALGOS = ["XGBoost", "GLM", "DRF", "GBM", "DeepLearning", "StackedEnsemble"]

# ONE_LAYERED default plan (ModelingPlans.java)
_DEFAULT_PLAN = [("XGBoost", "defaults"), ("GLM", "defaults"), ("DRF", "def_1"), ("GBM", "defaults"),
                 ("DeepLearning", "defaults"), ("DRF", "XRT"), ("XGBoost", "grid_1"), ("GBM", "grid_1"),
                 ("DeepLearning", "grid_1"), ("DeepLearning", "grid_2"), ("DeepLearning", "grid_3"),
                 ("GBM", "lr_annealing"), ("XGBoost", "lr_search"),
                 ("StackedEnsemble", "best_of_family"), ("StackedEnsemble", "all")]

_DEFAULT_STEPS = {"XGBoost": ["def_2", "def_1", "def_3"], "GLM": ["def_1"], "DRF": ["def_1", "XRT"],
                  "GBM": ["def_5", "def_2", "def_3", "def_4", "def_1"], "DeepLearning": ["def_1"],
                  "StackedEnsemble": ["best_of_family", "all"]}
_GRID_STEPS = {"XGBoost": ["grid_1"], "GBM": ["grid_1"], "DeepLearning": ["grid_1", "grid_2", "grid_3"]}
_EXPLOIT_STEPS = {"GBM": ["lr_annealing"], "XGBoost": ["lr_search"]}

_MAX_TREES = 10000  # reference: ntrees=10000, early stopping decides


def _work(algo, step):
    """(priority group, weight) of a plan step (ModelingStep.java:505 / 575:
    default models weigh 10, grids 30; WorkAllocations.remainingWorkRatio)."""
    if algo == "StackedEnsemble":
        return "se", 10
    if step.startswith("grid"):
        return "grid", 30
    if step in ("lr_annealing", "lr_search"):
        return "exploit", 10
    return "default", 10


def _estimators():
    from .. import estimators as E
    return {"XGBoost": E.H2OXGBoostEstimator, "GLM": E.H2OGeneralizedLinearEstimator,
            "DRF": E.H2ORandomForestEstimator, "GBM": E.H2OGradientBoostingEstimator,
            "DeepLearning": E.H2ODeepLearningEstimator}


def _step_params(algo, step):
    """Fixed parameters of the default model steps (modeling/*StepsProvider.java)."""
    tree_es = dict(ntrees=_MAX_TREES, score_tree_interval=5)
    if algo == "GBM":
        base = dict(sample_rate=0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8, **tree_es)
        depth, rows = {"def_1": (6, 1), "def_2": (7, 10), "def_3": (8, 10), "def_4": (10, 10),
                       "def_5": (15, 100)}[step]
        return dict(base, max_depth=depth, min_rows=rows)
    if algo == "XGBoost":
        depth, rows, sr = {"def_1": (10, 5, 0.6), "def_2": (15, 10, 0.6), "def_3": (5, 3, 0.8)}[step]
        return dict(tree_es, max_depth=depth, min_rows=rows, sample_rate=sr, col_sample_rate=0.8,
                    col_sample_rate_per_tree=0.8)
    if algo == "DRF":
        p = dict(ntrees=_MAX_TREES, score_tree_interval=5)
        if step == "XRT":
            p["histogram_type"] = "Random"
        return p
    if algo == "GLM":
        return dict(lambda_search=True, alpha=[0.0, 0.2, 0.4, 0.6, 0.8, 1.0])
    if algo == "DeepLearning":
        return dict(epochs=10, hidden=[10, 10, 10], adaptive_rate=True)
    raise KeyError(step)


def _grid_space(algo, step, classification):
    """Random-discrete hyper spaces of the grid steps."""
    if algo == "GBM":
        return dict(fixed=dict(ntrees=_MAX_TREES, score_tree_interval=5),
                    space=dict(max_depth=list(range(3, 18)), min_rows=[1, 5, 10, 15, 30, 100],
                               sample_rate=[0.5, 0.6, 0.7, 0.8, 0.9, 1.0], col_sample_rate=[0.4, 0.7, 1.0],
                               col_sample_rate_per_tree=[0.4, 0.7, 1.0], min_split_improvement=[1e-4, 1e-5]))
    if algo == "XGBoost":
        return dict(fixed=dict(ntrees=_MAX_TREES, score_tree_interval=5),
                    space=dict(max_depth=[3, 6, 9, 12, 15], min_rows=[0.01, 0.1, 1.0, 3.0, 5.0, 10.0, 15.0, 20.0],
                               sample_rate=[0.6, 0.8, 1.0], col_sample_rate=[0.6, 0.8, 1.0],
                               col_sample_rate_per_tree=[0.7, 0.8, 0.9, 1.0], booster=["gbtree", "dart"],
                               reg_lambda=[0.001, 0.01, 0.1, 1.0, 10.0, 100.0],
                               reg_alpha=[0.001, 0.01, 0.1, 0.5, 1.0]))
    if algo == "DeepLearning":
        hidden = {"grid_1": [[20], [50], [100]], "grid_2": [[20, 20], [50, 50], [100, 100]],
                  "grid_3": [[20, 20, 20], [50, 50, 50], [100, 100, 100]]}[step]
        ndrop = len(hidden[0])
        drops = [[r] * ndrop for r in (0.0, 0.1, 0.2, 0.3, 0.4, 0.5)]
        return dict(fixed=dict(epochs=10, adaptive_rate=True, activation="RectifierWithDropout"),
                    space=dict(hidden=hidden, hidden_dropout_ratios=drops, rho=[0.9, 0.95, 0.99],
                               epsilon=[1e-6, 1e-7, 1e-8, 1e-9], input_dropout_ratio=[0.0, 0.05, 0.1, 0.15, 0.2]))
    raise KeyError((algo, step))


def _expand_plan(plan):
    """Normalise a modeling plan to a list of (algo, step_id)."""
    out = []
    for item in plan:
        if isinstance(item, str):
            algo, spec = item, "all"
        elif isinstance(item, dict):
            algo = item["name"]
            spec = item.get("alias") or [s["id"] if isinstance(s, dict) else s for s in item.get("steps", [])] or "all"
        else:
            algo, spec = item[0], (item[1] if len(item) > 1 else "all")
        algo = {a.lower(): a for a in _ALGOS}.get(str(algo).lower(), algo)
        if isinstance(spec, str) and spec in ("all", "defaults", "grids", "exploitation"):
            steps = []
            if spec in ("all", "defaults"):
                steps += _DEFAULT_STEPS.get(algo, [])
            if spec in ("all", "grids"):
                steps += _GRID_STEPS.get(algo, [])
            if spec in ("all", "exploitation"):
                steps += _EXPLOIT_STEPS.get(algo, [])
        elif isinstance(spec, str):
            steps = [spec]
        else:
            steps = list(spec)
        for s in steps:
            if s == "defaults":
                out += [(algo, d) for d in _DEFAULT_STEPS.get(algo, [])]
            else:
                out.append((algo, s))
    return out


class H2OAutoML:
    def __init__(self, nfolds=-1, balance_classes=False, class_sampling_factors=None, max_after_balance_size=5.0,
                 max_runtime_secs=None, max_runtime_secs_per_model=None, max_models=None, distribution="AUTO",
                 stopping_metric="AUTO", stopping_tolerance=None, stopping_rounds=3, seed=None, project_name=None,
                 exclude_algos=None, include_algos=None, exploitation_ratio=-1, modeling_plan=None,
                 preprocessing=None, monotone_constraints=None, keep_cross_validation_predictions=False,
                 keep_cross_validation_models=False, keep_cross_validation_fold_assignment=False,
                 sort_metric="AUTO", export_checkpoints_dir=None, verbosity="warn", recovery_dir=None,
                 grid_models_per_step=None, **kw):
        self.nfolds = 5 if nfolds in (-1, None) else int(nfolds)
        self.max_runtime_secs = max_runtime_secs if max_runtime_secs not in (None, 0) else (None if max_models else 3600)
        self.max_runtime_secs_per_model = max_runtime_secs_per_model
        self.max_models = max_models
        self.stopping_metric = stopping_metric
        self.stopping_tolerance = stopping_tolerance
        self.stopping_rounds = stopping_rounds
        self.seed = seed if seed is not None else -1
        self.project_name = project_name or dkv.make_key("AutoML")
        self.exclude_algos = [a.lower() for a in (exclude_algos or [])]
        self.include_algos = [a.lower() for a in include_algos] if include_algos else None
        self.sort_metric = sort_metric
        self.balance_classes = balance_classes
        self.class_sampling_factors = class_sampling_factors
        self.max_after_balance_size = max_after_balance_size
        self.distribution = distribution
        self.monotone_constraints = monotone_constraints
        self.keep_cross_validation_predictions = keep_cross_validation_predictions
        self.keep_cross_validation_models = keep_cross_validation_models
        self.keep_cross_validation_fold_assignment = keep_cross_validation_fold_assignment
        self.exploitation_ratio = exploitation_ratio
        self.modeling_plan = modeling_plan
        self.preprocessing = preprocessing
        self.export_checkpoints_dir = export_checkpoints_dir
        self.recovery_dir = recovery_dir
        self.grid_models_per_step = grid_models_per_step
        self.verbosity = verbosity
        prev = dkv.get(self.project_name)
        # reference: training again under the same project_name extends the leaderboard
        self.models = list(prev.models) if isinstance(prev, H2OAutoML) else []
        self.event_log_rows = list(prev.event_log_rows) if isinstance(prev, H2OAutoML) else []
        self._leaderboard = None
        self.training_info = {}
        self._done_steps = []
        self._te = None
        self._t0 = time.time()

    # ------------------------------------------------------------------ helpers
    _VERB = {"debug": 0, "info": 1, "warn": 2, "warning": 2, "error": 3}

    def _log(self, stage, msg, level="Info"):
        self.event_log_rows.append({"timestamp": time.strftime("%H:%M:%S"), "level": level, "stage": stage,
                                    "message": msg})
        # the reference client prints the event log at or above `verbosity`
        v = self._VERB.get(str(self.verbosity or "warn").lower(), 2)
        if self.verbosity is not None and self._VERB.get(str(level).lower(), 1) >= v:
            print(f"{time.strftime('%H:%M:%S')}: {msg}", flush=True)

    def _allowed(self, algo):
        a = algo.lower()
        if self.include_algos is not None:
            return a in self.include_algos
        return a not in self.exclude_algos

    def _n_base(self):
        return len([m for m in self.models if m.algo != "stackedensemble"])

    def _budget_left(self):
        if self.max_models and self._n_base() >= self.max_models:
            return False
        out = True
        if self.max_runtime_secs and time.time() - self._t0 > self.max_runtime_secs:
            out = False
        dl = getattr(self, "_step_deadline", None)
        if dl is not None and time.time() > dl:
            out = False       # this grid step's share of the budget is spent
        # the clock is rank 0's (every rank must start the same models), and a
        # REST cancel of the AutoML job stops here between models
        from ..core import job as jobmod
        from ..parallel import cloud
        j = jobmod.current()
        clocked = bool(self.max_runtime_secs) or dl is not None
        if j is not None:
            prog = (self._n_base() / self.max_models) if self.max_models else \
                ((time.time() - self._t0) / self.max_runtime_secs if self.max_runtime_secs else 0.0)
            out = bool(j.tick(min(prog, 0.99), extra=(out,) if clocked else ())[0]) if clocked else \
                (j.tick(min(prog, 0.99)) or out)
        elif clocked and cloud.is_distributed():
            out = bool(cloud.agree([out])[0])
        return out

    def _set_stopping_tolerance(self, frame):
        """AutoML.java:357: an unset stopping tolerance adapts to the training
        frame, min(0.05, max(0.001, 1 / sqrt((1 - NA fraction) * nrows)))
        (HyperSpaceSearchCriteria.default_stopping_tolerance_for_frame); a user
        value under 70% of that default draws a warning."""
        n = int(frame.nrows)
        ncols = max(1, len(frame.names))
        na = 0
        for c in frame.names:
            try:
                na += int(frame.vec(c).nacnt())
            except Exception:
                pass
        naf = min(1.0, na / max(1, n * ncols))
        dflt = min(0.05, max(0.001, 1.0 / math.sqrt(max(1e-12, (1 - naf) * max(n, 1)))))
        if self.stopping_tolerance in (None, -1, "AUTO"):
            self.stopping_tolerance = dflt
            self._log("Validation", f"Setting stopping tolerance adaptively based on the training frame: {dflt}")
        else:
            self._log("Validation", f"Stopping tolerance set by the user: {self.stopping_tolerance}")
            if float(self.stopping_tolerance) < 0.7 * dflt:
                self._log("Validation", f"Stopping tolerance set by the user is < 70% of the recommended default of "
                                        f"{dflt}, so models may take a long time to converge or may not converge "
                                        f"at all.", level="Warn")

    def _assign_step_time(self, item, pending):
        """Time share of one step (ModelingStep.java:550): remaining budget x
        its weight / the remaining weight of the steps in its priority group
        plus the Stacked Ensembles, so one slow early model (e.g. a DRF
        running to early stopping) cannot eat the whole budget."""
        self._step_deadline = None
        if not self.max_runtime_secs or item[0] == "StackedEnsemble":
            return
        left = self.max_runtime_secs - (time.time() - self._t0)
        grp, w = _work(*item)
        rem = sum(_work(*it)[1] for it in pending if _work(*it)[0] in (grp, "se"))
        self._step_deadline = time.time() + max(1.0, left * w / max(rem, w))

    def _seed(self):
        return self.seed if self.seed not in (None, -1) else 42

    def _common(self, algo):
        c = dict(nfolds=self.nfolds, keep_cross_validation_predictions=True,
                 keep_cross_validation_models=self.keep_cross_validation_models,
                 fold_assignment="Modulo", seed=self._seed())
        if self.nfolds == 0:
            c.pop("fold_assignment")
        if algo in ("GBM", "XGBoost", "DRF", "DeepLearning"):
            c.update(stopping_rounds=self.stopping_rounds, stopping_tolerance=self.stopping_tolerance or 0.001,
                     stopping_metric=self.stopping_metric if self.stopping_metric != "AUTO" else "auto")
        if self.balance_classes and algo in ("GBM", "DRF", "DeepLearning", "XGBoost"):
            c.update(balance_classes=True, class_sampling_factors=self.class_sampling_factors,
                     max_after_balance_size=self.max_after_balance_size)
        if self.distribution not in (None, "AUTO") and algo in ("GBM", "XGBoost", "DeepLearning"):
            c["distribution"] = self.distribution
        if self.monotone_constraints and algo in ("GBM", "XGBoost"):
            c["monotone_constraints"] = self.monotone_constraints
        rt = self.max_runtime_secs_per_model
        if self.max_runtime_secs:
            left = max(1.0, self.max_runtime_secs - (time.time() - self._t0))
            dl = getattr(self, "_step_deadline", None)
            if dl is not None:
                left = min(left, max(1.0, dl - time.time()))
            rt = min(rt, left) if rt else left
        if rt:
            c["max_runtime_secs"] = rt
        return c

    # ------------------------------------------------------------------ model building
    def _build(self, cls, algo, name, params, data):
        if not self._budget_left():
            return None
        kw = self._common(algo)
        kw.update(params)
        kw["model_id"] = f"{name}_AutoML_{self.project_name}"
        t = time.time()
        try:
            est = cls(**kw)
            est.train(x=data["x"], y=data["y"], training_frame=data["train"], weights_column=data["weights"],
                      fold_column=data["fold"], validation_frame=data["valid"])
        except Exception as e:
            from ..core.job import JobCancelled
            if isinstance(e, JobCancelled):
                raise
            self._log("ModelTraining", f"{name} failed: {e!r}", level="Warn")
            return None
        self.models.append(est)
        self._log("ModelTraining", f"{est.model_id} trained in {time.time() - t:.1f}s")
        self._checkpoint_model(est)
        return est

    def _run_step(self, algo, step, data, classification):
        E = _estimators()
        if algo == "StackedEnsemble":
            return self._se_step(step, data)
        cls = E[algo]
        if step.startswith("def_") or step == "XRT":
            name = f"{algo}_{step.split('_')[-1]}" if step != "XRT" else "XRT_1"
            if algo == "DRF" and step == "def_1":
                name = "DRF_1"
            self._build(cls, algo, name, _step_params(algo, step), data)
        elif step.startswith("grid_"):
            g = _grid_space(algo, step, classification)
            # a stable per-step offset (str hash() is salted per process, which
            # made seeded AutoML grids draw different models on every run)
            rng = np.random.RandomState(self._seed() + zlib.crc32(f"{algo}:{step}".encode()) % 1000)
            nmax = self.grid_models_per_step or 10 ** 6
            for i in range(nmax):
                if not self._budget_left():
                    break
                hp = {k: v[rng.randint(len(v))] for k, v in g["space"].items()}
                self._build(cls, algo, f"{algo}_{step}_model_{i + 1}", dict(g["fixed"], **hp), data)
        elif step in ("lr_annealing", "lr_search"):
            self._exploit(algo, cls, step, data)
        else:
            raise ValueError(f"unknown step {algo}:{step}")

    def _exploit(self, algo, cls, step, data):
        """Refit the best model of `algo` with a smaller/annealed learning rate and keep
        it only if it improves the leaderboard metric (GBMStepsProvider lr_annealing,
        XGBoostSteps lr_search)."""
        fam = [m for m in self.models if m.algo == algo.lower() and m._spec is not None]
        if not fam:
            return
        lb = Leaderboard(fam, sort_metric=self.sort_metric)
        best = lb.models[0]
        # only the names this estimator takes (its _parms also carry the
        # shared defaults every estimator holds)
        base = {k: v for k, v in best._user_parms().items() if k not in ("model_id", "training_frame",
                                                                          "validation_frame", "response_column",
                                                                          "checkpoint")}
        if step == "lr_annealing":
            cands = [dict(learn_rate=0.05 if algo == "GBM" else 0.1, learn_rate_annealing=0.99)]
        else:
            cands = [dict(learn_rate=lr) for lr in (0.05, 0.01) if lr < float(base.get("learn_rate", 0.1))]
        for j, c in enumerate(cands):
            params = dict(base, **c)
            params.pop("nfolds", None)
            m = self._build(cls, algo, f"{algo}_{step}_selection_{j + 1}", params, data)
            if m is None:
                continue
            lb2 = Leaderboard([best, m], sort_metric=self.sort_metric)
            if lb2.models[0] is not m:
                self.models.remove(m)
                self._log("ModelSelection", f"{m.model_id} did not improve on {best.model_id}; discarded")
            else:
                best = m

    def _se_step(self, step, data):
        from ..models.ensemble import H2OStackedEnsembleEstimator
        if data["y"] is None or self.nfolds == 0 and data["blending"] is None:
            if data["y"] is not None:
                self._log("ModelTraining", "StackedEnsemble skipped: needs nfolds>0 or a blending_frame")
            return
        base_all = [m for m in self.models if m.algo != "stackedensemble"]
        if len(base_all) < 2:
            return
        lb = Leaderboard(base_all, sort_metric=self.sort_metric)
        if step == "best_of_family":
            fam = {}
            for m in lb.models:
                key = "xrt" if m._parms.get("histogram_type") == "Random" and m.algo == "drf" else m.algo
                fam.setdefault(key, m)
            base, name = list(fam.values()), "StackedEnsemble_BestOfFamily_1"
        else:
            base, name = lb.models, "StackedEnsemble_AllModels_1"
        if len(base) < 2:
            return
        t = time.time()
        try:
            # StackedEnsembleStepsProvider.java:146: the metalearner is
            # cross-validated with the AutoML nfolds, so the ensemble carries
            # cross-validation metrics comparable with the base models'
            se_kw = {"metalearner_nfolds": self.nfolds} if (self.nfolds and data["blending"] is None) else {}
            se = H2OStackedEnsembleEstimator(base_models=base, model_id=f"{name}_AutoML_{self.project_name}",
                                             seed=self._seed(), **se_kw)
            se.train(x=data["x"], y=data["y"], training_frame=data["train"], validation_frame=data["valid"],
                     blending_frame=data["blending"])
        except Exception as e:
            from ..core.job import JobCancelled
            if isinstance(e, JobCancelled):
                raise
            self._log("ModelTraining", f"{name} failed: {e!r}", level="Warn")
            return
        self.models.append(se)
        self._log("ModelTraining", f"{se.model_id} trained in {time.time() - t:.1f}s")
        self._checkpoint_model(se)

    # ------------------------------------------------------------------ preprocessing
    def _preprocess(self, train, x, y, classification):
        """TargetEncoding preprocessing (preprocessing/TargetEncoding.java): categorical
        predictors with cardinality >= 25 are replaced by KFold target encodings."""
        steps = [s if isinstance(s, str) else (s.get("type") or "") for s in (self.preprocessing or [])]
        if not any(str(s).lower().replace("_", "") == "targetencoding" for s in steps) or y is None:
            return train, x
        from ..models.targetencoder import H2OTargetEncoderEstimator
        cats = [c for c in x if train.vec(c).type == "enum" and len(train.vec(c).domain or []) >= 25]
        if not cats:
            return train, x
        te = H2OTargetEncoderEstimator(data_leakage_handling="KFold" if self.nfolds else "None",
                                       fold_column=None, blending=True, inflection_point=5, smoothing=10,
                                       noise=0.0, seed=self._seed())
        if self.nfolds:
            train = train[:, :]
            train["__automl_te_fold"] = train.modulo_kfold_column(self.nfolds)
            te._parms["fold_column"] = "__automl_te_fold"
        te.train(x=cats, y=y, training_frame=train)
        enc = te.transform(train, as_training=True)
        self._te = te
        new_x = [c for c in x if c not in cats] + [n for n in enc.names if n.endswith("_te")]
        self._log("Preprocessing", f"TargetEncoding of {len(cats)} column(s): {cats}")
        return enc, new_x

    # ------------------------------------------------------------------ recovery
    def _checkpoint_model(self, est):
        from ..models.persist import save_model
        for d in (self.export_checkpoints_dir, self.recovery_dir):
            if d:
                os.makedirs(d, exist_ok=True)
                try:
                    save_model(est, d, force=True)
                except Exception as e:  # a model without MOJO support cannot be checkpointed
                    self._log("Checkpoint", f"{est.model_id} not saved: {e!r}", level="Warn")

    def _state_path(self):
        return os.path.join(self.recovery_dir, f"{self.project_name}.automl.json")

    def _write_state(self, args):
        if not self.recovery_dir:
            return
        st = {"project_name": self.project_name, "args": args, "done_steps": self._done_steps,
              "models": [m.model_id for m in self.models],
              "settings": {k: v for k, v in self.__dict__.items()
                           if not k.startswith("_") and k not in ("models", "event_log_rows", "training_info")
                           and isinstance(v, (int, float, str, bool, list, dict, type(None)))}}
        with open(self._state_path(), "w") as f:
            json.dump(st, f, default=str)

    def _save_inputs(self, train, valid, lbf, blend):
        from ..core.frame_io import save_frame
        os.makedirs(self.recovery_dir, exist_ok=True)
        out = {}
        for key, fr in (("train", train), ("valid", valid), ("leaderboard", lbf), ("blending", blend)):
            if fr is None:
                continue
            d = f"{self.project_name}.{key}_frame"
            if not os.path.exists(os.path.join(self.recovery_dir, d, "frame.json")):
                save_frame(fr, os.path.join(self.recovery_dir, d))
            out[key] = d
        return out

    # ------------------------------------------------------------------ train
    def train(self, x=None, y=None, training_frame=None, fold_column=None, weights_column=None,
              validation_frame=None, leaderboard_frame=None, blending_frame=None, _resume_state=None):
        self._t0 = time.time()
        if isinstance(y, int):
            y = training_frame.names[y]
        yv = training_frame.vec(y) if y is not None else None
        classification = yv is not None and yv.type == "enum"
        if x is None:
            x = [n for n in training_frame.names if n not in (y, fold_column, weights_column)]
        x = [training_frame.names[i] if isinstance(i, int) else i for i in x]
        args = {"x": x, "y": y, "fold_column": fold_column, "weights_column": weights_column}
        if self.recovery_dir and _resume_state is None:
            args["frames"] = self._save_inputs(training_frame, validation_frame, leaderboard_frame, blending_frame)
        if _resume_state is not None:
            args = _resume_state["args"]
            self._done_steps = list(_resume_state["done_steps"])
        self._log("Workflow", f"AutoML build started: {self.project_name}")
        self._set_stopping_tolerance(training_frame)
        train, xx = self._preprocess(training_frame, x, y, classification)
        valid = validation_frame
        if self._te is not None and valid is not None:
            valid = self._te.transform(valid)
        if self.nfolds == 0 and valid is None and blending_frame is None and y is not None:
            # AutoML.java: hold out 10% for early stopping when there is no CV
            tr, va = train.split_frame([0.9], seed=self._seed())
            train, valid = tr, va
            self._log("DataImport", "nfolds=0 and no validation frame: training frame split 90/10")
        data = {"x": xx, "y": y, "train": train, "valid": valid, "weights": weights_column,
                "fold": fold_column if fold_column not in (None, "") else None, "blending": blending_frame}
        if data["fold"] is not None:
            self.nfolds = 0  # fold column takes over
        plan = _expand_plan(self.modeling_plan) if self.modeling_plan else _expand_plan(_DEFAULT_PLAN)
        explore = [s for s in plan if s[1] not in ("lr_annealing", "lr_search") and s[0] != "StackedEnsemble"]
        exploit = [s for s in plan if s[1] in ("lr_annealing", "lr_search")]
        ses = [s for s in plan if s[0] == "StackedEnsemble"]
        if self.exploitation_ratio == 0:
            exploit = []
        self._write_state(args)
        order = [s for s in explore + exploit + ses if self._allowed(s[0])]
        for i, (algo, step) in enumerate(order):
            tag = f"{algo}:{step}"
            if tag in self._done_steps:
                continue
            self._step_deadline = None
            if algo != "StackedEnsemble" and not self._budget_left():
                continue     # out of time: skip the remaining base-model steps, still build the ensembles
            self._assign_step_time((algo, step), [it for it in order[i:]
                                                  if f"{it[0]}:{it[1]}" not in self._done_steps])
            self._run_step(algo, step, data, classification)
            self._step_deadline = None
            self._done_steps.append(tag)
            self._write_state(args)
        self._leaderboard = Leaderboard(self.models, sort_metric=self.sort_metric, frame=leaderboard_frame)
        self.training_info = {"start_epoch": int(self._t0), "stop_epoch": int(time.time()),
                              "duration_secs": round(time.time() - self._t0, 2),
                              "best_model": self.leader.model_id if self.leader else None,
                              "nfolds": self.nfolds, "models_trained": len(self.models)}
        self._log("Workflow", "AutoML build done")
        self._write_state(args)
        dkv.put(self.project_name, self)
        return self.leader

    # ------------------------------------------------------------------ results
    @property
    def leader(self):
        return self._leaderboard.models[0] if self._leaderboard and self._leaderboard.models else None

    @property
    def leaderboard(self):
        return self._leaderboard.as_frame() if self._leaderboard else None

    @property
    def event_log(self):
        import pandas as pd
        return H2OFrame(pd.DataFrame(self.event_log_rows)) if self.event_log_rows else None

    def get_best_model(self, algorithm=None, criterion=None):
        lb = Leaderboard(self.models, sort_metric=criterion or self.sort_metric)
        for m in lb.models:
            if algorithm is None or m.algo == algorithm.lower() or (algorithm.lower() == "basemodel" and m.algo != "stackedensemble"):
                return m
        return None

    def predict(self, test_data):
        if self._te is not None:
            test_data = self._te.transform(test_data)
        return self.leader.predict(test_data)

    def get_leaderboard(self, extra_columns=None):
        return self._leaderboard.as_frame(extra_columns=extra_columns)

    # ---- reference H2OAutoMLBaseMixin / H2OAutoML object API
    # (h2o-py/h2o/automl/_base.py:41-237, _estimator.py)
    @property
    def key(self):
        return self.project_name

    def detach(self):
        dkv.remove(self.project_name)

    def download_pojo(self, path="", get_genmodel_jar=False, genmodel_name=""):
        """POJO of the leader (_base.py:41)."""
        return self.leader.download_pojo(path, get_genmodel_jar=get_genmodel_jar, genmodel_name=genmodel_name)

    def download_mojo(self, path=".", get_genmodel_jar=False, genmodel_name="", **kw):
        """MOJO of the leader (_base.py:54); format="h2o" writes the reference
        h2o-genmodel layout."""
        return self.leader.download_mojo(path, get_genmodel_jar=get_genmodel_jar, genmodel_name=genmodel_name, **kw)

    def pareto_front(self, test_frame=None, x_metric=None, y_metric=None, **kwargs):
        """Pareto front of the leaderboard (_base.py:237): prediction time per
        row vs the sort metric by default, optimum from the metric directions."""
        from ..explanation import pareto_front
        from .leaderboard import make_leaderboard
        lb = self.get_leaderboard("ALL") if test_frame is None else \
            make_leaderboard(self, test_frame, extra_columns="ALL")
        x_metric = x_metric or "predict_time_per_row_ms"
        y_metric = y_metric or lb.columns[1]
        hib = ("auc", "aucpr")
        optimum = "{} {}".format("top" if y_metric.lower() in hib else "bottom",
                                 "right" if x_metric.lower() in hib else "left")
        kwargs.setdefault("title", f"Pareto Front for {self.project_name}")
        return pareto_front(lb, x_metric, y_metric, optimum=optimum, **kwargs)

    def _lb_models(self):
        return list(self._leaderboard.models) if self._leaderboard else []

    def explain(self, frame, **kw):
        from ..explanation import explain
        return explain(self._lb_models(), frame, **kw)

    def explain_row(self, frame, row_index, **kw):
        from ..explanation import explain_row
        return explain_row([self.leader], frame, row_index, **kw)

    def varimp(self, use_pandas=True, **kw):
        from ..explanation import varimp
        return varimp(self._lb_models(), use_pandas=use_pandas, **kw)

    def varimp_heatmap(self, **kw):
        from ..explanation import varimp_heatmap
        return varimp_heatmap(self._lb_models(), **kw)

    def model_correlation(self, frame, **kw):
        from ..explanation import model_correlation
        return model_correlation(self._lb_models(), frame, **kw)

    def model_correlation_heatmap(self, frame, **kw):
        from ..explanation import model_correlation_heatmap
        return model_correlation_heatmap(self._lb_models(), frame, **kw)

    def pd_multi_plot(self, frame, column, **kw):
        from ..explanation import pd_multi_plot
        return pd_multi_plot(self._lb_models(), frame, column, **kw)

    @property
    def modeling_steps(self):
        return [{"name": a, "steps": [{"id": s}]} for a, s in (t.split(":") for t in self._done_steps)]


def get_automl(project_name):
    return dkv.get(project_name)


def get_leaderboard(aml, extra_columns=None):
    return aml.get_leaderboard(extra_columns)


def resume_automl(recovery_dir):
    """Continue every AutoML run recorded in `recovery_dir` (h2o.resume)."""
    from ..core.frame_io import load_frame
    from ..models.persist import load_model
    out = []
    if not recovery_dir or not os.path.isdir(recovery_dir):
        return out
    for fn in sorted(os.listdir(recovery_dir)):
        if not fn.endswith(".automl.json"):
            continue
        with open(os.path.join(recovery_dir, fn)) as f:
            st = json.load(f)
        frames = st["args"].get("frames") or {}
        if "train" not in frames:
            continue
        s = dict(st["settings"])
        s.pop("modeling_plan", None)
        aml = H2OAutoML(**{k: v for k, v in s.items() if k in H2OAutoML.__init__.__code__.co_varnames},
                        modeling_plan=st["settings"].get("modeling_plan"))
        aml.models = []
        for mid in st["models"]:
            p = os.path.join(recovery_dir, mid)
            if os.path.exists(p):
                aml.models.append(load_model(p))
        ld = {k: load_frame(None, os.path.join(recovery_dir, d)) for k, d in frames.items()}
        a = st["args"]
        aml.train(x=a["x"], y=a["y"], training_frame=ld["train"], validation_frame=ld.get("valid"),
                  leaderboard_frame=ld.get("leaderboard"), blending_frame=ld.get("blending"),
                  fold_column=a.get("fold_column"), weights_column=a.get("weights_column"), _resume_state=st)
        out.append(aml)
    return out
