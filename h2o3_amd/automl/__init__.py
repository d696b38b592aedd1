"""AutoML.

Reference: h2o-automl (ai/h2o/automl/AutoML.java, ModelingPlans.java,
modeling/*StepsProvider.java, leaderboard/*, events/EventLog.java): a
modeling plan of default models (XGBoost x3, GLM, DRF, XRT, GBM x5, DL),
random grids for GBM / XGBoost / DL, then Stacked Ensembles ("BestOfFamily"
and "AllModels"), all cross-validated with shared folds, under
max_models / max_runtime_secs budgets; results in a leaderboard sorted by
the problem's default metric.
"""
from __future__ import annotations

import math
import time

import numpy as np

from ..core import dkv
from ..core.frame import H2OFrame
from .leaderboard import Leaderboard

_ALGOS = ["XGBoost", "GLM", "DRF", "GBM", "DeepLearning", "StackedEnsemble"]


class H2OAutoML:
    def __init__(self, nfolds=-1, balance_classes=False, class_sampling_factors=None, max_after_balance_size=5.0,
                 max_runtime_secs=None, max_runtime_secs_per_model=None, max_models=None, distribution="AUTO",
                 stopping_metric="AUTO", stopping_tolerance=None, stopping_rounds=3, seed=None, project_name=None,
                 exclude_algos=None, include_algos=None, exploitation_ratio=-1, modeling_plan=None,
                 preprocessing=None, monotone_constraints=None, keep_cross_validation_predictions=False,
                 keep_cross_validation_models=False, keep_cross_validation_fold_assignment=False,
                 sort_metric="AUTO", export_checkpoints_dir=None, verbosity="warn", **kw):
        self.nfolds = 5 if nfolds in (-1, None) else nfolds
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
        self.distribution = distribution
        self.monotone_constraints = monotone_constraints
        self.keep_cross_validation_predictions = keep_cross_validation_predictions
        self.modeling_plan = modeling_plan
        self.preprocessing = preprocessing
        self.event_log_rows = []
        self.models = []
        self._leaderboard = None
        self.training_info = {}

    # ------------------------------------------------------------------ helpers
    def _log(self, stage, msg, level="Info"):
        self.event_log_rows.append({"timestamp": time.strftime("%H:%M:%S"), "level": level, "stage": stage,
                                    "message": msg})

    def _allowed(self, algo):
        a = algo.lower()
        if self.include_algos is not None:
            return a in self.include_algos
        return a not in self.exclude_algos

    def _budget_left(self):
        if self.max_models and len([m for m in self.models if m.algo != "stackedensemble"]) >= self.max_models:
            return False
        if self.max_runtime_secs and time.time() - self._t0 > self.max_runtime_secs:
            return False
        return True

    def _common(self):
        c = dict(nfolds=self.nfolds, keep_cross_validation_predictions=True, fold_assignment="Modulo",
                 seed=self.seed if self.seed != -1 else 42)
        if self.max_runtime_secs_per_model:
            c["max_runtime_secs"] = self.max_runtime_secs_per_model
        return c

    def _plan(self, classification):
        from ..estimators import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator,
                                  H2OGradientBoostingEstimator, H2ORandomForestEstimator, H2OXGBoostEstimator)
        es = dict(stopping_rounds=self.stopping_rounds, stopping_tolerance=self.stopping_tolerance or 0.001,
                  score_tree_interval=5)
        plan = [
            ("XGBoost", "XGBoost_1", H2OXGBoostEstimator, dict(ntrees=100, max_depth=10, min_rows=5, sample_rate=0.6,
                                                               col_sample_rate_per_tree=0.8, learn_rate=0.3)),
            ("GLM", "GLM_1", H2OGeneralizedLinearEstimator, dict(lambda_search=True, alpha=0.5)),
            ("DRF", "DRF_1", H2ORandomForestEstimator, dict(ntrees=50)),
            ("XGBoost", "XGBoost_2", H2OXGBoostEstimator, dict(ntrees=100, max_depth=20, min_rows=10, sample_rate=0.6,
                                                               col_sample_rate_per_tree=0.8, learn_rate=0.3)),
            ("GBM", "GBM_1", H2OGradientBoostingEstimator, dict(ntrees=100, max_depth=6, min_rows=1, sample_rate=0.8,
                                                               col_sample_rate=0.8, col_sample_rate_per_tree=0.8, **es)),
            ("GBM", "GBM_2", H2OGradientBoostingEstimator, dict(ntrees=100, max_depth=7, min_rows=10, sample_rate=0.8,
                                                               col_sample_rate=0.8, col_sample_rate_per_tree=0.8, **es)),
            ("GBM", "GBM_3", H2OGradientBoostingEstimator, dict(ntrees=100, max_depth=8, min_rows=10, sample_rate=0.8,
                                                               col_sample_rate=0.8, col_sample_rate_per_tree=0.8, **es)),
            ("GBM", "GBM_4", H2OGradientBoostingEstimator, dict(ntrees=100, max_depth=10, min_rows=10, sample_rate=0.8,
                                                               col_sample_rate=0.8, col_sample_rate_per_tree=0.8, **es)),
            ("DeepLearning", "DeepLearning_1", H2ODeepLearningEstimator, dict(epochs=10, hidden=[10, 10, 10])),
            ("DRF", "XRT_1", H2ORandomForestEstimator, dict(ntrees=50, histogram_type="Random")),
            ("XGBoost", "XGBoost_3", H2OXGBoostEstimator, dict(ntrees=100, max_depth=5, min_rows=3, sample_rate=0.8,
                                                               col_sample_rate_per_tree=0.8, learn_rate=0.3)),
        ]
        # random grid steps (GBM / XGBoost / DL), reference: *StepsProvider grids
        rng = np.random.RandomState(self.seed if self.seed not in (None, -1) else 42)
        for i in range(30):
            plan.append(("GBM", f"GBM_grid_1_model_{i + 1}", H2OGradientBoostingEstimator,
                         dict(ntrees=100, max_depth=int(rng.choice([3, 4, 5, 6, 7, 8, 9, 10, 12, 15])),
                              min_rows=float(rng.choice([1, 5, 10, 15, 30, 100])),
                              learn_rate=float(rng.choice([0.001, 0.005, 0.01, 0.05, 0.08, 0.1, 0.5, 0.8])),
                              sample_rate=float(rng.choice([0.5, 0.6, 0.7, 0.8, 0.9, 1.0])),
                              col_sample_rate=float(rng.choice([0.4, 0.7, 1.0])), **es)))
            plan.append(("XGBoost", f"XGBoost_grid_1_model_{i + 1}", H2OXGBoostEstimator,
                         dict(ntrees=100, max_depth=int(rng.choice([3, 6, 9, 12, 15])),
                              min_rows=float(rng.choice([0.01, 0.1, 1, 3, 5, 10])),
                              learn_rate=float(rng.choice([0.01, 0.05, 0.1, 0.3])),
                              sample_rate=float(rng.choice([0.6, 0.8, 1.0])),
                              reg_lambda=float(rng.choice([0.001, 0.01, 0.1, 1, 10, 100])))))
        return plan

    # ------------------------------------------------------------------ train
    def train(self, x=None, y=None, training_frame=None, fold_column=None, weights_column=None,
              validation_frame=None, leaderboard_frame=None, blending_frame=None):
        from ..models.ensemble import H2OStackedEnsembleEstimator
        self._t0 = time.time()
        yv = training_frame.vec(y) if y is not None else None
        classification = yv is not None and yv.type == "enum"
        self._log("Workflow", f"AutoML build started: {self.project_name}")
        for algo, name, cls, params in self._plan(classification):
            if not self._budget_left():
                break
            if not self._allowed(algo):
                continue
            kw = self._common()
            kw.update(params)
            if self.monotone_constraints and algo in ("GBM", "XGBoost"):
                kw["monotone_constraints"] = self.monotone_constraints
            kw["model_id"] = f"{name}_AutoML_{self.project_name}"
            try:
                t = time.time()
                est = cls(**kw)
                est.train(x=x, y=y, training_frame=training_frame, weights_column=weights_column,
                          fold_column=fold_column, validation_frame=validation_frame)
                self.models.append(est)
                self._log("ModelTraining", f"{est.model_id} trained in {time.time() - t:.1f}s")
            except Exception as e:
                self._log("ModelTraining", f"{name} failed: {e!r}", level="Warn")
        if self._allowed("StackedEnsemble") and y is not None and len(self.models) >= 2:
            lb = Leaderboard(self.models, sort_metric=self.sort_metric, frame=leaderboard_frame)
            best_of_family = {}
            for m in lb.models:
                best_of_family.setdefault(m.algo, m)
            for se_name, base in (("StackedEnsemble_BestOfFamily", list(best_of_family.values())),
                                  ("StackedEnsemble_AllModels", lb.models)):
                if len(base) < 2:
                    continue
                try:
                    se = H2OStackedEnsembleEstimator(base_models=base, model_id=f"{se_name}_AutoML_{self.project_name}",
                                                     seed=self.seed)
                    se.train(x=x, y=y, training_frame=training_frame, validation_frame=validation_frame,
                             blending_frame=blending_frame)
                    self.models.append(se)
                    self._log("ModelTraining", f"{se.model_id} trained")
                except Exception as e:
                    self._log("ModelTraining", f"{se_name} failed: {e!r}", level="Warn")
        self._leaderboard = Leaderboard(self.models, sort_metric=self.sort_metric, frame=leaderboard_frame)
        self.training_info = {"start_epoch": int(self._t0), "stop_epoch": int(time.time()),
                              "duration_secs": round(time.time() - self._t0, 2)}
        self._log("Workflow", "AutoML build done")
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
        return H2OFrame(pd.DataFrame(self.event_log_rows), _local=True) if self.event_log_rows else None

    def get_best_model(self, algorithm=None, criterion=None):
        lb = Leaderboard(self.models, sort_metric=criterion or self.sort_metric)
        for m in lb.models:
            if algorithm is None or m.algo == algorithm.lower() or (algorithm.lower() == "basemodel" and m.algo != "stackedensemble"):
                return m
        return None

    def predict(self, test_data):
        return self.leader.predict(test_data)

    def get_leaderboard(self, extra_columns=None):
        return self._leaderboard.as_frame(extra_columns=extra_columns)


def get_automl(project_name):
    return dkv.get(project_name)


def get_leaderboard(aml, extra_columns=None):
    return aml.get_leaderboard(extra_columns)
