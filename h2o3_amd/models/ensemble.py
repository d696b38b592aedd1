"""Stacked Ensemble.

Reference: hex/ensemble/StackedEnsemble.java (level-one frame from the base
models' cross-validation holdout predictions — or predictions on a
`blending_frame` — then a metalearner), hex/ensemble/Metalearners.java
(AUTO = GLM with non-negative coefficients and lambda search; glm / gbm /
drf / deeplearning / naivebayes / xgboost), StackedEnsembleModel.java
(scoring: base-model predictions -> metalearner).
"""
from __future__ import annotations

import torch

from ..core.frame import H2OFrame
from ..core.vec import T_ENUM, T_REAL, Vec
from .base import H2OEstimator

SE_DEFAULTS = dict(base_models=[], metalearner_algorithm="auto", metalearner_nfolds=0,
                   metalearner_fold_assignment=None, metalearner_fold_column=None, metalearner_params=None,
                   metalearner_transform="NONE", max_runtime_secs=0.0, blending_frame=None, seed=-1,
                   score_training_samples=10000, keep_levelone_frame=False, export_checkpoints_dir=None,
                   auc_type="auto", gainslift_bins=-1)


def _resolve_models(base):
    from ..core import dkv
    out = []
    for b in base:
        if isinstance(b, str):
            o = dkv.get(b)
        else:
            o = b
        if hasattr(o, "models") and not isinstance(o, H2OEstimator):   # a grid / automl leaderboard
            out.extend(o.models)
        elif o is not None:
            out.append(o)
    return out


class H2OStackedEnsembleEstimator(H2OEstimator):
    algo = "stackedensemble"
    _defaults = SE_DEFAULTS

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, blending_frame=None, **kw):
        if blending_frame is not None:
            self._parms["blending_frame"] = blending_frame
        base = _resolve_models(self._parms.get("base_models") or [])
        self._base = base
        if x is None and base:
            x = base[0]._spec.x
        return super().train(x=x, y=y, training_frame=training_frame, validation_frame=validation_frame, **kw)

    def _level_one(self, models, frame, use_cv):
        cols, names = [], []
        for m in models:
            if use_cv:
                raw = getattr(m, "_cv_holdout", None)
                if raw is None:
                    raise ValueError(f"base model {m.model_id} has no cross-validation holdout predictions: train it "
                                     "with nfolds>1 and keep_cross_validation_predictions=True (or use a blending_frame)")
            else:
                raw = m._predict_raw(frame)
            if self._spec.nclasses == 2:
                cols.append(raw[:, -1])
                names.append(m.model_id)
            elif self._spec.nclasses > 2:
                for k in range(raw.shape[1]):
                    cols.append(raw[:, k])
                    names.append(f"{m.model_id}/{self._spec.response_domain[k]}")
            else:
                cols.append(raw[:, 0])
                names.append(m.model_id)
        if str(self._parms.get("metalearner_transform") or "NONE").lower() == "logit" and self._spec.nclasses >= 2:
            # MetalearnerTransform.Logit (StackedEnsembleModel.java:95): logit of
            # the base-model probabilities, clamped to [1e-9, 1 - 1e-9]
            cols = [torch.logit(c.to(torch.float64).clamp(1e-9, 1 - 1e-9)) for c in cols]
        vecs = [Vec(c.to(torch.float32).contiguous(), T_REAL) for c in cols]
        return vecs, names

    def _fit(self, spec):
        from ..estimators import (H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                                  H2ORandomForestEstimator, H2ODeepLearningEstimator, H2ONaiveBayesEstimator,
                                  H2OXGBoostEstimator)
        p = self._parms
        base = self._base
        if not base:
            raise ValueError("StackedEnsemble needs base_models")
        blend = p.get("blending_frame")
        frame = blend if blend is not None else spec.frame
        vecs, names = self._level_one(base, frame, use_cv=blend is None)
        y = frame.vec(spec.y)
        mt = str(p.get("metalearner_transform") or "NONE").lower()
        if mt not in ("none", "logit"):
            raise ValueError(f"metalearner_transform must be NONE or Logit, got {mt}")
        fcol = p.get("metalearner_fold_column")
        nf = int(p.get("metalearner_nfolds") or 0)
        if fcol and nf:
            raise ValueError("Cannot specify fold_column and nfolds at the same time.")
        extra_v, extra_n = [], []
        if fcol:
            if fcol not in frame.names:
                raise ValueError(f"metalearner_fold_column '{fcol}' is not in the training frame")
            extra_v, extra_n = [frame.vec(fcol)], [fcol]
        lvl1 = H2OFrame.from_vecs(vecs + extra_v + [y], names + extra_n + [spec.y])
        self._names = names
        algo = (p.get("metalearner_algorithm") or "auto").lower()
        mp = dict(p.get("metalearner_params") or {})
        # Metalearner.setCrossValidationParams
        if fcol:
            mp.setdefault("fold_column", fcol)
        elif nf:
            mp.setdefault("nfolds", nf)
            if nf > 1 and p.get("metalearner_fold_assignment"):
                mp.setdefault("fold_assignment", p["metalearner_fold_assignment"])
        if p.get("seed", -1) not in (None, -1):
            mp.setdefault("seed", p["seed"])
        if algo in ("auto", "glm"):
            fam = "binomial" if spec.nclasses == 2 else ("multinomial" if spec.nclasses > 2 else "gaussian")
            mp.setdefault("family", fam)
            if algo == "auto":
                # Metalearners.AUTOMetalearner.setCustomParams: non-negative
                # weights (not for multinomial / ordinal), no standardization,
                # lambda search without early stopping when a validation
                # frame is given, scoring history every 5 iterations otherwise
                mp.setdefault("non_negative", str(mp["family"]).lower() not in ("multinomial", "ordinal"))
                mp.setdefault("standardize", False)
                mp.setdefault("generate_scoring_history", True)
                if spec.valid is not None:
                    mp.setdefault("lambda_search", True)
                    mp.setdefault("early_stopping", False)
                else:
                    mp.setdefault("score_iteration_interval", 5)
            meta = H2OGeneralizedLinearEstimator(**mp)
        else:
            cls = {"gbm": H2OGradientBoostingEstimator, "drf": H2ORandomForestEstimator,
                   "deeplearning": H2ODeepLearningEstimator, "naivebayes": H2ONaiveBayesEstimator,
                   "xgboost": H2OXGBoostEstimator}[algo]
            meta = cls(**mp)
        lvl1_valid = None
        if spec.valid is not None and algo in ("auto", "glm"):
            # StackedEnsemble.java: the metalearner sees a level-one validation
            # frame of base-model predictions on the validation rows
            vv, _ = self._level_one(base, spec.valid, use_cv=False)
            lvl1_valid = H2OFrame.from_vecs(vv + [spec.valid.vec(spec.y)], names + [spec.y])
        meta.train(x=names, y=spec.y, training_frame=lvl1, validation_frame=lvl1_valid)
        self._meta = meta
        if getattr(meta, "_cross_validation_metrics", None) is not None:
            # StackedEnsembleModel.java:371: the ensemble's cross-validation
            # metrics are the metalearner's, cross-validated on the level-one
            # frame of base-model holdout predictions (honest, unlike training
            # metrics of base models refit on all rows)
            self._cross_validation_metrics = meta._cross_validation_metrics
        if p.get("keep_levelone_frame"):
            self._output["levelone_frame"] = lvl1
        self._output["model_summary"] = {"base_models": [m.model_id for m in base], "metalearner": meta.algo}

    def metalearner(self):
        return self._meta

    def _label_threshold(self):
        """Labels come from the metalearner's scoring of the level-one frame
        (StackedEnsembleModel.java:251-258 metalearner.score), i.e. the
        metalearner's default threshold -- as the MOJO's metalearner does."""
        if getattr(self, "_meta", None) is not None and hasattr(self._meta, "_label_threshold"):
            return self._meta._label_threshold()
        return super()._label_threshold()

    def _predict_raw(self, frame):
        vecs, names = self._level_one(self._base, frame, use_cv=False)
        lvl1 = H2OFrame.from_vecs(vecs, names)
        return self._meta._predict_raw(lvl1)

    def levelone_frame_id(self):
        return self._output.get("levelone_frame")
