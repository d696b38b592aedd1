"""ModelSelection: best-subset GLM search.

Reference: hex/modelselection/ModelSelection.java, ModelSelectionModel.java,
ModelSelectionUtils.java (modes allsubsets / maxr / maxrsweep / backward;
max_predictor_number / min_predictor_number; allsubsets and maxr pick the
best-R2 subset for every size; maxrsweep does the same with sweep
operations on the cross-product matrix; backward drops the predictor with
the smallest |z| while its p-value exceeds p_values_threshold; the result
frame lists model_name, model_id, best_r2_value / z / p values and
predictor names per subset size).

MI355X design: one weighted Gram of [X, y] (the matrix-core Gram kernel)
is all the search needs -- the R2 of any subset is 1 - RSS/TSS from a
small Cholesky solve on that cross-product matrix, so allsubsets / maxr
evaluate thousands of candidate subsets without touching the rows again;
only the final per-size models are fitted as real GLMs.
"""
from __future__ import annotations

import itertools
import math

import numpy as np
import pandas as pd
import torch

from ...core.frame import H2OFrame
from ...core.vec import T_ENUM
from ..base import H2OEstimator
from ..datainfo import DataInfo
from ...ops import linalg_ops
from ...parallel import collectives as coll
from .glm import H2OGeneralizedLinearEstimator

MS_DEFAULTS = dict(mode="maxr", max_predictor_number=1, min_predictor_number=1, p_values_threshold=0.0,
                   family="AUTO", link="family_default", lambda_=0.0, alpha=0.0, standardize=True,
                   intercept=True, nparallelism=0, build_glm_model=True, influence=None, seed=-1,
                   compute_p_values=True, max_iterations=0,
                   # GLM parameters forwarded to the inner GLMs (model_selection.py in h2o-py)
                   score_iteration_interval=-1, tweedie_variance_power=0.0, tweedie_link_power=1.0, theta=1e-10,
                   solver="AUTO", lambda_search=False, early_stopping=True, nlambdas=-1,
                   missing_values_handling="MeanImputation", plug_values=None, remove_collinear_columns=False,
                   non_negative=False, objective_epsilon=-1.0, beta_epsilon=1e-4, gradient_epsilon=-1.0,
                   startval=None, prior=-1.0, cold_start=False, lambda_min_ratio=-1.0, beta_constraints=None,
                   max_active_predictors=-1, obj_reg=-1.0, balance_classes=False, class_sampling_factors=None,
                   max_after_balance_size=5.0, max_confusion_matrix_size=20)

_GLM_PASS = ("score_iteration_interval", "tweedie_variance_power", "tweedie_link_power", "theta", "solver",
             "lambda_search", "early_stopping", "nlambdas", "missing_values_handling", "plug_values",
             "remove_collinear_columns", "non_negative", "objective_epsilon", "beta_epsilon", "gradient_epsilon",
             "prior", "cold_start", "lambda_min_ratio", "beta_constraints", "max_active_predictors", "obj_reg",
             "balance_classes", "class_sampling_factors", "max_after_balance_size", "seed", "startval")


class H2OModelSelectionEstimator(H2OEstimator):
    algo = "modelselection"
    _defaults = MS_DEFAULTS

    # ---------------------------------------------------------- R2 engine
    def _cross(self, spec):
        di = DataInfo(spec.frame, spec.x, standardize=False, use_all_factor_levels=False, pad_to=0)
        X, ok = di.expand(spec.frame, dtype=torch.float32, pad=False)
        y = spec.y_tensor(dtype=torch.float64).to(torch.float32)
        w = spec.w_tensor()
        w = torch.ones_like(y) if w is None else w.to(torch.float32)
        ok = ok & ~torch.isnan(y)
        w = torch.where(ok, w, torch.zeros_like(w))
        A = torch.cat([torch.ones_like(y).view(-1, 1), torch.nan_to_num(X), torch.nan_to_num(y).view(-1, 1)], 1)
        G = linalg_ops.weighted_gram(A, w).to(torch.float64)
        coll.allreduce_(G)
        # predictor -> expanded column indices (offset 1 for the intercept)
        groups = {}
        for j, nm in enumerate(di.coef_names):
            src = next((c for c in spec.x if nm == c or nm.startswith(c + ".")), nm)
            groups.setdefault(src, []).append(j + 1)
        return G.cpu().numpy(), groups

    def _r2(self, G, cols):
        idx = [0] + cols
        yi = G.shape[0] - 1
        sw = G[0, 0]
        ybar = G[0, yi] / sw
        tss = G[yi, yi] - sw * ybar * ybar
        A = G[np.ix_(idx, idx)]
        b = G[idx, yi]
        try:
            beta = np.linalg.solve(A + 1e-12 * np.eye(len(idx)), b)
        except np.linalg.LinAlgError:
            beta = np.linalg.lstsq(A, b, rcond=None)[0]
        rss = G[yi, yi] - 2 * beta @ b + beta @ A @ beta
        return 1 - rss / tss if tss > 0 else 0.0

    def _subset_r2(self, G, groups, preds):
        return self._r2(G, [j for p in preds for j in groups[p]])

    # ---------------------------------------------------------- search modes
    def _allsubsets(self, G, groups, preds, kmax):
        best = {}
        for k in range(1, kmax + 1):
            cand = max(itertools.combinations(preds, k), key=lambda s: self._subset_r2(G, groups, s))
            best[k] = list(cand)
        return best

    def _maxr(self, G, groups, preds, kmax):
        best = {}
        cur = []
        for k in range(1, kmax + 1):
            rest = [p for p in preds if p not in cur]
            add = max(rest, key=lambda q: self._subset_r2(G, groups, cur + [q]))
            cur = cur + [add]
            improved = True
            while improved and k > 1:
                improved = False
                r0 = self._subset_r2(G, groups, cur)
                for i in range(len(cur)):
                    for q in [p for p in preds if p not in cur]:
                        trial = cur[:i] + [q] + cur[i + 1:]
                        r = self._subset_r2(G, groups, trial)
                        if r > r0 + 1e-12:
                            cur, r0, improved = trial, r, True
            best[k] = list(cur)
        return best

    def _check_init(self, spec, mode, preds):
        """ModelSelection.java initModelSelectionParameters."""
        p = self._parms
        fam = str(p.get("family") or "AUTO").lower()
        if mode not in ("maxr", "allsubsets", "maxrsweep", "backward"):
            raise ValueError(f"mode must be one of allsubsets, maxr, maxrsweep, backward; got {mode}")
        if mode != "backward":
            if spec.nclasses > 1:
                raise ValueError("ERRR on field: response: 'allsubsets' and 'maxr' only works with regression.")
            if fam not in ("auto", "gaussian"):
                raise ValueError("ERRR on field: _family: ModelSelection only supports Gaussian family for "
                                 "'allsubset' and 'maxr' mode.")
            k = int(p.get("max_predictor_number", 1))
            if k < 1 or k > len(preds):
                raise ValueError("ERRR on field: max_predictor_number: max_predictor_number must exceed 0 and be no "
                                 "greater than the number of predictors of the training frame.")
        else:
            if spec.valid is not None:
                raise ValueError("ERRR on field: validation_frame: is not supported for ModelSelection "
                                 "mode='backward'")
            if p.get("lambda_search"):
                raise ValueError("ERRR on field: lambda_search: backward selection does not support lambda_search.")
            lam = p.get("lambda_")
            if lam not in (None, 0, 0.0) and not (isinstance(lam, (list, tuple)) and list(lam) == [0]):
                raise ValueError("ERRR on field: lambda: must be set to 0 for backward selection")
            if fam in ("multinomial", "ordinal"):
                raise ValueError("ERRR on field: family: backward selection does not support multinomial or ordinal")
            mn = int(p.get("min_predictor_number", 1))
            if mn <= 0:
                raise ValueError("ERRR on field: min_predictor_number: must be >= 1.")
            if mn > len(preds):
                raise ValueError("ERRR on field: min_predictor_number: cannot exceed the total number of predictors "
                                 f"({len(preds)})in the dataset.")
        if int(p.get("nparallelism", 0) or 0) < 0:
            raise ValueError("ERRR on field: nparallelism: must be >= 0.")

    def _glm(self, spec, preds):
        p = self._parms
        fw = {k: p[k] for k in _GLM_PASS if k in p}
        if int(p.get("max_iterations") or 0) > 0:
            fw["max_iterations"] = int(p["max_iterations"])
        m = H2OGeneralizedLinearEstimator(family=p.get("family") or "AUTO", link=p.get("link"),
                                          lambda_=p.get("lambda_", 0.0), alpha=p.get("alpha", 0.0),
                                          standardize=p.get("standardize", True), intercept=p.get("intercept", True),
                                          compute_p_values=bool(p.get("compute_p_values", True)) or
                                          str(p.get("mode") or "maxr").lower() == "backward", **fw)
        m.train(x=list(preds), y=spec.y, training_frame=spec.frame, weights_column=spec.weights_column)
        return m

    def _fit(self, spec):
        p = self._parms
        mode = str(p.get("mode") or "maxr").lower()
        preds = list(spec.x)
        self._check_init(spec, mode, preds)
        kmax = min(int(p.get("max_predictor_number", 1)), len(preds))
        rows = []
        self._models = {}
        if mode == "backward":
            kmin = max(1, int(p.get("min_predictor_number", 1)))
            thr = float(p.get("p_values_threshold", 0.0))
            cur = list(preds)
            while True:
                m = self._glm(spec, cur)
                self._models[len(cur)] = m
                tab = m.coef_with_p_values()
                z = {r["names"]: r for r in tab.to_dict("records")} if hasattr(tab, "to_dict") else {}
                rows.append({"model_name": f"best {len(cur)} predictors model", "model_id": m.model_id,
                             "coefficient_names": [c for c in m.coef() if c != "Intercept"],
                             "z_values": [z[c]["z_value"] for c in m.coef() if c in z and c != "Intercept"],
                             "p_values": [z[c]["p_value"] for c in m.coef() if c in z and c != "Intercept"],
                             "predictor_names": list(cur)})
                if len(cur) <= kmin:
                    break
                # predictor-level max p-value (categoricals: min over their levels, reference)
                pv = {}
                for c in cur:
                    vals = [z[n]["p_value"] for n in z if n == c or n.startswith(c + ".")]
                    pv[c] = min(vals) if vals else 1.0
                worst = max(cur, key=lambda c: pv[c])
                if pv[worst] <= thr and thr > 0:
                    break
                cur = [c for c in cur if c != worst]
            self._result = pd.DataFrame(rows)
            return
        G, groups = self._cross(spec)
        best = self._allsubsets(G, groups, preds, kmax) if mode == "allsubsets" else self._maxr(G, groups, preds, kmax)
        for k in range(1, kmax + 1):
            sel = best[k]
            r2 = self._subset_r2(G, groups, sel)
            mid = None
            if p.get("build_glm_model", True):
                m = self._glm(spec, sel)
                self._models[k] = m
                mid = m.model_id
            rows.append({"model_name": f"best {k} predictors model", "model_id": mid, "best_r2_value": r2,
                         "predictor_names": list(sel)})
        self._result = pd.DataFrame(rows)

    # ---------------------------------------------------------- API
    def result(self):
        df = self._result.copy()
        df["predictor_names"] = [", ".join(v) for v in df["predictor_names"]]
        for c in ("coefficient_names", "z_values", "p_values"):
            if c in df:
                df[c] = [", ".join(map(str, v)) for v in df[c]]
        return H2OFrame(df)

    def get_best_R2_values(self):
        return list(self._result["best_r2_value"]) if "best_r2_value" in self._result else None

    def get_best_model_predictors(self):
        return list(self._result["predictor_names"])

    def coef(self, predictor_size=None):
        if predictor_size is None:
            return [self._models[k].coef() for k in sorted(self._models)]
        return self._models[predictor_size].coef()

    def coef_norm(self, predictor_size=None):
        if predictor_size is None:
            return [self._models[k].coef_norm() for k in sorted(self._models)]
        return self._models[predictor_size].coef_norm()

    def get_best_model(self, predictor_size):
        return self._models[predictor_size]

    def _predict_raw(self, frame):
        k = max(self._models)
        return self._models[k]._predict_raw(frame)

    def _score_all(self, spec):
        if self._models:
            self._training_metrics = self._models[max(self._models)]._training_metrics
