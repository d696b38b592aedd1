"""ANOVA GLM (type III sums of squares over main effects and interactions).

Reference: hex/anovaglm/ANOVAGLM.java, ANOVAGLMModel.java,
ANOVAGLMUtils.java (predictors and their interactions up to
highest_interaction_term; categorical columns are effects (sum-to-zero)
coded so type III tests are meaningful; one GLM for the full model plus
one per left-out term; SS = deviance(reduced) - deviance(full), df =
#columns of the term, F = (SS/df) / (residual deviance / residual df)
with its p-value; result table columns predictors_interactions, family,
link, ss, df, f_values, p_values).

MI355X design: the transformed design is materialised once on the device
and every reduced model is the same fused IRLS GLM pass on a column
subset -- the models share the HBM-resident columns (no re-parse).
"""
from __future__ import annotations

import itertools
import math

import numpy as np
import pandas as pd
import torch
from scipy import stats

from ...core.frame import H2OFrame
from ...core.vec import T_ENUM, T_REAL, Vec
from ..base import H2OEstimator
from .glm import H2OGeneralizedLinearEstimator

ANOVA_DEFAULTS = dict(family="AUTO", link="family_default", highest_interaction_term=2, type=3, lambda_=0.0,
                      alpha=0.0, standardize=True, compute_p_values=True, save_transformed_framekeys=False,
                      nparallelism=4, seed=-1, max_iterations=0, early_stopping=False,
                      # GLM parameters forwarded to every inner GLM (anovaglm.py in h2o-py)
                      tweedie_variance_power=0.0, tweedie_link_power=1.0, theta=1e-10, solver="AUTO",
                      missing_values_handling="MeanImputation", plug_values=None, non_negative=False, prior=-1.0,
                      lambda_search=False, balance_classes=False, class_sampling_factors=None,
                      max_after_balance_size=5.0)

_GLM_PASS = ("tweedie_variance_power", "tweedie_link_power", "theta", "solver", "missing_values_handling",
             "plug_values", "non_negative", "prior", "lambda_search", "balance_classes", "class_sampling_factors",
             "max_after_balance_size", "max_iterations", "early_stopping", "seed")


class H2OANOVAGLMEstimator(H2OEstimator):
    algo = "anovaglm"
    _defaults = ANOVA_DEFAULTS

    def _effect_cols(self, frame, c):
        v = frame.vec(c)
        if v.type == T_ENUM:
            dom = self._doms[c]
            codes = self._adapt_enum(v, dom).long()
            L = len(dom)
            out = []
            for i in range(L - 1):
                col = torch.where(codes == i, 1.0, torch.where(codes == L - 1, -1.0, 0.0))
                out.append((f"{c}_{dom[i]}", col.to(torch.float32)))
            return out
        return [(c, v.as_float(torch.float32))]

    def _transformed(self, frame):
        base = {c: self._effect_cols(frame, c) for c in self._x}
        cols, term_cols = [], {}
        for term in self._terms:
            parts = [base[c] for c in term]
            names = []
            for combo in itertools.product(*parts):
                nm = ":".join(n for n, _ in combo)
                val = combo[0][1]
                for _, t in combo[1:]:
                    val = val * t
                cols.append((nm, val))
                names.append(nm)
            term_cols[":".join(term)] = names
        vecs = [Vec(v.contiguous(), T_REAL) for _, v in cols]
        names = [n for n, _ in cols]
        if self._y in frame.names:
            vecs.append(frame.vec(self._y))
            names.append(self._y)
        if self._w and self._w in frame.names:
            vecs.append(frame.vec(self._w))
            names.append(self._w)
        return H2OFrame.from_vecs(vecs, names), term_cols

    def _fit(self, spec):
        p = self._parms
        self._x, self._y, self._w = list(spec.x), spec.y, spec.weights_column
        self._doms = {c: list(spec.frame.vec(c).domain) for c in self._x if spec.frame.vec(c).type == T_ENUM}
        # ANOVAGLM.java:105-121 init checks
        if len(self._x) < 2:
            raise ValueError("ERRR on field: predictors: there must be at least two predictors.")
        h = int(p.get("highest_interaction_term", 2))
        if h == 0:
            h = len(self._x)
        if h < 1 or h > len(self._x):
            raise ValueError("ERRR on field: highest_interaction_term: must be >= 1 or <= number of predictors.")
        if spec.nclasses > 2:
            raise ValueError("ERRR on field: family: multinomial and ordinal are not supported at this point.")
        if int(p.get("type", 3)) != 3:
            raise ValueError("type: only type III sums of squares are supported (as in the reference)")
        self._terms = [t for k in range(1, min(h, len(self._x)) + 1) for t in itertools.combinations(self._x, k)]
        tf, term_cols = self._transformed(spec.frame)
        all_cols = [c for t in term_cols.values() for c in t]
        fam = p.get("family") or "AUTO"

        def glm(xs):
            fw = {k: p[k] for k in _GLM_PASS if k in p}
            if not fw.get("max_iterations"):
                fw.pop("max_iterations", None)
            m = H2OGeneralizedLinearEstimator(family=fam, link=p.get("link"), lambda_=p.get("lambda_", 0.0),
                                              alpha=p.get("alpha", 0.0), standardize=p.get("standardize", True),
                                              compute_p_values=False, **fw)
            m.train(x=xs, y=self._y, training_frame=tf, weights_column=self._w)
            return m

        full = glm(all_cols)
        self._full = full
        dev_full = full.residual_deviance()
        n = tf.nrow
        res_df = n - len(all_cols) - 1
        rows = []
        gaussian = full._fam.family == "gaussian"
        for tname, tcols in term_cols.items():
            red = glm([c for c in all_cols if c not in tcols])
            ss = red.residual_deviance() - dev_full
            df = len(tcols)
            if gaussian:
                F = (ss / df) / (dev_full / res_df) if res_df > 0 and dev_full > 0 else float("nan")
                pv = float(stats.f.sf(F, df, res_df)) if F == F else float("nan")
            else:
                F = ss / df
                pv = float(stats.chi2.sf(ss, df))
            rows.append((tname, full._fam.family, full._fam.link, ss, df, F, pv))
        self._result = pd.DataFrame(rows, columns=["predictors_interactions", "family", "link", "ss", "df",
                                                   "f_values", "p_values"])
        self._output["result"] = self._result
        self._tf = tf if p.get("save_transformed_framekeys") else None

    def result(self):
        return H2OFrame(self._result)

    def summary(self):
        return self._result

    def _predict_raw(self, frame):
        tf, _ = self._transformed(frame)
        return self._full._predict_raw(tf)

    def _score_all(self, spec):
        self._training_metrics = self._full._training_metrics
