"""RuleFit (Friedman & Popescu 2008).

Reference: hex/rulefit/RuleFit.java, RuleFitModel.java, Rule.java,
Condition.java, RuleEnsemble.java (tree ensembles of depths
min_rule_length..max_rule_length generate candidate rules -- every
leaf is the conjunction of the (merged) conditions on its path -- rules
become 0/1 features, optional linear terms are added, a sparse (lasso)
GLM selects rules; rule_importance lists coefficient, support and rule
text; remove_duplicates drops rules with identical support patterns).

MI355X design: rule features are never evaluated condition-by-condition:
the scoring kernel gives the leaf of every row in every tree, and a rule
(a leaf's path) indicator is "the row's leaf is this leaf" -- one gather
through a per-tree identity table.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_ENUM, T_INT, T_REAL, Vec
from ..parallel import cloud
from .base import H2OEstimator

RULEFIT_DEFAULTS = dict(algorithm="AUTO", min_rule_length=3, max_rule_length=3, max_num_rules=-1,
                        model_type="RULES_AND_LINEAR", rule_generation_ntrees=50, remove_duplicates=True,
                        lambda_=None, distribution="AUTO", seed=-1, weights_column=None, max_categorical_levels=10)


def _cond_text(tree, j, left, names, domains):
    f = names[tree.feat[j]]
    na = tree.na_left[j] == left
    if tree.is_cat[j] and tree.cat_left[j] is not None:
        dom = domains.get(f, [])
        mask = tree.cat_left[j]
        lv = [dom[i] for i in range(min(len(dom), len(mask))) if bool(mask[i]) == left]
        s = f"({f} in {{{', '.join(map(str, lv))}}}"
    else:
        s = f"({f} {'<' if left else '>='} {float(tree.thr[j]):.6g}"
    return s + (f" or {f} is NA)" if na else ")")


class H2ORuleFitEstimator(H2OEstimator):
    algo = "rulefit"
    _defaults = RULEFIT_DEFAULTS

    def _wants_categorical_response(self):
        return str(self._parms.get("distribution") or "").lower() in ("bernoulli", "multinomial")

    def _tree_models(self, spec):
        from .tree.drf import H2ORandomForestEstimator
        from .tree.gbm import H2OGradientBoostingEstimator
        p = self._parms
        algo = str(p.get("algorithm") or "AUTO").upper()
        lo, hi = int(p.get("min_rule_length", 3)), int(p.get("max_rule_length", 3))
        if lo > hi:                                        # RuleFitModel.java:79
            raise ValueError(f"min_rule_length cannot be greater than max_rule_length. Current values:  "
                             f"min_rule_length = {lo}, max_rule_length = {hi}.")
        depths = list(range(lo, hi + 1))
        nt = max(1, int(p.get("rule_generation_ntrees", 50)) // len(depths))
        seed = p.get("seed", -1)
        models = []
        for d in depths:
            kw = dict(ntrees=nt, max_depth=d, seed=seed if seed not in (-1, None) else 1234 + d)
            if algo == "GBM":
                m = H2OGradientBoostingEstimator(**kw, learn_rate=0.1)
            else:
                m = H2ORandomForestEstimator(**kw)
            m.train(x=list(spec.x), y=spec.y, training_frame=spec.frame, weights_column=spec.weights_column)
            models.append(m)
        return models

    def _rules(self):
        """Rules = tree LEAVES (Rule.extractRulesFromTree): the conjunction of
        the path's conditions with conditions on one feature and operator
        merged (thresholds tightened, level sets intersected; NA matches only
        if every merged condition admits it), sorted by feature name, named
        M<model>T<tree>N<node> -- plus _<class> for the per-class trees of a
        multinomial ensemble (Rule.java:107-118, the tree number counting
        iterations).  Returns (model idx, tree idx, leaf id, text,
        #conditions, varname, [(feature, op, threshold or level codes, NA)],
        forest position, class idx or None)."""
        out = []
        sp = self._spec
        classes = list(sp.response_domain) if sp.nclasses > 2 else None
        for mi, m in enumerate(self._trees):
            names = list(m._spec.x)
            doms = getattr(m, "_x_domains", {})
            K = m._n_tree_classes() if classes else 1
            for ft, t in enumerate(m._forest.trees):
                ti, kc = (ft // K, int(m._forest.tclass[ft])) if classes else (ft, None)
                left = np.asarray(t.left)
                right = np.asarray(t.right)
                par = {}
                for j in range(len(left)):
                    if left[j] >= 0:
                        par[int(left[j])] = (j, True)
                        par[int(right[j])] = (j, False)
                for leaf in range(len(left)):
                    if left[leaf] >= 0:
                        continue
                    conds = {}
                    k = leaf
                    while k in par:
                        j, is_left = par[k]
                        f = names[t.feat[j]]
                        na = bool(t.na_left[j] == is_left)
                        if t.is_cat[j] and t.cat_left[j] is not None:
                            mask = t.cat_left[j]
                            dom = doms.get(f, [])
                            lv = {i for i in range(len(dom)) if i < len(mask) and bool(mask[i]) == is_left}
                            key = (f, "in")
                            if key in conds:
                                conds[key] = (conds[key][0] & lv, conds[key][1] and na)
                            else:
                                conds[key] = (lv, na)
                        else:
                            op = "<" if is_left else ">="
                            thr = float(t.thr[j])
                            key = (f, op)
                            if key in conds:
                                old = conds[key][0]
                                thr = min(old, thr) if op == "<" else max(old, thr)
                                conds[key] = (thr, conds[key][1] and na)
                            else:
                                conds[key] = (thr, na)
                        k = j
                    parts, struct = [], []
                    for (f, op), (v, na) in sorted(conds.items(), key=lambda kv: kv[0]):
                        struct.append((f, op, sorted(v) if op == "in" else v, na))
                        if op == "in":
                            dom = doms.get(f, [])
                            s_ = f"({f} in {{{', '.join(str(dom[i]) for i in sorted(v))}}}"
                        else:
                            s_ = f"({f} {op} {v:.6g}"
                        parts.append(s_ + (f" or {f} is NA)" if na else ")"))
                    vn = f"M{mi}T{ti}N{leaf}" + (f"_{classes[kc]}" if classes else "")
                    out.append((mi, ti, leaf, " & ".join(parts), len(parts), vn, struct, ft, kc))
        return out

    def _rule_matrix(self, frame):
        cols = []
        for mi, m in enumerate(self._trees):
            X = m._score_matrix(frame)
            leaf = m._forest.predict(X, m._n_tree_classes(), leaf=True).long()   # [n, T]
            for ti, t in enumerate(m._forest.trees):
                anc = self._anc[(mi, ti)]                                          # [n_nodes, n_nodes] bool
                cols.append(anc[leaf[:, ti]])                                      # [n, n_nodes]
        full = torch.cat(cols, 1) if cols else torch.zeros((frame.nlocal, 0), dtype=torch.bool)
        return full[:, self._keep_cols]

    def _fit(self, spec):
        from .glm.glm import H2OGeneralizedLinearEstimator
        p = self._parms
        self._trees = self._tree_models(spec)
        # ancestor tables: anc[leaf, node] = node on the path root->leaf
        self._anc = {}
        offsets = []
        base = 0
        for mi, m in enumerate(self._trees):
            for ti, t in enumerate(m._forest.trees):
                nn = t.n_nodes
                # a row satisfies exactly one rule per tree: its leaf's
                A = torch.eye(nn, dtype=torch.bool)
                self._anc[(mi, ti)] = A.to(cloud.device())
                offsets.append((mi, ti, base, nn))
                base += nn
        rules = self._rules()
        col_of = {(mi, ti): b for mi, ti, b, _ in offsets}
        idx = [col_of[(r[0], r[7])] + r[2] for r in rules]
        self._keep_cols = torch.as_tensor(idx, dtype=torch.long, device=cloud.device())
        R = self._rule_matrix(spec.frame)
        texts = [r[3] for r in rules]
        varnames = [r[5] for r in rules]
        if p.get("remove_duplicates", True) and R.shape[1]:
            # identical support patterns (hash of the packed column) -> keep the shortest rule
            Rh = R.to(torch.float64)
            g = torch.Generator(device="cpu").manual_seed(7)
            g.manual_seed(7 + 1000003 * cloud.rank())
            proj = Rh.T @ torch.rand(R.shape[0], 2, generator=g, dtype=torch.float64).to(Rh.device)
            from ..parallel import collectives as coll
            coll.allreduce_(proj)  # same keys on every rank
            keys = [(round(float(a), 9), round(float(b), 9)) for a, b in proj.cpu().tolist()]
            seen = {}
            for i, k in enumerate(keys):
                if k not in seen or rules[i][4] < rules[seen[k]][4]:
                    seen[k] = i
            keep = sorted(seen.values())
            R = R[:, keep]
            texts = [texts[i] for i in keep]
            varnames = [varnames[i] for i in keep]
            self._keep_cols = self._keep_cols[torch.as_tensor(keep, device=self._keep_cols.device)]
        self._rule_texts = texts
        mtype = str(p.get("model_type") or "RULES_AND_LINEAR").upper()
        self._rule_names = list(varnames)
        fr = self._design(spec.frame, R, mtype)
        glm_kw = dict(alpha=1.0, lambda_search=p.get("lambda_") is None, seed=p.get("seed", -1))
        if p.get("lambda_") is not None:
            glm_kw["lambda_"] = p["lambda_"]
        dist = str(p.get("distribution") or "AUTO").lower()
        if spec.nclasses == 2:
            glm_kw["family"] = "binomial"
        elif spec.nclasses > 2:
            glm_kw["family"] = "multinomial"
        elif dist not in ("auto", "gaussian"):
            glm_kw["family"] = dist
        mnr = int(p.get("max_num_rules", -1) or -1)
        if mnr > 0:
            # RuleFit.java:228: the Lasso path stops once more than
            # max_num_rules + 1 predictors are active
            glm_kw["max_active_predictors"] = mnr + 1
            glm_kw["lambda_search"] = True
            glm_kw.pop("lambda_", None)
        self._glm = H2OGeneralizedLinearEstimator(**glm_kw)
        xs = [c for c in fr.names if c != spec.y]
        self._glm.train(x=xs, y=spec.y, training_frame=fr)
        self._mtype = mtype
        # rule importance table
        coef = self._glm.coef() if spec.nclasses <= 2 else {}
        rows = []
        sup = R.to(torch.float64).mean(0).cpu().numpy() if R.shape[1] else np.zeros(0)
        if spec.nclasses > 2:
            # multinomial: a rule's coefficient in the linear model of its own
            # tree's class (RuleFitUtils.getRules strips the class suffix)
            tabs = self._glm._output.get("coefficients_table_multinomials", {})
            cls_of = {r[5]: r[8] for r in rules}
            dom = list(spec.response_domain)
            for i, nm in enumerate(self._rule_names):
                c = float(tabs.get(dom[cls_of[nm]], {}).get(nm, 0.0))
                if c != 0.0:
                    rows.append((nm, c, float(sup[i]), texts[i]))
        for i, nm in enumerate(self._rule_names if spec.nclasses <= 2 else []):
            c = coef.get(nm, 0.0)
            if c != 0.0:
                rows.append((nm, c, float(sup[i]), texts[i]))
        if mtype != "RULES":
            for x in spec.x:
                for k, v in coef.items():
                    if (k == f"linear.{x}" or k.startswith(f"linear.{x}.")) and v != 0.0:
                        rows.append((k, v, 1.0, k))
        rows.sort(key=lambda r: -abs(r[1]))
        self._output["rule_importance"] = pd.DataFrame(rows, columns=["variable", "coefficient", "support", "rule"])

    def _design(self, frame, R, mtype):
        vecs, names = [], []
        if mtype in ("RULES_AND_LINEAR", "RULES"):
            for i in range(R.shape[1]):
                vecs.append(Vec(R[:, i].to(torch.float32).contiguous(), T_INT))
                names.append(self._rule_names[i])
        if mtype in ("RULES_AND_LINEAR", "LINEAR"):
            for x in self._spec.x:
                v = frame.vec(x)
                vecs.append(v)
                names.append(f"linear.{x}")
        if self._spec.y in frame.names:
            vecs.append(frame.vec(self._spec.y))
            names.append(self._spec.y)
        return H2OFrame.from_vecs(vecs, names)

    def rule_importance(self):
        return self._output["rule_importance"]

    def predict_rules(self, frame, rule_ids):
        R = self._rule_matrix(frame)
        pos = {n: i for i, n in enumerate(self._rule_names)}
        ids = [pos[r] for r in rule_ids]
        return H2OFrame.from_vecs([Vec(R[:, i].to(torch.float32).contiguous(), T_INT) for i in ids], list(rule_ids))

    def _predict_raw(self, frame):
        R = self._rule_matrix(frame)
        fr = self._design(frame, R, self._mtype)
        return self._glm._predict_raw(fr)
