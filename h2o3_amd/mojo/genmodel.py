"""Standalone MOJO scorer (numpy only — no torch, no GPU, no cluster).

Reference: h2o-genmodel (hex/genmodel/MojoModel.java, ModelMojoReader.java,
algos/*/ *MojoModel.score0, easy/EasyPredictModelWrapper.java).  Load a
MOJO zip written by h2o3_amd.mojo.writer and score pandas DataFrames or
row dicts: categorical values are mapped through the stored domains
(unseen levels -> NA, like the reference's adaptation), numeric NA = NaN.
"""
from __future__ import annotations

import io
import json
import math
import zipfile

import numpy as np


def scoring_names(domain):
    """Prediction columns (hex/Model.java makeScoringNames): "predict", then
    one probability column per class, integer labels prefixed with "p"."""
    out = ["predict"]
    for d in domain:
        d = str(d)
        t = d[1:] if d[:1] in "+-" else d
        out.append("p" + d if t.isdigit() and -2**31 <= int(d) < 2**31 else d)
    return out


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def _softmax(z):
    z = z - z.max(1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(1, keepdims=True)



def _glrm_impute(name, u):
    """GlrmLoss.impute of a numeric loss."""
    n = name.lower()
    if n == "poisson":
        return np.exp(u)
    if n in ("logistic", "hinge"):
        return (u > 0).astype(np.float64)
    return u


def _glrm_mimpute(multi_loss, U):
    """GlrmLoss.mimpute: argmax (Categorical) or the first level minimising
    the ordinal loss (Ordinal)."""
    if multi_loss.lower() != "ordinal" or U.shape[1] <= 1:
        return U.argmax(1)
    w = U.shape[1]
    loss = np.concatenate([np.zeros((U.shape[0], 1)), -np.cumsum(np.minimum(U[:, :w - 1], 1.0), 1)], 1)
    best = np.zeros(U.shape[0], dtype=np.int64)
    bl = loss[:, 0].copy()
    for a in range(1, w):
        b = loss[:, a] < bl
        best[b] = a
        bl[b] = loss[b, a]
    return best

class MojoModel:
    def __init__(self, zbytes):
        self._z = zipfile.ZipFile(io.BytesIO(zbytes))
        self.meta = json.loads(self._z.read("model.json"))
        self.info = {}
        sec = None
        for line in self._z.read("model.ini").decode().splitlines():
            line = line.strip()
            if line.startswith("["):
                sec = line
            elif sec == "[info]" and "=" in line:
                k, v = line.split("=", 1)
                self.info[k.strip()] = v.strip()
        self.algo = self.meta["algo"]
        self.details = json.loads(self._z.read("experimental/modelDetails.json")) \
            if "experimental/modelDetails.json" in self._z.namelist() else None
        self._arr = {}
        for n in self._z.namelist():
            if n.startswith("arrays/") and n.endswith(".npy"):
                self._arr[n[7:-4]] = np.load(io.BytesIO(self._z.read(n)), allow_pickle=False)
        self.nclasses = int(self.meta.get("nclasses", 1))
        self.response_domain = self.meta.get("response_domain")
        if self.algo == "stackedensemble":
            self._base = [MojoModel(self._z.read(f"models/{i}.zip")) for i in range(len(self.meta["base"]))]
            self._meta_model = MojoModel(self._z.read("models/meta.zip"))
        if self.algo == "rulefit":
            self._rf_trees = [MojoModel(self._z.read(f"models/tree_{i}.zip"))
                              for i in range(len(self.meta["rf_trees"]))]
            self._rf_glm = MojoModel(self._z.read("models/glm.zip"))

    @staticmethod
    def load(path):
        """Load a MOJO: this platform's layout (model.json + arrays/), or the
        reference's h2o-genmodel layout (model.ini + trees/ / domains/ ...,
        zip or unpacked directory) via mojo.h2o_mojo."""
        from . import h2o_mojo
        if h2o_mojo.is_h2o_layout(path):
            return h2o_mojo.H2OMojoModel(path)
        with open(path, "rb") as f:
            return MojoModel(f.read())

    # ---------------------------------------------------------------- inputs
    def _col(self, df, c, dom=None):
        if c not in df:
            return np.full(len(df), np.nan)
        s = df[c]
        if dom is not None:
            idx = {d: i for i, d in enumerate(dom)}
            out = np.full(len(s), np.nan)
            for i, v in enumerate(s.values if hasattr(s, "values") else s):
                if v is None or (isinstance(v, float) and math.isnan(v)):
                    continue
                key = v if isinstance(v, str) else (str(int(v)) if float(v).is_integer() else str(v))
                j = idx.get(key, idx.get(str(v)))
                if j is not None:
                    out[i] = j
            return out
        return np.asarray(s, dtype=np.float64)

    def _tree_matrix(self, df):
        xd = self.meta.get("x_domains", {})
        return np.stack([self._col(df, c, xd.get(c)) for c in self.meta["x"]], 1) if self.meta["x"] else \
            np.zeros((len(df), 0))

    def _interactions(self, df, recipe):
        """Replay the GLM interaction recipe (models/glm/interactions.py) on a
        pandas frame."""
        import pandas as pd
        df = df.copy()
        for r in recipe:
            a, b = df.get(r["a"]), df.get(r["b"])
            if r["kind"] == "nn":
                df[r["name"]] = pd.to_numeric(a, errors="coerce").astype(float) * \
                    pd.to_numeric(b, errors="coerce").astype(float)
            elif r["kind"] == "cc":
                lv = set(r["levels"])
                vals = [f"{x}_{y}" if x is not None and y is not None and f"{x}_{y}" in lv else None
                        for x, y in zip(a.astype(object).where(a.notna(), None).map(self._lvl),
                                        b.astype(object).where(b.notna(), None).map(self._lvl))]
                df[r["name"]] = vals
            else:
                xv = pd.to_numeric(b, errors="coerce").astype(float).fillna(0.0).values
                av = a.astype(object).where(a.notna(), None).map(self._lvl)
                for lvl in r["levels"]:
                    df[f"{r['name']}.{lvl}"] = np.where(av == lvl, xv, 0.0)
        return df

    def _gam_columns(self, df):
        """Smoother columns <col>_<cr|tp|is|ms>_<i> from the stored knots and
        centering matrices (mojo/gam_np.py)."""
        from .gam_np import basis, tp_basis
        g = self.meta["gam"]
        suf = {0: "cr", 1: "tp", 2: "is", 3: "ms"}
        df = df.copy()
        for gi, c in enumerate(g["cols"]):
            if g["bs"][gi] == 1:
                cc_ = list(c) if isinstance(c, (list, tuple)) else [c]
                Xm = np.stack([np.where(np.isnan(self._col(df, cc)), g["means"][cc], self._col(df, cc))
                               for cc in cc_], 1)
                t = g["tp"][str(gi)]
                Xc = tp_basis(Xm, g["knots"][gi], self._arr[f"gamZcs{gi}"], t["terms"], t["means"], t["ostd"],
                              t["standardize"]) @ self._arr[f"gamZ{gi}"]
                name = "_".join(cc_) if isinstance(c, (list, tuple)) else c
            else:
                x = self._col(df, c)
                x = np.where(np.isnan(x), g["means"][c], x)
                Xc = basis(x, g["bs"][gi], g["knots"][gi], g["orders"][gi]) @ self._arr[f"gamZ{gi}"]
                name = c
            for i in range(Xc.shape[1]):
                df[f"{name}_{suf[g['bs'][gi]]}_{i}"] = Xc[:, i].astype(np.float32).astype(np.float64)
        return df

    @staticmethod
    def _lvl(v):
        if v is None:
            return None
        if isinstance(v, float) and v.is_integer():
            return str(int(v))
        return str(v)

    def _expand(self, df):
        di = self.meta["di"]
        if di.get("ia"):
            df = self._interactions(df, di["ia"])
        n = len(df)
        X = np.zeros((n, di["P"]))
        for c in di["cat_cols"]:
            codes = self._col(df, c, di["domains"][c])
            codes = np.where(np.isnan(codes), di["cat_modes"][c], codes).astype(int)
            if not di["use_all"]:
                codes = codes - 1
            ok = codes >= 0
            X[np.nonzero(ok)[0], di["cat_offsets"][c] + codes[ok]] = 1.0
        base = sum(len(d) if di["use_all"] else len(d) - 1 for d in (di["domains"][c] for c in di["cat_cols"]))
        for j, c in enumerate(di["num_cols"]):
            x = self._col(df, c)
            x = np.where(np.isnan(x), di["plug"][j], x)
            if di["standardize"]:
                x = (x - di["means"][j]) / di["sigmas"][j]
            X[:, base + j] = x
        return X

    # ---------------------------------------------------------------- scoring
    def _leaves(self, X):
        """Terminal node id of every row in every tree: [n, T]."""
        A = self._arr
        feat, thr, left, right = A["forest_feat"], A["forest_thr"], A["forest_left"], A["forest_right"]
        nal, coff, clen, bits = A["forest_na_left"], A["forest_cat_off"], A["forest_cat_len"], A["forest_cat_bits"]
        roots = A["forest_roots"]
        n = X.shape[0]
        ar = np.arange(n)
        out = np.zeros((n, len(roots)), dtype=np.int64)
        for t in range(len(roots)):
            nd = np.full(n, roots[t])
            while True:
                l = left[nd]
                act = l >= 0
                if not act.any():
                    break
                x = X[ar, feat[nd]]
                isn = np.isnan(x)
                co = coff[nd]
                code = np.where(isn, -1, np.nan_to_num(x, nan=-1)).astype(np.int64)
                inr = (code >= 0) & (code < clen[nd])
                bit = bits[np.clip(co + np.maximum(code, 0), 0, len(bits) - 1)] != 0
                gocat = np.where(isn | ~inr, nal[nd] != 0, bit)
                gonum = np.where(isn, nal[nd] != 0, x.astype(np.float32) < thr[nd].astype(np.float32))
                go = np.where(co >= 0, gocat, gonum)
                nd = np.where(act, np.where(go, l, right[nd]), nd)
            out[:, t] = nd - roots[t]
        return out

    def _forest(self, X, K, leaf=False):
        A = self._arr
        feat, thr, left, right = A["forest_feat"], A["forest_thr"], A["forest_left"], A["forest_right"]
        nal, coff, clen, bits, val = A["forest_na_left"], A["forest_cat_off"], A["forest_cat_len"], \
            A["forest_cat_bits"], A["forest_value"]
        roots, tcls = A["forest_roots"], A["forest_tclass"]
        n = X.shape[0]
        out = np.zeros((n, K))
        ar = np.arange(n)
        for t in range(len(roots)):
            nd = np.full(n, roots[t])
            while True:
                l = left[nd]
                act = l >= 0
                if not act.any():
                    break
                x = X[ar, feat[nd]]
                isn = np.isnan(x)
                co = coff[nd]
                code = np.where(isn, -1, np.nan_to_num(x, nan=-1)).astype(np.int64)
                inr = (code >= 0) & (code < clen[nd])
                bit = bits[np.clip(co + np.maximum(code, 0), 0, len(bits) - 1)] != 0
                gocat = np.where(isn | ~inr, nal[nd] != 0, bit)
                # split values are f32 and compared in f32 (reference: float split points)
                gonum = np.where(isn, nal[nd] != 0, x.astype(np.float32) < thr[nd].astype(np.float32))
                go = np.where(co >= 0, gocat, gonum)
                nd = np.where(act, np.where(go, l, right[nd]), nd)
            out[ar, tcls[t]] += val[nd]
        return out

    # ------------------------------------------------------------ contributions
    def _node_left(self, j, X):
        """Split decision of packed node j for every row of X (the scoring
        walk's rule: f32 thresholds, categorical level bitsets, NA direction)."""
        A = self._arr
        x = X[:, int(A["forest_feat"][j])]
        isn = np.isnan(x)
        nal = A["forest_na_left"][j] != 0
        co = int(A["forest_cat_off"][j])
        if co >= 0:
            code = np.where(isn, -1, np.nan_to_num(x, nan=-1)).astype(np.int64)
            inr = (code >= 0) & (code < A["forest_cat_len"][j])
            bits = A["forest_cat_bits"]
            bit = bits[np.clip(co + np.maximum(code, 0), 0, len(bits) - 1)] != 0
            return np.where(isn | ~inr, nal, bit)
        return np.where(isn, nal, x.astype(np.float32) < np.float32(A["forest_thr"][j]))

    def predict_contributions(self, df, output_format="Original", top_n=None, bottom_n=None, compare_abs=False):
        """TreeSHAP feature contributions of a GBM / DRF / XGBoost MOJO (the
        reference's EasyPredictModelWrapper.predictContributions /
        PredictContributions): one column per feature plus BiasTerm, in link
        space (GBM / XGBoost: the row sum is the raw margin incl. init_f; DRF
        binomial: the reference's 1/(F+1) - contribution(P(class 0)) form,
        summing to P(class 1))."""
        from .treeshap_np import contributions_frame, tree_shap
        m = self.meta
        if self.algo not in ("gbm", "drf", "xgboost"):
            raise ValueError(f"contributions are not available for a {self.algo} MOJO")
        if self.nclasses > 2:
            raise ValueError("Calculating contributions is currently not supported for multinomial models.")
        A = self._arr
        if "forest_weight" not in A:
            raise ValueError("this MOJO carries no node weights (written before contributions were supported)")
        if m.get("catenc") and not getattr(df, "_catenc_done", False):
            df = encode_df(df, m["catenc"])
        X = self._tree_matrix(df)
        n, F = X.shape
        roots, tcls = A["forest_roots"], A["forest_tclass"]
        left, right, val, cov, feat = A["forest_left"], A["forest_right"], A["forest_value"], \
            A["forest_weight"], A["forest_feat"]
        phi = np.zeros((n, F + 1))
        trees = [t for t in range(len(roots)) if tcls[t] == 0]
        scale = 1.0 / max(1, len(trees)) if self.algo == "drf" else 1.0
        for t in trees:
            tree_shap(left, right, cov, val, feat, lambda j: self._node_left(j, X), n, phi, scale=scale,
                      root=int(roots[t]))
        if self.algo in ("gbm", "xgboost"):
            phi[:, -1] += float(np.asarray(m["init_f"]).reshape(-1)[0])
        elif self.nclasses == 2:
            phi[:, :-1] += 1.0 / (F + 1)
            phi[:, -1] += 1.0 / (F + 1) - 1.0
        return contributions_frame(phi, list(m["x"]), top_n=top_n, bottom_n=bottom_n, compare_abs=compare_abs)

    def predict_raw(self, df):
        m = self.meta
        a = self.algo
        if m.get("catenc") and not getattr(df, "_catenc_done", False):
            df = encode_df(df, m["catenc"])
        if a in ("gbm", "xgboost"):
            X = self._tree_matrix(df)
            K = m["K"]
            f = self._forest(X, K) + np.asarray(m["init_f"]).reshape(1, -1)
            if K > 1:
                return _softmax(f)
            link = m["link"]
            mu = _sigmoid(f[:, 0]) if link == "logit" else (np.exp(f[:, 0]) if link == "log" else f[:, 0])
            return np.stack([1 - mu, mu], 1) if self.nclasses == 2 else mu.reshape(-1, 1)
        if a == "drf":
            X = self._tree_matrix(df)
            K = m["K"]
            s = self._forest(X, K) / max(1, m["ntrees"] // K)
            if self.nclasses == 2 and m["binomial_single"]:
                p1 = np.clip(s[:, 0], 0, 1)
                return np.stack([1 - p1, p1], 1)
            if self.nclasses > 1:
                s = np.clip(s, 0, None)
                return s / np.maximum(s.sum(1, keepdims=True), 1e-30)
            return s[:, :1]
        if a == "isolationforest":
            X = self._tree_matrix(df)
            ml = self._forest(X, 1)[:, 0] / m["ntrees"]
            rng = m["max_len"] - m["min_len"]
            sc = (m["max_len"] - ml) / rng if rng > 0 else np.zeros_like(ml)
            return np.stack([sc, ml], 1)
        if a == "rulefit":
            import pandas as pd
            cols = []
            for mi, tm in enumerate(self._rf_trees):
                leaves = tm._leaves(tm._tree_matrix(df))
                for ti in range(m["rf_trees"][mi]):
                    cols.append(self._arr[f"anc_{mi}_{ti}"][leaves[:, ti]])
            R = np.concatenate(cols, 1)[:, self._arr["keep_cols"]] if cols else np.zeros((len(df), 0))
            d = {}
            if m["mtype"] in ("RULES_AND_LINEAR", "RULES"):
                for i, nm in enumerate(m["rule_names"]):
                    d[nm] = R[:, i].astype(np.float64)
            if m["mtype"] in ("RULES_AND_LINEAR", "LINEAR"):
                for x in m["x"]:
                    d[f"linear.{x}"] = df[x].values if x in df else np.full(len(df), np.nan)
            return self._rf_glm.predict_raw(pd.DataFrame(d))
        if a == "gam":
            df = self._gam_columns(df)
            a = "glm"
        if a == "glm":
            X = self._expand(df)
            if m.get("multi") == "multinomial":
                return _softmax(X @ self._arr["B"] + self._arr["b0"].reshape(1, -1))
            if m.get("multi") == "ordinal":
                eta = X @ self._arr["beta"]
                th = self._arr["theta"]
                thc = np.cumsum(np.concatenate([th[:1], np.log1p(np.exp(th[1:]))]))
                cdf = _sigmoid(thc.reshape(1, -1) - eta.reshape(-1, 1))
                cdf = np.concatenate([np.zeros((len(eta), 1)), cdf, np.ones((len(eta), 1))], 1)
                return np.clip(np.diff(cdf, axis=1), 0, None)
            b = self._arr["beta_std"]
            eta = X @ b[:-1] + b[-1]
            link = m["link"]
            if link == "logit":
                mu = _sigmoid(eta)
            elif link == "log":
                mu = np.exp(eta)
            elif link == "inverse":
                mu = 1.0 / eta
            else:
                mu = eta
            return np.stack([1 - mu, mu], 1) if self.nclasses == 2 else mu.reshape(-1, 1)
        if a == "glrm":
            return self._glrm_reconstruct(df)
        if a == "kmeans":
            X = self._expand(df)
            nc = sum(len(d) if self.meta["di"]["use_all"] else len(d) - 1
                     for d in (self.meta["di"]["domains"][c] for c in self.meta["di"]["cat_cols"]))
            X[:, :nc] *= float(m.get("cat_scale", 1.0))
            C = self._arr["centers_std"]
            d = ((X[:, None, :] - C[None]) ** 2).sum(2)
            return d.argmin(1).reshape(-1, 1).astype(float)
        if a == "pca":
            X = self._expand(df)
            return (X - self._arr["mean"]) @ self._arr["evecs"]
        if a == "deeplearning":
            h = self._expand(df)
            for L in m["layers"]:
                kind, i = L[0], L[1]
                if kind == "linear":
                    h = h @ self._arr[f"W{i}"].T + self._arr[f"b{i}"]
                elif kind == "maxout":
                    z = h @ self._arr[f"W{i}"].T + self._arr[f"b{i}"]
                    h = z.reshape(len(h), -1, L[2]).max(2)
                elif kind == "tanh":
                    h = np.tanh(h)
                elif kind == "relu":
                    h = np.maximum(h, 0)
                elif kind == "elu":
                    h = np.where(h > 0, h, np.expm1(h))
                elif kind == "scale":
                    h = h * L[2]
            if m["autoencoder"]:
                return h
            if m["K"] > 1:
                return _softmax(h)
            return h * m["ysd"] + m["ymu"]
        if a == "naivebayes":
            n = len(df)
            logp = np.log(np.maximum(self._arr["prior"], 1e-300))[None].repeat(n, 0)
            nbp = m["nb_params"]
            for c, spec in m["nb"].items():
                if spec[0] == "cat":
                    codes = self._col(df, c, spec[2])
                    pr = self._arr[f"nb_{spec[1]}"].T[np.nan_to_num(codes, nan=0).astype(int)]
                    pr = np.where(pr <= nbp["eps_prob"], nbp["min_prob"], pr)
                    contrib = np.where(np.isnan(codes)[:, None], 0.0, np.log(np.maximum(pr, 1e-300)))
                else:
                    x = self._col(df, c)
                    mean, sd = self._arr[f"nb_{spec[1]}_mean"], self._arr[f"nb_{spec[1]}_sd"]
                    sd = np.where(sd <= nbp["eps_sdev"], nbp["min_sdev"], sd)
                    z = (x[:, None] - mean[None]) / sd[None]
                    contrib = np.where(np.isnan(x)[:, None], 0.0, -0.5 * z * z - np.log(sd[None] * math.sqrt(2 * math.pi)))
                logp = logp + contrib
            return _softmax(logp)
        if a == "extendedisolationforest":
            X = np.nan_to_num(self._expand(df))
            A = self._arr
            n = X.shape[0]
            tot = np.zeros(n)
            for r in A["eif_roots"]:
                nd = np.full(n, r)
                for _ in range(m["height"] + 1):
                    l = A["eif_left"][nd]
                    act = l >= 0
                    if not act.any():
                        break
                    proj = ((X - A["eif_point"][nd]) * A["eif_normal"][nd]).sum(1)
                    nd = np.where(act, np.where(proj <= 0, l, A["eif_right"][nd]), nd)
                tot += A["eif_value"][nd]
            ml = tot / m["ntrees"]
            psi = m["psi"]
            c = 0.0 if psi <= 1 else (1.0 if psi == 2 else 2.0 * (math.log(psi - 1) + 0.5772156649) - 2.0 * (psi - 1) / psi)
            return np.stack([np.power(2.0, -ml / c), ml], 1)
        if a == "isotonicregression":
            x = self._col(df, m["x"][0])
            tx, ty = self._arr["thresholds_x"], self._arr["thresholds_y"]
            p = np.interp(np.clip(x, tx[0], tx[-1]), tx, ty)
            if m["out_of_bounds"].lower() != "clip":
                p = np.where((x < tx[0]) | (x > tx[-1]), np.nan, p)
            return np.where(np.isnan(x), np.nan, p).reshape(-1, 1)
        if a == "coxph":
            X = self._expand(df)
            beta = self._arr["beta"]
            lp = X @ beta
            keys = list(self._arr["strata_keys"])
            means = self._arr["strata_means"]
            key = np.zeros(len(df), dtype=np.int64)
            for c in m["stratify_by"]:
                dom = m["strata_domains"].get(c)
                codes = self._col(df, c, dom) if dom is not None else np.asarray(df[c], dtype=float)
                codes = np.where(np.isnan(codes), -1, codes).astype(np.int64)
                key = key * ((len(dom) + 1) if dom else 1_000_003) + codes + 1
            base = np.array([means[keys.index(k)] @ beta if k in keys else np.nan for k in key])
            return (lp - base).reshape(-1, 1)
        if a == "upliftdrf":
            X = self._tree_matrix(df)
            s = self._forest(X, 2) / max(1, m["ntrees"])
            return np.stack([s[:, 0] - s[:, 1], s[:, 0], s[:, 1]], 1)
        if a == "word2vec":
            vocab = self._z.read("vocabulary.txt").decode().split("\n")
            idx = {w: i for i, w in enumerate(vocab)}
            V = self._arr["vectors"]
            col = df[df.columns[0]]
            out = np.full((len(col), V.shape[1]), np.nan)
            for i, wd in enumerate(col):
                j = idx.get(wd) if isinstance(wd, str) else None
                if j is not None:
                    out[i] = V[j]
            return out
        if a == "targetencoder":
            cols = []
            tp = m["te_params"]
            for c, t in m["te"].items():
                dom = t["domain"]
                codes = self._col(df, c, dom)
                codes = np.where(np.isnan(codes), len(dom), codes).astype(int)
                for k, suf in enumerate(m["suffix"]):
                    num, den = np.asarray(t["num"][k])[codes], np.asarray(t["den"][k])[codes]
                    prior = m["prior"][k]
                    mean = np.where(den > 0, num / np.where(den > 0, den, 1), prior)
                    if tp.get("blending"):
                        kk, ff = float(tp.get("inflection_point", 10)), float(tp.get("smoothing", 20))
                        lam = 1 / (1 + np.exp((kk - den) / ff))
                        mean = lam * mean + (1 - lam) * prior
                    cols.append(mean)
            return np.stack(cols, 1) if cols else np.zeros((len(df), 0))
        if a == "stackedensemble":
            import pandas as pd
            cols = {}
            names = m["level1_names"]
            j = 0
            for b in self._base:
                raw = b.predict_raw(df)
                if self.nclasses == 2:
                    cols[names[j]] = raw[:, -1]
                    j += 1
                elif self.nclasses > 2:
                    for k in range(raw.shape[1]):
                        cols[names[j]] = raw[:, k]
                        j += 1
                else:
                    cols[names[j]] = raw[:, 0]
                    j += 1
            if str(m.get("metalearner_transform", "NONE")).lower() == "logit" and self.nclasses >= 2:
                cols = {k: np.log(np.clip(v, 1e-9, 1 - 1e-9) / (1 - np.clip(v, 1e-9, 1 - 1e-9)))
                        for k, v in cols.items()}
            return self._meta_model.predict_raw(pd.DataFrame(cols))
        raise NotImplementedError(a)

    # ---------------------------------------------------------------- GLRM
    def _glrm_layout(self, df):
        g = self.meta["glrm"]
        mats, masks = [], []
        for kind, c, w in g["blocks"]:
            if kind == "cat":
                codes = self._col(df, c, g["doms"][c])
                ok = ~np.isnan(codes)
                oh = np.zeros((len(codes), w))
                oh[np.nonzero(ok)[0], codes[ok].astype(int)] = 1.0
                mats.append(oh)
                masks.append(np.repeat(ok.reshape(-1, 1), w, 1))
            else:
                x = self._col(df, c)
                mu, sd, lo, hi = g["stats"][c]
                tr = g["transform"]
                if tr == "STANDARDIZE":
                    x = (x - mu) / sd
                elif tr == "NORMALIZE":
                    x = (x - lo) / max(hi - lo, 1e-12)
                elif tr == "DEMEAN":
                    x = x - mu
                elif tr == "DESCALE":
                    x = x / sd
                masks.append((~np.isnan(x)).reshape(-1, 1))
                mats.append(np.nan_to_num(x).reshape(-1, 1))
        return np.concatenate(mats, 1), np.concatenate(masks, 1).astype(np.float64)

    def _glrm_loss_grad(self, A, M, U, want_grad=True):
        """Per-row loss and dLoss/dU (hex/genmodel/algos/glrm/GlrmLoss.java)."""
        g = self.meta["glrm"]
        tot = np.zeros(U.shape[0])
        G = np.zeros_like(U) if want_grad else None
        j = 0
        ml = g["multi_loss"].lower()
        for kind, c, w in g["blocks"]:
            a, m, u = A[:, j:j + w], M[:, j:j + w], U[:, j:j + w]
            if kind == "num":
                name = g["loss_by_col"].get(c, g["loss"]).lower()
                a, m, u = a[:, 0], m[:, 0], u[:, 0]
                d = u - a
                if name == "quadratic":
                    L, dL = d * d, 2 * d
                elif name == "absolute":
                    L, dL = np.abs(d), np.sign(d)
                elif name == "huber":
                    ad = np.abs(d)
                    L = np.where(ad <= 1, 0.5 * ad * ad, ad - 0.5)
                    dL = np.where(ad <= 1, d, np.sign(d))
                elif name == "poisson":
                    L = np.exp(u) - a * u + np.where(a > 0, a * np.log(np.maximum(a, 1e-300)) - a, 0.0)
                    dL = np.exp(u) - a
                elif name in ("hinge", "logistic"):
                    aa = np.where(a > 0, 1.0, -1.0)
                    if name == "hinge":
                        L = np.maximum(1 - aa * u, 0)
                        dL = np.where(1 - aa * u >= 0, -aa, 0.0)
                    else:
                        L = np.logaddexp(0, -aa * u)
                        dL = -aa / (1 + np.exp(aa * u))
                elif name == "periodic":
                    cc = 2 * math.pi / g["period"]
                    L = 1 - np.cos((a - u) * cc)
                    dL = -cc * np.sin((a - u) * cc)
                else:
                    raise ValueError(name)
                tot += L * m
                if want_grad:
                    G[:, j] = dL * m
            else:
                rowm = m[:, 0]
                if ml == "ordinal":
                    # GlrmLoss.Ordinal: sum_{i < w-1} (a > i ? max(1 - u_i, 0) : 1)
                    lvl = a.argmax(1).reshape(-1, 1)
                    ar = np.arange(w).reshape(1, -1)
                    below = ar < lvl
                    L = np.where(below, np.maximum(1 - u, 0), np.where(ar < w - 1, 1.0, 0.0))
                    dL = np.where(below & (1 - u >= 0), -1.0, 0.0)
                else:
                    below = a > 0
                    L = np.where(below, np.maximum(1 - u, 0), np.maximum(1 + u, 0))
                    dL = np.where(below, np.where(1 - u >= 0, -1.0, 0.0), np.where(1 + u >= 0, 1.0, 0.0))
                tot += L.sum(1) * rowm
                if want_grad:
                    G[:, j:j + w] = dL * rowm.reshape(-1, 1)
            j += w
        return tot, G

    @staticmethod
    def _glrm_reg(name, X):
        n = (name or "None").lower()
        if n == "quadratic":
            return (X * X).sum(1)
        if n == "l2":
            return np.sqrt((X * X).sum(1))
        if n == "l1":
            return np.abs(X).sum(1)
        return np.zeros(X.shape[0])

    @staticmethod
    def _glrm_prox(name, X, sg):
        n = (name or "None").lower()
        if n == "none":
            return X
        if n == "quadratic":
            return X / (1 + 2 * sg)
        if n == "l2":
            nr = np.maximum(np.sqrt((X * X).sum(1, keepdims=True)), 1e-300)
            return X * np.maximum(1 - sg / nr, 0)
        if n == "l1":
            return np.sign(X) * np.maximum(np.abs(X) - sg, 0)
        if n == "nonnegative":
            return np.maximum(X, 0)
        if n in ("onesparse", "unitonesparse"):
            idx = X.argmax(1)
            out = np.zeros_like(X)
            r = np.arange(X.shape[0])
            out[r, idx] = np.maximum(X[r, idx], 0) if n == "onesparse" else 1.0
            return out
        if n == "simplex":
            u = -np.sort(-X, 1)
            css = np.cumsum(u, 1) - 1
            ind = np.arange(1, X.shape[1] + 1)
            rho = ((u - css / ind) > 0).cumsum(1).argmax(1)
            theta = css[np.arange(X.shape[0]), rho] / (rho + 1)
            return np.maximum(X - theta.reshape(-1, 1), 0)
        raise ValueError(name)

    def _glrm_solve_x(self, A, M):
        """Per-row proximal gradient on x with Y fixed (same recurrence as the
        in-cluster GLRM predict: least-squares start, 1/(2||Y||^2) first step,
        x1.05 on improvement, /2 otherwise)."""
        g = self.meta["glrm"]
        Y = self._arr["Y"]
        k = Y.shape[0]
        rx, gx = g["regularization_x"], g["gamma_x"]
        Gm = Y @ Y.T + 1e-6 * np.eye(k)
        X = self._glrm_prox(rx, np.linalg.solve(Gm, Y @ (A * M).T).T, 0.0)
        n = X.shape[0]
        step = np.full((n, 1), 0.5 / max(float((Y * Y).sum()), 1e-12))
        obj = self._glrm_loss_grad(A, M, X @ Y, False)[0] + gx * self._glrm_reg(rx, X)
        live = np.ones(n, dtype=bool)
        for _ in range(int(g["iters"])):
            gX = self._glrm_loss_grad(A, M, X @ Y)[1] @ Y.T
            Xn = self._glrm_prox(rx, X - step * gX, step * gx)
            on = self._glrm_loss_grad(A, M, Xn @ Y, False)[0] + gx * self._glrm_reg(rx, Xn)
            better = (on < obj) & live
            rel = (obj - on) / np.maximum(np.abs(obj), 1e-300)
            X = np.where(better.reshape(-1, 1), Xn, X)
            obj = np.where(better, on, obj)
            step = np.where(better.reshape(-1, 1), step * 1.05, np.where(live.reshape(-1, 1), step / 2, step))
            live = live & ~(better & (rel < 1e-9)) & (step.reshape(-1) >= 1e-8)
            if not live.any():
                break
        return X

    def _glrm_reconstruct(self, df):
        A, M = self._glrm_layout(df)
        X = self._glrm_solve_x(A, M)
        self._glrm_x = X
        return X @ self._arr["Y"]

    def glrm_reconstruct(self, df):
        """DataFrame of reconstr_<col> like GLRM predict()/reconstruct()."""
        import pandas as pd
        g = self.meta["glrm"]
        U = self._glrm_reconstruct(df)
        out = {}
        j = 0
        for kind, c, w in g["blocks"]:
            u = U[:, j:j + w]
            if kind == "num":
                x = _glrm_impute(g["loss_by_col"].get(c, g["loss"]), u[:, 0].copy())
                if g["impute_original"]:
                    mu, sd, lo, hi = g["stats"][c]
                    tr = g["transform"]
                    if tr == "STANDARDIZE":
                        x = x * sd + mu
                    elif tr == "NORMALIZE":
                        x = x * (hi - lo) + lo
                    elif tr == "DEMEAN":
                        x = x + mu
                    elif tr == "DESCALE":
                        x = x * sd
                out[f"reconstr_{c}"] = x
            else:
                out[f"reconstr_{c}"] = np.array(g["doms"][c], dtype=object)[_glrm_mimpute(g["multi_loss"], u)]
            j += w
        return pd.DataFrame(out)

    def predict(self, df):
        """Returns a pandas DataFrame shaped like the in-cluster predict()."""
        import pandas as pd
        if self.algo == "glrm":
            return self.glrm_reconstruct(df)
        raw = self.predict_raw(df)
        if self.algo == "isolationforest":
            return pd.DataFrame({"predict": raw[:, 0], "mean_length": raw[:, 1]})
        if self.algo == "extendedisolationforest":
            return pd.DataFrame({"anomaly_score": raw[:, 0], "mean_length": raw[:, 1]})
        if self.algo == "coxph":
            return pd.DataFrame({"lp": raw[:, 0]})
        if self.algo == "upliftdrf":
            return pd.DataFrame(raw, columns=["uplift_predict", "p_y1_with_treatment", "p_y1_without_treatment"])
        if self.algo == "word2vec":
            return pd.DataFrame(raw, columns=[f"C{i + 1}" for i in range(raw.shape[1])])
        if self.algo == "targetencoder":
            names = [f"{c}{s}_te" for c in self.meta["te"] for s in self.meta["suffix"]]
            out = df.copy()
            for i, nm in enumerate(names):
                out[nm] = raw[:, i]
            return out
        if self.nclasses > 1 and self.response_domain:
            dom = self.response_domain
            if self.nclasses == 2:
                lab = np.where(raw[:, 1] >= 0.5, dom[1], dom[0])
            else:
                lab = np.array(dom, dtype=object)[raw.argmax(1)]
            out = {"predict": lab}
            for k, d in enumerate(scoring_names(dom)[1:]):
                out[d] = raw[:, k]
            return pd.DataFrame(out)
        if raw.shape[1] == 1:
            return pd.DataFrame({"predict": raw[:, 0]})
        return pd.DataFrame(raw, columns=[f"C{i + 1}" for i in range(raw.shape[1])])

    def predict_row(self, row: dict):
        import pandas as pd
        return self.predict(pd.DataFrame([row])).iloc[0].to_dict()


class EasyPredictModelWrapper:
    """h2o-genmodel's convenience wrapper (predictBinomial / predictRegression...).
    enable_contributions=True adds the row's TreeSHAP contributions to each
    prediction (EasyPredictModelWrapper.Config.setEnableContributions,
    EasyPredictModelWrapper.java:196); works with either MOJO layout."""

    def __init__(self, model, enable_contributions=False):
        self.m = model
        self.enable_contributions = bool(enable_contributions)

    def predict(self, row: dict):
        out = self.m.predict_row(row)
        if self.enable_contributions:
            out["contributions"] = self.predict_contributions(row)
        return out

    def predict_contributions(self, row: dict):
        """{feature: contribution, ..., "BiasTerm": bias} of one row."""
        import pandas as pd
        df = self.m.predict_contributions(pd.DataFrame([row]))
        return {k: float(v) for k, v in df.iloc[0].items()}


def load(path):
    return MojoModel.load(path)


def _level_index(v, pos):
    if v is None or (isinstance(v, float) and v != v):
        return -1
    if isinstance(v, str):
        return pos.get(v, -1)
    key = str(int(v)) if float(v).is_integer() else str(v)
    return pos.get(key, pos.get(str(v), -1))


def encode_df(df, d):
    """The model's categorical_encoding on a pandas frame (the numpy twin of
    models/catenc.py CategoricalEncoder.transform; h2o-genmodel
    CategoricalEncoding)."""
    import pandas as pd
    sch = d["scheme"]
    out, exp = {}, {}
    for c in df.columns:
        st = d["cols"].get(c)
        if st is None or c not in d["x_in"]:
            out[c] = df[c].values
            continue
        dom = st["domain"]
        L = len(dom)
        pos = {v: i for i, v in enumerate(dom)}
        codes = np.array([_level_index(v, pos) for v in df[c].tolist()], dtype=np.int64)
        if sch == "OneHotExplicit":
            idx = np.where(codes < 0, L, codes)
            for j, nm in enumerate([f"{c}.{x}" for x in dom] + [f"{c}.missing(NA)"]):
                exp[nm] = (idx == j).astype(np.float64)
        elif sch == "Binary":
            val = np.where(codes < 0, 0, codes + 1)
            nb = 1 + int(np.floor(np.log2(L))) if L > 0 else 1
            for k in range(nb):
                exp[f"{c}:{k}"] = ((val >> k) & 1).astype(np.float64)
        elif sch == "LabelEncoder":
            out[c] = np.where(codes < 0, np.nan, codes.astype(np.float64))
        elif sch == "EnumLimited":
            if not st.get("limited"):
                out[c] = df[c].values
            else:
                lut = np.asarray(st["lut"], dtype=np.int64)
                nc = lut[np.where(codes < 0, L, codes)]
                nd = np.array(list(st["new_domain"]) + [None], dtype=object)
                out[st["name"]] = nd[np.where(nc < 0, len(nd) - 1, nc)]
        elif sch == "Eigen":
            proj = np.asarray(st["proj"], dtype=np.float32).astype(np.float64)
            out[f"{c}.Eigen"] = np.where(codes < 0, np.nan, proj[np.clip(codes, 0, None)] if L else 0.0)
        else:   # SortByResponse: same level names, reordered domain (names carry the meaning)
            out[c] = df[c].values
    res = pd.DataFrame({**out, **exp}, index=df.index)
    res._catenc_done = True
    return res
