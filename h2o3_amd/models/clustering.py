"""K-Means, PCA, SVD, Naive Bayes.

References: hex/kmeans/KMeans.java (Lloyd iterations as MRTasks, init
Random / PlusPlus / Furthest / User, standardize, estimate_k by the
reduction in within-SS), hex/pca/PCA.java (GramSVD / Power / Randomized /
GLRM methods, importance table), hex/svd/SVD.java, hex/naivebayes/
NaiveBayes.java (Laplace smoothing, gaussian numeric likelihoods,
min_sdev/eps_sdev, min_prob/eps_prob).

MI355X design: the expanded design matrix is one HBM tensor; K-Means
lives in models/kmeans.py (one fused HIP pass per Lloyd iteration); PCA/SVD take the weighted Gram from the f32-MFMA Gram kernel and finish
with a tiny f64 eigendecomposition; every reduction is one all_reduce.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_ENUM, T_INT, T_REAL, Vec
from ..ops import cluster_ops, linalg_ops
from ..parallel import cloud
from ..parallel import collectives as coll
from ..core.groupsum import group_sum
from . import metrics as mm
from .base import H2OEstimator
from .datainfo import DataInfo


def _seed(p, default=1234):
    s = p.get("seed", -1)
    return default if s is None or s == -1 else int(s) & 0x7FFFFFFF


# ====================================================================== KMeans
from .kmeans import KMEANS_DEFAULTS, H2OKMeansEstimator  # noqa: E402,F401  (fused HIP Lloyd pass)


# ====================================================================== PCA / SVD
def _transform_info(frame, x, transform, use_all, mvh="MeanImputation"):
    t = (transform or "NONE").upper()
    di = DataInfo(frame, x, standardize=t in ("STANDARDIZE", "DESCALE", "DEMEAN", "NORMALIZE"),
                  use_all_factor_levels=use_all, pad_to=32, missing_values_handling=mvh)
    if t in ("DEMEAN",):
        di.sigmas = [1.0] * len(di.sigmas)
    if t == "DESCALE":
        di.means = [0.0] * len(di.means)
    if t == "NORMALIZE":
        out = []
        for c in di.num_cols:
            v = frame.vec(c)
            r = v.rollups()
            out.append(max(r["max"] - r["min"], 1e-12))
        di.sigmas = out
    return di


def _top_eig(G, k, method, iters, seed):
    """Top-k eigenpairs of the symmetric (all-reduced, identical on every
    rank) Gram G by hex/svd/SVD.java's methods: GramSVD = exact
    eigendecomposition, Power = power iterations with deflation (stops at
    1e-10 change or max_iterations), Randomized = max_iterations subspace
    iterations from a seeded Gaussian block then a Rayleigh-Ritz step."""
    G = G.to(torch.float64).cpu()
    P = G.shape[0]
    k = min(k, P)
    m = (method or "GramSVD").lower()
    gen = torch.Generator(device="cpu").manual_seed(seed)
    if m == "power":
        V = torch.zeros((P, k), dtype=torch.float64)
        lam = torch.zeros(k, dtype=torch.float64)
        R = G.clone()
        for j in range(k):
            v = torch.randn(P, generator=gen, dtype=torch.float64)
            v = v / v.norm().clamp_min(1e-300)
            for _ in range(max(1, iters)):
                w = R @ v
                nw = w.norm()
                if float(nw) == 0:
                    break
                w = w / nw
                done = float((w - v).abs().max()) < 1e-10
                v = w
                if done:
                    break
            lam[j] = v @ (R @ v)
            V[:, j] = v
            R = R - lam[j] * torch.outer(v, v)
        return lam, V
    if m == "randomized":
        Q = torch.randn((P, k), generator=gen, dtype=torch.float64)
        for _ in range(max(1, iters)):
            Q, _ = torch.linalg.qr(G @ Q)
        lb, W = torch.linalg.eigh(Q.T @ G @ Q)
        order = torch.argsort(lb, descending=True)
        return lb[order], Q @ W[:, order]
    lam, V = torch.linalg.eigh(G)
    order = torch.argsort(lam, descending=True)[:k]
    return lam[order], V[:, order]


def gram_and_mean(X, P):
    """(X'X [P,P], column means [P], row count) of the model matrix, all-reduced,
    from ONE pass of the Gram kernel: when the expansion left a padding column
    (pad_to=32), it is set to 1 so that the same pass yields the column sums
    (G[P, :P]) and the row count (G[P, P]) -- no f64 copy of X for the mean.
    X's padding columns carry no model weight (every projection zeroes rows >=
    P of V), so the 1s stay."""
    if X.shape[1] > P and X.device.type == "cuda":
        X[:, P] = 1.0
        G = linalg_ops.weighted_gram(X)[:P + 1, :P + 1]
        coll.allreduce_(G)
        n = float(G[P, P])
        return G[:P, :P].contiguous(), G[P, :P] / max(n, 1.0), n
    G = linalg_ops.weighted_gram(X)[:P, :P]
    coll.allreduce_(G)
    s = X[:, :P].sum(0, dtype=torch.float64)
    coll.allreduce_(s)
    n = coll.allreduce_scalar(float(X.shape[0]))
    return G, s / max(n, 1.0), n


PCA_DEFAULTS = dict(transform="none", k=1, max_iterations=1000, seed=-1, use_all_factor_levels=False,
                    compute_metrics=True, impute_missing=False, pca_method="GramSVD", pca_impl="mtj_evd_symmmatrix",
                    max_runtime_secs=0.0, export_checkpoints_dir=None)


class H2OPrincipalComponentAnalysisEstimator(H2OEstimator):
    algo = "pca"
    supervised_learning = False
    _defaults = PCA_DEFAULTS

    def _fit(self, spec):
        p = self._parms
        di = _transform_info(spec.frame, spec.x, p.get("transform"), bool(p.get("use_all_factor_levels")),
                             mvh="MeanImputation" if p.get("impute_missing") else "Skip")
        self._dinfo = di
        X, ok = di.expand(spec.frame)
        if not bool(ok.all()):
            X = X[ok]      # impute_missing=False: rows with an NA are skipped (PCA.java)
        k = int(p.get("k", 1))
        method = (p.get("pca_method") or "GramSVD").lower()
        P = di.P
        G, mean, n = gram_and_mean(X, P)
        if method in ("gramsvd", "glrm"):
            if not di.standardize:
                # covariance about the mean (reference demeans via the Gram's intercept row)
                G = G - n * torch.outer(mean, mean)
            cov = G / max(n - 1, 1)
            impl = str(p.get("pca_impl") or "mtj_evd_symmmatrix").lower()
            if impl == "mtj_svd_densematrix":
                # PCAImplementation.MTJ_SVD_DENSEMATRIX: singular values of the
                # covariance (= its eigenvalues, PSD), not an eigensolver
                U_, S_, _ = torch.linalg.svd(cov.cpu())
                evals, evecs = S_, U_
            else:   # MTJ_EVD_DENSEMATRIX / MTJ_EVD_SYMMMATRIX / JAMA: symmetric eigensolver
                evals, evecs = torch.linalg.eigh(cov.cpu())
                order = torch.argsort(evals, descending=True)
                evals, evecs = evals[order], evecs[:, order]
        else:  # Power / Randomized (hex/svd/SVD.java): iterations on the covariance
            # X'X comes from ONE pass of the hand-written MFMA Gram (gram.hip via
            # weighted_gram, f64 across row blocks); the centred cross-product
            # Xc'(Xc Q) of every subspace / power iteration is (G - n mu mu') Q,
            # so the iterations run on the P x P matrix and never re-read X
            if not di.standardize:
                G = G - n * torch.outer(mean, mean)
            cov = G / max(n - 1, 1)
            iters = min(int(p.get("max_iterations", 1000)), 1000)
            evals, evecs = _top_eig(cov, k, method, iters, _seed(p))
        k = min(k, evecs.shape[1])
        sd = torch.sqrt(evals.clamp_min(0))
        tot = float(evals.clamp_min(0).sum())
        self._evecs = evecs[:, :k].to(torch.float64)
        self._mean = mean.cpu() if not di.standardize else torch.zeros(P, dtype=torch.float64)
        var = evals[:k].clamp_min(0)
        self._output["eigenvectors"] = self._evecs.numpy()
        self._output["std_deviation"] = sd[:k].numpy()
        self._output["importance"] = {"Standard deviation": sd[:k].tolist(),
                                      "Proportion of Variance": (var / tot).tolist() if tot > 0 else [0.0] * k,
                                      "Cumulative Proportion": (torch.cumsum(var, 0) / tot).tolist() if tot > 0 else [0.0] * k}
        self._output["coef_names"] = di.coef_names
        self._output["model_summary"] = self._output["importance"]
        self._k = k

    def _predict_raw(self, frame):
        X, _ = self._dinfo.expand(frame)
        P = self._dinfo.P
        # projections X v_j on the MFMA skinny-GEMM kernel for large frames
        # (cluster_ops.xv; columns past P are padding), minus the mean's
        V = torch.zeros((X.shape[1], self._evecs.shape[1]), dtype=torch.float64)
        V[:P] = self._evecs
        Z = cluster_ops.xv(X, V).to(torch.float64)
        return Z - (self._mean.to(torch.float64) @ self._evecs).to(X.device).view(1, -1)

    def predict(self, test_data, **kw):
        Z = self._predict_raw(test_data)
        return H2OFrame.from_vecs([Vec(Z[:, j].contiguous(), T_REAL) for j in range(Z.shape[1])],
                                  [f"PC{j + 1}" for j in range(Z.shape[1])])

    transform = predict

    def _score_unsupervised(self, spec):
        # compute_metrics=False: no training metrics (PCAModel.makeMetricBuilder skipped)
        self._training_metrics = mm.ModelMetricsDimReduction(nobs=spec.frame.nrows) \
            if self._parms.get("compute_metrics", True) else None

    def varimp(self, use_pandas=False):
        return self._output["importance"]

    @property
    def rotation(self):
        return self._output["eigenvectors"]


SVD_DEFAULTS = dict(transform="none", svd_method="GramSVD", nv=1, max_iterations=1000, seed=-1, keep_u=True,
                    u_name=None, v_name=None, use_all_factor_levels=True, max_runtime_secs=0.0,
                    export_checkpoints_dir=None)


class H2OSingularValueDecompositionEstimator(H2OEstimator):
    algo = "svd"
    supervised_learning = False
    _defaults = SVD_DEFAULTS

    def _fit(self, spec):
        p = self._parms
        di = _transform_info(spec.frame, spec.x, p.get("transform"), bool(p.get("use_all_factor_levels", True)))
        self._dinfo = di
        X, ok = di.expand(spec.frame)
        nv = int(p.get("nv", 1))
        P = di.P
        G = linalg_ops.weighted_gram(X)[:P, :P]
        coll.allreduce_(G)
        ev, V = _top_eig(G, nv, p.get("svd_method") or "GramSVD", int(p.get("max_iterations", 1000)), _seed(p))
        d = torch.sqrt(ev.clamp_min(0))
        self._V = V
        self._d = d
        self._output["d"] = d.tolist()
        self._output["v"] = V.numpy()
        if p.get("keep_u", True):
            # U = X V / d: the skinny MFMA projection kernel for large frames
            Vp = torch.zeros((X.shape[1], V.shape[1]), dtype=torch.float64)
            Vp[:P] = V
            U = cluster_ops.xv(X, Vp).to(torch.float64) / d.to(X.device).clamp_min(1e-300)
            self._u = H2OFrame.from_vecs([Vec(U[:, j].contiguous(), T_REAL) for j in range(U.shape[1])],
                                         [f"u{j + 1}" for j in range(U.shape[1])])
            # u_name / v_name: DKV keys of the U and V frames (SVDModel._u_key / _v_key)
            from ..core import dkv
            uk = p.get("u_name") or f"SVDUMatrix_{self.model_id}"
            dkv.put(uk, self._u)
            self._output["u_key"] = {"name": uk}
        import pandas as pd
        vk = p.get("v_name") or f"SVDVMatrix_{self.model_id}"
        from ..core import dkv
        dkv.put(vk, H2OFrame(pd.DataFrame(V.numpy(), columns=[f"Vec{j + 1}" for j in range(V.shape[1])])))
        self._output["v_key"] = {"name": vk}

    def d(self):
        return self._output["d"]

    def v(self):
        return self._output["v"]

    def u(self):
        return getattr(self, "_u", None)

    def _predict_raw(self, frame):
        X, _ = self._dinfo.expand(frame)
        Vp = torch.zeros((X.shape[1], self._V.shape[1]), dtype=torch.float64)
        Vp[: self._dinfo.P] = self._V
        return cluster_ops.xv(X, Vp).to(torch.float64)

    def predict(self, test_data, **kw):
        Z = self._predict_raw(test_data)
        return H2OFrame.from_vecs([Vec(Z[:, j].contiguous(), T_REAL) for j in range(Z.shape[1])],
                                  [f"v{j + 1}" for j in range(Z.shape[1])])

    def _score_unsupervised(self, spec):
        self._training_metrics = mm.ModelMetricsDimReduction(nobs=spec.frame.nrows)


# ====================================================================== Naive Bayes
NB_DEFAULTS = dict(laplace=0.0, min_sdev=0.001, eps_sdev=0.0, min_prob=0.001, eps_prob=0.0,
                   compute_metrics=True, seed=-1, max_confusion_matrix_size=20, balance_classes=False,
                   class_sampling_factors=None, max_after_balance_size=5.0)


class H2ONaiveBayesEstimator(H2OEstimator):
    algo = "naivebayes"
    _defaults = NB_DEFAULTS

    def _score_all(self, spec):
        # compute_metrics=False (NaiveBayes.java): no training / validation metrics
        if not self._parms.get("compute_metrics", True):
            self._training_metrics = self._validation_metrics = None
            return
        super()._score_all(spec)

    def _fit(self, spec):
        if not spec.is_classification:
            raise ValueError("Naive Bayes requires a categorical response")
        p = self._parms
        K = spec.nclasses
        y = spec.y_tensor().long()
        ok = y >= 0
        lap = float(p.get("laplace", 0.0))
        cnt = torch.bincount(y[ok], minlength=K).to(torch.float64)
        coll.allreduce_(cnt)
        self._prior = (cnt + lap) / (cnt.sum() + K * lap) if lap > 0 else cnt / cnt.sum()
        self._tables = {}
        num_cols = []
        for c in spec.x:
            v = spec.frame.vec(c)
            if v.type == T_ENUM:
                L = len(v.domain)
                m = ok & (v.data >= 0)
                # (class, level) counts: integer bincount over the combined key
                t = torch.bincount(y[m] * L + v.data[m].long(), minlength=K * L).to(torch.float64).view(K, L)
                coll.allreduce_(t)
                prob = (t + lap) / (t.sum(1, keepdim=True) + L * lap)
                self._tables[c] = ("cat", prob, list(v.domain))
            else:
                num_cols.append(c)
        if num_cols:
            # every numeric column's per-class moments in one pass: one-hot(class)^T
            # [x | x^2 | non-NA] as f64 GEMMs over row chunks (NaN rows of a column
            # drop out of that column only, as in NaiveBayes.java's per-column NA skip)
            P = len(num_cols)
            yk = torch.where(ok, y, torch.zeros_like(y))
            wok = ok.to(torch.float64)
            st = torch.zeros((K, 3 * P), dtype=torch.float64, device=y.device)
            n = y.shape[0]
            step = max(1, (1 << 26) // max(3 * P, 1))
            for a in range(0, n, step):
                X = torch.stack([spec.frame.vec(c).as_float(torch.float64)[a:a + step] for c in num_cols], 1)
                M = (~torch.isnan(X)).to(torch.float64) * wok[a:a + step].view(-1, 1)
                X = torch.nan_to_num(X) * M
                st += group_sum(yk[a:a + step], torch.cat([X, X * X, M], 1), K)
            coll.allreduce_(st)
            s1, s2, cnt_c = st[:, :P], st[:, P:2 * P], st[:, 2 * P:]
            mean = s1 / cnt_c.clamp_min(1)
            var = (s2 - cnt_c * mean ** 2) / (cnt_c - 1).clamp_min(1)
            sd = torch.sqrt(var.clamp_min(0))
            for j, c in enumerate(num_cols):
                self._tables[c] = ("num", mean[:, j].contiguous(), sd[:, j].contiguous())
        self._output["apriori"] = self._prior.cpu().tolist()
        self._output["pcond"] = {c: (t[1].cpu().numpy().tolist(), t[2] if t[0] == "cat" else t[2].cpu().tolist())
                                 for c, t in self._tables.items()}

    def _predict_raw(self, frame):
        p = self._parms
        n = frame.nlocal
        logp = torch.log(self._prior.clamp_min(1e-300)).view(1, -1).repeat(n, 1).to(cloud.device())
        min_sdev, eps_sdev = float(p["min_sdev"]), float(p["eps_sdev"])
        min_prob, eps_prob = float(p["min_prob"]), float(p["eps_prob"])
        num = [(c, t) for c, t in self._tables.items() if t[0] == "num" and c in frame.names]
        for c, t in self._tables.items():
            if c not in frame.names or t[0] != "cat":
                continue
            v = frame.vec(c)
            codes = self._adapt_enum(v, t[2]).long()
            pr = t[1].T[codes.clamp(min=0)]               # [n, K]
            pr = torch.where(pr <= eps_prob, torch.full_like(pr, min_prob), pr)
            contrib = torch.log(pr.clamp_min(1e-300))
            logp = logp + torch.where((codes < 0).view(-1, 1), torch.zeros_like(contrib), contrib)
        if num:
            # all numeric columns at once: Gaussian log densities [rows, P, K] per row chunk
            mean = torch.stack([t[1] for _, t in num], 0)                # [P, K]
            sd = torch.stack([t[2] for _, t in num], 0)
            sd = torch.where(sd <= eps_sdev, torch.full_like(sd, min_sdev), sd)
            lnorm = torch.log(sd * math.sqrt(2 * math.pi))
            K = mean.shape[1]
            step = max(1, (1 << 25) // max(len(num) * K, 1))
            for a in range(0, n, step):
                X = torch.stack([frame.vec(c).as_float(torch.float64)[a:a + step] for c, _ in num], 1)
                z = (X.unsqueeze(2) - mean.unsqueeze(0)) / sd.unsqueeze(0)
                contrib = -0.5 * z * z - lnorm.unsqueeze(0)
                contrib = torch.where(torch.isnan(X).unsqueeze(2), torch.zeros_like(contrib), contrib)
                logp[a:a + step] += contrib.sum(1)
        return torch.softmax(logp, 1)
