"""K-Means clustering.

Reference: hex/kmeans/KMeans.java —
  * initial centers (KMeans.java:123): user points, Random rows, or for
    PlusPlus / Furthest one random row plus 5 rounds of distance-weighted
    oversampling (SumSqr + Sampler, probability 3k * d / sum d) reclustered
    down to k (recluster, KMeans.java:1011);
  * Lloyd iterations (LloydsIterationTask, KMeans.java:731) until fewer than
    max(1, 1e-4 * rows) rows change cluster or max_iterations;
  * empty clusters re-seeded at the worst row (cleanupBadClusters, :194);
  * estimate_k (:329-420): k grows from 1 by splitting the cluster with the
    widest bounding-box range at its center (splitLargestCluster / SplitTask)
    until the relative within-SS improvement drops below
    min(0.02 + 10/rows + 2.5/ncols^2, 0.8);
  * categorical columns: mismatch distance 1 and the per-cluster mode as
    the center (GenModel.KMeans_distance, max_cats); NAs imputed with the
    column mean / mode (Kmeans_preprocessData).
  * cluster_size_constraints: the assignment step becomes a transportation
    LP (the reference's KMeansSimplexSolver).

MI355X design: the standardized design matrix is ONE f32 HBM tensor
[rows, P] (P padded to 4) with each categorical column one-hot encoded at
1/sqrt(2), so the squared euclidean distance of a one-hot block IS the
reference's 0/1 mismatch; every Lloyd iteration is ONE fused HIP kernel
pass (ops/csrc/kmeans.hip: f32 MFMA distances, arg-min, LDS per-cluster
sums) followed by ONE all-reduce of a [k*P + 2k + 1] f64 vector.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_INT, Vec
from ..ops import cluster_ops
from ..parallel import cloud
from ..parallel import collectives as coll
from . import metrics as mm
from .base import H2OEstimator
from .datainfo import DataInfo
from ..core.groupsum import group_extreme

KMEANS_DEFAULTS = dict(k=1, estimate_k=False, user_points=None, max_iterations=10, standardize=True, seed=-1,
                       init="Furthest", categorical_encoding="auto", max_runtime_secs=0.0,
                       cluster_size_constraints=None, score_each_iteration=False)

CAT_SCALE = math.sqrt(0.5)       # one-hot at 1/sqrt(2): squared distance of a level mismatch = 1
TOLERANCE = 1e-4                  # KMeans.java:29


def _seed(p, default=1234):
    s = p.get("seed", -1)
    return default if s is None or s == -1 else int(s) & 0x7FFFFFFF


def _row_uniform(rows, seed):
    """Counter-based uniform in (0, 1) per global row index (integer hash,
    32-bit lanes in int64 so no product overflows)."""
    m = 0xFFFFFFFF
    x = (rows ^ (int(seed) & m)) & m
    x = (((x >> 16) ^ x) * 0x45D9F3B) & m
    x = (((x >> 16) ^ x) * 0x45D9F3B) & m
    x = (x >> 16) ^ x
    return (x.to(torch.float64) + 0.5) / 4294967296.0


class H2OKMeansEstimator(H2OEstimator):
    algo = "kmeans"
    supervised_learning = False
    _defaults = KMEANS_DEFAULTS
    _cat_scale = CAT_SCALE

    # ------------------------------------------------------------------ data
    def _design(self, frame):
        """Standardized / imputed design matrix in the clustering space."""
        X, ok = self._dinfo.expand(frame, dtype=torch.float32, pad=True)
        nc = self._dinfo.n_cat_expanded
        if nc:
            X[:, :nc] *= CAT_SCALE
        return X, ok

    def _cat_blocks(self):
        di = self._dinfo
        return [(di.cat_offsets[c], len(di.domains[c])) for c in di.cat_cols]

    def _fix_cats(self, C):
        """Categorical blocks of the centers -> one-hot of the most frequent
        level (max_cats, KMeans.java:1059): the block holds level sums."""
        for off, L in self._cat_blocks():
            blk = C[:, off:off + L]
            top = blk.argmax(1)
            blk.zero_()
            blk.scatter_(1, top.view(-1, 1), CAT_SCALE)
        return C

    def _offsets(self, n_local):
        ns = coll.all_gather_object(int(n_local))
        off = int(sum(ns[:cloud.rank()]))
        return off, int(sum(ns))

    def _rows_global(self, X, rows):
        """Rows by GLOBAL index (row shards concatenated in rank order): every
        rank fills the rows it owns, one all-reduce."""
        off, _ = self._offsets(X.shape[0])
        out = torch.zeros((len(rows), X.shape[1]), dtype=torch.float64, device=X.device)
        for i, r in enumerate(rows):
            if off <= r < off + X.shape[0]:
                out[i] = X[r - off].to(torch.float64)
        coll.allreduce_(out)
        return out

    # ------------------------------------------------------------------ init
    def _init_centers(self, X, w, k, rng):
        p = self._parms
        up = p.get("user_points")
        if up is not None:
            from ..core import dkv
            up = dkv.get(up) if isinstance(up, str) else up
            U, _ = self._design(up)
            return coll.all_gather_var(U.to(torch.float64))[:k]      # the points frame is row-sharded too
        _, ntot = self._offsets(X.shape[0])
        init = (p.get("init") or "Furthest").lower()

        def rand_row():
            return max(0, int(rng.random_sample() * ntot) - 1)     # randomRow, KMeans.java:1054
        if init == "random":
            return self._rows_global(X, [rand_row() for _ in range(k)])
        C = self._rows_global(X, [rand_row()])
        if k == 1:
            return C
        # 5 rounds of k-means|| oversampling (SumSqr + Sampler)
        dmin = torch.empty(X.shape[0], dtype=torch.float32, device=X.device)
        # the sampler's uniform is a hash of (seed, round, GLOBAL row): the same
        # candidates whatever the row sharding (1 rank or N), unlike a per-rank
        # generator stream
        off, _ = self._offsets(X.shape[0])
        grow = torch.arange(X.shape[0], device=X.device, dtype=torch.int64) + int(off)
        seed0 = int(rng.randint(0, 2 ** 31 - 1))
        for rnd in range(5):
            cluster_ops.lloyd_pass(X, C, accumulate=False, dmin=dmin)
            tot = coll.allreduce_scalar(float(dmin.to(torch.float64).sum()))
            if tot <= 0:
                break
            u = _row_uniform(grow, seed0 * 7919 + rnd)
            pick = torch.nonzero(3.0 * k * dmin.to(torch.float64) > u * tot).flatten()
            S = coll.all_gather_var(X[pick].to(torch.float64))
            C = torch.cat([C, S.to(C.device)], 0)
            if C.shape[0] > 64 * k + 1024:        # bounded candidate set
                break
        return self._recluster(C.cpu().numpy(), k, init, rng)

    @staticmethod
    def _recluster(points, k, init, rng):
        """recluster (KMeans.java:1011) on the host: the sampled candidates
        are few (O(k) per round)."""
        res = [points[0]]
        d = ((points - points[0]) ** 2).sum(1)
        while len(res) < min(k, len(points)):
            if init == "plusplus":
                s = d.sum()
                thr = rng.random_sample() * s
                idx = np.nonzero(d >= thr)[0]
                i = int(idx[0]) if len(idx) else int(np.argmax(d))
            else:
                i = int(np.argmax(d)) if d.max() > 0 else 0
            res.append(points[i])
            d = np.minimum(d, ((points - points[i]) ** 2).sum(1))
        while len(res) < k:
            res.append(points[len(res) % len(points)])
        return torch.as_tensor(np.stack(res), dtype=torch.float64, device=cloud.device())

    # ------------------------------------------------------------------ lloyd
    def _lloyd(self, X, w, C, assign, nrows_tot, t_end):
        """Lloyd iterations from centers C (f64 [k, P]) until convergence."""
        p = self._parms
        k, P = C.shape
        maxit = int(p.get("max_iterations", 10))
        it = 0
        reinit = 0
        hist = []
        st = None
        while True:
            st = cluster_ops.lloyd_pass(X, C, w, assign, accumulate=True, xabs_max=self._xabs(X, w))
            coll.allreduce_(st.vec)
            wts = st.weights
            newC = torch.where(wts.view(-1, 1) > 0, st.sums / wts.clamp_min(1e-300).view(-1, 1), C)
            newC = self._fix_cats(newC)
            empty = torch.nonzero(wts <= 0).flatten().tolist()
            if empty and not p.get("estimate_k"):
                # cleanupBadClusters: re-seed the first empty cluster at the worst row
                newC[empty[0]] = self._worst_row(X, C)
                if len(empty) > 1 and reinit < k:
                    reinit += 1
                    C = C.clone()
                    C[empty[0]] = newC[empty[0]]
                    continue
                reinit = 0
            it += 1
            hist.append({"timestamp": time.time(), "iterations": it, "number_of_reassigned_observations": st.changed,
                         "within_cluster_sum_of_squares": float(st.withinss.sum())})
            C = newC
            if self._tick(it, maxit, deadline=t_end)[1] or st.changed < max(1.0, nrows_tot * TOLERANCE) or \
                    it >= maxit:
                break
        return C, st, it, hist

    def _xabs(self, X, w):
        """max |w x| of the training matrix, once per fit (fixed-point sums)."""
        key = (X.data_ptr(), X.shape, None if w is None else w.data_ptr())
        if getattr(self, "_xabs_key", None) != key:
            self._xabs_key, self._xabs_val = key, cluster_ops.abs_bound(X, w)
        return self._xabs_val

    def _worst_row(self, X, C):
        dmin = torch.empty(X.shape[0], dtype=torch.float32, device=X.device)
        cluster_ops.lloyd_pass(X, C, accumulate=False, dmin=dmin)
        v, i = (dmin.max(0) if dmin.numel() else (torch.tensor(-1.0), torch.tensor(0)))
        off, _ = self._offsets(X.shape[0])
        cand = coll.all_gather_object((float(v), off + int(i)))
        r = max(range(len(cand)), key=lambda j: (cand[j][0], -j))
        return self._rows_global(X, [cand[r][1]])[0]

    def _bounds(self, X, assign, k, chunk=1 << 20):
        """Per-cluster bounding boxes (IterationTask._lo/_hi), f64 [k, P]."""
        P = X.shape[1]
        lo = torch.full((k, P), float("inf"), dtype=torch.float64, device=X.device)
        hi = torch.full((k, P), float("-inf"), dtype=torch.float64, device=X.device)
        for a in range(0, X.shape[0], chunk):
            xc = X[a:a + chunk].to(torch.float64)
            ac = assign[a:a + chunk]
            lo = torch.minimum(lo, group_extreme(ac, xc, k, "min"))
            hi = torch.maximum(hi, group_extreme(ac, xc, k, "max"))
        coll.allreduce_(lo, "min")
        coll.allreduce_(hi, "max")
        return lo, hi

    def _split_largest(self, X, w, C, assign):
        """splitLargestCluster + SplitTask (KMeans.java:451, :1110)."""
        k, P = C.shape
        lo, hi = self._bounds(X, assign, k)
        rng_ = (hi - lo).to(torch.float32)
        nc = self._dinfo.n_cat_expanded
        rng_[:, :nc] = -1                                      # never split along a categorical
        rng_[:, self._dinfo.P:] = -1                           # padding
        rng_ = torch.nan_to_num(rng_, nan=-1.0, posinf=-1.0, neginf=-1.0)
        flat = int(torch.argmax(rng_.reshape(-1)))
        clu, dim = flat // P, flat % P
        split = float(C[clu, dim])
        m = assign == clu
        move = m & (X[:, dim].to(torch.float64) > split)
        stay = m & ~move
        ww = torch.ones(X.shape[0], dtype=torch.float64, device=X.device) if w is None else w.to(torch.float64)
        st = torch.stack([(X.to(torch.float64) * (ww * stay).view(-1, 1)).sum(0),
                          (X.to(torch.float64) * (ww * move).view(-1, 1)).sum(0)])
        cnt = torch.stack([(ww * stay).sum(), (ww * move).sum()])
        coll.allreduce_(st)
        coll.allreduce_(cnt)
        newC = torch.cat([C, C[clu:clu + 1]], 0).clone()
        if float(cnt[0]) > 0:
            newC[clu] = st[0] / cnt[0]
        if float(cnt[1]) > 0:
            newC[k] = st[1] / cnt[1]
        assign[move] = k
        return newC

    # ------------------------------------------------------------------ fit
    def _fit(self, spec):
        p = self._parms
        t0 = time.time()
        t_end = t0 + float(p["max_runtime_secs"]) if float(p.get("max_runtime_secs") or 0) > 0 else None
        di = DataInfo(spec.frame, spec.x, standardize=bool(p.get("standardize", True)), use_all_factor_levels=True,
                      pad_to=4)
        self._dinfo = di
        X, ok = self._design(spec.frame)
        if not bool(ok.all()):
            X = X[ok]
        w = spec.w_tensor()
        fw = self.__dict__.get("_fold_w")
        if fw is not None:
            # CV fold model: holdout rows carry weight 0 (the reference trains
            # fold models on the whole frame with a fold-weight column, so the
            # standardization is the full frame's)
            w = fw.to(torch.float32) if w is None else w * fw.to(w.dtype)
        w = None if w is None else w[ok]
        _, nrows_tot = self._offsets(X.shape[0])
        rng = np.random.RandomState(_seed(p))
        K = int(p.get("k", 1))
        estimate = bool(p.get("estimate_k"))
        constraints = p.get("cluster_size_constraints")
        assign = torch.full((X.shape[0],), -1, dtype=torch.int32, device=X.device)
        hist = []
        if constraints is not None:
            C, st, it, hist = self._constrained(X, w, K, rng, [float(c) for c in constraints], t_end)
            self._k_history = [K]
        elif estimate:
            # k grows from 1; the first Lloyd pass lands on the grand mean
            C = self._init_centers(X, w, 1, rng)
            cutoff = min(0.02 + 10.0 / max(nrows_tot, 1) + 2.5 / max(len(spec.x), 1) ** 2, 0.8)
            prev_ss, best = 0.0, None
            self._k_history = []
            for k in range(1, K + 1):
                C, st, it, h = self._lloyd(X, w, C, assign, nrows_tot, t_end)
                hist += h
                now = float(st.withinss.sum())
                rel = 1.0 if prev_ss == 0 else (prev_ss - now) / prev_ss
                prev_ss = now
                if k > 1 and rel < cutoff:
                    C, st, it, assign = best
                    break
                self._k_history.append(k)
                best = (C.clone(), st, it, assign.clone())
                if self._tick(k, K, deadline=t_end)[1] or k == K:
                    break
                C = self._split_largest(X, w, C, assign)
        else:
            C = self._init_centers(X, w, K, rng)
            C, st, it, hist = self._lloyd(X, w, C, assign, nrows_tot, t_end)
            self._k_history = [C.shape[0]]
        self._C_std = C.to(torch.float32)
        self._iterations = it
        self._scoring_history = hist
        self._train_X, self._train_w = X, w
        self._output["centers"] = self._centers_raw(C)
        self._output["centers_std"] = C[:, :di.P].cpu().numpy()
        self._output["coef_names"] = di.coef_names
        self._output["model_summary"] = {"number_of_rows": nrows_tot, "number_of_clusters": C.shape[0],
                                         "number_of_categorical_columns": len(di.cat_cols),
                                         "number_of_iterations": it}

    def _centers_raw(self, C):
        """Centers per input column: numeric destandardized, categorical as
        the level label (the reference 'centers' table)."""
        di = self._dinfo
        Ch = C.cpu().numpy()
        out = []
        for r in range(Ch.shape[0]):
            row = []
            for c in di.x:
                if c in di.cat_offsets:
                    off = di.cat_offsets[c]
                    L = len(di.domains[c])
                    row.append(di.domains[c][int(np.argmax(Ch[r, off:off + L]))])
                elif c in di.num_cols:
                    j = di.num_cols.index(c)
                    v = Ch[r, di.n_cat_expanded + j]
                    row.append(float(v * di.sigmas[j] + di.means[j]) if di.standardize else float(v))
            out.append(row)
        return out

    # ------------------------------------------------------------------ constrained
    def _constrained(self, X, w, k, rng, cons, t_end):
        """Constrained K-means: the assignment minimizes total distance with
        at least cons[c] rows per cluster — a transportation LP whose
        constraint matrix is totally unimodular, so the HiGHS optimum is
        integral (the reference solves the same problem with its own
        network simplex, KMeansSimplexSolver.java).  Rows are gathered to
        the host: this mode is for the small data the reference supports it
        on."""
        from scipy.optimize import linprog
        from scipy.sparse import coo_matrix
        p = self._parms
        if len(cons) != k:
            raise ValueError("cluster_size_constraints must have k entries")
        Xg = coll.all_gather_var(X.to(torch.float64)).cpu().numpy()
        n, P = Xg.shape
        if sum(cons) > n:
            raise ValueError("the sum of cluster_size_constraints exceeds the number of rows")
        C = self._init_centers(X, w, k, rng).cpu().numpy()
        maxit = int(p.get("max_iterations", 10))
        prev = None
        hist = []
        it = 0
        rows = np.repeat(np.arange(n), k)
        cols_ = np.arange(n * k)
        A_eq = coo_matrix((np.ones(n * k), (rows, cols_)), shape=(n, n * k))
        A_ub = coo_matrix((-np.ones(n * k), (np.tile(np.arange(k), n), cols_)), shape=(k, n * k))
        for it in range(1, maxit + 1):
            D = ((Xg[:, None, :] - C[None]) ** 2).sum(2)
            res = linprog(D.reshape(-1), A_ub=A_ub, b_ub=-np.asarray(cons), A_eq=A_eq, b_eq=np.ones(n),
                          bounds=(0, 1), method="highs")
            if not res.success:
                raise RuntimeError(f"constrained k-means LP failed: {res.message}")
            a = res.x.reshape(n, k).argmax(1)
            newC = np.stack([Xg[a == j].mean(0) if (a == j).any() else C[j] for j in range(k)])
            newC = self._fix_cats(torch.as_tensor(newC)).numpy()
            changed = n if prev is None else int((a != prev).sum())
            hist.append({"timestamp": time.time(), "iterations": it, "number_of_reassigned_observations": changed,
                         "within_cluster_sum_of_squares": float(D[np.arange(n), a].sum())})
            prev = a
            C = newC
            if self._tick(it, maxit, deadline=t_end)[1] or changed < max(1.0, n * TOLERANCE):
                break
        self._constrained_assign = prev
        Ct = torch.as_tensor(C, dtype=torch.float64, device=X.device)
        return Ct, None, it, hist

    # ------------------------------------------------------------------ scoring
    def _assign(self, X):
        a = torch.empty(X.shape[0], dtype=torch.int32, device=X.device)
        cluster_ops.lloyd_pass(X, self._C_std, accumulate=False, assign=a)
        return a

    def _predict_raw(self, frame):
        X, _ = self._design(frame)
        return self._assign(X).view(-1, 1).to(torch.float32)

    def predict(self, test_data, **kw):
        X, _ = self._design(test_data)
        return H2OFrame.from_vecs([Vec(self._assign(X).contiguous(), T_INT)], ["predict"])

    def _cluster_metrics(self, X, w):
        """size / withinss with the final centers (one fused pass) and
        totss about the grand center (GenModel.KMeans_distance to the
        standardized mean / modes, KMeans.java:563)."""
        k = self._C_std.shape[0]
        st = cluster_ops.lloyd_pass(X, self._C_std, w, accumulate=True)
        coll.allreduce_(st.vec)
        gc = torch.zeros((1, X.shape[1]), dtype=torch.float64, device=X.device)
        di = self._dinfo
        for c in di.cat_cols:
            gc[0, di.cat_offsets[c] + di.cat_modes[c]] = CAT_SCALE
        if not di.standardize:
            for j, mu in enumerate(di.means):
                gc[0, di.n_cat_expanded + j] = mu
        tot = cluster_ops.lloyd_pass(X, gc, w, accumulate=True)
        coll.allreduce_(tot.vec)
        within = st.withinss.cpu().tolist()
        tw = float(sum(within))
        totss = float(tot.withinss.sum())
        return mm.ModelMetricsClustering(tot_withinss=tw, totss=totss, betweenss=totss - tw, withinss=within,
                                         size=st.weights.cpu().tolist(), nobs=int(float(st.weights.sum())),
                                         k=k)

    def _score_unsupervised(self, spec):
        self._training_metrics = self._cluster_metrics(self._train_X, self._train_w)
        self._output["model_summary"].update({
            "within_cluster_sum_of_squares": self._training_metrics.tot_withinss(),
            "total_sum_of_squares": self._training_metrics.totss(),
            "between_cluster_sum_of_squares": self._training_metrics.betweenss()})
        self._train_X = None
        if spec.valid is not None:
            self._validation_metrics = self._unsupervised_perf(spec.valid)

    def _cross_validate_unsup(self, spec):
        """N-fold CV of a clustering model (ModelBuilder CV +
        ModelMetricsClustering.MetricBuilderClustering.reduceForCV): fold model
        i trains on the whole frame with fold i's rows at weight 0, scores
        its holdout rows; the CV metrics pool the holdout rows' within-cluster
        squared distances (tot_withinss) and their per-column sums / sums of
        squares (totss about the pooled mean, x != mode counts for the
        categorical columns); no per-cluster size / withinss (cluster ids of
        different fold models do not line up)."""
        folds, k = self._fold_ids(spec)
        self._cv_fold_assignment = folds
        fr = spec.frame
        cv_models = []
        acc = None
        for i in range(k):
            sub = self._cv_sub(i, k)
            sub._fold_w = folds != i
            sub._fit(spec)
            sub._score_all(spec)
            sub._fold_w = None
            te_mask = folds == i
            X, ok = sub._design(fr[te_mask])
            if not bool(ok.all()):
                X = X[ok]
            sub._validation_metrics = sub._cluster_metrics(X, None)
            di = sub._dinfo
            nc = di.n_cat_expanded
            Xn = X[:, nc:di.P].to(torch.float64)
            mis = torch.zeros(1, dtype=torch.float64, device=X.device)
            for c in di.cat_cols:
                mis += (X[:, di.cat_offsets[c] + di.cat_modes[c]] == 0).sum().to(torch.float64)
            v = torch.cat([Xn.sum(0), (Xn * Xn).sum(0), mis,
                           torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device)])
            coll.allreduce_(v)
            acc = v if acc is None else acc + v
            acc_tw = float(sub._validation_metrics.tot_withinss())
            sub._cv_tw = acc_tw
            cv_models.append(sub)
        tw = float(sum(m._cv_tw for m in cv_models))
        nn = (acc.numel() - 2) // 2
        cs, css, mis, cnt = acc[:nn], acc[nn:2 * nn], float(acc[2 * nn]), float(acc[2 * nn + 1])
        nrows = float(fr.nrows) if spec.weights_column is None else cnt
        if int(self._parms.get("k", 1)) == 1:
            totss = tw
        else:
            totss = float((css - cs * cs / max(nrows, 1.0)).sum()) + mis
        self._cross_validation_metrics = mm.ModelMetricsClustering(tot_withinss=tw, totss=totss,
                                                                   betweenss=totss - tw, nobs=int(cnt))
        self._cv_models = cv_models if self._parms.get("keep_cross_validation_models", True) else []
        rows = {}
        for m in cv_models:
            for kk, vv in m._validation_metrics._m.items():
                if isinstance(vv, (int, float)) and not isinstance(vv, bool):
                    rows.setdefault(kk, []).append(vv)
        self._output["cross_validation_metrics_summary"] = {
            kk: {"mean": float(np.mean(v)), "sd": float(np.std(v, ddof=1)) if len(v) > 1 else 0.0, "values": v}
            for kk, v in rows.items()}

    def _mt(self, train=False, valid=False, xval=False):
        if xval:
            return self._cross_validation_metrics
        if valid:
            return self._validation_metrics
        return self._training_metrics

    def _unsupervised_perf(self, frame):
        X, ok = self._design(frame)
        if not bool(ok.all()):
            X = X[ok]
        return self._cluster_metrics(X, None)

    # ------------------------------------------------------------------ accessors
    def centers(self):
        return [list(r) for r in self._output["centers"]]

    def centers_std(self):
        return self._output["centers_std"].tolist()

    def size(self, train=False, valid=False):
        return self._training_metrics.get("size")

    def tot_withinss(self, train=False, valid=False, xval=False):
        return self._mt(train, valid, xval).tot_withinss()

    def betweenss(self, train=False, valid=False, xval=False):
        return self._mt(train, valid, xval).betweenss()

    def totss(self, train=False, valid=False, xval=False):
        return self._mt(train, valid, xval).totss()

    def withinss(self, train=False, valid=False, xval=False):
        return self._mt(train, valid, xval).withinss()

    def centroid_stats(self, train=False, valid=False):
        """Per-cluster (centroid, size, within_cluster_sum_of_squares) table of
        the training (or validation) metrics (ModelMetricsClustering
        centroid_stats; h2o-py model/models/clustering.py:189)."""
        import pandas as pd

        def one(mt):
            if mt is None:
                return None
            size = mt.get("size") if hasattr(mt, "get") else None
            wss = mt.withinss() if hasattr(mt, "withinss") else None
            if size is None or wss is None:
                return None
            return pd.DataFrame({"centroid": list(range(1, len(size) + 1)), "size": [float(v) for v in size],
                                 "within_cluster_sum_of_squares": [float(v) for v in wss]})
        res = {}
        if train or not valid:
            res["train"] = one(self._training_metrics)
        if valid:
            res["valid"] = one(self._validation_metrics)
        return list(res.values())[0] if len(res) == 1 else res

    def num_iterations(self):
        return self._iterations

    def scoring_history(self):
        return self._scoring_history
