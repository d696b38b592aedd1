"""Generalized Low Rank Models.

Reference: hex/glrm/GLRM.java + GLRMModel.java + hex/genmodel/algos/glrm
(GlrmLoss: Quadratic, Absolute, Huber, Poisson, Hinge, Logistic,
Periodic; multi-losses Categorical / Ordinal for enum columns;
GlrmRegularizer: None, Quadratic, L2, L1, NonNegative, OneSparse,
UnitOneSparse, Simplex; alternating proximal gradient on X and Y with the
reference's step rule: grow 1.05x after an improving step, halve and
retry otherwise; init Random / SVD / PlusPlus / User; transform of the
numeric columns; archetypes Y, representation frame X, reconstruction =
predict, `impute_original` undoes the transform).

MI355X design: A (n x p_expanded, one-hot enum blocks), X (n x k) and Y
(k x p) all live on the device; each half-iteration is two GEMMs (X Y and
the gradient products) plus fused elementwise loss gradients obtained
from torch autograd over the masked loss -- no per-row loops.  Row
shards stay local (X is row-sharded like the data); the Y gradient is an
all-reduce of a k x p matrix.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_ENUM, T_REAL, Vec
from ..parallel import cloud
from ..parallel import collectives as coll
from .base import H2OEstimator
from ..ops import linalg_ops

GLRM_DEFAULTS = dict(k=1, loss="Quadratic", loss_by_col=None, loss_by_col_idx=None, multi_loss="Categorical",
                     period=1, regularization_x="None", regularization_y="None", gamma_x=0.0, gamma_y=0.0,
                     max_iterations=1000, max_updates=2000, init_step_size=1.0, min_step_size=1e-4, seed=-1,
                     init="PlusPlus", svd_method="Randomized", user_y=None, user_x=None, expand_user_y=True,
                     impute_original=False, recover_svd=False, transform="NONE", representation_name=None,
                     loading_name=None)


def _num_loss(name, a, u, period):
    n = name.lower()
    if n == "quadratic":
        return (a - u) ** 2
    if n == "absolute":
        return (a - u).abs()
    if n == "huber":
        d = (a - u).abs()
        return torch.where(d <= 1, 0.5 * d * d, d - 0.5)
    if n == "poisson":
        return torch.exp(u) - a * u + torch.where(a > 0, a * torch.log(a.clamp_min(1e-300)) - a, torch.zeros_like(a))
    if n == "hinge":
        aa = torch.where(a > 0, torch.ones_like(a), -torch.ones_like(a))
        return torch.clamp(1 - aa * u, min=0)
    if n == "logistic":
        aa = torch.where(a > 0, torch.ones_like(a), -torch.ones_like(a))
        return torch.nn.functional.softplus(-aa * u)
    if n == "periodic":
        return 1 - torch.cos((a - u) * (2 * math.pi / period))
    raise ValueError(f"unknown loss {name}")


def _num_impute(name, u):
    """GlrmLoss.impute: the data value a numeric loss reconstructs from u."""
    n = name.lower()
    if n == "poisson":
        return torch.exp(u)
    if n in ("logistic", "hinge"):
        return (u > 0).to(u.dtype)
    return u


def _cat_impute(multi_loss, U):
    """GlrmLoss.mimpute: Categorical -> argmax; Ordinal -> the level a whose
    ordinal loss sum_{i<a} (1 - min(1, u_i)) + (w-1-a) is smallest."""
    if multi_loss.lower() != "ordinal":
        return U.argmax(1)
    w = U.shape[1]
    if w <= 1:
        return torch.zeros(U.shape[0], dtype=torch.long, device=U.device)
    dec = torch.cumsum(torch.clamp(U[:, :w - 1], max=1.0), 1)            # sum_{i<a} min(1, u_i), a = 1..w-1
    loss = torch.cat([torch.zeros_like(dec[:, :1]), -dec], 1)              # relative to the a = 0 loss
    best = torch.zeros(U.shape[0], dtype=torch.long, device=U.device)
    bl = loss[:, 0].clone()
    for a in range(1, w):                                                  # strict improvement only (first minimum)
        b = loss[:, a] < bl
        best = torch.where(b, torch.full_like(best, a), best)
        bl = torch.where(b, loss[:, a], bl)
    return best


def _reg(name, M):
    n = (name or "None").lower()
    if n == "none" or n == "nonnegative" or n in ("onesparse", "unitonesparse", "simplex"):
        return M.new_zeros(())
    if n == "quadratic":
        return (M * M).sum()
    if n == "l2":
        return torch.sqrt((M * M).sum(1)).sum()
    if n == "l1":
        return M.abs().sum()
    raise ValueError(f"unknown regularizer {name}")


def _reg_rows(name, M):
    """Per-row regularizer values (rows of X are independent at scoring)."""
    n = (name or "None").lower()
    if n == "quadratic":
        return (M * M).sum(1)
    if n == "l2":
        return torch.sqrt((M * M).sum(1))
    if n == "l1":
        return M.abs().sum(1)
    return M.new_zeros((M.shape[0],))


def _prox(name, M, step_gamma):
    n = (name or "None").lower()
    if n == "none":
        return M
    if n == "quadratic":
        return M / (1 + 2 * step_gamma)
    if n == "l2":
        nr = torch.sqrt((M * M).sum(1, keepdim=True)).clamp_min(1e-300)
        return M * torch.clamp(1 - step_gamma / nr, min=0)
    if n == "l1":
        return torch.sign(M) * torch.clamp(M.abs() - step_gamma, min=0)
    if n == "nonnegative":
        return M.clamp_min(0)
    if n == "onesparse":
        idx = M.argmax(1, keepdim=True)
        out = torch.zeros_like(M)
        out.scatter_(1, idx, M.gather(1, idx).clamp_min(0))
        return out
    if n == "unitonesparse":
        idx = M.argmax(1, keepdim=True)
        return torch.zeros_like(M).scatter_(1, idx, 1.0)
    if n == "simplex":  # Euclidean projection onto the probability simplex (row-wise)
        u, _ = torch.sort(M, 1, descending=True)
        css = torch.cumsum(u, 1) - 1
        ind = torch.arange(1, M.shape[1] + 1, device=M.device, dtype=M.dtype)
        cond = u - css / ind > 0
        rho = cond.to(torch.int64).cumsum(1).argmax(1, keepdim=True)
        theta = css.gather(1, rho) / (rho + 1).to(M.dtype)
        return torch.clamp(M - theta, min=0)
    raise ValueError(f"unknown regularizer {name}")


class H2OGeneralizedLowRankEstimator(H2OEstimator):
    algo = "glrm"
    supervised_learning = False
    _defaults = GLRM_DEFAULTS

    # ------------------------------------------------------------ data layout
    def _layout(self, frame, cols, fit=False):
        p = self._parms
        blocks, mats, masks = [], [], []
        dev = cloud.device()
        if fit:
            self._stats = {}
        for c in cols:
            v = frame.vec(c)
            if v.type == T_ENUM or (not fit and c in self._doms):
                dom = self._doms[c] if not fit else list(v.domain)
                if fit:
                    self._doms[c] = dom
                codes = self._adapt_enum(v, dom).long() if not fit else v.data.long()
                oh = torch.zeros((frame.nlocal, len(dom)), dtype=torch.float32, device=dev)
                okr = codes >= 0
                oh[torch.nonzero(okr).view(-1), codes[okr]] = 1.0
                mats.append(oh)
                masks.append(okr.view(-1, 1).expand(-1, len(dom)))
                blocks.append(("cat", c, len(dom)))
            else:
                x = v.as_float(torch.float32)
                if fit:
                    okx = ~torch.isnan(x)
                    s = torch.stack([x[okx].sum().double(), (x[okx].double() ** 2).sum(), okx.sum().double(),
                                     torch.where(okx, x, torch.full_like(x, float("inf"))).min().double(),
                                     torch.where(okx, x, torch.full_like(x, -float("inf"))).max().double()])
                    s3, lo_, hi_ = s[:3].clone(), s[3:4].clone(), s[4:5].clone()
                    coll.allreduce_(s3)
                    coll.allreduce_(lo_, "min")
                    coll.allreduce_(hi_, "max")
                    s = torch.cat([s3, lo_, hi_])
                    mu = float(s[0] / s[2])
                    sd = math.sqrt(max(float(s[1] / s[2]) - mu * mu, 0) * float(s[2]) / max(float(s[2]) - 1, 1))
                    self._stats[c] = (mu, sd if sd > 0 else 1.0, float(s[3]), float(s[4]))
                mu, sd, lo, hi = self._stats[c]
                tr = str(p.get("transform") or "NONE").upper()
                if tr == "STANDARDIZE":
                    x = (x - mu) / sd
                elif tr == "NORMALIZE":
                    x = (x - lo) / max(hi - lo, 1e-12)
                elif tr == "DEMEAN":
                    x = x - mu
                elif tr == "DESCALE":
                    x = x / sd
                m = ~torch.isnan(x)
                mats.append(torch.nan_to_num(x).view(-1, 1))
                masks.append(m.view(-1, 1))
                blocks.append(("num", c, 1))
        A = torch.cat(mats, 1) if mats else torch.zeros((frame.nlocal, 0), device=dev)
        M = torch.cat(masks, 1).to(torch.float32) if masks else torch.zeros_like(A)
        return A, M, blocks

    def _col_loss(self, c):
        """Loss of numeric column c (loss_by_col overrides loss)."""
        p = self._parms
        if p.get("loss_by_col"):
            for name, i in zip(p["loss_by_col"], p.get("loss_by_col_idx") or []):
                if (self._cols[i] if isinstance(i, int) else i) == c:
                    return name
        return p.get("loss") or "Quadratic"

    def _multi_loss(self):
        return "Ordinal" if str(self._parms.get("multi_loss") or "Categorical").lower() == "ordinal" else "Categorical"

    def _loss_groups(self, blocks, device):
        """Columns grouped for one vectorized loss evaluation per group:
        numeric columns by loss name, the categorical one-vs-all columns
        together; ordinal categorical blocks keep their own term."""
        key = (id(blocks), str(device))
        if getattr(self, "_lg_key", None) == key:
            return self._lg
        p = self._parms
        lbc = {}
        if p.get("loss_by_col"):
            idx = p.get("loss_by_col_idx") or []
            for name, i in zip(p["loss_by_col"], idx):
                lbc[self._cols[i] if isinstance(i, int) else i] = name
        ordinal = str(p.get("multi_loss") or "Categorical").lower() == "ordinal"
        num, cat, ords, j = {}, [], [], 0
        for kind, c, w in blocks:
            if kind == "num":
                num.setdefault(lbc.get(c, p.get("loss") or "Quadratic"), []).append(j)
            elif ordinal:
                ords.append((j, w))
            else:
                cat += list(range(j, j + w))
            j += w
        t = lambda v: torch.as_tensor(v, dtype=torch.long, device=device)  # noqa: E731
        self._lg = ({k: t(v) for k, v in num.items()}, t(cat) if cat else None, ords)
        self._lg_key = key
        return self._lg

    def _loss(self, A, M, U, blocks, per_row=False):
        p = self._parms
        num, cat, ords = self._loss_groups(blocks, U.device)
        tot = U.new_zeros((U.shape[0],))
        period = float(p.get("period", 1))
        for name, idx in num.items():
            if idx.numel() == A.shape[1]:                    # every column: no gather
                tot = tot + (_num_loss(name, A, U, period) * M).sum(1)
            else:
                tot = tot + (_num_loss(name, A[:, idx], U[:, idx], period) * M[:, idx]).sum(1)
        if cat is not None:                                  # one-vs-all hinge over every level column
            a, u = A[:, cat], U[:, cat]
            L = torch.where(a > 0, torch.clamp(1 - u, min=0), torch.clamp(1 + u, min=0))
            tot = tot + (L * M[:, cat]).sum(1)
        for j, w in ords:
            # GlrmLoss.Ordinal: sum_{i < w-1} (a > i ? max(1 - u_i, 0) : 1)
            a, m, u = A[:, j:j + w - 1], M[:, j:j + w], U[:, j:j + w - 1]
            lvl = A[:, j:j + w].argmax(1, keepdim=True)
            ar = torch.arange(w - 1, device=a.device).view(1, -1)
            L = torch.where(lvl > ar, torch.clamp(1 - u, min=0), torch.ones_like(u))
            tot = tot + L.sum(1) * m[:, 0]
        return tot if per_row else tot.sum()

    def _grad_u(self, A, M, U, blocks):
        """d loss / d U (U = X Y) with U as the only autograd leaf: the X and
        Y gradients are then gU Y' and X' gU."""
        Uv = U.detach().requires_grad_(True)
        gU, = torch.autograd.grad(self._loss(A, M, Uv, blocks), Uv)
        return gU

    # ------------------------------------------------------------ fit
    def _fit(self, spec):
        p = self._parms
        self._doms = {}
        self._cols = list(spec.x)
        A, M, blocks = self._layout(spec.frame, self._cols, fit=True)
        self._blocks = blocks
        n, P = A.shape
        k = int(p.get("k", 1))
        seed = p.get("seed", -1)
        g = torch.Generator(device="cpu").manual_seed(int(seed) if seed not in (-1, None) else 12345)
        init = str(p.get("init") or "PlusPlus").lower()
        if init == "user" and p.get("user_y") is None and p.get("user_x") is None:
            raise ValueError("ERRR on field: _init: init = User requires user_y and/or user_x")
        if p.get("user_y") is not None and init == "user":
            Y = self._user_y(p["user_y"], blocks, k).to(A.device)
        elif init == "user":
            Y = torch.randn((k, P), generator=g).to(A.device)
        elif init == "svd":
            Y = self._svd_init(A, M, k, spec.frame.nrows, g)
        elif init == "plusplus":
            # k-means++ seeded archetypes from data rows (rank 0's rows,
            # broadcast so every rank starts from the same Y)
            nl = A.shape[0]
            if nl:
                idx = [int(torch.randint(nl, (1,), generator=g))]
                d2 = ((A - A[idx[0]]) ** 2).sum(1)
                for _ in range(1, k):
                    pr = (d2 / d2.sum().clamp_min(1e-30)).cpu()
                    i = int(torch.multinomial(pr, 1, generator=g)) if float(d2.sum()) > 0 \
                        else int(torch.randint(nl, (1,), generator=g))
                    idx.append(i)
                    d2 = torch.minimum(d2, ((A - A[i]) ** 2).sum(1))
                Y = A[idx].clone()
            else:
                Y = torch.zeros((k, P), device=A.device)
            if cloud.is_distributed():
                Y = coll.broadcast_(Y.contiguous(), 0)
        else:
            Y = torch.randn((k, P), generator=g).to(A.device)
        if Y.shape[0] < k:
            Y = torch.cat([Y, torch.randn((k - Y.shape[0], P), generator=g).to(A.device) * 0.01], 0)
        if p.get("user_x") is not None and init == "user":
            X = self._user_x(p["user_x"], spec.frame, k).to(A.device)
        else:
            X = None
        if X is None:
            X = self._init_x(A, M, Y, g)
        gx, gy = float(p.get("gamma_x", 0.0)), float(p.get("gamma_y", 0.0))
        rx, ry = p.get("regularization_x"), p.get("regularization_y")

        def objective(X_, Y_):
            # X is row-sharded (loss and its regularizer are summed over the
            # ranks), Y is replicated: every rank sees the same objective, so the
            # step-size control flow (and the collective count) agrees
            loc = self._loss(A, M, X_ @ Y_, blocks) + gx * _reg(rx, X_)
            return coll.allreduce_scalar(float(loc)) + gy * float(_reg(ry, Y_))

        step = float(p.get("init_step_size", 1.0))
        min_step = float(p.get("min_step_size", 1e-4))
        obj = objective(X, Y)
        hist = [obj]
        it = 0
        updates = 0
        scale = 1.0 / max(int(spec.frame.nrows), 1)    # global rows: the same Y step on every rank
        max_it, max_up = int(p.get("max_iterations", 1000)), int(p.get("max_updates", 2000))
        while it < max_it and updates < max_up and step >= min_step:
            it += 1
            self._tick(it, max_it)
            # X update
            gX = self._grad_u(A, M, X @ Y, blocks) @ Y.T
            Xn = _prox(rx, X - step * scale * gX, step * scale * gx)
            # Y update
            gY = linalg_ops.tmm(Xn, self._grad_u(A, M, Xn @ Y, blocks))
            coll.allreduce_(gY)
            Yn = _prox(ry, Y - step * scale * gY, step * scale * gy)
            on = objective(Xn, Yn)
            updates += 1
            if on < obj:
                rel = (obj - on) / max(abs(obj), 1e-300)
                X, Y, obj = Xn, Yn, on
                step *= 1.05
                hist.append(obj)
                if rel < 1e-8:
                    break
            else:
                step /= 2
        self._X, self._Y = X, Y
        self._step = step
        o = self._output
        o["objective"] = obj
        o["iterations"] = it
        o["updates"] = updates
        o["step_size"] = step
        o["archetypes"] = self._archetypes_df()
        o["scoring_history"] = hist
        # loading_name: the reference's deprecated alias of representation_name
        rep = p.get("representation_name") or p.get("loading_name") or f"GLRMLoading_{self.model_id}"
        self._rep_name = rep
        if p.get("recover_svd"):
            Q, R = torch.linalg.qr(X.double())
            U2, S2, V2 = torch.linalg.svd(R @ Y.double(), full_matrices=False)
            o["singular_vals"] = S2.cpu().numpy()
            o["eigenvectors"] = V2.T.cpu().numpy()
        from ..core import dkv
        dkv.put(rep, self.representation_frame())

    def _user_y(self, uy, blocks, k):
        """GLRM.java:404 initialXY (init=User): user_y holds k rows; with
        expand_user_y its columns are the original ones (a categorical column
        gives the level index, expanded to its one-hot block), otherwise it
        is already in the expanded layout."""
        df = uy.as_data_frame() if hasattr(uy, "as_data_frame") else __import__("pandas").DataFrame(uy)
        P = sum(w for _, _, w in blocks)
        expand = bool(self._parms.get("expand_user_y", True))
        ncol = len(blocks) if expand else P
        if df.shape[1] != ncol:
            raise ValueError(f"ERRR on field: _user_y: The user-specified Y must have the same number of columns "
                             f"({ncol}) as the training observations")
        if df.shape[0] != k:
            raise ValueError(f"ERRR on field: _user_y: The user-specified Y must have k = {k} rows")
        if df.isna().values.any():
            raise ValueError("ERRR on field: _user_y: The user-specified Y cannot contain any missing values")
        if not expand:
            Y = np.asarray(df.values, dtype=np.float64)
        else:
            Y = np.zeros((k, P))
            j = 0
            for ci, (kind, c, w) in enumerate(blocks):
                col = df.iloc[:, ci]
                if kind == "cat":
                    dom = self._doms[c]
                    for r in range(k):
                        v = col.iloc[r]
                        lv = dom.index(v) if isinstance(v, str) and v in dom else int(float(v))
                        if 0 <= lv < w:
                            Y[r, j + lv] = 1.0
                else:
                    Y[:, j] = col.values.astype(np.float64)
                j += w
        if not np.any(Y):
            raise ValueError("ERRR on field: _user_y: The user-specified Y cannot all be zero")
        return torch.as_tensor(Y, dtype=torch.float32)

    def _user_x(self, ux, frame, k):
        """user_x: the initial representation X (one row per training row,
        k columns), taken shard by shard like the training frame."""
        if ux.nrows != frame.nrows:
            raise ValueError("ERRR on field: _user_x: The user-specified X must have the same number of rows "
                             f"({frame.nrows}) as the training observations")
        if ux.ncols != k:
            raise ValueError(f"ERRR on field: _user_x: The user-specified X must have k = {k} columns")
        X = torch.stack([ux.vec(c).as_float(torch.float32) for c in ux.names], 1)
        if bool(torch.isnan(X).any()):
            raise ValueError("ERRR on field: _user_x: The user-specified X cannot contain any missing values")
        if coll.allreduce_scalar(float(X.abs().sum())) == 0:
            raise ValueError("ERRR on field: _user_x: The user-specified X cannot all be zero")
        return X

    def _svd_init(self, A, M, k, n, g):
        """init = SVD (GLRM.java:458): the top-k right singular vectors of
        the training matrix from its all-reduced Gram (identical on every
        rank), by the svd_method of hex/svd/SVD.java: GramSVD = exact
        eigendecomposition, Power = power iterations with deflation,
        Randomized = k subspace iterations from a seeded Gaussian start."""
        Am = (A * M).double()
        G = Am.T @ Am
        coll.allreduce_(G)
        P = G.shape[0]
        method = str(self._parms.get("svd_method") or "Randomized").lower()
        if method == "gramsvd":
            lam, V = torch.linalg.eigh(G)
            order = torch.argsort(lam, descending=True)[:k]
            lam, V = lam[order], V[:, order]
        elif method == "power":
            V = torch.zeros((P, k), dtype=torch.float64, device=G.device)
            lam = torch.zeros(k, dtype=torch.float64, device=G.device)
            R = G.clone()
            iters = max(1, min(int(self._parms.get("max_iterations", 1000)), 1000))
            for j in range(k):
                v = torch.randn(P, generator=g, dtype=torch.float64).to(G.device)
                v = v / v.norm().clamp_min(1e-300)
                for _ in range(iters):
                    w = R @ v
                    nw = w.norm()
                    if float(nw) == 0:
                        break
                    w = w / nw
                    if float((w - v).abs().max()) < 1e-10:
                        v = w
                        break
                    v = w
                lam[j] = v @ (R @ v)
                V[:, j] = v
                R = R - lam[j] * torch.outer(v, v)
        else:   # randomized subspace iteration, k passes (GLRM.java:468)
            Q = torch.randn((P, k), generator=g, dtype=torch.float64).to(G.device)
            for _ in range(max(1, k)):
                Q, _ = torch.linalg.qr(G @ Q)
            B = Q.T @ G @ Q
            lb, W = torch.linalg.eigh(B)
            order = torch.argsort(lb, descending=True)
            lam, V = lb[order], Q @ W[:, order]
        Y = (torch.sqrt(lam.clamp_min(0)).view(-1, 1) * V.T) / math.sqrt(max(n, 1))
        return Y.to(torch.float32)

    def _init_x(self, A, M, Y, g):
        # least squares start: X = A Y^T (Y Y^T)^-1 (quadratic-loss optimum for fixed Y)
        k = Y.shape[0]
        G = Y @ Y.T + 1e-6 * torch.eye(k, device=Y.device)
        return torch.linalg.solve(G, Y @ (A * M).T).T.contiguous()

    def _archetypes_df(self):
        names = []
        for kind, c, w in self._blocks:
            if kind == "num":
                names.append(c)
            else:
                names += [f"{c}.{d}" for d in self._doms[c]]
        Y = self._Y.detach().cpu().numpy()
        df = pd.DataFrame(Y, columns=names)
        df.insert(0, "archetype", [f"Arch{i + 1}" for i in range(Y.shape[0])])
        return df

    def archetypes(self):
        return self._output["archetypes"].drop(columns=["archetype"]).values

    def representation_frame(self):
        X = self._X.detach()
        return H2OFrame.from_vecs([Vec(X[:, i].contiguous().to(torch.float32), T_REAL) for i in range(X.shape[1])],
                                  [f"Arch{i + 1}" for i in range(X.shape[1])])

    # ------------------------------------------------------------ scoring
    def _solve_x(self, frame, iters=None):
        """Rows of X for new data with Y fixed, every row independent like the
        reference's per-row scorer (hex/genmodel/algos/glrm/GlrmMojoModel.java
        score0): proximal gradient with a per-row step that grows 1.05x after
        an improving step and halves otherwise; a row stops when its relative
        improvement drops below 1e-9 or its step below 1e-8.  Vectorised over
        all rows on the device; the MOJO scorer (mojo/genmodel.py) runs the
        same recurrence in numpy."""
        A, M, blocks = self._layout(frame, self._cols)
        Y = self._Y.detach()
        p = self._parms
        rx, gx = p.get("regularization_x"), float(p.get("gamma_x", 0.0))
        iters = int(iters or self._score_iters())
        n = A.shape[0]
        X = _prox(rx, self._init_x(A, M, Y, None), 0.0)
        step = torch.full((n, 1), self._score_step(), dtype=X.dtype, device=X.device)
        obj = self._loss(A, M, X @ Y, blocks, per_row=True) + gx * _reg_rows(rx, X)
        live = torch.ones(n, dtype=torch.bool, device=X.device)
        for _ in range(iters):
            Xv = X.clone().requires_grad_(True)
            gX, = torch.autograd.grad(self._loss(A, M, Xv @ Y, blocks), Xv)
            Xn = _prox(rx, X - step * gX, step * gx)
            on = self._loss(A, M, Xn @ Y, blocks, per_row=True) + gx * _reg_rows(rx, Xn)
            better = (on < obj) & live
            rel = (obj - on) / obj.abs().clamp_min(1e-300)
            X = torch.where(better.view(-1, 1), Xn, X)
            obj = torch.where(better, on, obj)
            step = torch.where(better.view(-1, 1), step * 1.05, torch.where(live.view(-1, 1), step / 2, step))
            live = live & ~(better & (rel < 1e-9)) & (step.view(-1) >= 1e-8)
            if not bool(live.any()):
                break
        return X.detach(), A, M

    def _score_step(self):
        # 1 / (2 ||Y||_F^2) bounds the quadratic loss's curvature in x: a
        # descent step for every row from the first iteration
        return 0.5 / max(float((self._Y.detach().double() ** 2).sum()), 1e-12)

    def _score_iters(self):
        return 2000

    def _reconstruct(self, X):
        p = self._parms
        U = (X @ self._Y).detach()
        vecs, names = [], []
        j = 0
        tr = str(p.get("transform") or "NONE").upper()
        for kind, c, w in self._blocks:
            u = U[:, j:j + w]
            if kind == "num":
                x = _num_impute(self._col_loss(c), u[:, 0])
                if p.get("impute_original"):
                    mu, sd, lo, hi = self._stats[c]
                    if tr == "STANDARDIZE":
                        x = x * sd + mu
                    elif tr == "NORMALIZE":
                        x = x * (hi - lo) + lo
                    elif tr == "DEMEAN":
                        x = x + mu
                    elif tr == "DESCALE":
                        x = x * sd
                vecs.append(Vec(x.contiguous().to(torch.float32), T_REAL))
            else:
                vecs.append(Vec(_cat_impute(self._multi_loss(), u).to(torch.int32), T_ENUM, self._doms[c]))
            names.append(f"reconstr_{c}")
            j += w
        return H2OFrame.from_vecs(vecs, names)

    def predict(self, test_data, **kw):
        X, _, _ = self._solve_x(test_data)
        return self._reconstruct(X)

    def reconstruct(self, test_data, reverse_transform=False):
        old = self._parms.get("impute_original")
        self._parms["impute_original"] = reverse_transform
        try:
            return self.predict(test_data)
        finally:
            self._parms["impute_original"] = old

    def transform_frame(self, test_data):
        X, _, _ = self._solve_x(test_data)
        return H2OFrame.from_vecs([Vec(X[:, i].contiguous(), T_REAL) for i in range(X.shape[1])],
                                  [f"Arch{i + 1}" for i in range(X.shape[1])])

    def _predict_raw(self, frame):
        X, _, _ = self._solve_x(frame)
        return (X @ self._Y).detach()

    def _score_all(self, spec):
        from . import metrics as mm
        A, M, blocks = self._layout(spec.frame, self._cols)
        U = (self._X @ self._Y).detach()
        num = torch.tensor(0.0, device=U.device)
        cat = torch.tensor(0.0, device=U.device)
        j = 0
        for kind, c, w in blocks:
            if kind == "num":
                num = num + (((A[:, j] - U[:, j]) ** 2) * M[:, j]).sum()
            else:
                pred = U[:, j:j + w].argmax(1)
                truth = A[:, j:j + w].argmax(1)
                cat = cat + ((pred != truth) & (M[:, j] > 0)).sum()
            j += w
        m = mm.ModelMetrics(numerr=float(num), caterr=float(cat), objective=self._output["objective"])
        m.kind = "glrm"
        self._training_metrics = m
