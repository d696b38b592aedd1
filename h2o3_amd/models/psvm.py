"""PSVM: parallel kernel SVM (Chang et al., "PSVM: Parallelizing Support
Vector Machines on Distributed Computers").

Reference: hex/psvm/PSVM.java, hex/psvm/psvm/IncompleteCholeskyFactorization.java,
hex/psvm/psvm/PrimalDualIPM.java, PSVMModel.java (gaussian kernel with
gamma (-1 = 1/#features), rank_ratio (-1 = sqrt(n)/n), pivoted incomplete
Cholesky K ~ H H', primal-dual interior point on the dual QP with
Sherman-Morrison-Woodbury solves against H, thresholds sv / fact /
feasible / surrogate-gap, mu_factor, positive / negative class weights;
the model keeps the support vectors and alpha*y; decision = sum alpha_i y_i
K(x_i, x) + b).

MI355X design: each ICF step is one kernel column = one GEMV-shaped
distance pass over the device-resident rows; the IPM's Newton system is
(diag + H~ H~')^-1 through a p x p Cholesky (p = rank) so every iteration
is two [n, p] GEMVs plus elementwise updates; scoring is a [n_test, n_sv]
distance GEMM + exp on the matrix cores.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..parallel import cloud
from ..parallel import collectives as coll
from .base import H2OEstimator
from .datainfo import DataInfo
from ..ops import linalg_ops

PSVM_DEFAULTS = dict(hyper_param=1.0, kernel_type="gaussian", gamma=-1.0, rank_ratio=-1.0, positive_weight=1.0,
                     negative_weight=1.0, disable_training_metrics=True, sv_threshold=1e-4, fact_threshold=1e-5,
                     feasible_threshold=1e-3, surrogate_gap_threshold=1e-3, mu_factor=10.0, max_iterations=200,
                     seed=-1)


def _kcol(X, xi, gamma):
    return torch.exp(-gamma * ((X - xi) ** 2).sum(1))


def icf(X, gamma, rank, tol):
    n = X.shape[0]
    H = torch.zeros((n, rank), dtype=torch.float64, device=X.device)
    diag = torch.ones(n, dtype=torch.float64, device=X.device)
    piv = []
    for j in range(rank):
        i = int(torch.argmax(diag))
        if float(diag[i]) < tol:
            H = H[:, :j]
            break
        piv.append(i)
        col = _kcol(X, X[i], gamma)
        if j:
            col = col - H[:, :j] @ H[i, :j]
        H[:, j] = col / math.sqrt(float(diag[i]))
        diag = diag - H[:, j] ** 2
        diag[i] = 0.0
    return H


def ipm(H, y, Cvec, mu_factor, feas_tol, gap_tol, max_iter):
    """Primal-dual IPM for min 1/2 a'Qa - 1'a, y'a = 0, 0 <= a <= C,
    Q = diag(y) H H' diag(y).  Returns (alpha, b)."""
    n, p = H.shape
    Ht = H * y.view(-1, 1)
    a = Cvec / 2
    # shift to satisfy y'a = 0 approximately
    lam = torch.ones(n, dtype=H.dtype, device=H.device)
    xi = torch.ones(n, dtype=H.dtype, device=H.device)
    nu = 0.0
    eye = torch.eye(p, dtype=H.dtype, device=H.device)
    for it in range(max_iter):
        Qa = Ht @ (Ht.T @ a)
        rd = Qa - 1 + nu * y - lam + xi
        rp = float(y @ a)
        gap = float(lam @ a + xi @ (Cvec - a))
        if float(rd.abs().max()) < feas_tol and abs(rp) < feas_tol and gap / n < gap_tol:
            break
        mu = gap / (2 * n) / mu_factor
        sig = lam / a + xi / (Cvec - a)
        z = -rd + (mu / a - lam) - (mu / (Cvec - a) - xi)
        # M = Ht Ht' + diag(sig): SMW with p x p Cholesky
        Di = 1.0 / sig
        Sm = eye + linalg_ops.tmm(Ht, Ht * Di.view(-1, 1))
        Lc = torch.linalg.cholesky(Sm)

        def Minv(v):
            t = Ht.T @ (Di * v)
            t = torch.cholesky_solve(t.view(-1, 1), Lc).view(-1)
            return Di * v - Di * (Ht @ t)

        Mz, My = Minv(z), Minv(y)
        dnu = (float(y @ Mz) + rp) / float(y @ My)
        da = Mz - dnu * My
        dlam = (mu - lam * a - lam * da) / a
        dxi = (mu - xi * (Cvec - a) + xi * da) / (Cvec - a)
        s = 1.0
        for v, dv in ((a, da), (lam, dlam), (xi, dxi), (Cvec - a, -da)):
            neg = dv < 0
            if bool(neg.any()):
                s = min(s, float((-v[neg] / dv[neg]).min()))
        s = min(1.0, 0.99 * s)
        a = a + s * da
        lam = lam + s * dlam
        xi = xi + s * dxi
        nu = nu + s * dnu
    return a, nu


class H2OSupportVectorMachineEstimator(H2OEstimator):
    algo = "psvm"
    _defaults = PSVM_DEFAULTS

    def _wants_categorical_response(self):
        return True

    def _score_all(self, spec):
        # PSVM.java:200: training metrics only with disable_training_metrics=False
        # (the default skips the O(n * #SV) scoring pass); validation always
        if not self._parms.get("disable_training_metrics", True):
            self._training_metrics = self._metrics_from_raw(spec, spec.frame, self._predict_raw(spec.frame))
        else:
            self._training_metrics = None
        if spec.valid is not None:
            self._validation_metrics = self._metrics_from_raw(spec, spec.valid, self._predict_raw(spec.valid))

    def _fit(self, spec):
        kt = str(self._parms.get("kernel_type") or "gaussian").lower()
        if kt != "gaussian":
            # PSVMModel.KernelType has the gaussian kernel only
            raise ValueError(f"kernel_type: unsupported kernel '{kt}' (only 'gaussian')")
        p = self._parms
        if spec.nclasses != 2:
            raise ValueError("PSVM supports binary classification only")
        di = DataInfo(spec.frame, spec.x, standardize=False, use_all_factor_levels=True, pad_to=0)
        self._dinfo = di
        X, ok = di.expand(spec.frame, dtype=torch.float64, pad=False)
        yl = spec.y_tensor().long()
        ok = ok & (yl >= 0)
        X, yl = coll.all_gather_var(X[ok]), coll.all_gather_var(yl[ok])
        y = torch.where(yl == 1, 1.0, -1.0).to(torch.float64)
        n, F = X.shape
        gamma = float(p.get("gamma", -1.0))
        gamma = 1.0 / F if gamma <= 0 else gamma
        rr = float(p.get("rank_ratio", -1.0))
        rank = int(math.sqrt(n)) if rr <= 0 else max(1, int(rr * n))
        rank = max(1, min(rank, n))
        H = icf(X, gamma, rank, float(p.get("fact_threshold", 1e-5)))
        C = float(p.get("hyper_param", 1.0))
        Cvec = torch.where(y > 0, C * float(p.get("positive_weight", 1.0)),
                           C * float(p.get("negative_weight", 1.0))).to(torch.float64)
        a, b = ipm(H, y, Cvec, float(p.get("mu_factor", 10.0)), float(p.get("feasible_threshold", 1e-3)),
                   float(p.get("surrogate_gap_threshold", 1e-3)), int(p.get("max_iterations", 200)))
        sv = a > float(p.get("sv_threshold", 1e-4)) * C
        self._sv = X[sv]
        self._ay = (a * y)[sv]
        self._gamma = gamma
        # bias: average over free support vectors of y - f_nobias (fallback: IPM multiplier)
        free = sv & (a < Cvec * (1 - 1e-3))
        if bool(free.any()):
            f = self._decision_nobias(X[free])
            self._b = float((y[free] - f).mean())
        else:
            self._b = float(b)
        self._output["svs_count"] = int(sv.sum())
        self._output["bsv_count"] = int((sv & ~free).sum())
        self._output["rho"] = -self._b
        self._output["rank"] = int(H.shape[1])
        self._output["gamma"] = gamma

    def _decision_nobias(self, Xq, chunk=8192):
        out = []
        S = self._sv
        sn = (S * S).sum(1).view(1, -1)
        for s in range(0, Xq.shape[0], chunk):
            q = Xq[s:s + chunk]
            d2 = (q * q).sum(1, keepdim=True) + sn - 2 * q @ S.T
            out.append(torch.exp(-self._gamma * d2.clamp_min(0)) @ self._ay)
        return torch.cat(out) if out else torch.zeros(0, dtype=torch.float64, device=Xq.device)

    def decision_function(self, frame):
        X, _ = self._dinfo.expand(frame, dtype=torch.float64, pad=False)
        return self._decision_nobias(X) + self._b

    def _predict_raw(self, frame):
        f = self.decision_function(frame)
        lab = (f > 0).to(torch.float32)
        # PSVM reports the label; class "probabilities" are the hard label
        return torch.stack([1 - lab, lab], 1)
