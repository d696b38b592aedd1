"""Cox proportional hazards.

Reference: hex/coxph/CoxPH.java (Newton-Raphson on the partial
likelihood, Efron / Breslow ties, counting-process (start, stop] data,
stratification, lre_min convergence), CoxPHModel.java (coef, exp_coef,
se_coef, z_coef, loglik, null loglik, concordance; predict = linear
predictor centred at the per-stratum covariate means).

MI355X design: no per-event loops over rows.  Rows are bucketed by event
time index with searchsorted; every risk-set sum (R0, R1) is a difference
array + cumulative sum over event times; the Hessian's sum over risk sets
of w e^eta x x' collapses to ONE weighted Gram (X' diag(a) X, the same
matrix-core Gram kernel GLM uses) with a per-row scalar weight a_i built
from prefix sums of 1/R0 over the event times inside the row's risk
interval; the Efron correction terms are an [E, P] GEMM.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_ENUM, T_REAL, Vec
from ..ops import linalg_ops
from ..parallel import cloud
from ..parallel import collectives as coll
from .base import H2OEstimator
from .datainfo import DataInfo

COX_DEFAULTS = dict(start_column=None, stop_column=None, stratify_by=None, ties="efron", init=0.0, lre_min=9.0,
                    max_iterations=20, use_all_factor_levels=False, interactions=None, interactions_only=None,
                    interaction_pairs=None, calc_cumhaz=True, single_node_mode=False)


def _stratum_terms(X, start, stop, ev, w, beta, efron):
    """loglik, gradient, Hessian (negative) for one stratum (float64 tensors)."""
    P = X.shape[1]
    eta = X @ beta
    r = w * torch.exp(eta)
    evm = ev > 0
    times = torch.unique(stop[evm])
    m = times.numel()
    if m == 0:
        z = torch.zeros(P, dtype=X.dtype, device=X.device)
        return 0.0, z, torch.zeros((P, P), dtype=X.dtype, device=X.device)
    # risk interval (jstart, jstop] in event-time indices
    jstop = torch.searchsorted(times, stop, right=True)
    jstart = torch.searchsorted(times, start, right=True) if start is not None else torch.zeros_like(jstop)
    valid = jstop > jstart
    R0d = torch.zeros(m + 1, dtype=X.dtype, device=X.device)
    R1d = torch.zeros((m + 1, P), dtype=X.dtype, device=X.device)
    R0d.index_add_(0, jstart[valid], r[valid])
    R0d.index_add_(0, jstop[valid], -r[valid])
    rx = r.view(-1, 1) * X
    R1d.index_add_(0, jstart[valid], rx[valid])
    R1d.index_add_(0, jstop[valid], -rx[valid])
    R0 = torch.cumsum(R0d, 0)[:m]
    R1 = torch.cumsum(R1d, 0)[:m]
    # events at each time
    je = torch.searchsorted(times, stop[evm])
    D0 = torch.zeros(m, dtype=X.dtype, device=X.device).index_add_(0, je, r[evm])
    D1 = torch.zeros((m, P), dtype=X.dtype, device=X.device).index_add_(0, je, rx[evm])
    dcnt = torch.bincount(je, minlength=m)
    wsum = torch.zeros(m, dtype=X.dtype, device=X.device).index_add_(0, je, w[evm])
    wbar = wsum / dcnt.clamp_min(1).to(X.dtype)
    # Efron expansion: one entry per (time j, l < d_j)
    jl = torch.repeat_interleave(torch.arange(m, device=X.device), dcnt)
    start_of = torch.cumsum(dcnt, 0) - dcnt
    l = torch.arange(jl.numel(), device=X.device) - start_of[jl]
    frac = (l.to(X.dtype) / dcnt[jl].to(X.dtype)) if efron else torch.zeros(jl.numel(), dtype=X.dtype,
                                                                             device=X.device)
    R0l = R0[jl] - frac * D0[jl]
    R1l = R1[jl] - frac.view(-1, 1) * D1[jl]
    wl = wbar[jl]
    ll = float((w[evm] * eta[evm]).sum() - (wl * torch.log(R0l)).sum())
    grad = (w[evm].view(-1, 1) * X[evm]).sum(0) - ((wl / R0l).view(-1, 1) * R1l).sum(0)
    # Hessian part 1: sum over (j,l) of wbar (R2 - frac D2) / R0l as per-row weights
    c = wl / R0l
    C = torch.zeros(m, dtype=X.dtype, device=X.device).index_add_(0, jl, c)
    Cf = torch.zeros(m, dtype=X.dtype, device=X.device).index_add_(0, jl, c * frac)
    Pc = torch.cat([torch.zeros(1, dtype=X.dtype, device=X.device), torch.cumsum(C, 0)])
    a = torch.where(valid, Pc[jstop] - Pc[jstart], torch.zeros_like(r))
    a_ev = torch.zeros_like(r)
    a_ev[evm] = Cf[je]
    a = r * (a - a_ev)
    H1 = linalg_ops.weighted_gram(X.to(torch.float32), a.to(torch.float32)) if (
        X.device.type == "cuda" and P % 32 == 0) else X.T @ (X * a.view(-1, 1))
    H2 = R1l.T @ (R1l * (wl / (R0l * R0l)).view(-1, 1))
    return ll, grad, H1.to(X.dtype) - H2


class H2OCoxProportionalHazardsEstimator(H2OEstimator):
    algo = "coxph"
    _defaults = COX_DEFAULTS

    def _wants_categorical_response(self):
        return False

    def _resolve_columns(self, x, y, training_frame):
        p = self._parms
        skip = {p.get("start_column"), p.get("stop_column"), y} | set(p.get("stratify_by") or [])
        if x is None:
            x = [c for c in training_frame.names if c not in skip and c not in (p.get("weights_column"),
                                                                                 p.get("offset_column"))]
        return super()._resolve_columns([c for c in x if c not in skip], y, training_frame)

    def _cross_validate(self, spec):
        pass

    def _strata(self, frame):
        sb = self._parms.get("stratify_by") or []
        if not sb:
            return torch.zeros(frame.nlocal, dtype=torch.long, device=cloud.device())
        key = torch.zeros(frame.nlocal, dtype=torch.long, device=cloud.device())
        for c in sb:
            v = frame.vec(c)
            codes = self._adapt_enum(v, self._strata_domains[c]).long() if c in getattr(self, "_strata_domains", {}) \
                else v.data.long()
            key = key * (len(v.domain) + 1 if v.domain else 1_000_003) + codes.clamp(min=-1) + 1
        return key

    def _fit(self, spec):
        p = self._parms
        fr = spec.frame
        self._strata_domains = {c: list(fr.vec(c).domain) for c in (p.get("stratify_by") or [])
                                if fr.vec(c).domain is not None}
        di = DataInfo(fr, spec.x, standardize=False, use_all_factor_levels=bool(p.get("use_all_factor_levels")),
                      missing_values_handling="Skip", pad_to=0)
        self._dinfo = di
        X, ok = di.expand(fr, dtype=torch.float64, pad=False)
        stop = fr.vec(p["stop_column"]).as_float(torch.float64)
        start = fr.vec(p["start_column"]).as_float(torch.float64) if p.get("start_column") else None
        yv = fr.vec(spec.y)
        ev = (yv.data.long() == 1).to(torch.float64) if yv.type == T_ENUM else yv.as_float(torch.float64)
        w = spec.w_tensor()
        w = torch.ones_like(stop) if w is None else w.to(torch.float64)
        ok = ok & ~torch.isnan(stop) & ~torch.isnan(ev)
        if start is not None:
            ok = ok & ~torch.isnan(start)
        strata = self._strata(fr)
        # gather to rank 0 semantics: every rank needs the global risk sets
        X, stop, ev, w, strata = (coll.all_gather_var(t[ok]) for t in (X, stop, ev, w, strata))
        start = coll.all_gather_var(start[ok]) if start is not None else None
        us = torch.unique(strata)
        self._strata_keys = us.cpu().tolist()
        P = X.shape[1]
        beta = torch.full((P,), float(p.get("init") or 0.0), dtype=torch.float64, device=X.device)
        efron = str(p.get("ties", "efron")).lower() == "efron"
        lre = float(p.get("lre_min", 9.0))
        groups = [(strata == s) for s in us]

        def terms(b):
            L, G, H = 0.0, torch.zeros(P, dtype=torch.float64, device=X.device), \
                torch.zeros((P, P), dtype=torch.float64, device=X.device)
            for g in groups:
                l_, g_, h_ = _stratum_terms(X[g], start[g] if start is not None else None, stop[g], ev[g], w[g], b,
                                            efron)
                L += l_
                G += g_
                H += h_
            return L, G, H

        ll0, G, H = terms(beta)
        self._null_loglik = ll0 if float(p.get("init") or 0.0) == 0.0 else terms(torch.zeros_like(beta))[0]
        ll = ll0
        it = 0
        for it in range(1, int(p.get("max_iterations", 20)) + 1):
            try:
                step = torch.linalg.solve(H, G)
            except RuntimeError:
                step = torch.linalg.lstsq(H, G.view(-1, 1)).solution.view(-1)
            nb = beta + step
            lln, Gn, Hn = terms(nb)
            halv = 0
            while (not math.isfinite(lln) or lln < ll - 1e-12) and halv < 20:
                step = step / 2
                nb = beta + step
                lln, Gn, Hn = terms(nb)
                halv += 1
            conv = abs(lln - ll) <= 10 ** (-lre) * max(abs(lln), 1e-300) or \
                (abs(lln) > 0 and -math.log10(max(abs(lln - ll) / abs(lln), 1e-300)) >= lre)
            beta, ll, G, H = nb, lln, Gn, Hn
            if conv:
                break
        self._beta = beta
        cov = torch.linalg.pinv(H)
        se = torch.sqrt(torch.clamp(torch.diagonal(cov), min=0))
        names = di.coef_names
        # per-stratum covariate means (reference centres the linear predictor)
        self._means = {}
        for s, g in zip(self._strata_keys, groups):
            self._means[s] = (X[g] * w[g].view(-1, 1)).sum(0) / w[g].sum()
        b = beta.cpu().numpy()
        o = self._output
        o["coefficients_table"] = pd.DataFrame({"names": names, "coefficients": b, "exp_coef": np.exp(b),
                                                "exp_neg_coef": np.exp(-b), "se_coef": se.cpu().numpy(),
                                                "z_coef": b / np.maximum(se.cpu().numpy(), 1e-300)})
        o["loglik"] = ll
        o["null_loglik"] = self._null_loglik
        o["iter"] = it
        o["n"] = int(X.shape[0])
        o["total_event"] = int(ev.sum())
        o["var_coef"] = cov.cpu().numpy()
        o["loglik_test"] = 2 * (ll - self._null_loglik)
        lp = self._lp_tensor(X, strata)
        o["concordance"] = _concordance(stop, ev, lp, strata)

    def _lp_tensor(self, X, strata):
        lp = X @ self._beta
        base = torch.zeros_like(lp)
        for s, mu in self._means.items():
            base = torch.where(strata == s, (mu @ self._beta).expand_as(lp), base)
        return lp - base

    def coef(self):
        t = self._output["coefficients_table"]
        return dict(zip(t["names"], t["coefficients"]))

    def concordance(self):
        return self._output["concordance"]

    def _predict_raw(self, frame):
        X, ok = self._dinfo.expand(frame, dtype=torch.float64, pad=False)
        lp = self._lp_tensor(X, self._strata(frame))
        lp = torch.where(ok, lp, torch.full_like(lp, float("nan")))
        return lp.to(torch.float32).view(-1, 1)

    def predict(self, test_data, **kw):
        return H2OFrame.from_vecs([Vec(self._predict_raw(test_data)[:, 0].contiguous(), T_REAL)], ["lp"])

    def _score_all(self, spec):
        from . import metrics as mm
        m = mm.ModelMetrics(concordance=self._output["concordance"], loglik=self._output["loglik"])
        m.kind = "coxph"
        self._training_metrics = m


def _concordance(stop, ev, lp, strata, max_rows=20000):
    """Harrell's C over comparable pairs (event earlier, same stratum)."""
    n = stop.numel()
    if n > max_rows:
        g = torch.Generator(device="cpu").manual_seed(0)
        idx = torch.randperm(n, generator=g)[:max_rows].to(stop.device)
        stop, ev, lp, strata = stop[idx], ev[idx], lp[idx], strata[idx]
    conc = disc = ties = 0.0
    evi = torch.nonzero(ev > 0).view(-1)
    for s in range(0, evi.numel(), 1024):
        i = evi[s:s + 1024]
        comp = (stop.view(1, -1) > stop[i].view(-1, 1)) & (strata.view(1, -1) == strata[i].view(-1, 1))
        d = lp[i].view(-1, 1) - lp.view(1, -1)
        conc += float((comp & (d > 0)).sum())
        disc += float((comp & (d < 0)).sum())
        ties += float((comp & (d == 0)).sum())
    tot = conc + disc + ties
    return (conc + 0.5 * ties) / tot if tot > 0 else float("nan")
