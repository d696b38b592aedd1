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


class _Seg:
    """Segmented sums by a fixed integer key: rows sorted by key once, each
    sum a direct segmented reduction over the sorted values (no differencing
    of a global prefix sum: r = w e^eta spans many orders of magnitude, and a
    small per-event-time sum would cancel against the running total).
    Replaces index_add_ into few bins (every row of a stratum without a start
    column lands in bin 0: a million f64 atomics on one address serialise)."""

    def __init__(self, key, m):
        self.order = torch.argsort(key, stable=True)
        ks = key[self.order]
        bounds = torch.searchsorted(ks, torch.arange(m + 1, device=key.device, dtype=ks.dtype))
        self.lengths = (bounds[1:] - bounds[:-1]).to(torch.int64)
        self.m = m

    def __call__(self, v):
        vs = v[self.order]
        if vs.shape[0] == 0:
            return torch.zeros((self.m,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        return torch.segment_reduce(vs, "sum", lengths=self.lengths, axis=0, unsafe=True, initial=0.0)


class _Stratum:
    """Risk-set structure of one stratum, independent of beta: event times,
    each row's risk interval (jstart, jstop] in event-time indices, the
    events per time and the Efron (time, l) expansion."""

    def __init__(self, X, start, stop, ev, w, efron):
        self.X, self.w = X, w
        self.evm = ev > 0
        self.times = torch.unique(stop[self.evm])
        m = self.m = self.times.numel()
        if m == 0:
            return
        jstop = torch.searchsorted(self.times, stop, right=True)
        jstart = torch.searchsorted(self.times, start, right=True) if start is not None else torch.zeros_like(jstop)
        self.valid = jstop > jstart
        self.jstart, self.jstop = jstart, jstop
        self.seg_start = _Seg(jstart[self.valid], m + 1)
        self.seg_stop = _Seg(jstop[self.valid], m + 1)
        self.je = je = torch.searchsorted(self.times, stop[self.evm])
        self.seg_ev = _Seg(je, m)
        self.dcnt = dcnt = torch.bincount(je, minlength=m)
        wsum = self.seg_ev(w[self.evm])
        self.wbar = wsum / dcnt.clamp_min(1).to(X.dtype)
        self.jl = jl = torch.repeat_interleave(torch.arange(m, device=X.device), dcnt)
        start_of = torch.cumsum(dcnt, 0) - dcnt
        l_ = torch.arange(jl.numel(), device=X.device) - start_of[jl]
        self.frac = (l_.to(X.dtype) / dcnt[jl].to(X.dtype)) if efron else \
            torch.zeros(jl.numel(), dtype=X.dtype, device=X.device)
        self.seg_jl = _Seg(jl, m)
        self.wl = self.wbar[jl]
        self.Xev_w = (w[self.evm].view(-1, 1) * X[self.evm]).sum(0)

    def terms(self, beta):
        """loglik, gradient, Hessian (negative) at beta (float64)."""
        X, w = self.X, self.w
        P = X.shape[1]
        if self.m == 0:
            z = torch.zeros(P, dtype=X.dtype, device=X.device)
            return 0.0, z, torch.zeros((P, P), dtype=X.dtype, device=X.device)
        eta = X @ beta
        r = w * torch.exp(eta)
        rx = r.view(-1, 1) * X
        v = self.valid
        R0 = torch.cumsum(self.seg_start(r[v]) - self.seg_stop(r[v]), 0)[:self.m]
        R1 = torch.cumsum(self.seg_start(rx[v]) - self.seg_stop(rx[v]), 0)[:self.m]
        D0 = self.seg_ev(r[self.evm])
        D1 = self.seg_ev(rx[self.evm])
        jl, frac, wl = self.jl, self.frac, self.wl
        R0l = R0[jl] - frac * D0[jl]
        R1l = R1[jl] - frac.view(-1, 1) * D1[jl]
        ll = float((w[self.evm] * eta[self.evm]).sum() - (wl * torch.log(R0l)).sum())
        grad = self.Xev_w - ((wl / R0l).view(-1, 1) * R1l).sum(0)
        # Hessian part 1: sum over (j,l) of wbar (R2 - frac D2) / R0l as per-row weights
        c = wl / R0l
        C = self.seg_jl(c)
        Cf = self.seg_jl(c * frac)
        Pc = torch.cat([torch.zeros(1, dtype=X.dtype, device=X.device), torch.cumsum(C, 0)])
        a = torch.where(v, Pc[self.jstop] - Pc[self.jstart], torch.zeros_like(r))
        a_ev = torch.zeros_like(r)
        a_ev[self.evm] = Cf[self.je]
        a = r * (a - a_ev)
        H1 = linalg_ops.weighted_gram(X.to(torch.float32), a.to(torch.float32)) if (
            X.device.type == "cuda" and P % 32 == 0) else X.T @ (X * a.view(-1, 1))
        H2 = R1l.T @ (R1l * (wl / (R0l * R0l)).view(-1, 1))
        return ll, grad, H1.to(X.dtype) - H2


def _stratum_terms(X, start, stop, ev, w, beta, efron):
    """loglik, gradient, Hessian (negative) for one stratum (float64 tensors)."""
    return _Stratum(X, start, stop, ev, w, efron).terms(beta)


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

        strat = [_Stratum(X[g], start[g] if start is not None else None, stop[g], ev[g], w[g], efron)
                 for g in groups]

        def terms(b):
            L, G, H = 0.0, torch.zeros(P, dtype=torch.float64, device=X.device), \
                torch.zeros((P, P), dtype=torch.float64, device=X.device)
            for st in strat:
                l_, g_, h_ = st.terms(b)
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
