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
from ..core.groupsum import index_add as _ia

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
        self.key = key
        self.order = torch.argsort(key, stable=True)
        ks = key[self.order]
        bounds = torch.searchsorted(ks, torch.arange(m + 1, device=key.device, dtype=ks.dtype))
        self.lengths = (bounds[1:] - bounds[:-1]).to(torch.int64)
        self.m = m

    def __call__(self, v):
        if v.dim() == 2 and v.is_cuda and v.shape[0] > 0:
            # [n, P] sums on the wave-merged grouped-sum kernel: torch's 2-D
            # segment_reduce runs ~67 ms at 1M x 10 on this stack
            from ..ops import metrics_ops
            if metrics_ops.available(v):
                return metrics_ops.group_sum(self.key, v, self.m).to(v.dtype)
        vs = v[self.order]
        if vs.shape[0] == 0:
            return torch.zeros((self.m,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        return torch.segment_reduce(vs, "sum", lengths=self.lengths, axis=0, unsafe=True, initial=0.0)


def _cumsum0(x):
    """cumsum over dim 0; a 2-D [m, P] input scans along its rows'
    contiguous copy (torch's outer-dimension scan kernel took 130 ms for
    [500k, 10] f64 on this stack)."""
    if x.dim() == 2 and x.is_cuda:
        return torch.cumsum(x.T.contiguous(), 1).T
    return torch.cumsum(x, 0)


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
        R1 = _cumsum0(self.seg_start(rx[v]) - self.seg_stop(rx[v]))[:self.m]
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
            X.device.type == "cuda" and P % 32 == 0) else linalg_ops.tmm(X, X * a.view(-1, 1))
        H2 = linalg_ops.tmm(R1l, R1l * (wl / (R0l * R0l)).view(-1, 1))
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
        # interactions / interaction_pairs / interactions_only (Model.InteractionSpec):
        # interactions-only columns feed the interaction features but are not
        # main effects themselves
        from .glm.interactions import interaction_pairs
        io = [c for c in (p.get("interactions_only") or []) if c]
        for c in io:
            if c not in fr.names:
                raise ValueError(f"ERRR on field: interactions_only: {c} not found in the training frame")
        pairs = interaction_pairs(spec.x, p.get("interactions"), p.get("interaction_pairs"))
        used = {c for pr in pairs for c in pr}
        for c in io:
            if c not in used:
                import warnings
                warnings.warn(f"Column '{c}' was marked to be used for interactions only but it is not actually "
                              "required in any interaction.")
        x_main = [c for c in spec.x if c not in io]
        di = DataInfo(fr, x_main, standardize=False, use_all_factor_levels=bool(p.get("use_all_factor_levels")),
                      missing_values_handling="Skip", pad_to=0, interactions=pairs or None)
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
        if p.get("calc_cumhaz", True):
            self._cumhaz(X, stop, ev, w, strata, efron)

    def _cumhaz(self, X, stop, ev, w, strata, efron):
        """calc_cumhaz (CoxPH.java:503 calcCumhaz_0): the Breslow baseline
        hazard / survival per stratum at every distinct stop time, with
        risks exp((x - mean) . beta) (numeric covariates de-meaned as the
        reference's DEMEAN DataInfo), and the cumulative hazard of the
        mean covariate vector with its two variance terms (Efron or
        Breslow tie handling) for survfit-style curves.  One sort + segment
        sums on the device; the per-time recursion is a cumsum."""
        di = self._dinfo
        beta = self._beta
        xc = X.clone()
        nb = di.n_cat_expanded
        if xc.shape[1] > nb:
            xc[:, nb:] = xc[:, nb:] - xc[:, nb:].mean(0, keepdim=True)
        risk = w * torch.exp(xc @ beta)
        times, tix = torch.unique(stop, return_inverse=True)
        T = times.numel()
        keys = self._strata_keys
        S = len(keys)
        sidx = torch.zeros_like(tix)
        for i, k in enumerate(keys):
            sidx = torch.where(strata == k, torch.full_like(tix, i), sidx)
        flat = sidx * T + tix
        def seg(v):
            out = torch.zeros(S * T, dtype=torch.float64, device=X.device)
            _ia(out, flat, v)
            return out.view(S, T)
        size_ev = seg(w * ev)
        risk_all = seg(risk)
        total = torch.zeros(S, dtype=torch.float64, device=X.device)
        _ia(total, sidx, risk)
        # risk still at stake before time t: total minus the rows that left earlier
        at_risk = total.view(-1, 1) - (torch.cumsum(risk_all, 1) - risk_all)
        haz = torch.where(size_ev > 0, size_ev / at_risk.clamp_min(1e-300), torch.zeros_like(size_ev))
        surv = torch.exp(-torch.cumsum(haz, 1))
        tn = times.cpu().numpy()
        names = ["t"] + ([",".join(str(v) for v in self._strata_label(k)) for k in keys] if self._strata_domains
                         else [])
        hz_cols = {"t": tn}
        sv_cols = {"t": tn}
        if not self._strata_domains:
            hz_cols["baseline hazard"] = haz[0].cpu().numpy()
            sv_cols["baseline survival"] = surv[0].cpu().numpy()
        else:
            for i, nm in enumerate(names[1:]):
                hz_cols[nm] = haz[i].cpu().numpy()
                sv_cols[nm] = surv[i].cpu().numpy()
        self._output["baseline_hazard"] = H2OFrame(pd.DataFrame(hz_cols))
        self._output["baseline_survival"] = H2OFrame(pd.DataFrame(sv_cols))
        # cumhaz_0 / var_cumhaz_1 / var_cumhaz_2 over the times with any row
        ev_cnt = seg(ev * (w > 0)).sum(0)
        sz = size_ev.sum(0)
        rs_all = risk_all.sum(0)
        rcum = torch.flip(torch.cumsum(torch.flip(rs_all, [0]), 0), [0])      # risk of stop >= t
        xr = torch.zeros((T, X.shape[1]), dtype=torch.float64, device=X.device)
        _ia(xr, tix, xc * risk.view(-1, 1))
        rcum_x = torch.flip(_cumsum0(torch.flip(xr, [0])), [0])
        rev = torch.zeros(T, dtype=torch.float64, device=X.device)
        _ia(rev, tix, risk * ev)
        xrev = torch.zeros_like(xr)
        _ia(xrev, tix, xc * (risk * ev).view(-1, 1))
        present = torch.zeros(T, dtype=torch.bool, device=X.device)
        present[tix] = True
        ch = torch.zeros(T, dtype=torch.float64, device=X.device)
        v1 = torch.zeros_like(ch)
        v2 = torch.zeros_like(xr)
        if efron:
            cmax = int(ev_cnt.max().item()) if T else 0
            for e in range(cmax):
                m = ev_cnt > e
                frac = torch.where(m, e / ev_cnt.clamp_min(1), torch.zeros_like(ev_cnt))
                h = torch.where(m, 1.0 / (rcum - frac * rev).clamp_min(1e-300), torch.zeros_like(rcum))
                avg = torch.where(m, sz / ev_cnt.clamp_min(1), torch.zeros_like(sz))
                ch += avg * h
                v1 += avg * h * h
                v2 += (avg * h * h).view(-1, 1) * (rcum_x - frac.view(-1, 1) * xrev)
        else:
            ch = sz / rcum.clamp_min(1e-300)
            v1 = sz / (rcum * rcum).clamp_min(1e-300)
            v2 = (rcum_x / rcum.clamp_min(1e-300).view(-1, 1)) * ch.view(-1, 1)
        keep = present
        self._output["cumhaz_0"] = torch.cumsum(ch[keep], 0).cpu().numpy()
        self._output["var_cumhaz_1"] = torch.cumsum(v1[keep], 0).cpu().numpy()
        self._output["var_cumhaz_2"] = _cumsum0(v2[keep]).cpu().numpy()
        self._output["time"] = tn[keep.cpu().numpy()]

    def _strata_label(self, key):
        """Level names of a stratum key built by _strata (mixed radix)."""
        sb = self._parms.get("stratify_by") or []
        out = []
        k = int(key)
        for c in reversed(sb):
            dom = self._strata_domains.get(c)
            base = len(dom) + 1 if dom else 1_000_003
            code = k % base - 1
            k //= base
            out.append(dom[code] if dom and 0 <= code < len(dom) else "NA" if dom else code)
        return list(reversed(out))

    @property
    def baseline_hazard_frame(self):
        return self._output.get("baseline_hazard")

    @property
    def baseline_survival_frame(self):
        return self._output.get("baseline_survival")

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
