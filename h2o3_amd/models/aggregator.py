"""Aggregator: exemplar-based row reduction.

Reference: hex/aggregator/Aggregator.java + AggregatorModel.java (rows are
normalised/standardised, a row joins the nearest exemplar within `radius`
or becomes a new exemplar; the radius is adapted until the number of
exemplars is within rel_tol_num_exemplars of target_num_exemplars; output
`aggregated_frame` = exemplar rows + `counts`, optional mapping frame).

MI355X design: rows are processed in large chunks; the distances of a
chunk to all current exemplars are one GEMM (||x||^2 + ||e||^2 - 2 x e^T)
on the device, only rows farther than the radius from every exemplar go
through the greedy (sequential) new-exemplar pass, and membership counts
are a device bincount of the per-row argmin.  The radius search runs on a
device-resident sample, the final pass on all rows.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_ENUM, T_INT, T_REAL, Vec
from ..parallel import cloud
from ..parallel import collectives as coll
from .base import H2OEstimator
from .datainfo import DataInfo

AGG_DEFAULTS = dict(target_num_exemplars=5000, rel_tol_num_exemplars=0.5, transform="NORMALIZE",
                    categorical_encoding="AUTO", save_mapping_frame=False, num_iteration_without_new_exemplar=500,
                    seed=-1)


def _leader(C: torch.Tensor, radius2: float, budget=None, block=1024):
    """Sequential leader pass over candidate rows C (in order): a row becomes
    an exemplar unless it lies within radius of an earlier accepted one.
    Blocked: the distances to the exemplars accepted in earlier blocks are
    one GPU matrix product, only the survivors of a block are resolved
    sequentially against each other (their pairwise closeness precomputed
    in f64).  Returns accepted positions into C."""
    acc: list[int] = []
    A = C[:0].to(torch.float64)
    for s in range(0, C.shape[0], block):
        cb = C[s:s + block].to(torch.float64)
        if A.shape[0]:
            d = (cb * cb).sum(1, keepdim=True) + (A * A).sum(1).view(1, -1) - 2 * cb @ A.T
            fi = torch.nonzero(d.min(1).values > radius2).view(-1)
        else:
            fi = torch.arange(cb.shape[0], device=C.device)
        if fi.numel() == 0:
            continue
        F = cb[fi]
        nb = F.shape[0]
        # in-block greedy as a fixed point: a row is accepted once every earlier
        # close row is rejected, rejected once an earlier close row is accepted
        L = (torch.cdist(F, F) ** 2 <= radius2) & torch.ones(nb, nb, dtype=torch.bool, device=C.device).tril(-1)
        und = torch.ones(nb, dtype=torch.bool, device=C.device)
        accd = torch.zeros_like(und)
        while bool(und.any()):
            live = und | accd
            new_acc = und & ~(L & live.view(1, -1)).any(1)
            new_rej = und & (L & accd.view(1, -1)).any(1)
            accd |= new_acc
            und &= ~(new_acc | new_rej)
        keep = torch.nonzero(accd).view(-1)
        if budget is not None and len(acc) + keep.numel() > budget:
            keep = keep[:max(budget - len(acc) + 1, 0)]
        acc.extend(int(s + t) for t in fi[keep].cpu().tolist())
        A = torch.cat([A, F[keep]], 0)
        if budget is not None and len(acc) > budget:
            break
    return acc


def _exemplars(X: torch.Tensor, radius2: float, chunk=65536, max_ex=None):
    """Greedy leader clustering.  Returns (exemplar row indices, assignment)."""
    n = X.shape[0]
    ex_idx = []
    E = X[:0]
    for s in range(0, n, chunk):
        xb = X[s:s + chunk]
        if E.shape[0]:
            d = (xb * xb).sum(1, keepdim=True) + (E * E).sum(1).view(1, -1) - 2 * xb @ E.T
            far = d.min(1).values > radius2
        else:
            far = torch.ones(xb.shape[0], dtype=torch.bool, device=X.device)
        cand = torch.nonzero(far).view(-1)
        if cand.numel():
            budget = None if max_ex is None else max_ex - sum(int(t.numel()) for t in ex_idx)
            new = _leader(xb[cand], radius2, budget)
            sel = cand[torch.as_tensor(new, device=X.device, dtype=torch.long)]
            ex_idx.append(sel + s)
            E = torch.cat([E, xb[sel]], 0)
            if max_ex is not None and E.shape[0] > max_ex:
                break
    ex = torch.cat(ex_idx) if ex_idx else torch.zeros(0, dtype=torch.long, device=X.device)
    return ex, E


def _assign(X, E, chunk=65536):
    out = torch.empty(X.shape[0], dtype=torch.long, device=X.device)
    en = (E * E).sum(1).view(1, -1)
    for s in range(0, X.shape[0], chunk):
        xb = X[s:s + chunk]
        d = (xb * xb).sum(1, keepdim=True) + en - 2 * xb @ E.T
        out[s:s + chunk] = d.argmin(1)
    return out


class H2OAggregatorEstimator(H2OEstimator):
    _extra_params = ("seed",)   # deterministic sampling (not a reference client argument)
    algo = "aggregator"
    supervised_learning = False
    _defaults = AGG_DEFAULTS

    def _fit(self, spec):
        p = self._parms
        tr = str(p.get("transform") or "NORMALIZE").upper()
        di = DataInfo(spec.frame, spec.x, standardize=False, use_all_factor_levels=True, pad_to=0)
        X, ok = di.expand(spec.frame, dtype=torch.float32, pad=False)
        # column transform (reference: NONE / STANDARDIZE / NORMALIZE / DEMEAN / DESCALE)
        mu = X.mean(0)
        sd = X.std(0).clamp_min(1e-12)
        lo, hi = X.min(0).values, X.max(0).values
        if tr == "STANDARDIZE":
            X = (X - mu) / sd
        elif tr == "NORMALIZE":
            X = (X - lo) / (hi - lo).clamp_min(1e-12)
        elif tr == "DEMEAN":
            X = X - mu
        elif tr == "DESCALE":
            X = X / sd
        X = torch.nan_to_num(X)
        if cloud.is_distributed():
            X = coll.all_gather_var(X)
        n, P = X.shape
        target = int(p.get("target_num_exemplars", 5000))
        tol = float(p.get("rel_tol_num_exemplars", 0.5))
        if n <= target:
            ex = torch.arange(n, device=X.device)
            E = X
        else:
            gen = torch.Generator(device="cpu").manual_seed(int(p.get("seed", -1)) if p.get("seed", -1) != -1 else 42)
            perm = torch.randperm(n, generator=gen).to(X.device)
            Xs = X[perm]
            # radius search: binary search in log-space on a sample, then full pass
            samp = Xs[: min(n, max(20 * target, 50000))]
            span = float(((samp.max(0).values - samp.min(0).values) ** 2).sum())
            lo_r, hi_r = 1e-8 * max(span, 1e-12), max(span, 1e-12)
            r2 = math.sqrt(lo_r * hi_r)
            # Aggregator.java:197: stop once the exemplar count has not grown for
            # num_iteration_without_new_exemplar too-few rounds
            stall_max = int(p.get("num_iteration_without_new_exemplar", 500))
            prev, stall = -1, 0
            for _ in range(30):
                ex_s, _ = _exemplars(samp, r2, max_ex=int(target * (1 + tol) * 4))
                k = ex_s.numel() * (n / samp.shape[0]) ** 0.5 if samp.shape[0] < n else ex_s.numel()
                if abs(k - target) <= tol * target:
                    break
                if k > target:
                    lo_r = r2
                else:
                    hi_r = r2
                    if ex_s.numel() == prev:
                        stall += 1
                    if stall > stall_max:
                        break
                    prev = ex_s.numel()
                r2 = math.sqrt(lo_r * hi_r)
            for _ in range(20):
                ex_p, E = _exemplars(Xs, r2, max_ex=int(target * (1 + tol)) + 1)
                if ex_p.numel() <= target * (1 + tol):
                    break
                r2 *= 1.5
            ex = perm[ex_p]
        a = _assign(X, E)
        counts = torch.bincount(a, minlength=E.shape[0])
        self._ex_rows = ex.cpu().numpy()
        self._counts = counts.cpu().numpy()
        self._mapping = a.cpu().numpy() if p.get("save_mapping_frame") else None
        # aggregated frame = original exemplar rows + counts
        src = spec.frame
        if cloud.is_distributed():
            agg = None
        else:
            agg = src[list(map(int, self._ex_rows)), :]
            agg = agg[:, list(spec.x)] if spec.x else agg
            agg["counts"] = H2OFrame.from_vecs([Vec(torch.as_tensor(self._counts, dtype=torch.float32,
                                                                    device=cloud.device()), T_INT)], ["counts"])
        self._agg = agg
        self._output["num_exemplars"] = int(E.shape[0])
        self._output["radius"] = math.sqrt(r2) if n > target else 0.0

    @property
    def aggregated_frame(self):
        return self._agg

    @property
    def mapping_frame(self):
        if self._mapping is None:
            return None
        return H2OFrame.from_vecs([Vec(torch.arange(len(self._mapping), dtype=torch.float32), T_INT),
                                   Vec(torch.as_tensor(self._mapping, dtype=torch.float32), T_INT)],
                                  ["Row", "ExemplarIdx"])

    def _score_all(self, spec):
        pass

    def _predict_raw(self, frame):
        raise NotImplementedError("Aggregator has no predict(); use aggregated_frame")
