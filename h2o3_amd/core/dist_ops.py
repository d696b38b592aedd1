"""Munging prims computed shard-locally with collectives -- no frame gathers,
no pandas -- identical code at one rank and at W ranks.

Reference:
* hex/quantile/Quantile.java:100,190 -- exact quantiles by iterative
  histogram refinement (a 1024-bin histogram per pass over the rows, the bin
  holding the target rank becomes the next pass's range);
* water/rapids/ast/prims/advmath/AstTable.java:27 -- per-chunk hash counts
  reduced across nodes (1-column integer fast path "Count", slow path
  "Counts", dense 2-column triples or the sparse 2-D layout);
* water/rapids/ast/prims/mungers/AstPivot.java:73 -- first non-NA value per
  (index, class), header from the class column;
* water/rapids/ast/prims/mungers/AstMelt.java:66 -- a per-chunk MRTask that
  emits, row by row, one output row per value column (row-major);
* water/rapids/ast/prims/mungers/AstRankWithinGroupBy.java -- sort by
  (group-by asc, sort columns), rank within each group, NA sort keys get NA;
* water/fvec/CreateInteractions.java -- interaction domains by descending
  level count, max_factors / min_occurrence pruning into "other";
* water/rapids/ast/prims/advmath/AstUnique.java, AstHist.java,
  AstCorrelation.java, AstDistance / AstDropDuplicates.

MI355X design.  Every prim is a pass over this rank's HBM-resident rows
(torch.unique / bincount / index_add / scatter_reduce) whose partial result
is reduced with ONE bucketed all-reduce, or -- when the partial is
dictionary-sized (unique keys, level counts) -- all-gathered and merged on
every rank.  Row-sized work that needs global order (duplicate detection,
group-wise selection) routes rows once with all_to_all (core/dist_munge.exchange)
to a hash or range owner and routes the verdict back.  At one rank the
collectives are no-ops and the same code runs.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..parallel import cloud
from ..parallel import collectives as coll
from .vec import T_ENUM, T_INT, T_REAL, T_TIME, Vec
from .groupsum import index_add as _ia

_BINS = 1024          # histogram bins per refinement pass (Quantile.java's nbins)
_GATHER_AT = 4096     # candidate values gathered and sorted exactly below this count


def _dev():
    return cloud.device()


def _dist():
    return cloud.is_distributed()


def _ar(t, op="sum"):
    if _dist():
        coll.allreduce_(t, op)
    return t


def _gather(t):
    return coll.all_gather_var(t.contiguous()) if _dist() else t


def _sharded_from_replicated(vecs, names):
    """A small result every rank holds in full -> row shards (the frame
    layout of core/frame._local_slice)."""
    from .frame import H2OFrame, _reshard
    fr = H2OFrame.from_vecs(vecs, names)
    return _reshard(fr) if _dist() else fr


def lexsort(keys):
    """Stable permutation sorting rows by keys[0], then keys[1], ... (each a
    1-D tensor; NaN must be mapped beforehand)."""
    n = keys[0].numel() if keys else 0
    idx = torch.arange(n, device=keys[0].device if keys else _dev())
    for k in reversed(keys):
        idx = idx[torch.argsort(k[idx], stable=True)]
    return idx


def global_key(v: Vec) -> torch.Tensor:
    """f64 sort / group key of a column, NaN for NA, consistent over ranks
    (enum: code; numeric / time: value; strings: rank in the global sorted
    dictionary of the column's values)."""
    if v.type == T_ENUM:
        c = v.data.to(torch.float64)
        return torch.where(v.data < 0, torch.full_like(c, math.nan), c)
    if v.on_host:
        arr = v.to_numpy()
        loc = sorted(set(x for x in arr if x is not None))
        allv = sorted(set().union(*coll.all_gather_object(loc))) if _dist() else loc
        m = {s: i for i, s in enumerate(allv)}
        return torch.tensor([m[x] if x is not None else math.nan for x in arr], dtype=torch.float64, device=_dev())
    return v.as_float(torch.float64)


# ------------------------------------------------------------------ order statistics
def _count(t):
    return int(_ar(torch.tensor([t.numel()], dtype=torch.int64, device=_dev()))[0])


def _range(t):
    big = math.inf
    mm = torch.tensor([float(t.min()) if t.numel() else big, -float(t.max()) if t.numel() else big],
                      dtype=torch.float64, device=_dev())
    _ar(mm, "min")
    return float(mm[0]), -float(mm[1])


def kth_smallest(x: torch.Tensor, k: int) -> float:
    """The k-th smallest (0-based) value of the multiset of every rank's x
    (no NaN): 1024-bin histogram refinement, each pass keeps only the bin
    holding rank k (Quantile.java:190), exact once few candidates remain."""
    cand, off = x, 0
    while True:
        n = _count(cand)
        if n <= _GATHER_AT:
            allv = torch.sort(_gather(cand)).values
            return float(allv[k - off])
        a, b = _range(cand)
        if a == b:
            return a
        # floor of a monotone map: bins respect the value order
        bins = ((cand - a) * (_BINS / (b - a))).floor().clamp_(0, _BINS - 1).long()
        cnt = _ar(torch.bincount(bins, minlength=_BINS))
        cum = torch.cumsum(cnt, 0)
        j = int(torch.searchsorted(cum, torch.tensor([k - off], dtype=cum.dtype, device=cum.device), right=True))
        off += int(cum[j - 1]) if j > 0 else 0
        cand = cand[bins == j]


def kth_smallest_many(x: torch.Tensor, ks) -> dict:
    """{k: k-th smallest (0-based)} for many ranks k at once over every rank's
    x (no NaN), exact.  Quantile.java's refinement, vectorised over targets:
    each pass is ONE pass over the surviving candidates -- every targeted bin
    of the previous pass becomes a group with its own 1024 sub-bins over the
    bin's edges, counted by one all-reduced bincount over all groups -- and
    groups with few values are finished exactly from a gather of their values.
    No per-group min / max scatter (a handful of slots taking 10^8 atomic
    updates): ranges come from the bin edges, and a group whose range has
    shrunk to rounding width gets its exact min / max by a masked reduction."""
    ks_l = sorted(set(int(k) for k in ks))
    if not ks_l:
        return {}
    dev = x.device
    cand = x.to(torch.float64)
    lo, hi = _range(cand)
    tk = torch.tensor(ks_l, dtype=torch.int64, device=dev)       # target ranks
    res = torch.full((tk.numel(),), math.nan, dtype=torch.float64, device=dev)
    if lo == hi:
        return dict(zip(ks_l, [lo] * len(ks_l)))
    gid = torch.zeros(cand.numel(), dtype=torch.int64, device=dev)
    tg = torch.zeros_like(tk)                                      # their group
    goff = torch.zeros(1, dtype=torch.int64, device=dev)          # rank offset per group
    ga = torch.tensor([lo], dtype=torch.float64, device=dev)      # group range [a, a + span]
    gspan = torch.tensor([hi - lo], dtype=torch.float64, device=dev)
    tpos = torch.arange(tk.numel(), device=dev)
    level = 0
    while tk.numel():
        G = goff.numel()
        cnt = _ar(torch.bincount(gid, minlength=G))
        # a range at rounding width (or a group still large after 4 passes,
        # i.e. narrowed 1024^4-fold: repeated values): exact min / max of those
        tiny = (gspan <= torch.maximum(ga.abs(), (ga + gspan).abs()) * 1e-12) | (level >= 4)
        level += 1
        const = torch.zeros(G, dtype=torch.bool, device=dev)
        for g in torch.nonzero(tiny & (cnt > _GATHER_AT)).view(-1).tolist():
            v = cand[gid == g]
            a, b = _range(v)
            if a == b:
                const[g] = True
                ga[g] = a
            else:
                ga[g], gspan[g] = a, b - a
        small = (cnt <= _GATHER_AT) | const
        if bool(small.any()):
            pick = small[gid] & ~const[gid]
            gv, gg = _gather(cand[pick]), _gather(gid[pick])
            o = lexsort([gg.to(torch.float64), gv])
            gv, gg = gv[o], gg[o]
            st = torch.searchsorted(gg, torch.arange(G, device=dev))
            ts = small[tg]
            g_s = tg[ts]
            pos = (st[g_s] + tk[ts] - goff[g_s]).clamp(0, max(gv.numel() - 1, 0))
            val = torch.where(const[g_s], ga[g_s], gv[pos] if gv.numel() else ga[g_s])
            res[tpos[ts]] = val
            tk, tg, tpos = tk[~ts], tg[~ts], tpos[~ts]
        if not tk.numel():
            break
        rem = ~small
        remap = torch.cumsum(rem.to(torch.int64), 0) - 1
        keep = rem[gid]
        cand, gid = cand[keep], remap[gid[keep]]
        R = int(rem.sum())
        a, span, off_r = ga[rem], gspan[rem], goff[rem]
        # floor of a monotone map: sub-bins respect the value order
        sub = ((cand - a[gid]) * (_BINS / span[gid])).floor().clamp_(0, _BINS - 1).long()
        idx = gid * _BINS + sub
        cum = torch.cumsum(_ar(torch.bincount(idx, minlength=R * _BINS)).view(R, _BINS), 1)
        tr = remap[tg]
        j = torch.searchsorted(cum[tr], (tk - off_r[tr]).view(-1, 1), right=True).view(-1)
        below = torch.where(j > 0, cum[tr, (j - 1).clamp(min=0)], torch.zeros_like(j))
        key = tr * _BINS + j
        ukey, inv = torch.unique(key, return_inverse=True)
        noff = torch.zeros(ukey.numel(), dtype=torch.int64, device=dev).scatter_(0, inv, off_r[tr] + below)
        ur, uj = torch.div(ukey, _BINS, rounding_mode="floor"), ukey % _BINS
        w = span[ur] / _BINS
        na = a[ur] + uj.to(torch.float64) * w
        # the edge sub-bins absorb the clamp: keep the group's full outer range there
        nspan = torch.where(uj == _BINS - 1, a[ur] + span[ur] - na, w)
        lut = torch.full((R * _BINS,), -1, dtype=torch.int64, device=dev)
        lut[ukey] = torch.arange(ukey.numel(), device=dev)
        ng = lut[idx]
        live = ng >= 0
        cand, gid = cand[live], ng[live]
        tg, goff, ga, gspan = inv, noff, na, nspan
    return dict(zip(ks_l, res.tolist()))


def weighted_lower(x: torch.Tensor, w: torch.Tensor, t: float) -> float:
    """Smallest value v with (sum of weights of values <= v) >= t over every
    rank's (x, w) -- the weighted quantile rule of quantile_values."""
    cand, cw, off = x, w, 0.0
    while True:
        n = _count(cand)
        if n <= _GATHER_AT:
            xs, ws = _gather(cand), _gather(cw)
            o = torch.argsort(xs, stable=True)
            c = torch.cumsum(ws[o], 0) + off
            i = int(torch.searchsorted(c, torch.tensor([t], dtype=c.dtype, device=c.device)).clamp(max=xs.numel() - 1))
            return float(xs[o][i])
        a, b = _range(cand)
        if a == b:
            return a
        bins = ((cand - a) * (_BINS / (b - a))).floor().clamp_(0, _BINS - 1).long()
        ws = _ar(_ia(torch.zeros(_BINS, dtype=torch.float64, device=cand.device), bins, cw))
        cum = torch.cumsum(ws, 0) + off
        j = int(torch.searchsorted(cum, torch.tensor([t], dtype=cum.dtype, device=cum.device)).clamp(max=_BINS - 1))
        off = float(cum[j - 1]) if j > 0 else off
        m = bins == j
        cand, cw = cand[m], cw[m]


def quantile_values(v: Vec, probs, method="interpolate", weights=None):
    """Quantiles of a column, exact, without gathering it (R type-7
    interpolation or low / high / average; weighted: the smallest value whose
    cumulative weight reaches p * total)."""
    x = v.as_float(torch.float64)
    ok = ~torch.isnan(x)
    x = x[ok]
    n = _count(x)
    if n == 0:
        return [math.nan] * len(probs)
    if weights is not None:
        w = weights[ok].to(torch.float64)
        tot = float(_ar(w.sum().view(1))[0])
        return [weighted_lower(x, w, p * tot) for p in probs]
    cache = {}

    def kth(k):
        if k not in cache:
            cache[k] = kth_smallest(x, k)
        return cache[k]
    out = []
    for p in probs:
        h = (n - 1) * p
        lo = int(math.floor(h))
        hi = min(lo + 1, n - 1)
        if method == "low":
            out.append(kth(lo))
        elif method == "high":
            out.append(kth(hi))
        elif method == "average":
            out.append((kth(lo) + kth(hi)) / 2 if h != lo else kth(lo))
        else:
            a = kth(lo)
            out.append(a + (h - lo) * (kth(hi) - a) if h != lo else a)
    return out


# ------------------------------------------------------------------ group-wise median / mode
def segment_median_mode(gid: torch.Tensor, x: torch.Tensor, G: int, op: str, combine: str = "interpolate") -> torch.Tensor:
    """Per-group median (torch.quantile 0.5 rule) or mode (most frequent value,
    ties -> smallest) of x over groups gid in [0, G), NaN ignored; one sort,
    no per-group loop."""
    dev = x.device
    res = torch.full((G,), math.nan, dtype=torch.float64, device=dev)
    ok = ~torch.isnan(x)
    g, v = gid[ok], x[ok].to(torch.float64)
    if v.numel() == 0:
        return res
    o = lexsort([g.to(torch.float64), v])
    g, v = g[o], v[o]
    if op == "median":
        cnt = torch.bincount(g, minlength=G)
        start = torch.cumsum(cnt, 0) - cnt
        has = cnt > 0
        lo = start + (cnt - 1).clamp(min=0) // 2
        hi = start + cnt // 2
        lo, hi = lo[has], hi[has]
        a, b = v[lo], v[hi]
        cm = str(combine).lower()
        # even counts: the two middle values combined like Quantile's
        # combine_method (lo / hi / the average)
        res[has] = a if cm in ("lo", "low") else b if cm in ("hi", "high") else torch.where(lo == hi, a, a + 0.5 * (b - a))
        return res
    # mode: runs of equal (group, value); per group the longest run, ties -> smallest value
    new = torch.ones(v.numel(), dtype=torch.bool, device=dev)
    new[1:] = (g[1:] != g[:-1]) | (v[1:] != v[:-1])
    rs = torch.nonzero(new).view(-1)
    rl = torch.diff(torch.cat([rs, torch.tensor([v.numel()], device=dev)]))
    rg, rv = g[rs], v[rs]
    o2 = lexsort([rg.to(torch.float64), -rl.to(torch.float64), rv])
    rg, rv = rg[o2], rv[o2]
    first = torch.ones(rg.numel(), dtype=torch.bool, device=dev)
    first[1:] = rg[1:] != rg[:-1]
    res[rg[first]] = rv[first]
    return res


def group_median_mode(gid: torch.Tensor, x: torch.Tensor, G: int, op: str, combine: str = "interpolate") -> torch.Tensor:
    """segment_median_mode over row-sharded (gid, x): each group's rows are
    routed once (all_to_all) to the rank owning a contiguous range of group
    ids, which computes its groups; the G-sized results are all-gathered."""
    if not _dist():
        return segment_median_mode(gid, x, G, op, combine)
    from .dist_munge import exchange
    W = cloud.world()
    dest = (gid * W) // max(G, 1)
    got = exchange([Vec(gid, T_INT), Vec(x.to(torch.float64), T_REAL)], dest)
    r = cloud.rank()
    g0 = (r * G + W - 1) // W            # first gid with gid * W // G == r
    g1 = ((r + 1) * G + W - 1) // W
    loc = segment_median_mode(got[0].data - g0, got[1].data, max(g1 - g0, 0), op, combine)
    return _gather(loc)


# ------------------------------------------------------------------ unique / table / hist
def unique(fr, include_nas=False):
    """AstUnique: the sorted distinct values of the first column (a
    dictionary-sized all-gather of per-rank uniques), row-sharded."""
    from .vec import make_string
    v = fr._vecs[0]
    name = fr.names[:1]
    if v.type == T_ENUM:
        codes = torch.unique(_gather(torch.unique(v.data)))
        if not include_nas:
            codes = codes[codes >= 0]
        return _sharded_from_replicated([Vec(codes.to(torch.int32), T_ENUM, v.domain)], name)
    if v.on_host:
        loc = set(x for x in v.data if x is not None or include_nas)
        allv = set().union(*coll.all_gather_object(sorted(loc, key=lambda s: (s is None, s)))) if _dist() else loc
        vals = sorted(allv, key=lambda s: (s is None, s))
        return _sharded_from_replicated([make_string(vals)], name)
    x = v.as_float(torch.float64)
    nan = torch.isnan(x)
    u = torch.unique(_gather(torch.unique(x[~nan])))
    if include_nas and int(_ar(torch.tensor([int(nan.any())], device=_dev()), "max")[0]):
        u = torch.cat([u, torch.tensor([math.nan], dtype=u.dtype, device=u.device)])
    return _sharded_from_replicated([Vec(u.to(torch.float32) if v.data.dtype == torch.float32 else u, v.type)], name)


def _key_counts(keys):
    """Global (distinct key rows [K, d] sorted lexicographically, counts [K])
    over rows with no NaN key: per-rank unique with counts, all-gathered
    (distinct-key sized), merged."""
    K = torch.stack(keys, 1)
    K = K[~torch.isnan(K).any(1)]
    u, c = torch.unique(K, dim=0, return_counts=True)
    if _dist():
        u, c = _gather(u), _gather(c)
        u, inv = torch.unique(u, dim=0, return_inverse=True)
        c = _ia(torch.zeros(u.shape[0], dtype=torch.int64, device=u.device), inv, c)
    return u, c


def _key_vec(vals, v: Vec):
    if v.type == T_ENUM:
        return Vec(vals.to(torch.int32), T_ENUM, v.domain)
    if v.on_host:
        from .vec import make_string
        arr = v.to_numpy()
        loc = sorted(set(x for x in arr if x is not None))
        allv = sorted(set().union(*coll.all_gather_object(loc))) if _dist() else loc
        return make_string([allv[int(i)] for i in vals.tolist()])
    return Vec(vals, T_INT if v.type == T_INT else v.type)


def _is_int_col(v: Vec, x: torch.Tensor) -> bool:
    if v.type == T_ENUM:
        return True
    if v.on_host or v.type == T_TIME:
        return False
    ok = ~torch.isnan(x)
    bad = int(_ar(torch.tensor([int((x[ok] != torch.round(x[ok])).any())], device=_dev()), "max")[0])
    return bad == 0


def table(fr, data2=None, dense=True):
    """AstTable.  One column: [col, "Count"] for integer / categorical columns
    spanning <= 1e6 values (the fast path), [col, "Counts"] otherwise; two
    columns: dense triples [c1, c2, "Counts"] or, dense=False, one row per c1
    value and one count column per c2 value."""
    vecs = list(fr._vecs)
    names = list(fr.names)
    if data2 is not None:
        vecs += list(data2._vecs)
        names += list(data2.names)
    if len(vecs) > 2:
        raise ValueError("table expects one or two columns")
    keys = [global_key(v) for v in vecs]
    if len(vecs) == 1:
        v, x = vecs[0], keys[0]
        u, c = _key_counts([x])
        u = u[:, 0]
        fast = _is_int_col(v, x)
        if fast and u.numel():
            fast = float(u.max() - u.min()) + 1 <= 1e6
        return _sharded_from_replicated([_key_vec(u, v), Vec(c.to(torch.float64), T_INT)],
                                        [names[0], "Count" if fast else "Counts"])
    u, c = _key_counts(keys)
    if dense:
        return _sharded_from_replicated([_key_vec(u[:, 0], vecs[0]), _key_vec(u[:, 1], vecs[1]),
                                         Vec(c.to(torch.float64), T_INT)], [names[0], names[1], "Counts"])
    rows, ri = torch.unique(u[:, 0], return_inverse=True)
    cols, ci = torch.unique(u[:, 1], return_inverse=True)
    M = torch.zeros((rows.numel(), cols.numel()), dtype=torch.float64, device=u.device)
    M[ri, ci] = c.to(torch.float64)
    out, onames = [_key_vec(rows, vecs[0])], [names[0]]
    v2 = vecs[1]
    for j, cv in enumerate(cols.tolist()):
        out.append(Vec(M[:, j].contiguous(), T_INT))
        onames.append(v2.domain[int(cv)] if v2.type == T_ENUM else repr(float(cv)))
    return _sharded_from_replicated(out, onames)


def hist(fr, breaks="sturges"):
    """AstHist: breaks, counts, mids and density from one all-reduced
    bincount (range and n from all-reduces; "fd" uses the exact distributed
    quartiles)."""
    v = fr._vecs[0]
    x = v.as_float(torch.float64)
    x = x[~torch.isnan(x)]
    n = _count(x)
    lo, hi = _range(x)
    if isinstance(breaks, (list, tuple)):
        edges = np.asarray(breaks, dtype=float)
    else:
        if breaks in ("sturges", "doane") or breaks is None:
            k = int(math.ceil(math.log2(max(n, 1)) + 1))
        elif breaks == "rice":
            k = int(math.ceil(2 * n ** (1 / 3)))
        elif breaks == "sqrt":
            k = int(math.ceil(math.sqrt(n)))
        elif breaks == "scott":
            s = _ar(torch.stack([x.sum(), (x * x).sum()]))
            mean = float(s[0]) / max(n, 1)
            sd = math.sqrt(max(float(s[1]) / max(n, 1) - mean * mean, 0.0) * n / max(n - 1, 1))
            k = int(math.ceil((hi - lo) / (3.5 * sd / n ** (1 / 3)))) if sd > 0 else 1
        elif breaks == "fd":
            q1, q3 = quantile_values(Vec(x, T_REAL), [0.25, 0.75])
            iqr = q3 - q1
            k = int(math.ceil((hi - lo) / (2 * iqr / n ** (1 / 3)))) if iqr > 0 else 1
        else:
            k = int(breaks)
        edges = np.linspace(lo, hi, k + 1)
    e = torch.tensor(edges, dtype=torch.float64, device=x.device)
    idx = torch.clamp(torch.searchsorted(e, x, right=True) - 1, 0, len(edges) - 2)
    counts = _ar(torch.bincount(idx, minlength=len(edges) - 1).to(torch.float64))
    mids = (e[:-1] + e[1:]) / 2
    dens = counts / max(float(counts.sum()), 1.0) / torch.diff(e)
    return _sharded_from_replicated([Vec(e[1:].clone(), T_REAL), Vec(counts, T_REAL), Vec(mids.clone(), T_REAL),
                                     Vec(mids.clone(), T_REAL), Vec(dens, T_REAL)],
                                    ["breaks", "counts", "mids_true", "mids", "density"])


# ------------------------------------------------------------------ correlation / covariance
def _num_matrix(fr):
    return torch.stack([v.as_float(torch.float64) for v in fr._vecs], 1)


def _centered_cross(a, b):
    """(global column means of a and b, sum over rows of (a - ma)' (b - mb),
    n) by two all-reduces (means first, then the centred cross products)."""
    n = _count(a[:, 0]) if a.shape[1] else 0
    s = _ar(torch.cat([a.sum(0), b.sum(0)]))
    ma, mb = s[: a.shape[1]] / max(n, 1), s[a.shape[1]:] / max(n, 1)
    ac, bc = a - ma, b - mb
    cr = ac.T @ bc if ac.shape[1] * bc.shape[1] > 64 else \
        torch.stack([torch.stack([(ac[:, i] * bc[:, j]).sum() for j in range(bc.shape[1])])
                     for i in range(ac.shape[1])])
    sq = torch.cat([(ac * ac).sum(0), (bc * bc).sum(0)])
    red = _ar(torch.cat([cr.reshape(-1), sq]))
    p = a.shape[1]
    cr = red[: cr.numel()].view(cr.shape)
    return cr, red[cr.numel(): cr.numel() + p], red[cr.numel() + p:], n


def _small_matrix_frame(c, names):
    return _sharded_from_replicated([Vec(c[:, j].contiguous(), T_REAL) for j in range(c.shape[1])], list(names))


def cor(x, y=None, method="Pearson", use="everything"):
    """AstCorrelation: all-reduced centred cross products (Pearson) or ranks
    from the distributed sort (Spearman); use = everything / all.obs /
    complete.obs."""
    a = _num_matrix(x)
    b = _num_matrix(y) if y is not None else a
    use = (use or "everything").lower()
    if use not in ("everything", "all.obs", "complete.obs"):
        raise ValueError(f"use must be everything, all.obs or complete.obs, got {use}")
    if use != "everything":
        bad = torch.isnan(a).any(1) | torch.isnan(b).any(1)
        nbad = int(_ar(torch.tensor([int(bad.sum())], device=_dev()))[0])
        if use == "all.obs" and nbad:
            raise ValueError("Missing values in the data: use complete.obs or everything")
        if nbad:
            a, b = a[~bad], b[~bad]
    if method.lower() == "spearman":
        a = torch.stack([global_rank(a[:, j]) for j in range(a.shape[1])], 1)
        b = torch.stack([global_rank(b[:, j]) for j in range(b.shape[1])], 1) if y is not None else a
    cr, sa, sb, _ = _centered_cross(a, b)
    c = cr / torch.sqrt(torch.outer(sa, sb))
    if c.numel() == 1:
        return float(c)
    return _small_matrix_frame(c, (y or x).names)


def cov(x, y=None):
    a = _num_matrix(x)
    b = _num_matrix(y) if y is not None else a
    cr, _, _, n = _centered_cross(a, b)
    c = cr / (n - 1)
    if c.numel() == 1:
        return float(c)
    return _small_matrix_frame(c, (y or x).names)


def global_rank(x: torch.Tensor) -> torch.Tensor:
    """0-based position of every local value in the global stable sort
    (NaN first; ties by global row order), f64 -- the argsort(argsort)
    ranking, computed with the distributed sort's range partitioning."""
    from .dist_munge import sort_positions
    k = torch.where(torch.isnan(x), torch.full_like(x, -math.inf), x)
    return sort_positions([k]).to(torch.float64)


# ------------------------------------------------------------------ duplicates / pivot / melt / rank / interaction
def _row_offset(n_local):
    if not _dist():
        return 0
    ns = coll.all_gather_object(int(n_local))
    return int(sum(ns[: cloud.rank()]))


def _hash_rows(keys):
    """64-bit mix of the f64 bit patterns of the key columns (NaN canonical)."""
    h = torch.zeros(keys[0].numel(), dtype=torch.int64, device=keys[0].device)
    for k in keys:
        b = torch.where(torch.isnan(k), torch.full_like(k, math.nan), k + 0.0).view(torch.int64)
        h = h * 1000003 + b
        h = h ^ (h >> 29)
        h = h * 0x5851F42D4C957F2D
        h = h ^ (h >> 32)
    return h


def drop_duplicates(fr, columns=None, keep="first"):
    """AstDropDuplicates: rows whose key columns repeat an earlier (keep =
    first) or later (keep = last) row are dropped.  Rows are hash-routed to an
    owner rank (one all_to_all of the keys and global row ids), the owner
    picks the survivor of each exact key group, and the verdicts come back
    with a second all_to_all; the surviving rows stay where they are (the
    order of the frame is kept)."""
    from .frame import H2OFrame
    from .munging import _take
    cols = columns or fr.names
    cols = [fr.names[c] if isinstance(c, int) else c for c in cols]
    keys = [global_key(fr.vec(c)) for c in cols]
    n = fr.nlocal
    dev = _dev()
    gidx = torch.arange(n, device=dev, dtype=torch.int64) + _row_offset(n)
    if _dist():
        from .dist_munge import exchange
        W = cloud.world()
        dest = torch.remainder(_hash_rows(keys), W)
        src = torch.full((n,), cloud.rank(), dtype=torch.int64, device=dev)
        loc = torch.arange(n, device=dev, dtype=torch.int64)
        got = exchange([Vec(k, T_REAL) for k in keys] + [Vec(gidx, T_INT), Vec(src, T_INT), Vec(loc, T_INT)], dest)
        rk = [g.data for g in got[: len(keys)]]
        rg, rsrc, rloc = got[-3].data, got[-2].data, got[-1].data
        keep_r = _survivors(rk, rg, keep)
        back = exchange([Vec(rloc[keep_r], T_INT)], rsrc[keep_r])
        sel = torch.sort(back[0].data).values
    else:
        sel = torch.nonzero(_survivors(keys, gidx, keep)).view(-1)
    res = H2OFrame.from_vecs([_take(v, sel) for v in fr._vecs], fr.names)
    for v in res._vecs:
        v.replicated = False
    return res


def _survivors(keys, gidx, keep):
    """Mask of rows that are the first (last) of their exact key group by
    global row id."""
    n = gidx.numel()
    if n == 0:
        return torch.zeros(0, dtype=torch.bool, device=gidx.device)
    ks = [torch.where(torch.isnan(k), torch.full_like(k, -math.inf), k) for k in keys]
    ksn = [torch.isnan(k).to(torch.float64) for k in keys]       # NA == NA, distinct from -inf
    o = lexsort(ks + ksn + [gidx.to(torch.float64) if keep == "first" else -gidx.to(torch.float64)])
    same = torch.ones(n, dtype=torch.bool, device=gidx.device)
    same[0] = False
    for k in ks + ksn:
        ko = k[o]
        same[1:] &= ko[1:] == ko[:-1]
    m = torch.zeros(n, dtype=torch.bool, device=gidx.device)
    m[o[~same]] = True
    return m


def pivot(fr, index, column, value):
    """AstPivot: one row per index value (sorted), one column per class of
    `column` (all domain levels for a categorical, the distinct integer values
    otherwise), holding the first non-NA `value` of that (index, class) in
    row order."""
    iv, cv, vv = fr.vec(index), fr.vec(column), fr.vec(value)
    ik = global_key(iv)
    if int(_ar(torch.tensor([int(torch.isnan(ik).sum())], device=_dev()))[0]):
        raise ValueError(f"Index column '{index}' has > 0 NAs")
    ck = global_key(cv)
    rows = torch.unique(_gather(torch.unique(ik)))
    if cv.type == T_ENUM:
        classes = torch.arange(len(cv.domain or []), dtype=torch.float64, device=_dev())
        header = list(cv.domain or [])
    else:
        cl = ck[~torch.isnan(ck)].floor()
        classes = torch.unique(_gather(torch.unique(cl)))
        header = [str(int(c)) for c in classes.tolist()]
    if classes.numel() <= 1:
        raise ValueError(f"Column: '{column}'is constant. Perhaps use transpose?")
    R, C = rows.numel(), classes.numel()
    x = vv.as_float(torch.float64)
    ok = ~torch.isnan(x) & ~torch.isnan(ck)
    ri = torch.searchsorted(rows, ik[ok])
    ci = torch.searchsorted(classes, ck[ok].floor() if cv.type != T_ENUM else ck[ok])
    cell = ri * C + ci
    n = fr.nlocal
    gidx = (torch.arange(n, device=_dev(), dtype=torch.int64) + _row_offset(n))[ok]
    big = torch.iinfo(torch.int64).max
    first = torch.full((R * C,), big, dtype=torch.int64, device=_dev()).scatter_reduce(0, cell, gidx, "amin")
    first = _ar(first, "min")
    win = gidx == first[cell]
    val = _ia(torch.zeros(R * C, dtype=torch.float64, device=_dev()), cell[win], x[ok][win])
    has = _ia(torch.zeros(R * C, dtype=torch.float64, device=_dev()), cell[win], torch.ones_like(x[ok][win]))
    red = _ar(torch.stack([val, has]))
    M = torch.where(red[1] > 0, red[0], torch.full_like(red[0], math.nan)).view(R, C)
    out = [_key_vec(rows, iv)] + [Vec(M[:, j].contiguous(), T_REAL) for j in range(C)]
    return _sharded_from_replicated(out, [index] + header)


def melt(fr, id_vars, value_vars=None, var_name="variable", value_name="value", skipna=False):
    """AstMelt: row by row, one output row per value column (row-major, as
    the reference MRTask emits them), var column categorical over the value
    column names; purely shard-local (the output keeps the input's row
    distribution)."""
    from .frame import H2OFrame
    from .munging import _take
    id_vars = list(id_vars or [])
    if value_vars is None:
        value_vars = [c for c in fr.names if c not in id_vars]
    value_vars = list(value_vars)
    if not value_vars:
        raise ValueError("Empty list of value_vars provided, value_vars needs to have at least one column name.")
    for c in value_vars:
        v = fr.vec(c)
        if not (v.is_numeric and v.type != T_ENUM):
            raise ValueError("You can only use `melt` with numerical columns. Categorical (and other) columns are not "
                             "supported.")
    n, K = fr.nlocal, len(value_vars)
    dev = _dev()
    vals = torch.stack([fr.vec(c).as_float(torch.float64) for c in value_vars], 1).reshape(-1)   # row-major
    row = torch.arange(n, device=dev).repeat_interleave(K)
    var = torch.arange(K, device=dev, dtype=torch.int32).repeat(n)
    if skipna:
        keep = ~torch.isnan(vals)
        vals, row, var = vals[keep], row[keep], var[keep]
    out = [_take(fr.vec(c), row) for c in id_vars] + [Vec(var, T_ENUM, list(value_vars)), Vec(vals, T_REAL)]
    res = H2OFrame.from_vecs(out, id_vars + [var_name, value_name])
    for v in res._vecs:
        v.replicated = False
    return res


def rank_within_group_by(fr, group_by_cols, sort_cols, ascending=None, new_col_name="New_Rank_column",
                         sort_cols_sorted=False):
    """AstRankWithinGroupBy: the frame sorted by (group-by columns ascending,
    sort columns in their directions) with a 1-based rank within each group;
    rows with an NA sort key get an NA rank and are not counted.  Groups that
    straddle rank boundaries continue their count from the previous rank
    (one all-gather of per-rank boundary records)."""
    from .frame import H2OFrame
    from .munging import sort as frame_sort
    gb = [fr.names[c] if isinstance(c, int) else c for c in group_by_cols]
    sc = [fr.names[c] if isinstance(c, int) else c for c in sort_cols]
    asc = list(ascending) if ascending is not None else [True] * len(sc)
    s = frame_sort(fr, gb + sc, [True] * len(gb) + [bool(a) for a in asc])
    n = s.nlocal
    dev = _dev()
    gk = [global_key(s.vec(c)) for c in gb]
    gk = [torch.where(torch.isnan(k), torch.full_like(k, -math.inf), k) for k in gk]
    bad = torch.zeros(n, dtype=torch.bool, device=dev)
    for c in sc:
        bad |= torch.isnan(global_key(s.vec(c)))
    newg = torch.ones(n, dtype=torch.bool, device=dev)
    if n:
        same = torch.ones(n - 1, dtype=torch.bool, device=dev)
        for k in gk:
            same &= k[1:] == k[:-1]
        newg[1:] = ~same
    gstart = torch.cumsum(newg.to(torch.int64), 0) - 1           # local group ordinal
    cnt = (~bad).to(torch.int64)
    cum = torch.cumsum(cnt, 0)
    # counted rows before each group's start (exclusive prefix at the group start)
    starts = torch.nonzero(newg).view(-1)
    base = (cum - cnt)[starts] if n else cum
    rank = cum - base[gstart]
    if _dist():
        # a group running across rank boundaries continues the count of the
        # ranks before: walk back over the per-rank boundary records
        fk = [float(k[0]) for k in gk] if n else None
        lk = [float(k[-1]) for k in gk] if n else None
        tail = int(cnt[starts[-1]:].sum()) if n else 0
        recs = coll.all_gather_object((n, fk, lk, tail))
        carry = 0
        if n:
            for q in range(cloud.rank() - 1, -1, -1):
                m, fq, lq, tq = recs[q]
                if m == 0:
                    continue
                if lq != fk:
                    break
                carry += tq
                if fq != lq:
                    break
        if carry:
            rank = torch.where(gstart == 0, rank + carry, rank)
    out = torch.where(bad, torch.full_like(rank, -1), rank).to(torch.float64)
    out = torch.where(bad, torch.full_like(out, math.nan), out)
    res = H2OFrame.from_vecs(list(s._vecs) + [Vec(out, T_INT)], list(s.names) + [new_col_name])
    for v in res._vecs:
        v.replicated = False
    if sort_cols_sorted:
        res = frame_sort(res, sc, [bool(a) for a in asc])
    return res


def _interact(a_codes, a_dom, b_codes, b_dom, same, max_factors, min_occurrence):
    """One CreateInteractions step: (codes, domain) of the interaction of two
    categorical code vectors (NA = -1 -> level "NA")."""
    dev = a_codes.device
    a = a_codes.to(torch.int64)
    b = b_codes.to(torch.int64)
    key = a if same else (a + 1) * (len(b_dom) + 1) + (b + 1)
    valid = a >= 0 if same else torch.ones_like(a, dtype=torch.bool)
    u, c = torch.unique(key[valid], return_counts=True)
    if _dist():
        u, c = _gather(u), _gather(c)
        u, inv = torch.unique(u, return_inverse=True)
        c = _ia(torch.zeros(u.numel(), dtype=torch.int64, device=dev), inv, c)
    # descending count, ties by key (the reference's hash order is unspecified)
    o = lexsort([-c.to(torch.float64), u.to(torch.float64)])
    u, c = u[o], c[o]
    keepn = 0
    for cc in c.tolist():
        if keepn < max_factors and cc >= min_occurrence:
            keepn += 1
        else:
            break
    kept = u[:keepn]
    dom = []
    for k in kept.tolist():
        if same:
            dom.append(a_dom[k])
        else:
            ai, bi = k // (len(b_dom) + 1) - 1, k % (len(b_dom) + 1) - 1
            dom.append((a_dom[ai] if ai >= 0 else "NA") + "_" + (b_dom[bi] if bi >= 0 else "NA"))
    other = keepn < u.numel()
    if other:
        dom.append("other")
    ks, kpos = torch.sort(kept)
    pos = torch.searchsorted(ks, key).clamp(max=max(ks.numel() - 1, 0))
    hit = (ks.numel() > 0) & (ks[pos] == key) if ks.numel() else torch.zeros_like(key, dtype=torch.bool)
    codes = torch.where(hit, kpos[pos] if ks.numel() else torch.zeros_like(key),
                        torch.full_like(key, len(dom) - 1 if other else -1))
    if same:
        codes = torch.where(a < 0, torch.full_like(codes, -1), codes)
    return codes.to(torch.int32), dom


def interaction(data, factors, pairwise, max_factors, min_occurrence):
    """CreateInteractions: categorical interaction columns of the factors
    (all together, or every pair when pairwise and >= 3 factors); each
    column's domain lists the level combinations by descending count,
    keeping at most max_factors with >= min_occurrence rows, the rest "other".
    Counts are all-reduced as per-rank level-count dictionaries; the codes
    are computed shard-locally."""
    import itertools
    from .frame import H2OFrame
    names = [data.names[f] if isinstance(f, int) else f for f in factors]
    for nme in names:
        if data.vec(nme).type != T_ENUM:
            raise ValueError(f"interaction: column {nme} is not categorical")
    combos = list(itertools.combinations(names, 2)) if (pairwise and len(names) >= 3) else [tuple(names)]
    out, onames = [], []
    for cmb in combos:
        v0 = data.vec(cmb[0])
        codes, dom, name = v0.data, list(v0.domain or []), cmb[0]
        if len(cmb) == 1:
            codes, dom = _interact(codes, dom, codes, dom, True, max_factors, min_occurrence)
        for nxt in cmb[1:]:
            vb = data.vec(nxt)
            codes, dom = _interact(codes, dom, vb.data, list(vb.domain or []), False, max_factors, min_occurrence)
            name = name + "_" + nxt
        out.append(Vec(codes, T_ENUM, dom))
        onames.append(name)
    res = H2OFrame.from_vecs(out, onames)
    for v in res._vecs:
        v.replicated = False
    return res
