"""Frame munging: the Rapids prims behind the H2OFrame API.

Reference: water/rapids/ast/prims/mungers/* (AstGroup, AstMerge, AstSort,
AstCut, AstFillNA, AstMelt, AstPivot, AstRankWithinGroupBy, AstTable...),
water/rapids/ast/prims/advmath/* (AstQtile, AstKFold, AstStratifiedSplit,
AstCorrelation, AstHist, AstImpute, AstUnique...), hex/quantile/Quantile.java,
hex/SplitFrame.java, hex/createframe/*.

Design: group-by / merge / sort use GPU primitives (torch.unique with
inverse, argsort, searchsorted, index_add) on the HBM-resident columns.
With several ranks, sort / group-by / merge route rows with all_to_all
(core/dist_munge.py) and quantile / unique / table / hist / cor / cov /
pivot / melt / rank_within_group_by / interaction / drop_duplicates reduce
per-rank partials (core/dist_ops.py): no frame gathers, no pandas.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..parallel import cloud
from ..parallel import collectives as coll
from .frame import H2OFrame, _fmt_level, _local_slice, _reshard, _take, _to_enum, _vec_from_array
from .vec import NUMERIC_TYPES, T_ENUM, T_INT, T_REAL, T_STR, T_TIME, Vec, make_enum, make_numeric, make_string
from .groupsum import group_extreme, index_add as _ia


def _dev():
    return cloud.device()


# ---------------------------------------------------------------- quantiles
def quantile_values(v: Vec, probs, method="interpolate", weights=None):
    """Exact quantiles by distributed histogram refinement (core/dist_ops.py,
    hex/quantile/Quantile.java): no column gather at any W."""
    from .dist_ops import quantile_values as qv
    return qv(v, probs, method, weights)


def quantile(fr, prob=None, combine_method="interpolate", weights_column=None):
    from .dist_ops import _sharded_from_replicated
    probs = prob if prob is not None else [0.001, 0.01, 0.1, 0.25, 0.333, 0.5, 0.667, 0.75, 0.9, 0.99, 0.999]
    w = fr.vec(weights_column).as_float() if weights_column else None
    dev = _dev()
    vecs, names = [Vec(torch.tensor(probs, dtype=torch.float64, device=dev), T_REAL)], ["Probs"]
    for n, v in zip(fr.names, fr._vecs):
        if n == weights_column:
            continue
        q = quantile_values(v, probs, combine_method, w) if (v.is_numeric or v.is_time) else [float("nan")] * len(probs)
        vecs.append(Vec(torch.tensor(q, dtype=torch.float64, device=dev), T_REAL))
        names.append(f"{n}Quantiles")
    return _sharded_from_replicated(vecs, names)


def unique(fr, include_nas=False):
    from .dist_ops import unique as _u
    return _u(fr, include_nas)


def table(fr, data2=None, dense=True):
    from .dist_ops import table as _t
    return _t(fr, data2, dense)


def hist(fr, breaks="sturges"):
    from .dist_ops import hist as _h
    return _h(fr, breaks)


def _num_matrix(fr):
    return torch.stack([v.as_float(torch.float64) for v in fr._vecs], 1)


def _cross(ac, bc):
    """ac^T bc for [N, p] x [N, q] f64: per column pair reductions when p*q is
    small (a K = N f64 GEMM of a few columns runs on a poorly shaped library
    kernel: ~2 s at 20M rows), the GEMM otherwise."""
    p, q = ac.shape[1], bc.shape[1]
    if p * q <= 64:
        return torch.stack([torch.stack([(ac[:, i] * bc[:, j]).sum() for j in range(q)]) for i in range(p)])
    return ac.T @ bc


def cor(x, y=None, method="Pearson", use="everything"):
    """AstCorrelation without gathers (core/dist_ops.cor)."""
    from .dist_ops import cor as _c
    return _c(x, y, method, use)


def cov(x, y=None):
    from .dist_ops import cov as _c
    return _c(x, y)


def distance(x, y, measure="l2"):
    """AstDistance: rows of x (this rank's shard, the result stays sharded)
    against every row of y (the reference's MRTask over x broadcasts y)."""
    a = _num_matrix(x)
    b = _num_matrix(y.gather() if cloud.is_distributed() else y)
    m = measure.lower()
    if m == "l1":
        d = torch.cdist(a, b, p=1)
    elif m == "l2":
        d = torch.cdist(a, b, p=2)
    elif m == "cosine":
        d = (a @ b.T) / torch.outer(a.norm(dim=1), b.norm(dim=1))
    elif m == "cosine_sq":
        d = ((a @ b.T) / torch.outer(a.norm(dim=1), b.norm(dim=1))) ** 2
    else:
        raise ValueError(measure)
    return H2OFrame.from_tensor(d)


# ---------------------------------------------------------------- random / split
def _global_uniform(fr, seed):
    """Uniform [0,1) per global row, identical regardless of sharding."""
    seed = 42 if seed is None or seed == -1 else int(seed)
    g = torch.Generator(device="cpu").manual_seed(seed & 0x7FFFFFFFFFFF)
    n = fr.nrows
    off = fr.row_offset()
    r = torch.rand(n, generator=g, dtype=torch.float64)[off: off + fr.nlocal]
    return r.to(_dev())


def runif(fr, seed=None):
    r = _global_uniform(fr, seed)
    return H2OFrame.from_vecs([Vec(r, T_REAL)], ["rnd"])


def split_frame(fr, ratios, seed=None):
    """reference: hex/SplitFrame.java (random per-row assignment)."""
    r = _global_uniform(fr, seed)
    edges = np.cumsum([0.0] + list(ratios))
    out = []
    for i in range(len(ratios) + 1):
        lo = edges[i]
        hi = edges[i + 1] if i < len(ratios) else 1.0 + 1e-12
        m = (r >= lo) & (r < hi)
        out.append(fr[m])
    return out


def kfold_column(fr, n_folds=3, seed=-1):
    r = _global_uniform(fr, seed)
    f = torch.floor(r * n_folds).clamp(max=n_folds - 1)
    return H2OFrame.from_vecs([Vec(f.to(torch.float32), T_INT)], ["fold"])


def modulo_kfold_column(fr, n_folds=3):
    off = fr.row_offset()
    f = (torch.arange(off, off + fr.nlocal, device=_dev()) % n_folds).to(torch.float32)
    return H2OFrame.from_vecs([Vec(f, T_INT)], ["fold"])


def stratified_kfold_column(fr, n_folds=3, seed=-1):
    v = fr._vecs[0]
    y = v.data if v.type == T_ENUM else v.as_float().nan_to_num(-1).to(torch.int64)
    r = _global_uniform(fr, seed)
    f = torch.zeros(fr.nlocal, dtype=torch.float32, device=_dev())
    for c in torch.unique(y).tolist():
        idx = torch.nonzero(y == c).flatten()
        o = torch.argsort(r[idx])
        f[idx[o]] = (torch.arange(idx.numel(), device=_dev()) % n_folds).to(torch.float32)
    return H2OFrame.from_vecs([Vec(f, T_INT)], ["fold"])


def stratified_split(fr, test_frac=0.2, seed=-1):
    v = fr._vecs[0]
    y = v.data if v.type == T_ENUM else v.as_float().nan_to_num(-1).to(torch.int64)
    r = _global_uniform(fr, seed)
    out = np.empty(fr.nlocal, dtype=object)
    lab = torch.zeros(fr.nlocal, dtype=torch.int32, device=_dev())
    for c in torch.unique(y).tolist():
        idx = torch.nonzero(y == c).flatten()
        o = torch.argsort(r[idx])
        ntest = int(round(test_frac * idx.numel()))
        lab[idx[o[:ntest]]] = 1
    return H2OFrame.from_vecs([Vec(lab, T_ENUM, ["train", "test"])], ["test_train_split"])


# ---------------------------------------------------------------- rbind
def rbind(frames):
    frames = [f if isinstance(f, H2OFrame) else H2OFrame(f) for f in frames]
    base = frames[0]
    vecs = []
    for j, n in enumerate(base.names):
        parts = [f._vecs[j] for f in frames]
        t = parts[0].type
        if any(p.type == T_ENUM for p in parts):
            dom = []
            for p in parts:
                for d in (p.domain or []):
                    if d not in dom:
                        dom.append(d)
            codes = []
            for p in parts:
                if p.type == T_ENUM:
                    rm = torch.tensor([dom.index(d) for d in p.domain] or [0], dtype=torch.int32, device=_dev())
                    codes.append(torch.where(p.data < 0, p.data, rm[p.data.clamp(min=0).long()]))
                else:
                    vals = p.to_numpy()
                    codes.append(torch.tensor([dom.index(_fmt_level(x)) if x is not None and not (isinstance(x, float) and math.isnan(x)) and _fmt_level(x) in dom else -1 for x in vals], dtype=torch.int32, device=_dev()))
            vecs.append(Vec(torch.cat(codes), T_ENUM, dom))
        elif any(p.on_host for p in parts):
            vecs.append(make_string(np.concatenate([np.asarray(p.to_numpy(), dtype=object) for p in parts])))
        else:
            dt = torch.float64 if any(p.data.dtype == torch.float64 for p in parts) else torch.float32
            vv = Vec(torch.cat([p.as_float(dt) for p in parts]), t if all(p.type == t for p in parts) else T_REAL)
            vecs.append(vv)
    return H2OFrame.from_vecs(vecs, base.names)


# ---------------------------------------------------------------- sort / merge / group-by
def _key_tensor(v: Vec):
    if v.type == T_ENUM:
        return v.data.to(torch.float64)
    if v.on_host:
        arr = v.to_numpy()
        uniq = sorted(set(x for x in arr if x is not None))
        m = {s: i for i, s in enumerate(uniq)}
        return torch.tensor([m[x] if x is not None else float("nan") for x in arr], dtype=torch.float64, device=_dev())
    return v.as_float(torch.float64)


def sort(fr, by, ascending=True):
    from . import dist_munge
    if dist_munge.eligible(fr):
        return dist_munge.sort(fr, by, ascending)
    g = fr.gather()
    by = by if isinstance(by, (list, tuple)) else [by]
    asc = ascending if isinstance(ascending, (list, tuple)) else [ascending] * len(by)
    idx = torch.arange(g.nlocal, device=_dev())
    for b, a in reversed(list(zip(by, asc))):
        k = _key_tensor(g.vec(b))[idx]
        k = torch.where(torch.isnan(k), torch.full_like(k, -math.inf), k)  # NAs first (reference)
        o = torch.argsort(k if a else -k, stable=True)
        idx = idx[o]
    res = H2OFrame.from_vecs([_take(v, idx) for v in g._vecs], g.names)
    for v in res._vecs:
        v.replicated = g._vecs[0].replicated
    return _reshard(res) if cloud.is_distributed() else res


def _group_ids(frame, cols):
    """(unique key rows [G, ncols] in lexicographic order, group id per row).
    Each key column is ranked by a 1-D sort-unique, the ranks are combined
    mixed-radix (first column most significant, so the group order is the
    lexicographic order of torch.unique(dim=0)) and one more 1-D unique gives
    the groups -- a row-wise unique_dim sort is ~60x slower."""
    keys = [_key_tensor(frame.vec(c)) for c in cols]
    keys = [torch.where(torch.isnan(k), torch.full_like(k, -1e300), k) for k in keys]
    if not keys or keys[0].numel() == 0:
        K = torch.stack(keys, 1) if keys else torch.zeros((0, 0))
        return torch.unique(K, dim=0, return_inverse=True) if keys else (K, torch.zeros(0, dtype=torch.int64))
    vals, ranks = [], []
    for k in keys:
        u, r = torch.unique(k, return_inverse=True)
        vals.append(u)
        ranks.append(r)
    card = [int(u.numel()) for u in vals]
    tot = 1
    for c in card:
        tot *= max(c, 1)
    if tot >= (1 << 62):
        K = torch.stack(keys, 1)
        return torch.unique(K, dim=0, return_inverse=True)
    code = torch.zeros_like(ranks[0])
    for r, c in zip(ranks, card):
        code = code * c + r
    ucode, inv = torch.unique(code, return_inverse=True)
    cols_u = []
    rem = ucode
    for u, c in zip(reversed(vals), reversed(card)):
        cols_u.append(u[rem % c])
        rem = rem // c
    uniq = torch.stack(list(reversed(cols_u)), 1)
    return uniq, inv


class GroupBy:
    """reference: AstGroup (group-by with aggregates count/sum/mean/min/max/sd/var/ss/nrow/median/mode)."""

    def __init__(self, fr, by):
        self.fr = fr
        self.by = [fr.names[b] if isinstance(b, int) else b for b in (by if isinstance(by, (list, tuple)) else [by])]
        self.aggs = []
        self._res = None

    def _add(self, op, col, na):
        cols = [c for c in self.fr.names if c not in self.by] if col is None else (col if isinstance(col, (list, tuple)) else [col])
        for c in cols:
            self.aggs.append((op, c, na))
        return self

    def count(self, na="all"):
        self.aggs.append(("nrow", None, na))
        return self

    def sum(self, col=None, na="all"): return self._add("sum", col, na)
    def mean(self, col=None, na="all"): return self._add("mean", col, na)
    def min(self, col=None, na="all"): return self._add("min", col, na)
    def max(self, col=None, na="all"): return self._add("max", col, na)
    def sd(self, col=None, na="all"): return self._add("sd", col, na)
    def var(self, col=None, na="all"): return self._add("var", col, na)
    def ss(self, col=None, na="all"): return self._add("ss", col, na)
    def median(self, col=None, na="all"): return self._add("median", col, na)
    def mode(self, col=None, na="all"): return self._add("mode", col, na)

    def get_frame(self):
        if self._res is not None:
            return self._res
        from . import dist_munge
        if dist_munge.eligible(self.fr):
            res = dist_munge.group_by(self.fr, self.by, self.aggs)
            if res is not None:
                self._res = _reshard(res)
                return self._res
        fr = self.fr.gather() if cloud.is_distributed() else self.fr
        uniq, inv = _group_ids(fr, self.by)
        G = uniq.shape[0]
        out_vecs, out_names = [], []
        for j, b in enumerate(self.by):
            v = fr.vec(b)
            col = uniq[:, j]
            col = torch.where(col == -1e300, torch.full_like(col, float("nan")), col)
            if v.type == T_ENUM:
                out_vecs.append(Vec(torch.nan_to_num(col, nan=-1).to(torch.int32), T_ENUM, v.domain))
            else:
                out_vecs.append(Vec(col, v.type))
            out_names.append(b)
        for op, c, na in self.aggs:
            if op == "nrow":
                cnt = torch.bincount(inv, minlength=G).to(torch.float64)
                out_vecs.append(Vec(cnt, T_INT))
                out_names.append("nrow")
                continue
            x = fr.vec(c).as_float(torch.float64)
            nan = torch.isnan(x)
            if na == "rm" or na == "ignore":
                xz = torch.where(nan, torch.zeros_like(x), x)
                ok = (~nan).to(torch.float64)
            else:
                xz, ok = x, torch.ones_like(x)
            s = _ia(torch.zeros(G, dtype=torch.float64, device=x.device), inv, xz)
            n = _ia(torch.zeros(G, dtype=torch.float64, device=x.device), inv, ok)
            if op == "sum":
                r = s
            elif op == "mean":
                r = s / n
            elif op in ("min", "max"):
                fill = math.inf if op == "min" else -math.inf
                r = group_extreme(inv, torch.where(nan, torch.full_like(x, fill), x).to(torch.float64), G, op)
            elif op in ("sd", "var", "ss"):
                mean = s / n
                d = xz - mean[inv]
                ss = _ia(torch.zeros(G, dtype=torch.float64, device=x.device), inv, torch.where(ok > 0, d * d, torch.zeros_like(d)))
                r = ss if op == "ss" else (ss / (n - 1) if op == "var" else torch.sqrt(ss / (n - 1)))
            elif op in ("median", "mode"):
                from .dist_ops import segment_median_mode
                r = segment_median_mode(inv, x, G, op)
            out_vecs.append(Vec(r, T_REAL))
            out_names.append(f"{op}_{c}")
        res = H2OFrame.from_vecs(out_vecs, out_names)
        self._res = _reshard(res) if cloud.is_distributed() else res
        return self._res

    @property
    def frame(self):
        return self.get_frame()


def merge(x, y, all_x=False, all_y=False, by_x=None, by_y=None):
    """reference: water/rapids/ast/prims/mungers/AstMerge.java + Merge.java /
    BinaryMerge.java (radix-sort join).  Inner, left (all_x) or right (all_y)
    join on the key columns, result ordered by key; rows whose key has an NA
    never match (Merge.java drops NA-key rows of the right frame).

    Device path: both sides' keys get common order-preserving integer ids
    (per-column ranks over the union of values -- categorical keys by level
    name -- combined mixed-radix), the right frame is sorted by id, every left
    row finds its match range with two searchsorted calls, and the output row
    pairs come from one repeat_interleave; columns are gathered on the device.
    String / UUID key columns take the host (pandas) path."""
    if all_x and all_y:
        raise ValueError("all.x=TRUE and all.y=TRUE is not supported.  Choose one only.")
    from . import dist_munge
    if dist_munge.eligible(x, y):
        bx = by_x if by_x is not None else [n for n in x.names if n in y.names]
        bx = [x.names[c] if isinstance(c, int) else c for c in bx]
        byy = by_y if by_y is not None else (by_x if by_x is not None else bx)
        byy = [y.names[c] if isinstance(c, int) else c for c in byy]
        if not bx:
            raise ValueError("merge: no common columns to join on")
        res = dist_munge.merge(x, y, all_x, all_y, bx, byy)
        if res is not None:
            return res
    gx, gy = x.gather(), y.gather()
    if by_x is None:
        common = [n for n in gx.names if n in gy.names]
        by_x = by_y = common
    by_x = [gx.names[c] if isinstance(c, int) else c for c in by_x]
    by_y = [gy.names[c] if isinstance(c, int) else c for c in (by_y or by_x)]
    if not by_x:
        raise ValueError("merge: no common columns to join on")
    keys = _join_key_ids(gx, gy, by_x, by_y)
    if keys is None:
        res = _merge_host(gx, gy, all_x, all_y, by_x, by_y)
    else:
        kx, ky = keys
        if all_y:
            iy, ix = _join_pairs(ky, kx, keep_left=True)     # right join = left join from y's side
        else:
            ix, iy = _join_pairs(kx, ky, keep_left=all_x)
        res = _merged_frame(gx, gy, ix, iy, by_x, by_y)
    return _reshard(res) if cloud.is_distributed() else res


def _join_key_ids(gx, gy, by_x, by_y):
    """(kx, ky) int64 key ids shared by both frames (-1 = NA key), ordered like
    the key tuples; None when a key column pair needs the host path."""
    dev = _dev()
    ranks_x, ranks_y, cards = [], [], []
    na_x = torch.zeros(gx.nlocal, dtype=torch.bool, device=dev)
    na_y = torch.zeros(gy.nlocal, dtype=torch.bool, device=dev)
    for cx, cy in zip(by_x, by_y):
        vx, vy = gx.vec(cx), gy.vec(cy)
        if vx.on_host or vy.on_host:
            return None
        if (vx.type == T_ENUM) != (vy.type == T_ENUM):
            return None
        if vx.type == T_ENUM:
            union = sorted(set(vx.domain or []) | set(vy.domain or []))
            pos = {d: i for i, d in enumerate(union)}

            def ids(v):
                lut = torch.tensor([pos[d] for d in (v.domain or [])] or [0], dtype=torch.float64, device=dev)
                c = v.data.long()
                return torch.where(c >= 0, lut[c.clamp(min=0)], torch.full(c.shape, float("nan"), dtype=torch.float64,
                                                                          device=dev))
            ax, ay = ids(vx), ids(vy)
        else:
            ax, ay = vx.as_float(torch.float64), vy.as_float(torch.float64)
        na_x |= torch.isnan(ax)
        na_y |= torch.isnan(ay)
        both = torch.cat([ax, ay])
        ok = ~torch.isnan(both)
        u = torch.unique(both[ok])
        cards.append(max(int(u.numel()), 1))
        r = torch.searchsorted(u, torch.nan_to_num(both, nan=0.0))
        ranks_x.append(r[:gx.nlocal])
        ranks_y.append(r[gx.nlocal:])
    tot = 1
    for c in cards:
        tot *= c
    if tot >= (1 << 62):
        return None
    kx = torch.zeros(gx.nlocal, dtype=torch.int64, device=dev)
    ky = torch.zeros(gy.nlocal, dtype=torch.int64, device=dev)
    for rx, ry, c in zip(ranks_x, ranks_y, cards):
        kx = kx * c + rx
        ky = ky * c + ry
    return torch.where(na_x, torch.full_like(kx, -1), kx), torch.where(na_y, torch.full_like(ky, -1), ky)


def _join_pairs(kl, kr, keep_left):
    """Row index pairs (il, ir) of the join of key ids kl (left) with kr
    (right), ordered by (key, left row, right row); ir = -1 for kept
    unmatched left rows (keep_left), whose NA keys sort last."""
    dev = kl.device
    okr = kr >= 0
    rows_r = torch.nonzero(okr).view(-1)
    kr_ok = kr[rows_r]
    o = torch.argsort(kr_ok, stable=True)
    kr_s, rr_s = kr_ok[o], rows_r[o]
    lo = torch.searchsorted(kr_s, kl, right=False)
    hi = torch.searchsorted(kr_s, kl, right=True)
    cnt = torch.where(kl >= 0, hi - lo, torch.zeros_like(lo))
    out_cnt = torch.clamp(cnt, min=1) if keep_left else cnt
    left_rows = torch.arange(kl.numel(), device=dev)
    # left rows in key order (stable: original order within a key), NA keys last
    kl_sort = torch.where(kl >= 0, kl, torch.full_like(kl, torch.iinfo(torch.int64).max))
    lord = torch.argsort(kl_sort, stable=True)
    reps = out_cnt[lord]
    il = torch.repeat_interleave(left_rows[lord], reps)
    start = torch.repeat_interleave(lo[lord], reps)
    first = torch.cumsum(reps, 0) - reps
    within = torch.arange(il.numel(), device=dev) - torch.repeat_interleave(first, reps)
    matched = torch.repeat_interleave(cnt[lord] > 0, reps)
    ir = torch.where(matched, rr_s[(start + within).clamp(max=max(rr_s.numel() - 1, 0))] if rr_s.numel() else
                     torch.zeros_like(il), torch.full_like(il, -1))
    return il, ir


def _take_dev(v: Vec, idx):
    """Rows idx (int64 device tensor, -1 = NA row) of v."""
    na = idx < 0
    ii = idx.clamp(min=0)
    if v.on_host:
        arr = np.asarray(v.data, dtype=object)[ii.cpu().numpy()] if len(v.data) else \
            np.array([None] * idx.numel(), dtype=object)
        arr[na.cpu().numpy()] = None
        return Vec(arr, v.type)
    d = v.data[ii] if v.nlocal else torch.zeros(idx.numel(), dtype=v.data.dtype, device=idx.device)
    if v.type == T_ENUM:
        d = torch.where(na, torch.full_like(d, -1), d)
    else:
        d = torch.where(na, torch.full_like(d, float("nan")), d)
    return Vec(d, v.type, v.domain)


def _merged_frame(gx, gy, ix, iy, by_x, by_y):
    vecs, names = [], []
    for n, v in zip(gx.names, gx._vecs):
        vecs.append(_take_dev(v, ix))
        names.append(n)
    for n, v in zip(gy.names, gy._vecs):
        if n in by_y:
            continue
        nn = n if n not in names else n + "0"
        vecs.append(_take_dev(v, iy))
        names.append(nn)
    miss = ix < 0
    if bool(miss.any()):
        # right-join rows without a left match: their keys come from the right frame
        for kx, ky in zip(by_x, by_y):
            j = names.index(kx)
            filled = _take_dev(gy.vec(ky), torch.where(miss, iy, torch.full_like(iy, -1)))
            if vecs[j].type == T_ENUM and filled.type == T_ENUM and vecs[j].domain != filled.domain:
                filled = _recode(filled, vecs[j].domain)   # left domain, right-only levels appended
                vecs[j] = Vec(vecs[j].data, T_ENUM, filled.domain)
            vecs[j] = _coalesce(vecs[j], filled)
    return H2OFrame.from_vecs(vecs, names)


def _recode(v: Vec, domain):
    """Categorical v re-expressed in `domain` (levels missing from it are
    appended)."""
    dom = list(domain)
    pos = {d: i for i, d in enumerate(dom)}
    for d in v.domain or []:
        if d not in pos:
            pos[d] = len(dom)
            dom.append(d)
    lut = torch.tensor([pos[d] for d in (v.domain or [])] or [0], dtype=torch.int32, device=v.data.device)
    c = v.data.long()
    return Vec(torch.where(c >= 0, lut[c.clamp(min=0)], torch.full_like(v.data, -1)), T_ENUM, dom)


def _merge_host(gx, gy, all_x, all_y, by_x, by_y):
    """Host hash join (string / UUID keys): pandas over the key columns, NA
    keys never match, rows gathered on the device."""
    dx = gx[by_x].as_data_frame()
    dy = gy[by_y].as_data_frame()
    dx["__ix"] = np.arange(len(dx))
    dy["__iy"] = np.arange(len(dy))
    dy = dy.dropna(subset=by_y)
    how = "left" if all_x else ("right" if all_y else "inner")
    dxm = dx if all_x else dx.dropna(subset=by_x)
    m = dxm.merge(dy, left_on=by_x, right_on=by_y, how=how, sort=True)
    ix = torch.as_tensor(np.nan_to_num(m["__ix"].to_numpy(dtype=float), nan=-1).astype(np.int64), device=_dev())
    iy = torch.as_tensor(np.nan_to_num(m["__iy"].to_numpy(dtype=float), nan=-1).astype(np.int64), device=_dev())
    return _merged_frame(gx, gy, ix, iy, by_x, by_y)


def _take_with_na(v: Vec, idx):
    idx = np.asarray(idx, dtype=float)
    na = np.isnan(idx)
    ii = np.where(na, 0, idx).astype(np.int64)
    if v.on_host:
        arr = np.asarray(v.data, dtype=object)[ii] if len(v.data) else np.array([None] * len(ii), dtype=object)
        arr[na] = None
        return Vec(arr, v.type)
    t = torch.as_tensor(ii, device=_dev())
    nat = torch.as_tensor(na, device=_dev())
    d = v.data[t] if v.nlocal else torch.zeros(len(ii), dtype=v.data.dtype, device=_dev())
    if v.type == T_ENUM:
        d = torch.where(nat, torch.full_like(d, -1), d)
    else:
        d = torch.where(nat, torch.full_like(d, float("nan")), d)
    return Vec(d, v.type, v.domain)


def _coalesce(a: Vec, b: Vec):
    if a.on_host:
        arr = np.array([x if x is not None else y for x, y in zip(a.data, b.data)], dtype=object)
        return Vec(arr, a.type)
    m = a.isna()
    if a.type == T_ENUM:
        return Vec(torch.where(m, b.data, a.data), T_ENUM, a.domain)
    return Vec(torch.where(m, b.data.to(a.data.dtype), a.data), a.type)


# ---------------------------------------------------------------- impute / fill / scale / cut
def impute(fr, column=-1, method="mean", combine_method="interpolate", by=None, values=None):
    cols = range(fr.ncols) if column in (-1, None) else [fr._col_index(column)]
    res = []
    for j in cols:
        v = fr._vecs[j]
        if v.on_host:
            res.append(None)
            continue
        if values is not None:
            val = values[j] if isinstance(values, (list, tuple)) else values
        elif by is not None and len(by if isinstance(by, (list, tuple)) else [by]):
            res.append(_impute_by_group(fr, j, method, combine_method, by))
            continue
        elif v.type == T_ENUM or method == "mode":
            d = v.data if v.type == T_ENUM else v.as_float().to(torch.int64)
            ok = d[d >= 0]
            cnt = torch.bincount(ok.long())
            coll.allreduce_(cnt)
            val = int(torch.argmax(cnt))
        elif method == "median":
            val = quantile_values(v, [0.5], combine_method)[0]
        else:
            val = v.mean()
        if v.type == T_ENUM:
            fr._vecs[j] = Vec(torch.where(v.data < 0, torch.full_like(v.data, int(val)), v.data), T_ENUM, v.domain)
        else:
            x = v.data
            fr._vecs[j] = Vec(torch.where(torch.isnan(x), torch.full_like(x, float(val)), x), v.type)
        res.append(val)
    return res


def _impute_by_group(fr, j, method, combine_method, by):
    """AstImpute with group-by columns (advmath/AstImpute.java:72): each NA
    of column j takes its group's mean / median / mode; groups whose column is
    all NA stay NA.  Distributed like the reference's MRTask: group ids are
    mixed-radix codes over the GLOBAL per-column key dictionaries, means are
    one all-reduce of per-group (sum, count), medians / modes route each
    group's values to one owner rank (dist_ops.group_median_mode); only the
    G-sized group results cross ranks, never the frame.
    -> frame of the group keys and their fill value."""
    import pandas as pd
    from .dist_ops import global_key, group_median_mode
    by = list(by) if isinstance(by, (list, tuple)) else [by]
    bycols = [fr.names[b] if isinstance(b, (int, float)) else b for b in (int(b) if isinstance(b, float) else b
                                                                           for b in by)]
    dist = cloud.is_distributed()
    keys = [global_key(fr.vec(c)) for c in bycols]
    keys = [torch.where(torch.isnan(k), torch.full_like(k, -1e300), k) for k in keys]
    vals = [torch.unique(coll.all_gather_var(torch.unique(k).contiguous())) if dist else torch.unique(k)
            for k in keys]
    cards = [max(int(u.numel()), 1) for u in vals]
    if math.prod(cards) >= (1 << 62):
        raise ValueError("impute: too many distinct group-by key combinations")
    code = torch.zeros(fr.nlocal, dtype=torch.int64, device=_dev())
    for k, u, c in zip(keys, vals, cards):
        code = code * c + torch.searchsorted(u, k)
    uc = torch.unique(code)
    ucode = torch.unique(coll.all_gather_var(uc.contiguous())) if dist else uc
    G = int(ucode.numel())
    gid = torch.searchsorted(ucode, code)
    v = fr._vecs[j]
    enum = v.type == T_ENUM
    x = v.data.to(torch.float64) if enum else v.as_float(torch.float64)
    if enum:
        x = torch.where(v.data < 0, torch.full_like(x, math.nan), x)
    if enum or method == "mode":
        fill = group_median_mode(gid, x, G, "mode")
    elif method == "median":
        fill = group_median_mode(gid, x, G, "median", combine=str(combine_method))
    else:
        ok = ~torch.isnan(x)
        S = torch.zeros((2, G), dtype=torch.float64, device=x.device)
        _ia(S[0], gid[ok], x[ok])
        _ia(S[1], gid[ok], torch.ones_like(x[ok]))
        if dist:
            coll.allreduce_(S)
        fill = torch.where(S[1] > 0, S[0] / S[1].clamp(min=1), torch.full_like(S[0], math.nan))
    row_fill = fill[gid]
    lv = fr._vecs[j]
    if lv.type == T_ENUM:
        miss = (lv.data < 0) & ~torch.isnan(row_fill)
        fr._vecs[j] = Vec(torch.where(miss, torch.nan_to_num(row_fill, nan=-1).to(lv.data.dtype), lv.data),
                          T_ENUM, lv.domain)
    else:
        lx = lv.data
        fr._vecs[j] = Vec(torch.where(torch.isnan(lx), row_fill.to(lx.dtype), lx), lv.type)
    # the group keys, decoded from the codes (every rank the same)
    out = {}
    rem = ucode
    cols_u = []
    for u, c in zip(reversed(vals), reversed(cards)):
        cols_u.append(u[rem % c] if u.numel() else torch.full_like(rem, -1e300, dtype=torch.float64))
        rem = rem // c
    cols_u = list(reversed(cols_u))
    for c, col in zip(bycols, cols_u):
        kv = fr.vec(c)
        colh = col.cpu().numpy()
        if kv.type == T_ENUM:
            out[c] = [kv.domain[int(t)] if t >= 0 and t != -1e300 else None for t in colh]
        elif kv.on_host:
            loc = sorted(set(z for z in kv.to_numpy() if z is not None))
            allv = sorted(set().union(*coll.all_gather_object(loc))) if dist else loc
            out[c] = [allv[int(t)] if t != -1e300 else None for t in colh]
        else:
            out[c] = [None if t == -1e300 else t for t in colh]
    fv = fill.cpu().numpy()
    out[fr.names[j]] = [v.domain[int(t)] if t == t else None for t in fv] if enum else fv.tolist()
    return H2OFrame(pd.DataFrame(out), _local=not dist)


def _ffill(x, maxlen, dim):
    """Forward fill of NaNs along `dim` (up to maxlen consecutive NaNs after
    the last value): the index of the last valid element by a cummax scan."""
    n = x.shape[dim]
    shape = [1] * x.dim()
    shape[dim] = n
    pos = torch.arange(n, device=x.device).view(shape).expand_as(x)
    valid = ~torch.isnan(x)
    last = torch.cummax(torch.where(valid, pos, torch.full_like(pos, -1)), dim).values
    fill = (~valid) & (last >= 0) & (pos - last <= int(maxlen))
    return torch.where(fill, torch.gather(x, dim, last.clamp_min(0)), x)


def fillna(fr, method="forward", axis=0, maxlen=1):
    """AstFillNA: fill up to maxlen consecutive NAs with the previous
    (forward) or next (backward) value, down each column (axis 0) or along
    each row (axis 1); vectorized scans, no per-element loop.  Down columns
    of a row-sharded frame each rank fills its own shard and the runs that
    cross a shard boundary take the neighbouring ranks' carry (last / first
    valid value and its distance): one small all-gather, no frame gather."""
    if method not in ("forward", "backward"):
        raise ValueError("method must be 'forward' or 'backward'")
    g = fr
    num = [j for j, v in enumerate(g._vecs) if not v.on_host]
    out = list(g._vecs)
    back = method == "backward"
    if axis == 0:
        xs = {}
        for j in num:
            v = g._vecs[j]
            x = v.as_float(torch.float64)
            if v.type == T_ENUM:
                x = torch.where(v.data < 0, torch.full_like(x, float("nan")), x)
            xs[j] = x
            y = _ffill(x.flip(0) if back else x, maxlen, 0)
            out[j] = y.flip(0) if back else y
        if cloud.is_distributed() and num:
            out = _fill_across_shards(xs, out, num, back, int(maxlen))
        for j in num:
            out[j] = _fill_vec(g._vecs[j], out[j])
    elif num:
        X = torch.stack([(lambda v: torch.where(v.data < 0, torch.full_like(v.as_float(torch.float64), float("nan")),
                                                 v.as_float(torch.float64)) if v.type == T_ENUM
                          else v.as_float(torch.float64))(g._vecs[j]) for j in num], 1)
        Y = _ffill(X.flip(1) if back else X, maxlen, 1)
        Y = Y.flip(1) if back else Y
        for q, j in enumerate(num):
            out[j] = _fill_vec(g._vecs[j], Y[:, q].contiguous())
    return H2OFrame.from_vecs(out, g.names)


def _fill_across_shards(xs, out, num, back, maxlen):
    """Shard-boundary part of fillna down columns: per rank and column the
    (row count, last / first valid position, its value) are all-gathered;
    each rank's leading (forward) / trailing (backward) NA run then takes the
    nearest valid value of the preceding / following ranks within maxlen."""
    W, r = cloud.world(), cloud.rank()
    dev = _dev()
    info = []
    for j in num:
        x = xs[j]
        n = x.numel()
        valid = torch.nonzero(~torch.isnan(x)).view(-1)
        if valid.numel():
            p = int(valid[0]) if back else int(valid[-1])
            info.append([float(n), float(p), float(x[p])])
        else:
            info.append([float(n), -1.0, 0.0])
    t = torch.tensor(info, dtype=torch.float64, device=dev).view(1, -1)
    allinfo = coll.all_gather_dim0(t.contiguous()).view(W, len(num), 3).cpu().numpy()
    for c, j in enumerate(num):
        x = xs[j]
        n = x.numel()
        valid = torch.nonzero(~torch.isnan(x)).view(-1)
        gap, val, found = 0, 0.0, False
        ranks = range(r + 1, W) if back else range(r - 1, -1, -1)
        for q in ranks:
            nq, pq, vq = allinfo[q, c]
            if pq >= 0:
                gap += int(pq) if back else int(nq) - 1 - int(pq)
                val, found = vq, True
                break
            gap += int(nq)
        if not found or n == 0:
            continue
        pos = torch.arange(n, device=x.device)
        if back:
            run = pos > (int(valid[-1]) if valid.numel() else -1)     # trailing NAs
            dist = (n - 1 - pos) + gap + 1
        else:
            run = pos < (int(valid[0]) if valid.numel() else n)       # leading NAs
            dist = pos + gap + 1
        fill = run & (dist <= maxlen)
        out[j] = torch.where(fill, torch.full_like(out[j], float(val)), out[j])
    return out


def _fill_vec(v, y):
    if v.type == T_ENUM:
        return Vec(torch.nan_to_num(y, nan=-1).to(torch.int32), T_ENUM, v.domain)
    return Vec(y.to(v.data.dtype), v.type)


def scale_frame(fr, center=True, scale=True):
    out = []
    for v in fr._vecs:
        x = v.as_float(torch.float64)
        if center is True:
            x = x - v.mean()
        elif isinstance(center, (list, tuple)):
            pass
        if scale is True:
            r = v.rollups()
            sd = r["sigma"] if center is True else math.sqrt(coll.allreduce_scalar(float(torch.nansum(x * x))) / max(r["nrow"] - r["nacnt"] - 1, 1))
            x = x / sd if sd else x
        out.append(Vec(x.to(torch.float32), T_REAL))
    return H2OFrame.from_vecs(out, fr.names)


def cut(fr, breaks, labels=None, include_lowest=False, right=True, dig_lab=3):
    v = fr._vecs[0]
    x = v.as_float(torch.float64)
    b = torch.tensor(sorted(breaks), dtype=torch.float64, device=x.device)
    if right:
        idx = torch.searchsorted(b, x, right=False) - 1
        if include_lowest:
            idx = torch.where(x == b[0], torch.zeros_like(idx), idx)
    else:
        idx = torch.searchsorted(b, x, right=True) - 1
        if include_lowest:
            idx = torch.where(x == b[-1], torch.full_like(idx, len(breaks) - 2), idx)
    valid = (idx >= 0) & (idx < len(breaks) - 1) & ~torch.isnan(x)
    codes = torch.where(valid, idx, torch.full_like(idx, -1)).to(torch.int32)
    if labels is None:
        fmt = lambda z: f"{z:.{dig_lab}g}"
        labels = [(f"({fmt(breaks[i])},{fmt(breaks[i + 1])}]" if right else f"[{fmt(breaks[i])},{fmt(breaks[i + 1])})")
                  for i in range(len(breaks) - 1)]
    return H2OFrame.from_vecs([Vec(codes, T_ENUM, list(labels))], fr.names[:1])


# ---------------------------------------------------------------- apply / misc
def apply(fr, fun, axis=0):
    if axis == 0:
        res = {n: [fun(H2OFrame.from_vecs([v], [n]))] for n, v in zip(fr.names, fr._vecs)}
        vals = {n: [x[0] if not isinstance(x[0], H2OFrame) else x[0].flatten()] for n, x in res.items()}
        import pandas as pd
        return H2OFrame(pd.DataFrame(vals))
    # axis=1 (AstApply over rows): each rank applies `fun` to its own row shard
    # (the MRTask map); numeric results stay row-sharded, string results become
    # an enum column over the GLOBAL sorted set of levels -- no frame gather
    import pandas as pd
    df = fr.as_data_frame(local=True)
    out = df.apply(lambda row: fun(row), axis=1) if len(df) else pd.Series([], dtype=np.float64)
    numeric = bool(len(out) == 0 or pd.api.types.is_numeric_dtype(out) or pd.api.types.is_bool_dtype(out))
    if cloud.is_distributed():
        numeric = all(coll.all_gather_object(numeric))
    if numeric:
        t = torch.as_tensor(np.asarray(out.values, dtype=np.float64), device=_dev())
        return H2OFrame.from_vecs([Vec(t, T_REAL)], ["C1"])
    vals = [None if (x is None or (isinstance(x, float) and math.isnan(x))) else str(x) for x in out.values]
    levels = sorted(set(x for x in vals if x is not None))
    if cloud.is_distributed():
        levels = sorted(set().union(*coll.all_gather_object(levels)))
    pos = {lv: i for i, lv in enumerate(levels)}
    codes = torch.tensor([pos[x] if x is not None else -1 for x in vals], dtype=torch.int32, device=_dev())
    return H2OFrame.from_vecs([Vec(codes, T_ENUM, levels)], ["C1"])


def drop_duplicates(fr, columns=None, keep="first"):
    from .dist_ops import drop_duplicates as _d
    return _d(fr, columns, keep)


def pivot(fr, index, column, value):
    from .dist_ops import pivot as _p
    return _p(fr, index, column, value)


def melt(fr, id_vars, value_vars=None, var_name="variable", value_name="value", skipna=False):
    from .dist_ops import melt as _m
    return _m(fr, id_vars, value_vars, var_name, value_name, skipna)


def rank_within_group_by(fr, group_by_cols, sort_cols, ascending=None, new_col_name="New_Rank_column",
                         sort_cols_sorted=False):
    from .dist_ops import rank_within_group_by as _r
    return _r(fr, group_by_cols, sort_cols, ascending, new_col_name, sort_cols_sorted)


def topn(fr, column=0, nPercent=10, grabTopN=-1):
    """AstTopN (GrabTopNPQ, reducers/AstTopN.java:16): the top (grabTopN = 1)
    or bottom (-1) round(nPercent% of the rows) non-NA values of a column with
    their ORIGINAL global row indices.  Each rank keeps its own top-k of (value,
    global row) -- the MRTask map's priority queue --, the k-sized candidate
    lists are all-gathered (the reduce) and every rank selects the same final k,
    which come back row-sharded.  Ties keep the lower row index."""
    from .dist_ops import _sharded_from_replicated
    j = fr._col_index(column)
    v = fr._vecs[j]
    x = v.as_float(torch.float64)
    if v.type == T_ENUM:
        x = torch.where(v.data < 0, torch.full_like(x, math.nan), x)
    k = int(math.floor(nPercent * 0.01 * fr.nrows + 0.5))    # Java Math.round
    flip = 1.0 if grabTopN > 0 else -1.0
    ok = ~torch.isnan(x)
    key = torch.where(ok, x * flip, torch.full_like(x, -math.inf))
    kl = min(k, int(ok.sum()))
    rows = torch.arange(x.numel(), device=x.device, dtype=torch.int64) + fr.row_offset()
    if kl > 0:
        o = lexsort_desc_rows(key, rows)[:kl]
        cand_v, cand_r = x[o], rows[o]
    else:
        cand_v = torch.zeros(0, dtype=torch.float64, device=x.device)
        cand_r = torch.zeros(0, dtype=torch.int64, device=x.device)
    if cloud.is_distributed():
        cand_v = coll.all_gather_var(cand_v.contiguous())
        cand_r = coll.all_gather_var(cand_r.contiguous())
    o = lexsort_desc_rows(cand_v * flip, cand_r)[:k]
    vals, ridx = cand_v[o], cand_r[o]
    name = fr.names[j]
    is_int = v.type in (T_INT, T_ENUM) or (vals.numel() > 0 and bool((vals == torch.round(vals)).all()))
    vecs = [Vec(ridx.to(torch.float64), T_INT), Vec(vals, T_INT if is_int else T_REAL)]
    for q in vecs:
        q.replicated = True
    return _sharded_from_replicated(vecs, ["Original_Row_Indices", name])


def lexsort_desc_rows(key, rows):
    """Order by key descending, then row index ascending."""
    o = torch.argsort(rows, stable=True)
    return o[torch.argsort(-key[o], stable=True)]


def interaction(data, factors, pairwise, max_factors, min_occurrence):
    from .dist_ops import interaction as _i
    return _i(data, factors, pairwise, max_factors, min_occurrence)


def create_frame(frame_id=None, rows=10000, cols=10, randomize=True, real_fraction=None, categorical_fraction=None,
                 integer_fraction=None, binary_fraction=None, time_fraction=None, string_fraction=None, value=0,
                 real_range=100, factors=100, integer_range=100, binary_ones_fraction=0.02, missing_fraction=0.01,
                 has_response=False, response_factors=2, positive_response=False, seed=None):
    """reference: hex/createframe/recipes/SimpleCreateFrameRecipe.java."""
    import pandas as pd
    rng = np.random.RandomState(seed if seed not in (None, -1) else 42)
    fr_ = {"real": real_fraction, "cat": categorical_fraction, "int": integer_fraction, "bin": binary_fraction,
           "time": time_fraction, "str": string_fraction}
    given = {k: v for k, v in fr_.items() if v is not None}
    rest = 1.0 - sum(given.values())
    missing = [k for k, v in fr_.items() if v is None]
    default_share = {"real": 0.5, "cat": 0.2, "int": 0.2, "bin": 0.1, "time": 0.0, "str": 0.0}
    tot_def = sum(default_share[k] for k in missing) or 1
    for k in missing:
        fr_[k] = rest * default_share[k] / tot_def
    counts = {k: int(round(v * cols)) for k, v in fr_.items()}
    diff = cols - sum(counts.values())
    counts["real"] += diff
    data = {}
    ci = 1
    for kind, cnt in counts.items():
        for _ in range(max(cnt, 0)):
            name = f"C{ci}"
            ci += 1
            if kind == "real":
                x = rng.uniform(-real_range, real_range, rows) if randomize else np.full(rows, float(value))
            elif kind == "int":
                x = rng.randint(-integer_range, integer_range + 1, rows).astype(float)
            elif kind == "bin":
                x = (rng.rand(rows) < binary_ones_fraction).astype(float)
            elif kind == "cat":
                x = np.array([f"c{ci}.l{j}" for j in rng.randint(0, factors, rows)], dtype=object)
            elif kind == "time":
                x = pd.to_datetime(rng.randint(0, 2 ** 31, rows), unit="s").values
            else:
                x = np.array(["".join(rng.choice(list("abcdefgh"), 8)) for _ in range(rows)], dtype=object)
            if missing_fraction > 0 and kind not in ("time",):
                m = rng.rand(rows) < missing_fraction
                x = x.astype(object) if x.dtype == object else x.astype(float)
                x[m] = None if x.dtype == object else np.nan
            data[name] = x
    df = pd.DataFrame(data)
    types = {}
    if has_response:
        if response_factors == 1:
            resp = rng.uniform(0 if positive_response else -real_range, real_range, rows)
        else:
            resp = np.array([str(i) for i in rng.randint(0, response_factors, rows)], dtype=object)
            types["response"] = "enum"
        df.insert(0, "response", resp)
    for c in df.columns:
        if df[c].dtype == object and c != "response":
            types[c] = "enum" if counts["str"] == 0 or not c.startswith("C") else types.get(c)
    return H2OFrame(df, destination_frame=frame_id, column_types={k: v for k, v in types.items() if v})
