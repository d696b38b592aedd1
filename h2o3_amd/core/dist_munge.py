"""Row-sharded sort / group-by / merge without gathering frames.

Reference: water/rapids/ast/prims/mungers/AstSort + water/rapids/Merge.java
(radix sort: key MSB histograms decide which node owns which key range,
rows are shipped to their owners, sorted locally), AstGroup (per-chunk
partial aggregates reduced across nodes), BinaryMerge.java (both sides
range-partitioned on the join key, joined locally).

MI355X design.  Keys are turned into globally consistent integer ids from
all-gathered per-column UNIQUE values (not the columns), so only
key-dictionary-sized data is replicated.  Rows move once, with one
all_to_all_single per column (RCCL alltoall over xGMI; gloo on CPU), to the
rank owning their key range; each rank then sorts / joins its range with
the same device code as the one-rank path, so the result is the one-rank
result, sharded in rank order.  Group-by never moves rows: per-group partial
sums / counts / extrema are reduced with one bucketed all-reduce (a second
one for the centred sums of squares); median / mode route each group's
(group, value) pairs to the rank owning that group range.  Sort moves only
the keys to find each row's global position (sampled splitters, no key
gather), then every column once to its position's owner.

Frames with host (string / UUID) columns keep the gather path.
"""
from __future__ import annotations

import math

import torch

from ..parallel import cloud
from ..parallel import collectives as coll
from .vec import T_ENUM, T_INT, T_REAL, Vec
from .groupsum import group_extreme
from .groupsum import index_add as _ia


def eligible(*frames):
    return cloud.is_distributed() and all(not v.on_host and not v.replicated for f in frames for v in f._vecs)


def _dev():
    return cloud.device()


def exchange(vecs, dest):
    """Send row i of every Vec in `vecs` to rank dest[i]; returns the received
    Vecs (rows grouped by source rank, each source's rows in their original
    order) -- one counts exchange + one all_to_all_single per column."""
    W = cloud.world()
    dev = _dev()
    order = torch.argsort(dest, stable=True)
    send = torch.bincount(dest, minlength=W).to(torch.int64)
    recv = torch.empty_like(send)
    coll.all_to_all_single_(recv, send)
    sc, rc = send.tolist(), recv.tolist()
    out = []
    for v in vecs:
        d = v.data.index_select(0, order) if v.data.numel() else v.data
        if d.dtype == torch.bool:
            d = d.to(torch.uint8)
        r = torch.empty((int(sum(rc)),) + tuple(d.shape[1:]), dtype=d.dtype, device=dev)
        coll.all_to_all_single_(r, d.contiguous(), rc, sc)
        if v.data.dtype == torch.bool:
            r = r.to(torch.bool)
        nv = Vec(r, v.type, v.domain)
        out.append(nv)
    return out


def _splitters(sample, W):
    """W-1 ascending split values from an all-gathered sample of int64 keys."""
    s = torch.sort(coll.all_gather_var(sample)).values
    if s.numel() == 0:
        return torch.zeros(0, dtype=torch.int64, device=_dev())
    q = torch.arange(1, W, device=s.device, dtype=torch.float64) / W
    return s[(q * (s.numel() - 1)).round().long()]


# ------------------------------------------------------------------ sort
def _lex_ge(K, s):
    """Row-wise K >= s (lexicographic) for a key matrix K [n, d] and one
    splitter row s [d]."""
    cmp = torch.zeros(K.shape[0], dtype=torch.int8, device=K.device)
    for j in range(K.shape[1]):
        d = torch.sign(K[:, j] - s[j]).to(torch.int8)
        cmp = torch.where(cmp == 0, d, cmp)
    return cmp >= 0


def sort_positions(keys, samples_per_rank=256):
    """Global 0-based stable sort position (int64) of every local row for f64
    sort keys (NaN mapped beforehand, descending keys negated).  RadixOrder /
    AstSort without gathering keys: each rank contributes a sample of key
    rows, the W-1 splitters of the merged sample define key ranges, every row
    (keys + global row id, so ties keep row order and ranges split evenly)
    goes once to its range owner, which sorts its range; the positions go
    back with a second all_to_all.  At one rank: one local lexsort."""
    from .dist_ops import lexsort
    dev = _dev()
    n = keys[0].numel() if keys else 0
    W, r = cloud.world(), cloud.rank()
    off = int(sum(coll.all_gather_object(int(n))[:r])) if W > 1 else 0
    gid = torch.arange(n, device=dev, dtype=torch.int64) + off
    K = torch.stack([k.to(torch.float64) for k in keys] + [gid.to(torch.float64)], 1)
    if W == 1:
        pos = torch.empty(n, dtype=torch.int64, device=dev)
        pos[lexsort([K[:, j] for j in range(K.shape[1])])] = torch.arange(n, device=dev)
        return pos
    g = torch.Generator(device=dev)
    g.manual_seed(7919 + r)
    m = min(n, samples_per_rank)
    samp = K[torch.randperm(n, generator=g, device=dev)[:m]] if m else K[:0]
    S = coll.all_gather_var(samp)
    S = S[lexsort([S[:, j] for j in range(S.shape[1])])]
    if S.shape[0]:
        q = ((torch.arange(1, W, device=dev, dtype=torch.float64) / W) * (S.shape[0] - 1)).round().long()
        spl = S[q]
    else:
        spl = S
    dest = torch.zeros(n, dtype=torch.int64, device=dev)
    for i in range(spl.shape[0]):
        dest += _lex_ge(K, spl[i]).to(torch.int64)
    src = torch.full((n,), r, dtype=torch.int64, device=dev)
    loc = torch.arange(n, device=dev, dtype=torch.int64)
    got = exchange([Vec(K, T_REAL), Vec(src, T_INT), Vec(loc, T_INT)], dest)
    RK = got[0].data
    o = lexsort([RK[:, j] for j in range(RK.shape[1])])
    cnt = coll.all_gather_object(int(RK.shape[0]))
    base = int(sum(cnt[:r]))
    rpos = torch.empty(RK.shape[0], dtype=torch.int64, device=dev)
    rpos[o] = torch.arange(RK.shape[0], device=dev) + base
    back = exchange([Vec(rpos, T_INT), Vec(got[2].data, T_INT)], got[1].data)
    pos = torch.empty(n, dtype=torch.int64, device=dev)
    pos[back[1].data] = back[0].data
    return pos


def sort(fr, by, ascending):
    """Globally sorted frame (NAs first, stable), sharded in rank order:
    output rank r holds sorted positions [r*N/W, (r+1)*N/W).  Only the key
    columns travel to compute positions (sort_positions); every frame column
    then moves once, straight to the rank owning its sorted position."""
    from .munging import _key_tensor
    by = by if isinstance(by, (list, tuple)) else [by]
    asc = ascending if isinstance(ascending, (list, tuple)) else [ascending] * len(by)
    dev = _dev()
    W = cloud.world()
    n = fr.nlocal
    keys = []
    for b, a in zip(by, asc):
        k = _key_tensor(fr.vec(b))
        k = torch.where(torch.isnan(k), torch.full_like(k, -math.inf), k)
        keys.append(k if a else -k)
    mypos = sort_positions(keys)
    N = int(coll.allreduce_scalar(float(n)))
    bounds = torch.tensor([(N * q) // W for q in range(W + 1)], dtype=torch.int64, device=dev)
    dest = (torch.searchsorted(bounds, mypos, right=True) - 1).clamp(0, W - 1)
    got = exchange(list(fr._vecs) + [Vec(mypos, T_INT)], dest)
    order = torch.argsort(got[-1].data)
    from .frame import H2OFrame
    from .munging import _take
    return H2OFrame.from_vecs([_take(v, order) for v in got[:-1]], fr.names)


# ------------------------------------------------------------------ group-by
def _global_codes(fr, cols):
    """(global sorted key codes [G], per-column global unique values, cards,
    local code per row) -- the mixed-radix code of _group_ids over global
    per-column dictionaries."""
    from .munging import _key_tensor
    keys = [_key_tensor(fr.vec(c)) for c in cols]
    keys = [torch.where(torch.isnan(k), torch.full_like(k, -1e300), k) for k in keys]
    vals = [torch.unique(coll.all_gather_var(torch.unique(k))) for k in keys]
    cards = [max(int(u.numel()), 1) for u in vals]
    tot = 1
    for c in cards:
        tot *= c
    if tot >= (1 << 62):
        return None
    code = torch.zeros(fr.nlocal, dtype=torch.int64, device=_dev())
    for k, u, c in zip(keys, vals, cards):
        code = code * c + torch.searchsorted(u, k)
    ucode = torch.unique(coll.all_gather_var(torch.unique(code)))
    return ucode, vals, cards, code


def group_by(fr, by, aggs):
    """Result frame of GroupBy (every rank builds the same small frame)."""
    from .frame import H2OFrame
    got = _global_codes(fr, by)
    if got is None:
        return None
    ucode, vals, cards, code = got
    G = int(ucode.numel())
    gid = torch.searchsorted(ucode, code)
    dev = _dev()
    out_vecs, out_names = [], []
    rem = ucode
    cols_u = []
    for u, c in zip(reversed(vals), reversed(cards)):
        cols_u.append(u[rem % c])
        rem = rem // c
    cols_u = list(reversed(cols_u))
    for b, col in zip(by, cols_u):
        v = fr.vec(b)
        col = torch.where(col == -1e300, torch.full_like(col, float("nan")), col)
        if v.type == T_ENUM:
            out_vecs.append(Vec(torch.nan_to_num(col, nan=-1).to(torch.int32), T_ENUM, v.domain))
        else:
            out_vecs.append(Vec(col, v.type))
        out_names.append(b)
    # pass 1: counts, sums, extrema of every aggregate in one bucketed all-reduce
    sums, mins, maxs, meta = [], [], [], []
    for op, c, na in aggs:
        if op == "nrow":
            sums.append(torch.bincount(gid, minlength=G).to(torch.float64))
            meta.append((op, c, na, len(sums) - 1, None))
            continue
        x = fr.vec(c).as_float(torch.float64)
        nan = torch.isnan(x)
        rm = na in ("rm", "ignore")
        xz = torch.where(nan, torch.zeros_like(x), x) if rm else x
        ok = (~nan).to(torch.float64) if rm else torch.ones_like(x)
        s = _ia(torch.zeros(G, dtype=torch.float64, device=dev), gid, xz)
        nn = _ia(torch.zeros(G, dtype=torch.float64, device=dev), gid, ok)
        sums += [s, nn]
        mi = ma = None
        if op in ("min", "max"):
            fill = math.inf if op == "min" else -math.inf
            # NAs never win an extremum (the one-rank GroupBy semantics)
            t = group_extreme(gid, torch.where(nan, torch.full_like(x, fill), x).to(torch.float64), G, op)
            (mins if op == "min" else maxs).append(t)
            mi = len(mins) - 1 if op == "min" else None
            ma = len(maxs) - 1 if op == "max" else None
        meta.append((op, c, na, len(sums) - 2, (mi, ma)))
    S = torch.stack(sums) if sums else torch.zeros((0, G), dtype=torch.float64, device=dev)
    coll.allreduce_(S)
    if mins:
        Mi = torch.stack(mins).contiguous()
        coll.allreduce_(Mi, "min")
    if maxs:
        Ma = torch.stack(maxs).contiguous()
        coll.allreduce_(Ma, "max")
    # pass 2: centred sums of squares about the global group means
    sq, sq_idx = [], {}
    for op, c, na, si, _ in meta:
        if op in ("sd", "var", "ss"):
            x = fr.vec(c).as_float(torch.float64)
            nan = torch.isnan(x)
            rm = na in ("rm", "ignore")
            mean = S[si] / S[si + 1]
            xz = torch.where(nan, torch.zeros_like(x), x) if rm else x
            d = xz - mean[gid]
            okm = (~nan) if rm else torch.ones_like(nan)
            sq_idx[(op, c, na)] = len(sq)
            sq.append(_ia(torch.zeros(G, dtype=torch.float64, device=dev), gid, torch.where(okm, d * d, torch.zeros_like(d))))
    if sq:
        SQ = torch.stack(sq)
        coll.allreduce_(SQ)
    for op, c, na, si, mm in meta:
        if op == "nrow":
            out_vecs.append(Vec(S[si], T_INT))
            out_names.append("nrow")
            continue
        s, nn = S[si], S[si + 1]
        if op == "sum":
            res = s
        elif op == "mean":
            res = s / nn
        elif op == "min":
            res = Mi[mm[0]]
        elif op == "max":
            res = Ma[mm[1]]
        elif op in ("sd", "var", "ss"):
            ss = SQ[sq_idx[(op, c, na)]]
            res = ss if op == "ss" else (ss / (nn - 1) if op == "var" else torch.sqrt(ss / (nn - 1)))
        else:   # median / mode: rows routed to the owner of their group range
            from .dist_ops import group_median_mode
            res = group_median_mode(gid, fr.vec(c).as_float(torch.float64), G, op)
        out_vecs.append(Vec(res, T_REAL))
        out_names.append(f"{op}_{c}")
    for v in out_vecs:
        v.replicated = True
    return H2OFrame.from_vecs(out_vecs, out_names)


# ------------------------------------------------------------------ merge
def _key_ids(fx, fy, by_x, by_y):
    """Order-preserving int64 key ids, consistent over both frames and every
    rank, from all-gathered per-column unique values (-1 = NA key)."""
    dev = _dev()
    ranks_x, ranks_y, cards = [], [], []
    na_x = torch.zeros(fx.nlocal, dtype=torch.bool, device=dev)
    na_y = torch.zeros(fy.nlocal, dtype=torch.bool, device=dev)
    for cx, cy in zip(by_x, by_y):
        vx, vy = fx.vec(cx), fy.vec(cy)
        if (vx.type == T_ENUM) != (vy.type == T_ENUM):
            return None
        if vx.type == T_ENUM:
            union = sorted(set(vx.domain or []) | set(vy.domain or []))
            pos = {d: i for i, d in enumerate(union)}

            def ids(v):
                lut = torch.tensor([pos[d] for d in (v.domain or [])] or [0], dtype=torch.float64, device=dev)
                c = v.data.long()
                return torch.where(c >= 0, lut[c.clamp(min=0)], torch.full(c.shape, float("nan"),
                                                                          dtype=torch.float64, device=dev))
            ax, ay = ids(vx), ids(vy)
        else:
            ax, ay = vx.as_float(torch.float64), vy.as_float(torch.float64)
        na_x |= torch.isnan(ax)
        na_y |= torch.isnan(ay)
        loc = torch.cat([ax[~torch.isnan(ax)], ay[~torch.isnan(ay)]])
        u = torch.unique(coll.all_gather_var(torch.unique(loc)))
        cards.append(max(int(u.numel()), 1))
        ranks_x.append(torch.searchsorted(u, torch.nan_to_num(ax, nan=0.0)))
        ranks_y.append(torch.searchsorted(u, torch.nan_to_num(ay, nan=0.0)))
    tot = 1
    for c in cards:
        tot *= c
    if tot >= (1 << 62):
        return None
    kx = torch.zeros(fx.nlocal, dtype=torch.int64, device=dev)
    ky = torch.zeros(fy.nlocal, dtype=torch.int64, device=dev)
    for rx, ry, c in zip(ranks_x, ranks_y, cards):
        kx = kx * c + rx
        ky = ky * c + ry
    return torch.where(na_x, torch.full_like(kx, -1), kx), torch.where(na_y, torch.full_like(ky, -1), ky)


def merge(x, y, all_x, all_y, by_x, by_y):
    """Range-partitioned join: both frames' rows go to the rank owning their
    key-id range (splitters from a sample of the keys), NA-key rows of the
    kept side to the last rank; each rank joins its range locally."""
    from .frame import H2OFrame
    from .munging import _join_pairs, _merged_frame
    keys = _key_ids(x, y, by_x, by_y)
    if keys is None:
        return None
    kx, ky = keys
    W = cloud.world()
    dev = _dev()
    g = torch.Generator(device=dev)
    g.manual_seed(977 + cloud.rank())
    cand = torch.cat([kx[kx >= 0], ky[ky >= 0]])
    m = min(cand.numel(), 4096)
    samp = cand[torch.randperm(cand.numel(), generator=g, device=dev)[:m]] if m else cand
    spl = _splitters(samp, W)

    def dest(k, keep_na):
        d = torch.searchsorted(spl, k, right=True) if spl.numel() else torch.zeros_like(k)
        return torch.where(k < 0, torch.full_like(d, W - 1 if keep_na else -1), d)
    dx, dy = dest(kx, all_x), dest(ky, all_y)
    kxm, kym = dx >= 0, dy >= 0            # NA-key rows of the non-kept side never match: dropped
    vx = [Vec(v.data[kxm], v.type, v.domain) for v in x._vecs] + [Vec(kx[kxm], T_INT)]
    vy = [Vec(v.data[kym], v.type, v.domain) for v in y._vecs] + [Vec(ky[kym], T_INT)]
    gx_v = exchange(vx, dx[kxm])
    gy_v = exchange(vy, dy[kym])
    lx = H2OFrame.from_vecs(gx_v[:-1], x.names)
    ly = H2OFrame.from_vecs(gy_v[:-1], y.names)
    for v in lx._vecs + ly._vecs:
        v.replicated = False
    kxl, kyl = gx_v[-1].data, gy_v[-1].data
    if all_y:
        iy, ix = _join_pairs(kyl, kxl, keep_left=True)
    else:
        ix, iy = _join_pairs(kxl, kyl, keep_left=all_x)
    return _merged_frame(lx, ly, ix, iy, by_x, by_y)
