"""Global feature binning for the GPU tree engine.

Reference: hex/tree/DHistogram.java (bin layout, NA bin, `_step`/`_min`),
hex/tree/GlobalQuantilesCalc.java (QuantilesGlobal split points) and
SharedTreeModel.HistogramType.

The reference re-bins every (node, column) adaptively while it walks the
tree; on a GPU that means re-reading raw doubles at every level.  The
MI355X design bins each feature ONCE into a compact code matrix that stays
resident in HBM (uint8 when <= 255 bins, uint16 otherwise) — row-major for
the histogram kernel (one row's codes are contiguous: vector loads) and
column-major for the partition kernel (one split feature per node:
coalesced gathers).  Every histogram type maps to a set of per-feature cut
points; a split "code <= t" is exactly the float rule ``x < cuts[t]`` used at
scoring time, so training and scoring never disagree.

  QuantilesGlobal : nbins equal-frequency cut points (exact global order
                    statistics over every row of every rank)
  UniformAdaptive : the reference's top-level grid -- nbins_top_level uniform
                    cells over the exact [min, max] (one cell per integer for
                    narrow integer columns); each node then splits only at
                    max(nbins_top_level >> depth, nbins) uniform cuts over its
                    own observed range (engine.TreeGrower._adapt_hist,
                    DHistogram.java:366-386, DTree.java:337)
  Random          : the same grid, random cut subsets redrawn per node
  RoundRobin      : the same grid; each tree draws UniformAdaptive / Random /
                    QuantilesGlobal (DHistogram.java:226-233)
  UniformRobust   : uniform grid, outlier-robust range (0.1/99.9 pct)
  AUTO            : 254 quantile cells from a 1M-row sample, range from the
                    exact min / max (the GPU-native default)
Categorical columns: code = level (levels beyond nbins_cats are grouped
into contiguous buckets, as the reference does for high cardinality).
NA (and any out-of-domain value) maps to the last code of the histogram
stride (``na_code = Bs - 1``).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ...parallel import cloud
from ...parallel import collectives as coll


def _next_stride(nb: int) -> int:
    """Bins+NA rounded up to a multiple of 32 (pow2 for small)."""
    need = nb + 1
    s = 8
    while s < need and s < 256:
        s *= 2
    if s >= need:
        return s
    return ((need + 63) // 64) * 64


class BinnedData:
    def __init__(self):
        self.codes = None        # [N, Fp] row-major (uint8 / uint16)
        self.codes_col = None    # [F, N] column-major
        self.F = 0
        self.Fp = 0
        self.Bs = 0              # histogram stride (bins + NA, padded)
        self.na_code = 0
        self.nbins = []          # non-NA codes per feature
        self.is_cat = []
        self.cuts = []           # numeric: float64 array of len nbins-1 (x < cuts[t] -> code <= t)
        self.cat_card = []       # categorical: domain size
        self.cat_group = []      # levels per code for grouped high-cardinality cats
        self.names = []
        self.code_bytes = 1
        self.nrows_local = 0
        self.hist_type = "auto"      # lower-case histogram_type the cuts were built for
        self.nbins_node = 20         # nbins: floor of the per-node adaptive bin count
        self.nbins_top = 1024        # nbins_top_level
        self.qbounds = None          # RoundRobin: per-feature quantile boundary codes
        self.has_na = None           # per feature: any NA in the training rows (every rank)

    @property
    def dtype(self):
        return torch.uint8 if self.code_bytes == 1 else torch.uint16

    def split_value(self, f: int, t: int) -> float:
        """Float threshold for "code <= t goes left" on numeric feature f."""
        c = self.cuts[f]
        if t >= len(c):
            return float("inf")
        return float(c[t])

    def nbytes(self):
        n = 0
        for t in (self.codes, self.codes_col):
            if t is not None:
                n += t.numel() * t.element_size()
        return n


def _sample_rows(n, k, gen_device, seed):
    if n <= k:
        return None
    g = torch.Generator(device=gen_device)
    g.manual_seed(seed)
    return torch.randint(0, n, (k,), generator=g, device=gen_device)


def _global_finite(x):
    """(finite values of this rank's column as f64, global count, global min,
    global max, all values integral) -- exact, from all-reduces (the Vec
    rollups' min / max, not a row sample)."""
    xs = x[torch.isfinite(x)].to(torch.float64)
    n = xs.numel()
    big = float("inf")
    st = torch.tensor([float(n), float(xs.min()) if n else big, -float(xs.max()) if n else big,
                       float(bool((xs != torch.round(xs)).any())) if n else 0.0], dtype=torch.float64,
                      device=xs.device)
    if cloud.is_distributed():
        cnt = st[:1].clone()
        coll.allreduce_(cnt)
        mm = st[1:].clone()
        mm[2] = -mm[2]                    # "any non-integral" as a min of negatives
        coll.allreduce_(mm, "min")
        return xs, int(cnt[0]), float(mm[0]), -float(mm[1]), -float(mm[2]) == 0.0
    return xs, n, float(st[1]), -float(st[2]), float(st[3]) == 0.0


def _sample_quantile_cuts(xs, lo, B, seed):
    """AUTO: quantile cuts from a 1M-row sample (all-gathered over ranks)."""
    idx = _sample_rows(xs.shape[0], 1 << 20, xs.device, seed)
    samp = xs[idx] if idx is not None else xs
    if cloud.is_distributed():
        samp = coll.all_gather_var(samp)
    u = torch.unique(samp)
    if u.numel() <= B:
        uu = u.cpu().numpy()
        return (uu[:-1] + uu[1:]) / 2.0 if len(uu) > 1 else np.zeros(0)
    q = torch.linspace(0, 1, B + 1, dtype=torch.float64, device=samp.device)[1:-1]
    srt = torch.sort(samp).values
    pos = (q * (srt.numel() - 1)).round().long()
    c = torch.unique(srt[pos]).cpu().numpy()
    return c[c > lo]


def _exact_quantile_cuts(xs, n, lo, B, seed):
    """Cut points at the order statistics round(q (n-1)), q = k / B (exact,
    distributed histogram refinement: core/dist_ops.kth_smallest_many), or
    the midpoints between the distinct values when there are at most B."""
    from ...core.dist_ops import kth_smallest_many
    idx = _sample_rows(xs.shape[0], 1 << 20, xs.device, seed)
    samp = xs[idx] if idx is not None else xs
    u = torch.unique(coll.all_gather_var(torch.unique(samp)) if cloud.is_distributed() else samp)
    if u.numel() <= B:
        # few distinct values in the sample: exact when every value is one of them
        pos = torch.searchsorted(u, xs).clamp(max=max(u.numel() - 1, 0))
        miss = torch.tensor([float((u[pos] != xs).sum()) if u.numel() else float(xs.numel())],
                            dtype=torch.float64, device=xs.device)
        if cloud.is_distributed():
            coll.allreduce_(miss)
        if float(miss[0]) == 0.0:
            uu = u.cpu().numpy()
            return (uu[:-1] + uu[1:]) / 2.0 if len(uu) > 1 else np.zeros(0)
    q = np.linspace(0, 1, B + 1)[1:-1]
    ks = np.round(q * (n - 1)).astype(np.int64)
    if not cloud.is_distributed():
        # one rank holds every value: the order statistics of one device sort
        # (the distributed refinement below costs several passes + host loops)
        srt = torch.sort(xs).values
        c = np.unique(srt[torch.as_tensor(ks, device=srt.device)].cpu().numpy().astype(np.float64))
        return c[c > lo]
    vals = kth_smallest_many(xs, ks.tolist())
    c = np.unique(np.array([vals[int(k)] for k in ks], dtype=np.float64))
    return c[c > lo]


def compute_cuts(cols, is_cat, hist_type="AUTO", nbins=20, nbins_top_level=1024, nbins_cats=1024,
                 seed=1234, sample=1 << 20):
    """Per-feature cut points (list of float64 numpy arrays) and bin counts.

    QuantilesGlobal: exact global quantiles (all rows, every rank); AUTO:
    254 cells from a 1M-row sample.
    UniformAdaptive / Random / RoundRobin: the reference's top-level grid
    (DHistogram.initialHist): nbins_top_level uniform cells over the exact
    column [min, max], or one cell per integer when an integer column spans
    at most that many values; the per-node adaptive re-binning happens in
    the split search (engine.TreeGrower._adapt_hist)."""
    ht = (hist_type or "AUTO").lower()
    cuts, nb_list, groups = [], [], []
    for j, (col, cat) in enumerate(zip(cols, is_cat)):
        if cat:
            card = int(col[1])
            if card <= nbins_cats:
                nb_list.append(max(card, 1))
                groups.append(1)
            else:
                g = int(math.ceil(card / nbins_cats))
                nb_list.append(int(math.ceil(card / g)))
                groups.append(g)
            cuts.append(None)
            continue
        xs, n, lo, hi, is_int = _global_finite(col)
        if n == 0:
            cuts.append(np.zeros(0))
            nb_list.append(1)
            groups.append(1)
            continue
        if ht == "auto":
            # the GPU-native default: 254 quantile cells from a 1M-row sample
            c = _sample_quantile_cuts(xs, lo, min(254, max(nbins, 254)), seed + j)
        elif ht == "quantilesglobal":
            c = _exact_quantile_cuts(xs, n, lo, min(max(nbins, 2), 4095), seed + j)
        elif ht in ("uniformadaptive", "random", "roundrobin"):
            B = min(max(nbins_top_level, nbins), 4095)
            if hi <= lo:
                c = np.zeros(0)
            elif is_int and hi - lo + 1 <= B:
                c = np.arange(lo + 0.5, hi, 1.0)          # one cell per integer value
            else:
                c = np.unique(np.linspace(lo, hi, B + 1)[1:-1])
        else:
            B = min(max(nbins, 2), 4095)
            if ht == "uniformrobust" and n > 100:
                from ...core.dist_ops import kth_smallest_many
                k1, k2 = int(0.001 * (n - 1)), int(0.999 * (n - 1))
                v = kth_smallest_many(xs, [k1, k2])
                lo, hi = v[k1], v[k2]
            c = np.zeros(0) if hi <= lo else np.unique(np.linspace(lo, hi, B + 1)[1:-1])
        cuts.append(np.asarray(c, dtype=np.float64))
        nb_list.append(len(c) + 1)
        groups.append(1)
    return cuts, nb_list, groups


def quantile_bounds(cols, is_cat, cuts, nbins, seed=1234):
    """RoundRobin trees that draw QuantilesGlobal: for each numeric feature
    the fine-grid boundaries (code t: "code <= t" left) nearest to its nbins
    global quantile cuts, so those trees split only there."""
    out = []
    for j, (col, cat) in enumerate(zip(cols, is_cat)):
        if cat or cuts[j] is None or len(cuts[j]) == 0:
            out.append(None)
            continue
        xs, n, lo, hi, _ = _global_finite(col)
        q = _exact_quantile_cuts(xs, n, lo, max(nbins, 2), seed + j)
        fine = np.asarray(cuts[j])
        t = np.clip(np.searchsorted(fine, q), 0, len(fine) - 1)
        alt = np.clip(t - 1, 0, len(fine) - 1)
        t = np.where(np.abs(fine[alt] - q) < np.abs(fine[t] - q), alt, t)
        out.append(np.unique(t.astype(np.int64)))
    return out


def bin_frame_tensors(features, is_cat, cat_cards, names, hist_type="AUTO", nbins=20, nbins_top_level=1024,
                      nbins_cats=1024, seed=1234, want_col_major=True, cuts=None, nb_list=None,
                      groups=None) -> BinnedData:
    """features: list of local 1-D tensors (float for numeric with NaN=NA,
    int32 codes with -1=NA for categoricals)."""
    dev = cloud.device()
    F = len(features)
    N = features[0].shape[0] if F else 0
    if cuts is None:
        cols_for_cuts = [(None, cat_cards[j]) if is_cat[j] else features[j] for j in range(F)]
        cuts, nb_list, groups = compute_cuts(cols_for_cuts, is_cat, hist_type, nbins, nbins_top_level,
                                             nbins_cats, seed)
    maxb = max(nb_list) if nb_list else 1
    Bs = _next_stride(maxb)
    code_bytes = 1 if Bs <= 256 else 2
    dt = torch.uint8 if code_bytes == 1 else torch.int16
    na = Bs - 1
    align = 16 // code_bytes
    Fp = ((F + align - 1) // align) * align
    if Fp * code_bytes > 64:
        # wide rows: pad to whole 128-byte cache lines so a scattered row gather
        # (deep tree levels) touches ONE line instead of straddling two
        Fp = ((Fp * code_bytes + 127) // 128) * 128 // code_bytes
    col = torch.empty((max(Fp, 1), N), dtype=dt, device=dev)
    if Fp > F:
        col[F:] = na if code_bytes == 1 else (na if na < 32768 else na - 65536)
    has_na = torch.zeros(max(F, 1), dtype=torch.float32, device=dev)
    for j in range(F):
        x = features[j]
        if is_cat[j]:
            c = x.to(torch.int64)
            g = groups[j]
            if g > 1:
                c = torch.where(c >= 0, c // g, c)
            c = torch.where((c < 0) | (c >= nb_list[j]), torch.full_like(c, na), c)
        else:
            cu = torch.as_tensor(cuts[j], dtype=torch.float64 if x.dtype == torch.float64 else torch.float32,
                                 device=dev)
            xf = x if x.dtype in (torch.float32, torch.float64) else x.to(torch.float32)
            if x.dtype == torch.float32:
                # float32 cut points: make sure searchsorted agrees with the float64 rule
                cu = cu.to(torch.float32)
            c = torch.searchsorted(cu, xf.contiguous(), right=True) if cu.numel() else torch.zeros(N, dtype=torch.int64, device=dev)
            c = torch.where(torch.isnan(xf), torch.full_like(c, na), c)
        has_na[j] = (c == na).any().to(torch.float32)
        col[j] = c.to(dt) if code_bytes == 1 else c.to(torch.int32).to(torch.int16)
    # features with NAs anywhere in the training rows (every rank); a split on a
    # feature without any sends NAs of later data to the heavier child, as the
    # reference does when a node saw no NAs (DTree.java:1475-1478)
    coll.allreduce_(has_na, "max")
    bd = BinnedData()
    bd.F, bd.Fp, bd.Bs, bd.na_code = F, Fp, Bs, na
    bd.nbins = list(nb_list)
    bd.is_cat = list(is_cat)
    bd.cuts = [None if is_cat[j] else np.asarray(cuts[j], dtype=np.float64) for j in range(F)]
    # float32 data: store the float32-rounded cuts so scoring matches training exactly
    for j in range(F):
        if not is_cat[j] and features[j].dtype == torch.float32:
            bd.cuts[j] = bd.cuts[j].astype(np.float32).astype(np.float64)
    bd.has_na = [bool(v) for v in has_na[:F].tolist()]
    bd.cat_card = list(cat_cards)
    bd.cat_group = list(groups)
    bd.names = list(names)
    bd.code_bytes = code_bytes
    bd.nrows_local = N
    bd.hist_type = (hist_type or "AUTO").lower()
    bd.nbins_node = int(nbins)
    bd.nbins_top = int(max(nbins_top_level, nbins))
    bd.qbounds = quantile_bounds([features[j] if not is_cat[j] else None for j in range(F)], is_cat, bd.cuts,
                                 nbins, seed) if bd.hist_type == "roundrobin" else None
    bd.codes = col.t().contiguous()  # [N, Fp]
    bd.codes_col = col[:F] if want_col_major else None
    if not want_col_major:
        del col
    return bd
