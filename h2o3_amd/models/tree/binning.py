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

  QuantilesGlobal : nbins equal-frequency cut points (global sketch)
  UniformAdaptive : uniform grid over [min, max] with nbins_top_level cells
  UniformRobust   : uniform grid, outlier-robust range (0.1/99.9 pct)
  Random          : sorted uniform random cut points in [min, max]
  AUTO            : QuantilesGlobal with max(nbins, 254) bins, capped at 254
                    (the GPU-native default)
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


def compute_cuts(cols, is_cat, hist_type="AUTO", nbins=20, nbins_top_level=1024, nbins_cats=1024,
                 seed=1234, sample=1 << 20):
    """Per-feature cut points (list of float64 numpy arrays) and bin counts."""
    dev = cloud.device()
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
        x = col
        if ht in ("auto", "quantilesglobal"):
            B = min(254, max(nbins, 254)) if ht == "auto" else min(max(nbins, 2), 4095)
        elif ht in ("uniformadaptive",):
            B = min(max(nbins_top_level, nbins), 4095)
        else:
            B = min(max(nbins, 2), 4095)
        idx = _sample_rows(x.shape[0], sample, x.device, seed + j)
        xs = x[idx] if idx is not None else x
        xs = xs[torch.isfinite(xs)].to(torch.float64)
        if cloud.is_distributed():
            xs = coll.all_gather_var(xs)
        if xs.numel() == 0:
            cuts.append(np.zeros(0))
            nb_list.append(1)
            groups.append(1)
            continue
        lo, hi = float(xs.min()), float(xs.max())
        if ht in ("auto", "quantilesglobal"):
            u = torch.unique(xs)
            if u.numel() <= B:
                # few distinct values: cut exactly between them
                uu = u.cpu().numpy()
                c = (uu[:-1] + uu[1:]) / 2.0 if len(uu) > 1 else np.zeros(0)
                # cut "x < c" must separate uu[i] and uu[i+1]; midpoints do
            else:
                q = torch.linspace(0, 1, B + 1, dtype=torch.float64, device=xs.device)[1:-1]
                srt = torch.sort(xs).values
                pos = (q * (srt.numel() - 1)).round().long()
                c = torch.unique(srt[pos]).cpu().numpy()
                # a cut equal to the min would create an empty first bin
                c = c[c > lo]
        elif ht == "random":
            g = np.random.RandomState(seed + j)
            c = np.unique(np.sort(g.uniform(lo, hi, size=B - 1)))
        else:
            if ht == "uniformrobust" and xs.numel() > 100:
                srt = torch.sort(xs).values
                lo = float(srt[int(0.001 * (srt.numel() - 1))])
                hi = float(srt[int(0.999 * (srt.numel() - 1))])
            if hi <= lo:
                c = np.zeros(0)
            else:
                c = np.linspace(lo, hi, B + 1)[1:-1]
                c = np.unique(c)
        cuts.append(np.asarray(c, dtype=np.float64))
        nb_list.append(len(c) + 1)
        groups.append(1)
    return cuts, nb_list, groups


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
        col[j] = c.to(dt) if code_bytes == 1 else c.to(torch.int32).to(torch.int16)
    bd = BinnedData()
    bd.F, bd.Fp, bd.Bs, bd.na_code = F, Fp, Bs, na
    bd.nbins = list(nb_list)
    bd.is_cat = list(is_cat)
    bd.cuts = [None if is_cat[j] else np.asarray(cuts[j], dtype=np.float64) for j in range(F)]
    # float32 data: store the float32-rounded cuts so scoring matches training exactly
    for j in range(F):
        if not is_cat[j] and features[j].dtype == torch.float32:
            bd.cuts[j] = bd.cuts[j].astype(np.float32).astype(np.float64)
    bd.cat_card = list(cat_cards)
    bd.cat_group = list(groups)
    bd.names = list(names)
    bd.code_bytes = code_bytes
    bd.nrows_local = N
    bd.codes = col.t().contiguous()  # [N, Fp]
    bd.codes_col = col[:F] if want_col_major else None
    if not want_col_major:
        del col
    return bd
