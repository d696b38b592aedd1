"""Grouped sums without contended floating-point atomics.

`index_add_` / `bincount(weights=)` of millions of rows into a handful of
bins (class counts, per-class moments, per-cluster sums) serialises on a few
addresses: measured on MI355X, one f64 index_add_ of 2M rows into 2 bins took
~0.36 s (Naive Bayes on 2M x 50 spent 55 s in them).  For small bin counts
the sums are a one-hot GEMM on the matrix cores instead (f64 in, f64
accumulate; rows processed in chunks so the one-hot block stays ~256 MB);
large bin counts keep index_add_ (the atomics spread over many addresses).
On a GPU with the native library, f64 sums go to ops/csrc/metrics.hip's
group_sum kernel instead (wave-merged atomics, LDS-privatised for small
nbins * C): one pass for any bin count.  Rows whose idx is outside
[0, nbins) are skipped there; callers pass in-range indices.
"""
from __future__ import annotations

import torch

_ONEHOT_MAX_BINS = 1024
_ONEHOT_BLOCK = 1 << 25          # elements of one [rows, bins] one-hot block


def group_sum(idx: torch.Tensor, vals: torch.Tensor, nbins: int, dtype=torch.float64) -> torch.Tensor:
    """Sums of vals ([N] or [N, C]) grouped by idx (integer in [0, nbins)).
    Returns [nbins] (1-D vals) or [nbins, C]."""
    one_d = vals.dim() == 1
    v = (vals.view(-1, 1) if one_d else vals).to(dtype)
    idx = idx.reshape(-1).to(torch.int64)
    C = v.shape[1]
    if idx.device.type == "cuda" and dtype == torch.float64 and nbins * C < (1 << 31):
        from ..ops import metrics_ops
        if metrics_ops.available(idx):
            out = metrics_ops.group_sum(idx, v, nbins)
            return out[:, 0] if one_d else out
    if idx.device.type != "cuda" or nbins > _ONEHOT_MAX_BINS or idx.numel() == 0:
        out = torch.zeros((nbins, C), dtype=dtype, device=v.device).index_add_(0, idx, v)
        return out[:, 0] if one_d else out
    out = torch.zeros((nbins, C), dtype=dtype, device=v.device)
    chunk = max(1 << 16, _ONEHOT_BLOCK // max(nbins, 1))
    ar = torch.arange(nbins, device=idx.device).view(1, -1)
    for a in range(0, idx.numel(), chunk):
        oh = (idx[a:a + chunk].view(-1, 1) == ar).to(dtype)      # [c, nbins]
        out.addmm_(oh.T, v[a:a + chunk])
    return out[:, 0] if one_d else out


def index_add(out: torch.Tensor, idx: torch.Tensor, vals: torch.Tensor) -> torch.Tensor:
    """`out.index_add_(0, idx, vals)` that stays fast when millions of rows
    share a few indices: f64 GPU tensors go through the wave-merged
    group_sum kernel (torch's f64 index_add_ on this stack retries a
    compare-and-swap per row and serialises on a hot address: 56 s for 670k
    rows into one bin, measured); everything else is index_add_ itself."""
    if out.is_cuda and out.dtype == torch.float64 and out.is_contiguous() and out.shape[0] > 0:
        from ..ops import metrics_ops
        if metrics_ops.available(out):
            n = idx.numel()
            C = out[0].numel()
            out.view(out.shape[0], C).add_(metrics_ops.group_sum(idx, vals.reshape(n, C), out.shape[0]))
            return out
    return out.index_add_(0, idx, vals)


def group_extreme(idx: torch.Tensor, vals: torch.Tensor, nbins: int, op: str) -> torch.Tensor:
    """Per-group minimum (op "min") or maximum ("max") of vals ([N] or [N, C])
    by idx in [0, nbins), f64, +inf / -inf for empty groups.  f64 GPU input
    goes to the wave-merged HIP kernel (torch's float scatter_reduce amin /
    amax retries a compare-and-swap per row on a hot address)."""
    one_d = vals.dim() == 1
    v = vals.view(-1, 1) if one_d else vals
    idx = idx.reshape(-1).to(torch.int64)
    if v.is_cuda:
        from ..ops import metrics_ops
        if metrics_ops.available(v):
            out = metrics_ops.group_reduce(idx, v, nbins, op)
            return out[:, 0] if one_d else out
    fill = float("inf") if op == "min" else float("-inf")
    out = torch.full((nbins, v.shape[1]), fill, dtype=torch.float64, device=v.device)
    out.scatter_reduce_(0, idx.view(-1, 1).expand(-1, v.shape[1]), v.to(torch.float64),
                        reduce="amin" if op == "min" else "amax")
    return out[:, 0] if one_d else out
