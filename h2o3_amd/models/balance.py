"""balance_classes / class_sampling_factors / max_after_balance_size.

Reference: hex/ModelBuilder.java init (balance_classes -> the training frame
is re-sampled with water/util/MRUtils.sampleFrameStratified to the class
sampling factors, capped at max_after_balance_size x the original rows) and
hex/genmodel/GenModel.correctProbabilities (predicted class probabilities
are mapped back from the balanced class distribution to the prior one).

MI355X design.  Every rank re-samples its own row shard (the class counts
come from one all-reduce), so the balanced frame stays sharded and nothing
moves between GPUs: a row of class k is kept floor(f_k) times plus once more
with probability frac(f_k) (seeded per rank), as one repeat_interleave
gather per column.
"""
from __future__ import annotations

import numpy as np
import torch

from ..core.frame import H2OFrame, _take
from ..core.vec import T_ENUM
from ..parallel import cloud
from ..parallel import collectives as coll
from ..core.groupsum import index_add as _ia


def class_counts(frame, y, w=None):
    v = frame.vec(y)
    K = len(v.domain or [])
    codes = v.data.to(torch.int64)
    ok = codes >= 0
    wt = torch.ones_like(codes, dtype=torch.float64) if w is None else \
        torch.nan_to_num(frame.vec(w).as_float(torch.float64))
    c = torch.zeros(K, dtype=torch.float64, device=codes.device)
    _ia(c, codes[ok], wt[ok])
    coll.allreduce_(c)
    return c.cpu().numpy()


def sampling_factors(counts, factors=None, max_after=5.0):
    """MRUtils.sampleFrameStratified: the user's factors, or every class up to
    the majority class count; scaled down so the total stays under
    max_after_balance_size x the original size."""
    counts = np.asarray(counts, dtype=np.float64)
    n = counts.sum()
    if factors is not None:
        f = np.asarray([float(x) for x in factors], dtype=np.float64)
        if f.size != counts.size:
            raise ValueError(f"class_sampling_factors must have {counts.size} elements (one per class)")
    else:
        mx = counts.max() if counts.size else 0.0
        f = np.where(counts > 0, mx / np.where(counts > 0, counts, 1.0), 0.0)
    tot = float((counts * f).sum())
    cap = float(max_after) * n
    if max_after and max_after > 0 and tot > cap and tot > 0:
        f = f * (cap / tot)
    return f


def balance_frame(frame, y, factors, seed):
    """Row-resampled copy of `frame` (local shard only)."""
    codes = frame.vec(y).data.to(torch.int64)
    dev = codes.device
    f = torch.as_tensor(factors, dtype=torch.float64, device=dev)
    per = torch.where(codes >= 0, f[codes.clamp_min(0)], torch.ones_like(codes, dtype=torch.float64))
    base = torch.floor(per)
    g = torch.Generator(device=dev)
    g.manual_seed((int(seed) * 7919 + 104729 * (cloud.rank() + 1)) & 0x7FFFFFFF)
    extra = (torch.rand(per.shape, generator=g, device=dev, dtype=torch.float64) < (per - base)).to(torch.int64)
    reps = base.to(torch.int64) + extra
    idx = torch.repeat_interleave(torch.arange(codes.numel(), device=dev), reps)
    return H2OFrame.from_vecs([_take(v, idx) for v in frame._vecs], list(frame.names))


def correct_probabilities(raw, prior, model):
    """GenModel.correctProbabilities on [n, K] class probabilities."""
    pr = torch.as_tensor(prior, dtype=raw.dtype, device=raw.device)
    md = torch.as_tensor(model, dtype=raw.dtype, device=raw.device)
    ratio = torch.where((pr != 0) & (md != 0), pr / torch.where(md != 0, md, torch.ones_like(md)),
                        torch.ones_like(pr))
    out = raw * ratio.view(1, -1)
    s = out.sum(1, keepdim=True)
    return torch.where(s > 0, out / torch.where(s > 0, s, torch.ones_like(s)), raw)


def apply(est, frame, y):
    """Balance `frame` for estimator `est` when asked; returns the frame to
    train on and records the prior / model class distributions."""
    p = est._parms
    if not p.get("balance_classes") or y is None or frame.vec(y).type != T_ENUM:
        return frame
    w = p.get("weights_column")
    counts = class_counts(frame, y, w)
    f = sampling_factors(counts, p.get("class_sampling_factors"), float(p.get("max_after_balance_size") or 5.0))
    seed = p.get("seed", -1)
    out = balance_frame(frame, y, f, 1234 if seed in (None, -1) else seed)
    after = counts * f
    est._prior_class_dist = (counts / max(counts.sum(), 1e-300)).tolist()
    est._model_class_dist = (after / max(after.sum(), 1e-300)).tolist()
    est._output["prior_class_distribution"] = est._prior_class_dist
    est._output["model_class_distribution"] = est._model_class_dist
    return out
