"""Vec: one column of a Frame, resident in HBM as a single contiguous shard.

Reference: water/fvec/Vec.java (+ 25 compressed Chunk kinds such as
C1Chunk/C2SChunk/CXIChunk) and water/fvec/RollupStats.java.

MI355X-first design: the reference compresses each 4 MB chunk with a
per-chunk codec because JVM heap is small and rows are spread over many
nodes; here a rank owns a multi-GB row shard in 288 GB of HBM3E, so a column
is one dense tensor with a GPU-friendly dtype:

  real / int : float32 (float64 when an integer column exceeds 2^24 or the
               caller asks for it), NaN = NA
  enum       : int32 level codes, -1 = NA, plus a host-side domain
  time       : float64 milliseconds since epoch, NaN = NA
  string/uuid: host numpy object array (None = NA)

Rollups (min/max/mean/sigma/#NA/#zeros/isInt/cardinality) are computed in
one fused pass over the shard, all-reduced across ranks, and cached until
the Vec is mutated.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..parallel import cloud
from ..parallel import collectives as coll
from .memory import MANAGER as _MM

T_REAL, T_INT, T_ENUM, T_STR, T_TIME, T_UUID, T_BAD = "real", "int", "enum", "string", "time", "uuid", "bad"
NUMERIC_TYPES = (T_REAL, T_INT)


class Vec:
    __slots__ = ("_d", "_sp", "_clean", "_spf", "type", "domain", "_rollups", "_nrow_global", "replicated", "__weakref__")

    def __init__(self, data, vtype: str = T_REAL, domain=None):
        self._sp = None
        self._clean = None
        self._d = data
        if _MM.budget is not None:
            _MM.track(self)
        self.type = vtype
        self.domain = list(domain) if domain is not None else None
        self._rollups = None
        self._nrow_global = None
        self.replicated = False  # True when every rank holds the full column

    # ------------------------------------------------------------------ storage
    @property
    def data(self):
        """The column tensor (reloaded from the host / disk spill tier when the
        memory manager evicted it; core/memory.py)."""
        if self._sp is not None:
            return _MM.reload(self)
        if _MM.budget is not None:
            _MM.touch(self)
        return self._d

    @data.setter
    def data(self, value):
        if _MM.budget is not None:
            _MM.untrack(self)
        self._sp = None
        self._clean = None
        self._d = value
        if _MM.budget is not None:
            _MM.track(self)

    @property
    def spilled(self):
        return self._sp is not None

    # ------------------------------------------------------------------ basics
    @property
    def is_numeric(self):
        return self.type in NUMERIC_TYPES

    @property
    def is_categorical(self):
        return self.type == T_ENUM

    @property
    def is_string(self):
        return self.type in (T_STR, T_UUID)

    @property
    def is_time(self):
        return self.type == T_TIME

    @property
    def on_host(self):
        return self._sp is None and not isinstance(self._d, torch.Tensor)

    def __len__(self):
        return self.nlocal

    @property
    def nlocal(self):
        if self._sp is not None:
            return self._sp[3]           # spilled: the row count without a reload
        return len(self._d)

    def nrow(self):
        if self._nrow_global is None:
            dist_ = cloud.is_distributed() and not self.replicated
            self._nrow_global = int(coll.allreduce_scalar(self.nlocal)) if dist_ else self.nlocal
        return self._nrow_global

    def cardinality(self):
        return len(self.domain) if self.domain is not None else -1

    def invalidate(self):
        self._rollups = None
        self._nrow_global = None

    def copy(self):
        d = self.data.clone() if isinstance(self.data, torch.Tensor) else self.data.copy()
        v = Vec(d, self.type, self.domain)
        v.replicated = self.replicated
        return v

    # ------------------------------------------------------------------ views
    def as_float(self, dtype=torch.float32) -> torch.Tensor:
        """Numeric view with NaN for NA (enum codes -> float, NA -> NaN)."""
        if self.on_host:
            raise TypeError(f"cannot use {self.type} column as numeric")
        d = self.data
        if self.type == T_ENUM:
            f = d.to(dtype)
            return torch.where(d < 0, torch.full_like(f, float("nan")), f)
        return d.to(dtype)

    def isna(self) -> torch.Tensor:
        if self.on_host:
            return torch.tensor([x is None or (isinstance(x, float) and math.isnan(x)) for x in self.data],
                                dtype=torch.bool, device=cloud.device())
        if self.type == T_ENUM:
            return self.data < 0
        return torch.isnan(self.data)

    def to_numpy(self):
        if self.on_host:
            return self.data
        if self.type == T_ENUM:
            codes = self.data.cpu().numpy()
            dom = np.array(self.domain + [None], dtype=object)
            return dom[np.where(codes < 0, len(self.domain), codes)]
        return self.data.cpu().numpy()

    # ------------------------------------------------------------------ rollups
    def rollups(self) -> dict:
        if self._rollups is not None:
            return self._rollups
        if not self.on_host and self.data.is_cuda and self.type in NUMERIC_TYPES:
            # the frame kernel (ops/csrc/frame.hip): one launch per pass, one host read
            from ..ops import frame_ops
            if frame_ops.batchable(self) and frame_ops.rollups_many([self]) and self._rollups is not None:
                return self._rollups
        n = self.nrow()
        red = (lambda t, op="sum": t) if self.replicated else coll.allreduce_
        if self.on_host:
            na = sum(1 for x in self.data if x is None)
            na = int(na if self.replicated else coll.allreduce_scalar(na))
            r = dict(min=float("nan"), max=float("nan"), mean=float("nan"), sigma=float("nan"),
                     nacnt=na, zeros=0, isInt=False, nrow=n, pinfs=0, ninfs=0)
            self._rollups = r
            return r
        d = self.as_float(torch.float64)
        nan = torch.isnan(d)
        pinf = torch.isposinf(d)
        ninf = torch.isneginf(d)
        fin = ~(nan | pinf | ninf)
        dz = torch.where(fin, d, torch.zeros_like(d))
        cnt = fin.sum().to(torch.float64)
        s = dz.sum()
        big = torch.finfo(torch.float64).max
        mn = torch.where(fin, d, torch.full_like(d, big)).min() if d.numel() else torch.tensor(big, dtype=torch.float64, device=d.device)
        mx = torch.where(fin, d, torch.full_like(d, -big)).max() if d.numel() else torch.tensor(-big, dtype=torch.float64, device=d.device)
        isint = (torch.where(fin, dz - torch.round(dz), torch.zeros_like(dz)).abs().max() == 0) if d.numel() else torch.tensor(True, device=d.device)
        stats = torch.stack([cnt, s, nan.sum().to(torch.float64), (d == 0).sum().to(torch.float64),
                             pinf.sum().to(torch.float64), ninf.sum().to(torch.float64),
                             (~isint).to(torch.float64)])
        red(stats)
        mn_mx = torch.stack([mn, -mx])
        red(mn_mx, "min")
        cnt_, s_, na_, z_, pi_, ni_, notint = [float(x) for x in stats.tolist()]
        mean = s_ / cnt_ if cnt_ > 0 else float("nan")
        # second pass for a numerically stable variance
        if cnt_ > 1:
            ss = torch.where(fin, (d - mean) ** 2, torch.zeros_like(d)).sum().reshape(1)
            red(ss)
            sigma = math.sqrt(float(ss.item()) / (cnt_ - 1))
        else:
            sigma = float("nan") if cnt_ == 0 else 0.0
        mnv, mxv = float(mn_mx[0]), -float(mn_mx[1])
        if cnt_ == 0:
            mnv = mxv = float("nan")
        r = dict(min=mnv, max=mxv, mean=mean, sigma=sigma, nacnt=int(na_), zeros=int(z_),
                 isInt=(notint == 0 and self.type != T_TIME), nrow=n, pinfs=int(pi_), ninfs=int(ni_))
        self._rollups = r
        return r

    def min(self):
        return self.rollups()["min"]

    def max(self):
        return self.rollups()["max"]

    def mean(self):
        return self.rollups()["mean"]

    def sigma(self):
        return self.rollups()["sigma"]

    def nacnt(self):
        return self.rollups()["nacnt"]

    def is_const(self):
        r = self.rollups()
        if self.on_host:
            return False
        if r["nacnt"] == r["nrow"]:
            return True
        return r["min"] == r["max"] and r["nacnt"] == 0

    def is_binary(self):
        r = self.rollups()
        return self.is_numeric and r["isInt"] and r["min"] >= 0 and r["max"] <= 1


def make_numeric(values, device=None, dtype=None) -> Vec:
    device = device or cloud.device()
    t = torch.as_tensor(values)
    if dtype is None:
        dtype = torch.float32
        if t.dtype in (torch.float64, torch.int64, torch.int32):
            # keep float64 when float32 would lose integer precision
            tt = t.to(torch.float64)
            fin = torch.isfinite(tt)
            if fin.any():
                am = tt[fin].abs().max().item()
                if am > 2 ** 24 and bool((tt[fin] == torch.round(tt[fin])).all()):
                    dtype = torch.float64
    t = t.to(device=device, dtype=dtype)
    v = Vec(t, T_REAL)
    if v.nlocal and bool(torch.isfinite(t).any()):
        fin = torch.isfinite(t)
        if bool((t[fin] == torch.round(t[fin])).all()):
            v.type = T_INT
    return v


def make_enum(codes, domain, device=None) -> Vec:
    device = device or cloud.device()
    t = torch.as_tensor(codes).to(device=device, dtype=torch.int32)
    return Vec(t, T_ENUM, domain)


def make_enum_from_strings(values, device=None, domain=None) -> Vec:
    arr = np.asarray(values, dtype=object)
    mask = np.array([x is None or (isinstance(x, float) and math.isnan(x)) for x in arr], dtype=bool)
    strs = np.array([str(x) if not m else "" for x, m in zip(arr, mask)], dtype=object)
    if domain is None:
        local = sorted(set(strs[~mask].tolist()))
        if cloud.is_distributed():
            alls = coll.all_gather_object(local)
            local = sorted(set().union(*alls))
        domain = _sort_domain(local)
    idx = {s: i for i, s in enumerate(domain)}
    codes = np.array([idx.get(s, -1) if not m else -1 for s, m in zip(strs, mask)], dtype=np.int32)
    return make_enum(codes, domain, device)


def _sort_domain(levels):
    """H2O sorts categorical levels lexicographically, but numeric-looking
    levels numerically (water/parser/Categorical.java)."""
    def key(s):
        try:
            return (0, float(s), s)
        except ValueError:
            return (1, 0.0, s)
    if all(_isnum(s) for s in levels):
        return sorted(levels, key=key)
    return sorted(levels)


def _isnum(s):
    try:
        float(s)
        return True
    except ValueError:
        return False


def make_string(values) -> Vec:
    arr = np.asarray(values, dtype=object)
    arr = np.array([None if (x is None or (isinstance(x, float) and math.isnan(x))) else str(x) for x in arr],
                   dtype=object)
    return Vec(arr, T_STR)


def make_time(values_ms, device=None) -> Vec:
    device = device or cloud.device()
    t = torch.as_tensor(values_ms, dtype=torch.float64).to(device)
    return Vec(t, T_TIME)
