"""categorical_encoding: the nine schemes of hex/Model.java:355-365.

Reference: water/util/FrameUtils.java categoricalEncoder (:98) and its
encoders -- CategoricalOneHotEncoder (:702), CategoricalLabelEncoder (:797),
CategoricalBinaryEncoder (:862), CategoricalEnumLimitedEncoder (:966, the
top-N levels of water/fvec/CreateInteractions.java makeDomain), and
CategoricalEigenEncoder (:1038, hex/util/LinearAlgebraUtils.java toEigenArray);
SortByResponse is the ModelBuilder's domain reordering; the scoring side is
h2o-genmodel's hex/genmodel/CategoricalEncoding.java.

MI355X design.  An encoding is fitted once on the training frame (global
level counts / response means by one all-reduce over the row shards) and
kept on the model; every frame the model scores goes through the same
`transform` (string-level matching, so a test frame with another domain
order or unseen levels encodes like the reference's adaptTestForTrain).
The encoded columns are device tensors built by gathers/bit ops on the
codes -- no per-row host work:

  AUTO / Enum / OneHotInternal  the algorithm's own handling (identity here)
  OneHotExplicit   card+1 indicator columns `col.level`, `col.missing(NA)`
  Binary           1 + floor(log2(card)) bit columns `col:k` of (code + 1), NA -> 0
  LabelEncoder     the level index as a number (NA stays NA)
  EnumLimited      top `max_categorical_levels` levels by count (>= 2 rows),
                   the rest -> `other`; column `col.top_N_levels`
  Eigen            the level's coordinate in the leading eigenvector of the
                   centred one-hot Gram (`col.Eigen`), f32-rounded
  SortByResponse   levels re-ordered by mean response (same column)

Encoded columns replace the categorical column in place of the original
column order for the non-expanding schemes; the expanding ones (one-hot,
binary) append their columns after the numeric ones like the reference.
Eigen's leading eigenvector is degenerate (I - v v', eigenvalue 1 with
multiplicity card - 1), so which vector the reference's Jama solver returns
is implementation-defined: parity with reference Eigen models is unpinned.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..core.vec import T_ENUM, T_REAL, Vec
from ..parallel import collectives as coll
from ..core.groupsum import index_add as _ia

_CANON = {"auto": "AUTO", "enum": "Enum", "onehotinternal": "OneHotInternal", "onehotexplicit": "OneHotExplicit",
          "binary": "Binary", "eigen": "Eigen", "labelencoder": "LabelEncoder", "sortbyresponse": "SortByResponse",
          "enumlimited": "EnumLimited"}
IDENTITY = ("AUTO", "Enum", "OneHotInternal")


def canon(scheme) -> str:
    k = str(scheme or "auto").replace("_", "").replace("-", "").lower()
    if k not in _CANON:
        raise ValueError(f"categorical_encoding '{scheme}' is not one of {sorted(set(_CANON.values()))}")
    return _CANON[k]


def _codes_in(v: Vec, domain) -> torch.Tensor:
    """Codes of v in `domain` (level-name matching; NA / unseen -> -1)."""
    c = v.data.to(torch.int64)
    if list(v.domain or []) == list(domain):
        return c
    pos = {d: i for i, d in enumerate(domain)}
    lut = torch.tensor([pos.get(d, -1) for d in (v.domain or [])] + [-1], dtype=torch.int64, device=c.device)
    return lut[torch.where(c < 0, torch.full_like(c, len(lut) - 1), c)]


class CategoricalEncoder:
    """Fitted encoding of the categorical predictors of one model."""

    def __init__(self, scheme, max_levels=10):
        self.scheme = canon(scheme)
        self.max_levels = int(max_levels if max_levels and max_levels > 0 else 10)
        self.cols = {}            # column -> fitted state
        self.out_names = None     # encoded predictor names
        self.x_in = None          # original predictor names

    # ------------------------------------------------------------------ fit
    def fit(self, frame, x, y=None, w=None):
        self.x_in = list(x)
        yv = frame.vec(y) if (y is not None and y in frame.names) else None
        for c in self.x_in:
            v = frame.vec(c)
            if v.type != T_ENUM:
                continue
            dom = list(v.domain or [])
            codes = v.data.to(torch.int64)
            L = len(dom)
            st = {"domain": dom}
            if self.scheme in ("EnumLimited", "Eigen", "SortByResponse"):
                wt = None if w is None else frame.vec(w).as_float(torch.float64)
                cnt = torch.zeros(L + 1, dtype=torch.float64, device=codes.device)
                _ia(cnt, torch.where(codes < 0, torch.full_like(codes, L), codes),
                               torch.ones_like(codes, dtype=torch.float64) if wt is None else torch.nan_to_num(wt))
                coll.allreduce_(cnt)
                counts = cnt.cpu().numpy()
            if self.scheme == "EnumLimited":
                st.update(self._fit_limited(c, dom, counts))
            elif self.scheme == "Eigen":
                st["proj"] = self._fit_eigen(counts)
            elif self.scheme == "SortByResponse":
                if yv is None:
                    raise ValueError("categorical_encoding SortByResponse needs a response column")
                st["order"] = self._fit_sort(codes, L, yv)
            self.cols[c] = st
        self.out_names = self._names()
        return self

    def _fit_limited(self, col, dom, counts):
        """CreateInteractions.makeDomain for one column: levels by count
        (descending, stable), at most max_levels with >= 2 rows, the rest
        `other`; NA counts as the level "NA"."""
        L = len(dom)
        if L <= self.max_levels:
            return {"limited": False}
        order = sorted(range(L + 1), key=lambda j: (-counts[j], j))
        keep = []
        for j in order:
            if counts[j] <= 0:
                break
            if len(keep) < self.max_levels and counts[j] >= 2:
                keep.append(j)
            else:
                break
        new_dom = [dom[j] if j < L else "NA" for j in keep]
        truncated = len(keep) < sum(1 for j in range(L + 1) if counts[j] > 0)
        other = len(new_dom) if truncated else -1
        if truncated:
            new_dom.append("other")
        lut = np.full(L + 1, other, dtype=np.int64)
        for i, j in enumerate(keep):
            lut[j] = i
        return {"limited": True, "new_domain": new_dom, "lut": lut, "name": f"{col}.top_{self.max_levels}_levels"}

    @staticmethod
    def _fit_eigen(counts):
        """toEigenArray: one-hot Gram diagonal (NA imputed to the mode) ->
        uu = (diag(c) - c c'/N) / sqrt(c_i c_j) -> eigenvector of the
        largest eigenvalue (f32-rounded counts, as the reference rounds)."""
        c = counts[:-1].copy()
        if counts[-1] > 0 and c.size:
            c[int(np.argmax(c))] += counts[-1]          # imputeMissing: NA -> mode
        c = c.astype(np.float32).astype(np.float64)
        n = c.sum()
        if c.size == 0 or n <= 0:
            return np.zeros(c.size)
        s = np.sqrt(np.outer(c, c))
        with np.errstate(invalid="ignore", divide="ignore"):
            uu = (np.diag(c) - np.outer(c, c) / n) / s
        uu[~np.isfinite(uu)] = 0.0
        ev, vec = np.linalg.eigh(uu)
        return vec[:, int(np.argmax(ev))]

    @staticmethod
    def _fit_sort(codes, L, yv):
        """Mean response per level (classification: mean class index)."""
        yy = yv.data.to(torch.float64) if yv.type == T_ENUM else yv.as_float(torch.float64)
        if yv.type == T_ENUM:
            yy = torch.where(yv.data < 0, torch.full_like(yy, float("nan")), yy)
        ok = (codes >= 0) & ~torch.isnan(yy)
        s = torch.zeros(2 * L, dtype=torch.float64, device=codes.device)
        _ia(s[:L], codes[ok], yy[ok])
        _ia(s[L:], codes[ok], torch.ones_like(yy[ok]))
        coll.allreduce_(s)
        sh = s.cpu().numpy()
        mean = np.where(sh[L:] > 0, sh[:L] / np.maximum(sh[L:], 1), np.inf)
        return np.argsort(mean, kind="stable")

    # ------------------------------------------------------------ names
    def _names(self):
        nums, expanded = [], []
        for c in self.x_in:
            st = self.cols.get(c)
            if st is None:
                nums.append(c)
                continue
            dom = st["domain"]
            if self.scheme == "OneHotExplicit":
                expanded += [f"{c}.{d}" for d in dom] + [f"{c}.missing(NA)"]
            elif self.scheme == "Binary":
                expanded += [f"{c}:{k}" for k in range(self._nbits(len(dom)))]
            elif self.scheme == "EnumLimited":
                nums.append(st["name"] if st["limited"] else c)
            elif self.scheme == "Eigen":
                nums.append(f"{c}.Eigen")
            else:
                nums.append(c)
        return nums + expanded

    @staticmethod
    def _nbits(card):
        return 1 + int(math.floor(math.log2(card))) if card > 0 else 1

    # ------------------------------------------------------------ transform
    def transform(self, frame):
        """Encoded copy of `frame`: predictors replaced by their encoding,
        other columns (response, weights, offset, fold...) kept."""
        from ..core.frame import H2OFrame
        if getattr(frame, "_catenc_of", None) is self or self.is_encoded(frame):
            return frame
        names, vecs, tail_n, tail_v = [], [], [], []
        exp_n, exp_v = [], []
        xs = set(self.x_in)
        for n in frame.names:
            v = frame.vec(n)
            if n not in xs:
                tail_n.append(n)
                tail_v.append(v)
                continue
            st = self.cols.get(n)
            if st is None:
                names.append(n)
                vecs.append(v)
                continue
            if v.type != T_ENUM:      # a scoring frame with the column as numbers: treat as level names
                v = _as_enum(v, st["domain"])
            codes = _codes_in(v, st["domain"])
            L = len(st["domain"])
            if self.scheme == "OneHotExplicit":
                idx = torch.where(codes < 0, torch.full_like(codes, L), codes)
                for j in range(L + 1):
                    exp_v.append(Vec((idx == j).to(torch.float32), T_REAL))
                exp_n += [f"{n}.{d}" for d in st["domain"]] + [f"{n}.missing(NA)"]
            elif self.scheme == "Binary":
                val = torch.where(codes < 0, torch.zeros_like(codes), codes + 1)
                for k in range(self._nbits(L)):
                    exp_v.append(Vec(((val >> k) & 1).to(torch.float32), T_REAL))
                    exp_n.append(f"{n}:{k}")
            elif self.scheme == "LabelEncoder":
                names.append(n)
                vecs.append(Vec(torch.where(codes < 0, torch.full_like(codes, -1), codes).to(torch.float32)
                                .masked_fill(codes < 0, float("nan")), T_REAL))
            elif self.scheme == "EnumLimited":
                if not st["limited"]:
                    names.append(n)
                    vecs.append(v if list(v.domain or []) == st["domain"] else Vec(codes.to(torch.int32), T_ENUM,
                                                                                   st["domain"]))
                else:
                    lut = torch.as_tensor(st["lut"], device=codes.device)
                    nc = lut[torch.where(codes < 0, torch.full_like(codes, L), codes)]
                    names.append(st["name"])
                    vecs.append(Vec(nc.to(torch.int32), T_ENUM, list(st["new_domain"])))
            elif self.scheme == "Eigen":
                proj = torch.as_tensor(np.asarray(st["proj"], dtype=np.float32), device=codes.device)
                val = proj[codes.clamp_min(0)] if L else torch.zeros(codes.shape, device=codes.device)
                names.append(f"{n}.Eigen")
                vecs.append(Vec(torch.where(codes < 0, torch.full_like(val, float("nan")), val), T_REAL))
            elif self.scheme == "SortByResponse":
                order = st["order"]
                inv = np.empty(L, dtype=np.int64)
                inv[order] = np.arange(L)
                lut = torch.as_tensor(np.append(inv, -1), device=codes.device)
                nc = lut[torch.where(codes < 0, torch.full_like(codes, L), codes)]
                names.append(n)
                vecs.append(Vec(nc.to(torch.int32), T_ENUM, [st["domain"][j] for j in order]))
            else:
                names.append(n)
                vecs.append(v)
        out = H2OFrame.from_vecs(vecs + exp_v + tail_v, names + exp_n + tail_n)
        out._catenc_of = self
        return out

    def is_encoded(self, frame):
        """True when `frame` already holds this encoding's predictors (a
        subset / copy of an encoded frame): every encoded name present and,
        for the name-preserving schemes, already in encoded form."""
        fn = set(frame.names)
        if any(n not in fn for n in self.out_names):
            return False
        for c, st in self.cols.items():
            if self.scheme in ("OneHotExplicit", "Binary", "Eigen") or \
                    (self.scheme == "EnumLimited" and st.get("limited")):
                if c in fn:
                    return False
            elif self.scheme == "LabelEncoder":
                if frame.vec(c).type == T_ENUM:
                    return False
            elif self.scheme == "SortByResponse":
                if list(frame.vec(c).domain or []) != [st["domain"][j] for j in st["order"]]:
                    return False
        return True

    # ------------------------------------------------------------ (de)serialise
    def to_dict(self):
        cols = {}
        for c, st in self.cols.items():
            d = {"domain": st["domain"]}
            for k in ("limited", "new_domain", "name"):
                if k in st:
                    d[k] = st[k]
            if "lut" in st:
                d["lut"] = [int(v) for v in st["lut"]]
            if "proj" in st:
                d["proj"] = [float(v) for v in st["proj"]]
            if "order" in st:
                d["order"] = [int(v) for v in st["order"]]
            cols[c] = d
        return {"scheme": self.scheme, "max_levels": self.max_levels, "x_in": self.x_in, "cols": cols}

    @classmethod
    def from_dict(cls, d):
        e = cls(d["scheme"], d.get("max_levels", 10))
        e.x_in = list(d["x_in"])
        for c, st in d["cols"].items():
            st = dict(st)
            if "lut" in st:
                st["lut"] = np.asarray(st["lut"], dtype=np.int64)
            if "proj" in st:
                st["proj"] = np.asarray(st["proj"], dtype=np.float64)
            if "order" in st:
                st["order"] = np.asarray(st["order"], dtype=np.int64)
            e.cols[c] = st
        e.out_names = e._names()
        return e


def _as_enum(v, domain):
    """A numeric / string scoring column matched against a training domain by
    level name (numbers formatted like the parser's levels)."""
    from ..core.vec import make_enum_from_strings
    vals = v.to_numpy()
    out = []
    for x in vals:
        if x is None or (isinstance(x, float) and math.isnan(x)):
            out.append(None)
        elif isinstance(x, float) and float(x).is_integer():
            out.append(str(int(x)))
        else:
            out.append(str(x))
    return make_enum_from_strings(out, domain=list(domain))


def for_estimator(est):
    """The encoder an estimator asks for (None: the algorithm's own handling),
    after the per-algorithm validity rules of the reference."""
    p = est._parms
    if "categorical_encoding" not in p:
        return None
    scheme = canon(p.get("categorical_encoding"))
    algo = est.algo
    trees = algo in ("gbm", "drf", "isolationforest", "extendedisolationforest", "upliftdrf")
    if scheme == "OneHotInternal" and trees:
        raise ValueError("categorical_encoding: Cannot use OneHotInternal categorical encoding for tree methods.")
    if scheme == "Enum" and algo == "deeplearning":
        raise ValueError("categorical_encoding: Won't use explicit Enum encoding for categoricals - it's much "
                         "faster with OneHotInternal!")
    if scheme in IDENTITY:
        return None
    return CategoricalEncoder(scheme, p.get("max_categorical_levels", 10))
