"""String prims (reference: water/rapids/ast/prims/string/*).

Strings are host-resident (numpy object arrays); categorical columns are
transformed through their (small) domain, which is the reference's trick
too (AstToLower on an enum column rewrites only the domain).
"""
from __future__ import annotations

import math
import re

import numpy as np
import torch

from .vec import T_ENUM, T_INT, T_REAL, T_STR, Vec, make_enum_from_strings, make_string


def _map_strings(fr, fn, keep_enum=True):
    from .frame import H2OFrame
    out = []
    for v in fr._vecs:
        if v.type == T_ENUM and keep_enum:
            newdom = [fn(d) for d in v.domain]
            # merging of levels that became equal
            uniq = sorted(set(newdom))
            remap = torch.tensor([uniq.index(d) for d in newdom] or [0], dtype=torch.int32, device=v.data.device)
            codes = torch.where(v.data < 0, v.data, remap[v.data.clamp(min=0).long()])
            out.append(Vec(codes, T_ENUM, uniq))
        else:
            arr = v.to_numpy()
            out.append(make_string([None if x is None else fn(str(x)) for x in arr]))
    return H2OFrame.from_vecs(out, fr.names)


def _map_numeric(fr, fn):
    from .frame import H2OFrame
    out = []
    for v in fr._vecs:
        arr = v.to_numpy()
        vals = [float("nan") if x is None else float(fn(str(x))) for x in arr]
        out.append(Vec(torch.tensor(vals, dtype=torch.float32, device=_dev()), T_INT))
    return H2OFrame.from_vecs(out, fr.names)


def _dev():
    from ..parallel import cloud
    return cloud.device()


def tolower(fr): return _map_strings(fr, str.lower)
def toupper(fr): return _map_strings(fr, str.upper)
def trim(fr): return _map_strings(fr, str.strip)
def lstrip(fr, set=" "): return _map_strings(fr, lambda s: s.lstrip(set))
def rstrip(fr, set=" "): return _map_strings(fr, lambda s: s.rstrip(set))


def gsub(fr, pattern, replacement, ignore_case=False):
    rx = re.compile(pattern, re.I if ignore_case else 0)
    return _map_strings(fr, lambda s: rx.sub(replacement, s))


def sub(fr, pattern, replacement, ignore_case=False):
    rx = re.compile(pattern, re.I if ignore_case else 0)
    return _map_strings(fr, lambda s: rx.sub(replacement, s, count=1))


def substring(fr, start_index, end_index=None):
    return _map_strings(fr, lambda s: s[start_index:end_index], keep_enum=False)


def nchar(fr): return _map_numeric(fr, len)


def countmatches(fr, pattern):
    pats = pattern if isinstance(pattern, (list, tuple)) else [pattern]
    return _map_numeric(fr, lambda s: sum(s.count(p) for p in pats))


def entropy(fr):
    def ent(s):
        if not s:
            return 0.0
        c = {}
        for ch in s:
            c[ch] = c.get(ch, 0) + 1
        n = len(s)
        return -sum(v / n * math.log2(v / n) for v in c.values())
    return _map_numeric(fr, ent)


def strsplit(fr, pattern):
    from .frame import H2OFrame
    v = fr._vecs[0]
    arr = v.to_numpy()
    parts = [re.split(pattern, str(x)) if x is not None else [] for x in arr]
    k = max((len(p) for p in parts), default=0)
    vecs = [make_enum_from_strings([p[i] if i < len(p) else None for p in parts]) for i in range(k)]
    return H2OFrame.from_vecs(vecs, [f"C{i + 1}" for i in range(k)])


def tokenize(fr, split):
    from .frame import H2OFrame
    toks = []
    for v in fr._vecs:
        for x in v.to_numpy():
            if x is not None:
                toks.extend(t for t in re.split(split, str(x)) if t != "")
            toks.append(None)
    return H2OFrame.from_vecs([make_string(toks)], ["C1"])


def grep(fr, pattern, ignore_case=False, invert=False, output_logical=False):
    rx = re.compile(pattern, re.I if ignore_case else 0)
    v = fr._vecs[0]
    arr = v.to_numpy()
    hits = np.array([(rx.search(str(x)) is not None) != invert if x is not None else False for x in arr])
    from .frame import H2OFrame
    if output_logical:
        return H2OFrame.from_vecs([Vec(torch.tensor(hits.astype(np.float32), device=_dev()), T_INT)], ["C1"])
    idx = np.nonzero(hits)[0].astype(np.float32)
    return H2OFrame.from_vecs([Vec(torch.tensor(idx, device=_dev()), T_INT)], ["C1"])


def strdistance(fr, y, measure="lv", compare_empty=True):
    from .frame import H2OFrame
    a, b = fr._vecs[0].to_numpy(), y._vecs[0].to_numpy()

    def lev(s, t):
        if s is None or t is None:
            return float("nan")
        if not compare_empty and (s == "" or t == ""):
            return float("nan")
        prev = list(range(len(t) + 1))
        for i, cs in enumerate(s, 1):
            cur = [i]
            for j, ct in enumerate(t, 1):
                cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (cs != ct)))
            prev = cur
        return float(prev[-1])

    def jw(s, t):
        if s is None or t is None:
            return float("nan")
        if s == t:
            return 1.0
        ls, lt = len(s), len(t)
        if not ls or not lt:
            return 0.0
        md = max(ls, lt) // 2 - 1
        sm, tm = [False] * ls, [False] * lt
        m = 0
        for i in range(ls):
            for j in range(max(0, i - md), min(lt, i + md + 1)):
                if not tm[j] and s[i] == t[j]:
                    sm[i] = tm[j] = True
                    m += 1
                    break
        if not m:
            return 0.0
        k = tr = 0
        for i in range(ls):
            if sm[i]:
                while not tm[k]:
                    k += 1
                if s[i] != t[k]:
                    tr += 1
                k += 1
        jaro = (m / ls + m / lt + (m - tr / 2) / m) / 3
        p = 0
        while p < min(4, ls, lt) and s[p] == t[p]:
            p += 1
        return jaro + p * 0.1 * (1 - jaro)
    fn = lev if measure in ("lv", "levenshtein") else jw
    vals = [fn(None if x is None else str(x), None if z is None else str(z)) for x, z in zip(a, b)]
    return H2OFrame.from_vecs([Vec(torch.tensor(vals, dtype=torch.float64, device=_dev()), T_REAL)], ["C1"])


def num_valid_substrings(fr, path_to_words):
    with open(path_to_words) as f:
        words = set(w.strip() for w in f)
    return _map_numeric(fr, lambda s: sum(1 for i in range(len(s)) for j in range(i + 2, len(s) + 1) if s[i:j] in words))
