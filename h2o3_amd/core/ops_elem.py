"""Elementwise binary operators / ifelse over frames (Rapids operators).

Reference: water/rapids/ast/prims/operators/AstBinOp.java and friends.
NA semantics follow the reference: any NA operand gives NA, except the
logical ops where `NA & 0 = 0`, `NA | 1 = 1` (AstAnd/AstOr).
Categorical == / != against a string compares against the level's code.
"""
from __future__ import annotations

import numbers

import numpy as np
import torch

from .vec import NUMERIC_TYPES, T_ENUM, T_INT, T_REAL, T_STR, Vec


def _operand(fr, x, nlocal):
    from .frame import H2OFrame
    if isinstance(x, H2OFrame):
        return [v for v in x._vecs]
    return x


def _num(v: Vec, dt):
    return v.as_float(dt)


def _apply(op, a, b):
    nan = float("nan")
    if op == "+": return a + b
    if op == "-": return a - b
    if op == "*": return a * b
    if op == "/": return a / b
    if op == "//":
        r = torch.floor(a / b)
        return r
    if op == "%":
        return a - b * torch.floor(a / b)
    if op == "**": return torch.pow(a, b)
    na = torch.isnan(a) | torch.isnan(b) if isinstance(b, torch.Tensor) else torch.isnan(a) | (b != b)
    if op in ("==", "!=", "<", "<=", ">", ">="):
        r = {"==": a == b, "!=": a != b, "<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b}[op].to(a.dtype)
        return torch.where(na, torch.full_like(r, nan), r)
    if op == "&":
        an, bn = torch.isnan(a), (torch.isnan(b) if isinstance(b, torch.Tensor) else torch.tensor(b != b))
        az = (a == 0) & ~an
        bz = (b == 0) & ~bn
        r = ((a != 0) & (b != 0)).to(a.dtype)
        r = torch.where(an | bn, torch.full_like(r, nan), r)
        return torch.where(az | bz, torch.zeros_like(r), r)
    if op == "|":
        an, bn = torch.isnan(a), (torch.isnan(b) if isinstance(b, torch.Tensor) else torch.tensor(b != b))
        a1 = (a != 0) & ~an
        b1 = (b != 0) & ~bn
        r = ((a != 0) | (b != 0)).to(a.dtype)
        r = torch.where(an | bn, torch.full_like(r, nan), r)
        return torch.where(a1 | b1, torch.ones_like(r), r)
    raise ValueError(op)


def binop(fr, other, op, rev=False):
    from .frame import H2OFrame
    n = fr.nlocal
    out = []
    names = fr.names
    ovecs = other._vecs if isinstance(other, H2OFrame) else None
    if ovecs is not None and len(ovecs) != len(fr._vecs) and len(fr._vecs) == 1:
        # broadcast single column frame against the other frame
        return binop(other, fr, op, not rev)
    for i, v in enumerate(fr._vecs):
        ov = None
        if ovecs is not None:
            ov = ovecs[i if len(ovecs) > 1 else 0]
        # categorical vs string comparisons
        if op in ("==", "!=") and v.type == T_ENUM and isinstance(other, str):
            code = v.domain.index(other) if other in v.domain else -2
            r = (v.data == code)
            if op == "!=":
                r = ~r
            r = r.to(torch.float32)
            r = torch.where(v.data < 0, torch.full_like(r, float("nan")), r)
            out.append(Vec(r, T_INT))
            continue
        if op in ("==", "!=") and v.type == T_ENUM and ov is not None and ov.type == T_ENUM:
            a = np.array(v.to_numpy(), dtype=object)
            b = np.array(ov.to_numpy(), dtype=object)
            eq = np.array([x == y if x is not None and y is not None else np.nan for x, y in zip(a, b)], dtype=np.float64)
            if op == "!=":
                eq = np.where(np.isnan(eq), eq, 1 - eq)
            out.append(Vec(torch.tensor(eq, dtype=torch.float32, device=v.data.device), T_INT))
            continue
        if v.type == T_STR or (ov is not None and ov.type == T_STR):
            a = v.to_numpy()
            b = ov.to_numpy() if ov is not None else [other] * n
            if op in ("==", "!="):
                eq = np.array([float(x == y) if x is not None and y is not None else np.nan for x, y in zip(a, b)])
                if op == "!=":
                    eq = np.where(np.isnan(eq), eq, 1 - eq)
                out.append(Vec(torch.tensor(eq, dtype=torch.float32, device=fr._vecs[0].data.device if not fr._vecs[0].on_host else None), T_INT))
                continue
            raise TypeError("string columns only support == and !=")
        dt = torch.float64 if (v.data.dtype == torch.float64 or (ov is not None and not ov.on_host and ov.data.dtype == torch.float64)) else torch.float32
        if ov is not None and ov.type == T_ENUM and v.type != T_ENUM and op in ("==", "!="):
            a = _num(v, dt)
            b = _num(ov, dt)
        else:
            a = _num(v, dt) if v.type != T_ENUM or op not in ("==", "!=") else _num(v, dt)
            if ov is not None:
                b = _num(ov, dt)
            elif isinstance(other, (numbers.Number, bool, np.number)):
                b = float(other)
            elif other is None:
                b = float("nan")
            else:
                raise TypeError(f"unsupported operand {type(other)}")
        if rev:
            a, b = (b if isinstance(b, torch.Tensor) else torch.full_like(a, b)), a
        r = _apply(op, a, b) if isinstance(b, torch.Tensor) else _apply(op, a, torch.full_like(a, b))
        is_int = op in ("==", "!=", "<", "<=", ">", ">=", "&", "|") or (
            op in ("+", "-", "*", "%", "//") and v.type == T_INT and (ov is None or ov.type == T_INT) and
            (ov is not None or float(other).is_integer()))
        out.append(Vec(r, T_INT if is_int else T_REAL))
    return H2OFrame.from_vecs(out, names)


def ifelse(test, yes, no):
    from .frame import H2OFrame
    t = test._vecs[0].as_float()
    cond = t != 0
    na = torch.isnan(t)

    def val(x):
        if isinstance(x, H2OFrame):
            return x._vecs[0]
        return x
    y, n_ = val(yes), val(no)
    if isinstance(y, Vec) and y.type == T_ENUM or isinstance(n_, Vec) and n_.type == T_ENUM or isinstance(y, str) or isinstance(n_, str):
        ya = y.to_numpy() if isinstance(y, Vec) else np.array([y] * len(t), dtype=object)
        na_ = n_.to_numpy() if isinstance(n_, Vec) else np.array([n_] * len(t), dtype=object)
        c = cond.cpu().numpy()
        nn = na.cpu().numpy()
        res = [None if nn[i] else (ya[i] if c[i] else na_[i]) for i in range(len(t))]
        from .frame import _vec_from_array
        return H2OFrame.from_vecs([_vec_from_array(np.array(res, dtype=object), "enum")], ["C1"])
    a = y.as_float(torch.float64) if isinstance(y, Vec) else torch.full_like(t, float(y), dtype=torch.float64)
    b = n_.as_float(torch.float64) if isinstance(n_, Vec) else torch.full_like(t, float(n_), dtype=torch.float64)
    r = torch.where(cond, a, b)
    r = torch.where(na, torch.full_like(r, float("nan")), r)
    return H2OFrame.from_vecs([Vec(r.to(torch.float32) if r.abs().nan_to_num(0).max() < 2**24 else r, T_REAL)], test.names[:1])
