"""Rapids: the reference's S-expression language for frame munging.

Reference: water/rapids/Rapids.java (parser), water/rapids/Env.java (scopes
and DKV lookup), water/rapids/ast/prims/** (~250 primitives).  h2o-py builds
Rapids strings lazily and ships them over REST; this platform executes frames
eagerly, so Rapids is an *input language* here: `h2o.rapids("(+ 1 2)")`, the
REST `/99/Rapids` endpoint and scripts written against the reference go
through this interpreter, which maps each primitive onto the GPU frame ops of
H2OFrame / munging.

Grammar (Rapids.java:149): `(fn args...)` application, `{ x y . body }`
lambda, `[1 2 3]` / `[0:5]` (start:count[:stride]) number lists, `["a" 'b']`
string lists, quoted strings, numbers (incl. NaN / Inf / TRUE / FALSE), and
identifiers (locals, then DKV keys).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import dkv


class RapidsError(ValueError):
    pass


# ---------------------------------------------------------------- parser
class _Fun:
    def __init__(self, ids, body):
        self.ids, self.body = ids, body


class _Id(str):
    pass


class _Str(str):
    pass


class _Parser:
    def __init__(self, s):
        self.s, self.i = s, 0

    def ws(self):
        while self.i < len(self.s) and self.s[self.i] in " \t\n\r":
            self.i += 1
        return self.s[self.i] if self.i < len(self.s) else ""

    def eat(self, c):
        if self.ws() != c:
            raise RapidsError(f"expected '{c}' at {self.i}: ...{self.s[self.i:self.i + 20]}")
        self.i += 1

    def parse(self):
        c = self.ws()
        if c == "(":
            self.i += 1
            items = []
            while self.ws() != ")":
                if not self.ws():
                    raise RapidsError("unbalanced parenthesis")
                items.append(self.parse())
            self.i += 1
            return ("apply", items)
        if c == "{":
            self.i += 1
            ids = []
            while self.ws() != ".":
                ids.append(self.token())
            self.i += 1
            body = self.parse()
            self.eat("}")
            return _Fun(ids, body)
        if c == "[":
            self.i += 1
            if self.ws() in "\"'":
                out = []
                while self.ws() in "\"'" and self.ws():
                    out.append(self.string())
                    if self.ws() == ",":
                        self.i += 1
                self.eat("]")
                return ("strlist", out)
            out = []
            while self.ws() != "]":
                if not self.ws():
                    raise RapidsError("unterminated list")
                base = self.number()
                cnt, stride = 1, 1.0
                if self.ws() == ":":
                    self.i += 1
                    cnt = self.number()
                    if cnt < 1 or int(cnt) != cnt:
                        raise RapidsError(f"Count must be a positive integer, got {cnt}")
                    cnt = int(cnt)
                if self.ws() == ":":
                    self.i += 1
                    stride = self.number()
                out.extend(base + k * stride for k in range(cnt))
                if self.ws() == ",":
                    self.i += 1
            self.i += 1
            return ("numlist", out)
        if c in "\"'":
            return _Str(self.string())
        if not c:
            raise RapidsError("Expected an expression but ran out of text")
        t = self.token()
        num = _as_number(t)
        return num if num is not None else _Id(t)

    def token(self, stops=" \t\n\r()[]{}\"'"):
        self.ws()
        j = self.i
        while self.i < len(self.s) and self.s[self.i] not in stops:
            self.i += 1
        if j == self.i:
            raise RapidsError(f"empty token at {self.i}")
        return self.s[j:self.i]

    def number(self):
        t = self.token(" \t\n\r()[]{}\"':,")
        n = _as_number(t)
        if n is None:
            raise RapidsError(f"expected a number, got {t}")
        return n

    def string(self):
        q = self.s[self.i]
        self.i += 1
        out = []
        while self.i < len(self.s) and self.s[self.i] != q:
            ch = self.s[self.i]
            if ch == "\\" and self.i + 1 < len(self.s):
                self.i += 1
                ch = {"n": "\n", "t": "\t", "r": "\r"}.get(self.s[self.i], self.s[self.i])
            out.append(ch)
            self.i += 1
        self.i += 1
        return "".join(out)


def _as_number(t):
    tl = t.lower()
    if tl in ("nan", "na"):
        return float("nan")
    if tl in ("inf", "+inf", "infinity"):
        return float("inf")
    if tl in ("-inf", "-infinity"):
        return float("-inf")
    if t in ("TRUE", "True", "true"):
        return 1.0
    if t in ("FALSE", "False", "false"):
        return 0.0
    try:
        return float(t)
    except ValueError:
        return None


def parse(expr: str):
    p = _Parser(expr)
    ast = p.parse()
    if p.ws():
        raise RapidsError(f"trailing text: {p.s[p.i:p.i + 30]}")
    return ast


# ---------------------------------------------------------------- evaluation
class Env:
    def __init__(self, parent=None):
        self.vars, self.parent = {}, parent

    def lookup(self, name):
        e = self
        while e is not None:
            if name in e.vars:
                return e.vars[name]
            e = e.parent
        v = dkv.get(name)
        if v is None:
            if name in PRIMS:
                return ("prim", name)
            if name == "_":                            # the clients' "argument not given" placeholder
                return None
            raise RapidsError(f"Name lookup of '{name}' failed")
        if _is_frame(v):
            # Env.addGlobals: a defensive copy of the global frame (same columns,
            # own name / column lists), so structural changes (rename, :=,
            # append) never touch the stored frame; in-place prims
            # (h2o.impute) write back through _rapids_src
            c = _F().from_vecs(list(v._vecs), list(v.names))
            c._rapids_src = v
            return c
        return v


def evaluate(ast, env: Env):
    if isinstance(ast, float):
        return ast
    if isinstance(ast, _Str):
        return str(ast)
    if isinstance(ast, _Id):
        return env.lookup(ast)
    if isinstance(ast, _Fun):
        return ("lambda", ast, env)
    kind, items = ast
    if kind == "numlist":
        return list(items)
    if kind == "strlist":
        return list(items)
    if not items:
        raise RapidsError("empty application")
    head = items[0]
    if isinstance(head, _Id) and head in ("tmp=", "assign"):
        key = str(items[1])
        val = evaluate(items[2], env)
        if hasattr(val, "frame_id"):
            val = val.deep_copy(key) if head == "assign" else val
            val.frame_id = key
        dkv.put(key, val)
        return val
    if isinstance(head, _Id) and head == "rm":
        dkv.remove(str(items[1]))
        return 1.0
    if isinstance(head, _Id) and head == ",":
        out = None
        for it in items[1:]:
            out = evaluate(it, env)
        return out
    fn = evaluate(head, env) if not (isinstance(head, _Id) and head in PRIMS) else ("prim", str(head))
    args = [evaluate(a, env) for a in items[1:]]
    return call(fn, args)


def call(fn, args):
    if isinstance(fn, tuple) and fn[0] == "prim":
        return PRIMS[fn[1]](*args)
    if isinstance(fn, tuple) and fn[0] == "lambda":
        _, f, cenv = fn
        if len(args) != len(f.ids):
            raise RapidsError(f"function expects {len(f.ids)} args, got {len(args)}")
        e = Env(cenv)
        e.vars.update(zip(f.ids, args))
        return evaluate(f.body, e)
    raise RapidsError(f"not a function: {fn!r}")


def rapids(expr: str):
    """Execute a Rapids expression; frames are returned as H2OFrame, scalars as
    floats/strings, lists as lists (Rapids.exec)."""
    return evaluate(parse(expr), Env())


# ---------------------------------------------------------------- primitives
def _F():
    from .frame import H2OFrame
    return H2OFrame


def _is_frame(x):
    return hasattr(x, "_vecs")


def _scalar_frame(x):
    return _F()({"C1": [x]})


def _binop(op):
    pyop = {"+": lambda a, b: a + b, "-": lambda a, b: a - b, "*": lambda a, b: a * b,
            "/": lambda a, b: a / b if b != 0 else (math.nan if a == 0 else math.copysign(math.inf, a)),
            "^": lambda a, b: a ** b, "%": lambda a, b: math.fmod(a, b) if b else math.nan,
            "%%": lambda a, b: a % b if b else math.nan, "%/%": lambda a, b: a // b if b else math.nan,
            "intDiv": lambda a, b: float(int(a // b)) if b else math.nan,
            "==": lambda a, b: float(a == b), "!=": lambda a, b: float(a != b), "<": lambda a, b: float(a < b),
            "<=": lambda a, b: float(a <= b), ">": lambda a, b: float(a > b), ">=": lambda a, b: float(a >= b),
            "&": lambda a, b: float(bool(a) and bool(b)), "|": lambda a, b: float(bool(a) or bool(b)),
            "&&": lambda a, b: float(bool(a) and bool(b)), "||": lambda a, b: float(bool(a) or bool(b))}[op]
    fop = {"^": "**", "%%": "%", "%/%": "//", "intDiv": "//", "&&": "&", "||": "|"}.get(op, op)

    def f(a, b):
        if not _is_frame(a) and not _is_frame(b):
            if isinstance(a, str) or isinstance(b, str):
                return float(a == b) if op == "==" else float(a != b)
            return float(pyop(float(a), float(b)))
        from .ops_elem import binop
        if _is_frame(a):
            return binop(a, b, fop)
        return binop(b, a, fop, True)
    return f


def _unary(name):
    def f(x):
        if _is_frame(x):
            return getattr(x, name)()
        return float(getattr(_scalar_frame(x), name)().as_data_frame().iloc[0, 0])
    return f


def _cols(fr, sel):
    if isinstance(sel, (int, float, str)):
        sel = [sel]
    if sel and isinstance(sel[0], str):
        return fr[list(sel)]
    idx = [int(i) for i in sel]
    if idx and all(i < 0 for i in idx):
        drop = {-i - 1 for i in idx}
        idx = [i for i in range(fr.ncols) if i not in drop]
    return fr[:, idx]


def _rows(fr, sel):
    if _is_frame(sel):
        return fr[sel]
    if isinstance(sel, (int, float)):
        sel = [sel]
    idx = [int(i) for i in sel]
    if idx and all(i < 0 for i in idx):
        drop = {-i - 1 for i in idx}
        idx = [i for i in range(fr.nrows) if i not in drop]
    return fr[idx, :]


def _reduce(name, na_rm_default=False):
    def f(x, *rest):
        if not _is_frame(x):
            return float(x)
        vals = []
        for j in range(x.ncols):
            v = x.vec(j)
            t = v.as_float(torch.float64)
            ok = ~torch.isnan(t)
            na_rm = na_rm_default or (rest and bool(rest[0]))
            from ..parallel import collectives as _c
            if not na_rm and _c.allreduce_scalar(float((~ok).sum())) > 0:     # an NA on any rank
                vals.append(math.nan)
                continue
            t = t[ok]
            from ..parallel import collectives as coll
            if name == "sum":
                vals.append(coll.allreduce_scalar(float(t.sum())))
            elif name == "prod":
                # exact product over every rank's shard (no log-sum rounding)
                vals.append(float(np.prod(coll.all_gather_object(float(torch.prod(t))))))
            elif name == "min":
                vals.append(coll.allreduce_scalar(float(t.min()) if t.numel() else math.inf, "min"))
            elif name == "max":
                vals.append(coll.allreduce_scalar(float(t.max()) if t.numel() else -math.inf, "max"))
        if name == "sum":
            return float(sum(vals))
        if name == "prod":
            return float(np.prod(vals))
        return float(min(vals) if name == "min" else max(vals))
    return f


def _gb(fr, by, *aggs):
    """(GB frame [group cols] agg col na agg col na ...)"""
    from .munging import GroupBy
    names = fr.names
    gb = GroupBy(fr, [names[int(b)] if not isinstance(b, str) else b for b in (by if isinstance(by, list) else [by])])
    for k in range(0, len(aggs), 3):
        op, col, na = _name(aggs[k]), aggs[k + 1], _name(aggs[k + 2])
        col = names[int(col)] if not isinstance(col, str) else col
        if op in ("nrow", "count"):
            gb.count(na)
        else:
            getattr(gb, {"sumSquares": "ss"}.get(op, op))(col, na)
    return gb.get_frame()


def _name(x):
    """Bare identifiers that name a primitive (e.g. `mean`) used as string arguments."""
    return x[1] if isinstance(x, tuple) and x and x[0] == "prim" else x


def _assign_cols(dst, src, cols, rows):
    """(:= dst src col_list row_list): dst[rows, cols] = src, in place (AstRectangleAssign)"""
    fr = dst
    cols = cols if isinstance(cols, list) else [cols]
    for j, c in enumerate(cols):
        c = int(c) if not isinstance(c, str) else fr.names.index(c)
        val = src[:, j] if _is_frame(src) and src.ncols > 1 else src
        name = fr.names[c] if c < fr.ncols else f"C{c + 1}"
        if isinstance(rows, list) and rows:
            dev = fr.vec(0).data.device
            mask = torch.zeros(fr.nlocal, dtype=torch.bool, device=dev)
            r = torch.as_tensor([int(v) for v in rows], dtype=torch.int64, device=dev) - fr.row_offset()
            r = r[(r >= 0) & (r < fr.nlocal)]
            mask[r] = True                 # one scatter for the whole row list
            base = fr[name]
            from .ops_elem import ifelse
            mf = _F().from_vecs([type(fr.vec(0))(mask.to(torch.float32), "int")], ["m"])
            val = ifelse(mf, val, base)
        elif _is_frame(rows):
            from .ops_elem import ifelse
            val = ifelse(rows, val, fr[name])
        fr[name] = val
    return fr


_ROW_REDUCERS = {"sum", "sumNA", "mean", "min", "minNA", "max", "maxNA", "prod", "prod.na", "sd", "var"}


def _rowwise(fr, fun):
    """apply(fr, 1, f) for a reducer f (a primitive, or a one-argument lambda
    whose body is a reducer of its argument with constant options): one
    reduction along the columns of the shard's [rows, cols] matrix on the
    device, the result sharded like fr (AstApply margin 1 without a row loop)."""
    name, extra = None, []
    if isinstance(fun, tuple) and fun[0] == "prim":
        name = fun[1]
    elif isinstance(fun, tuple) and fun[0] == "lambda":
        f = fun[1]
        body = f.body
        if len(f.ids) == 1 and isinstance(body, tuple) and body[0] not in ("numlist", "strlist") and body[1]:
            head, *args = body[1]
            if isinstance(head, _Id) and str(head) in _ROW_REDUCERS and args and isinstance(args[0], _Id) \
                    and args[0] == f.ids[0] and all(isinstance(a, float) for a in args[1:]):
                name, extra = str(head), list(args[1:])
    if name not in _ROW_REDUCERS:
        return None
    from .vec import T_ENUM, T_REAL, Vec
    if any(fr.vec(j).type == T_ENUM or fr.vec(j).on_host for j in range(fr.ncols)):
        return None
    M = torch.stack([fr.vec(j).as_float(torch.float64) for j in range(fr.ncols)], 1)
    na_rm = name.endswith("NA") or name == "prod.na" or (bool(extra[0]) if extra else name in ("sd", "var"))
    base = name.replace("NA", "").replace(".na", "")
    nan = torch.isnan(M)
    if base == "sum":
        out = torch.nansum(M, 1)
    elif base == "mean":
        out = torch.nanmean(M, 1)
    elif base == "min":
        out = torch.where(nan, torch.full_like(M, math.inf), M).min(1).values
    elif base == "max":
        out = torch.where(nan, torch.full_like(M, -math.inf), M).max(1).values
    elif base == "prod":
        out = torch.where(nan, torch.ones_like(M), M).prod(1)
    else:
        cnt = (~nan).sum(1).to(torch.float64)
        mu = torch.nanmean(M, 1, keepdim=True)
        var = torch.nansum((M - mu) ** 2, 1) / (cnt - 1).clamp_min(1)
        out = torch.sqrt(var) if base == "sd" else var
    if not na_rm:
        out = torch.where(nan.any(1), torch.full_like(out, math.nan), out)
    return _F().from_vecs([Vec(out.contiguous(), T_REAL)], ["C1"])


def _apply(fr, margin, fun):
    margin = int(margin)
    if margin == 2:
        outs = [call(fun, [fr[:, j]]) for j in range(fr.ncols)]
        if all(not _is_frame(o) for o in outs):
            return _F()({n: [o] for n, o in zip(fr.names, outs)})
        res = outs[0]
        for o in outs[1:]:
            res = res.cbind(o)
        res.names = fr.names[:res.ncols]
        return res
    fast = _rowwise(fr, fun)
    if fast is not None:
        return fast
    rows = []
    g = fr.gather()
    for i in range(g.nrows):
        o = call(fun, [g[i, :]])
        rows.append(float(o) if not _is_frame(o) else float(o.as_data_frame().iloc[0, 0]))
    return _F()({"C1": rows})


def _ifelse(t, y, n):
    if not _is_frame(t):
        return y if t else n
    return t.ifelse(y, n)


def _time(name):
    def f(x):
        from . import timeops
        return getattr(timeops, name)(x)
    return f


def _str(name, *fixed):
    def f(x, *a):
        from . import strings
        return getattr(strings, name)(x, *a)
    return f


def _seq(frm, to, by=1.0):
    n = int(math.floor((to - frm) / by + 1e-10)) + 1
    return _F()({"C1": [frm + k * by for k in range(max(n, 0))]})


def _num(x):
    return float(x.as_data_frame().iloc[0, 0]) if _is_frame(x) else float(x)


PRIMS = {}
for _op in ("+", "-", "*", "/", "^", "%", "%%", "%/%", "intDiv", "==", "!=", "<", "<=", ">", ">=", "&", "|",
            "&&", "||"):
    PRIMS[_op] = _binop(_op)
for _nm, _meth in {"abs": "abs", "ceiling": "ceil", "floor": "floor", "trunc": "trunc", "sqrt": "sqrt", "exp": "exp",
                   "expm1": "expm1", "log": "log", "log10": "log10", "log2": "log2", "log1p": "log1p",
                   "sin": "sin", "cos": "cos", "tan": "tan", "asin": "asin", "acos": "acos", "atan": "atan",
                   "sinh": "sinh", "cosh": "cosh", "tanh": "tanh", "asinh": "asinh", "acosh": "acosh",
                   "atanh": "atanh", "sinpi": "sinpi", "cospi": "cospi", "tanpi": "tanpi", "sign": "sign",
                   "gamma": "gamma", "lgamma": "lgamma", "digamma": "digamma", "trigamma": "trigamma"}.items():
    PRIMS[_nm] = _unary(_meth)
PRIMS["not"] = PRIMS["!"] = lambda x: x.logical_negation() if _is_frame(x) else float(not x)
PRIMS["none"] = lambda x: x
PRIMS["round"] = lambda x, d=0.0: x.round(int(d)) if _is_frame(x) else float(round(x, int(d)))
PRIMS["signif"] = lambda x, d=6.0: x.signif(int(d)) if _is_frame(x) else float(f"{x:.{int(d)}g}")
for _nm in ("sum", "prod", "min", "max"):
    PRIMS[_nm] = _reduce(_nm)
PRIMS["sumNA"] = _reduce("sum", True)
PRIMS["minNA"] = _reduce("min", True)
PRIMS["maxNA"] = _reduce("max", True)
PRIMS["prod.na"] = _reduce("prod", True)
PRIMS["mean"] = lambda x, na_rm=0.0, axis=0.0: (x.mean(skipna=bool(na_rm), axis=int(axis))
                                                if int(axis) == 1 else x.mean(skipna=bool(na_rm), return_frame=True))
PRIMS["median"] = lambda x, na_rm=1.0: x.median(bool(na_rm))[0] if x.ncols == 1 else x.median(bool(na_rm))
PRIMS["sd"] = lambda x, na_rm=1.0: x.sd(bool(na_rm))[0] if x.ncols == 1 else x.sd(bool(na_rm))
PRIMS["var"] = lambda x, y=None, use="everything", symmetric=1.0: x.var(y if _is_frame(y) else None)
PRIMS["cor"] = lambda x, y=None, use="everything", method="Pearson": x.cor(y if _is_frame(y) else None,
                                                                             use=str(use), method=method)
PRIMS["nrow"] = lambda x: float(x.nrows)
PRIMS["ncol"] = lambda x: float(x.ncols)
PRIMS["dim"] = lambda x: [float(x.nrows), float(x.ncols)]
PRIMS["naCnt"] = lambda x: [float(c) for c in x.nacnt()]
PRIMS["any.na"] = lambda x: float(x.any_na_strict())
PRIMS["all"] = lambda x: float(x.all())
PRIMS["any"] = lambda x: float(x.any())
PRIMS["any.factor"] = lambda x: float(x.anyfactor())
for _nm in ("cumsum", "cumprod", "cummin", "cummax"):
    PRIMS[_nm] = (lambda m: lambda x, axis=0.0: getattr(x, m)(int(axis)))(_nm)
PRIMS["kurtosis"] = lambda x, na_rm=0.0: x.kurtosis(bool(na_rm))
PRIMS["skewness"] = lambda x, na_rm=0.0: x.skewness(bool(na_rm))
PRIMS["cols"] = PRIMS["cols_py"] = _cols
PRIMS["rows"] = _rows
PRIMS["cbind"] = lambda *fs: (fs[0].cbind(list(fs[1:])) if len(fs) > 1 else fs[0])
PRIMS["rbind"] = lambda *fs: fs[0].rbind(list(fs[1:])) if len(fs) > 1 else fs[0]
PRIMS["colnames="] = lambda fr, idx, names: _rename(fr, idx, names)
PRIMS["as.factor"] = lambda x: x.asfactor()
PRIMS["as.numeric"] = lambda x: x.asnumeric()
PRIMS["as.character"] = lambda x: x.ascharacter()
PRIMS["is.na"] = lambda x: x.isna() if _is_frame(x) else float(isinstance(x, float) and math.isnan(x))
PRIMS["is.factor"] = lambda x: [float(b) for b in x.isfactor()]
PRIMS["is.numeric"] = lambda x: [float(b) for b in x.isnumeric()]
PRIMS["is.character"] = lambda x: [float(b) for b in x.isstring()]
PRIMS["ifelse"] = _ifelse
def _levels(x):
    """AstLevels: one categorical column per input column holding the codes
    0..card-1 of its domain (NA-padded to the largest domain)."""
    from .vec import T_ENUM, Vec
    lv = x.levels()
    n = max([len(d or []) for d in lv] + [0])
    dev = x._vecs[0].data.device if x.ncols else None
    vecs = []
    for d in lv:
        d = list(d or [])
        codes = torch.full((n,), -1, dtype=torch.int32, device=dev)
        codes[:len(d)] = torch.arange(len(d), dtype=torch.int32, device=dev)
        vecs.append(Vec(codes, T_ENUM, d))
    from .frame import _reshard
    return _reshard(_F().from_vecs(vecs, [f"C{j + 1}" for j in range(len(lv))]))   # same table on every rank


PRIMS["levels"] = _levels
PRIMS["nlevels"] = lambda x: float(x.nlevels()[0])
PRIMS["setDomain"] = lambda x, inplace, levels: x.set_levels(levels)
PRIMS["relevel"] = lambda x, lvl: x.relevel(lvl)
PRIMS["relevel.by.freq"] = lambda x, w=None, topn=-1.0: x.relevel_by_frequency(w if isinstance(w, str) and w else None,
                                                                                int(topn))
PRIMS["appendLevels"] = lambda x, lv: x.append_levels(lv)
PRIMS["setLevel"] = lambda x, lv: x.set_level(lv)
PRIMS["na.omit"] = lambda x: x.na_omit()
PRIMS["scale"] = PRIMS["scale_inplace"] = lambda x, c=1.0, s=1.0: x.scale(c if isinstance(c, list) else bool(c),
                                                                          s if isinstance(s, list) else bool(s))
PRIMS["flatten"] = lambda x: x.flatten() if x.shape == (1, 1) else x
PRIMS["getrow"] = lambda x: x.getrow()
PRIMS["sort"] = lambda x, cols, asc=None: x.sort([x.names[int(c)] if not isinstance(c, str) else c for c in
                                                  (cols if isinstance(cols, list) else [cols])],
                                                 ascending=[bool(a) for a in asc] if isinstance(asc, list) else True)
PRIMS["merge"] = lambda l, r, ax=0.0, ay=0.0, bx=None, by=None, method="auto": l.merge(
    r, bool(ax), bool(ay), [l.names[int(i)] for i in bx] if bx else None, [r.names[int(i)] for i in by] if by else None)
PRIMS["GB"] = _gb
PRIMS["h2o.runif"] = lambda x, seed=-1.0: x.runif(int(seed))
PRIMS["unique"] = lambda x, na=0.0: x.unique(bool(na))
PRIMS["table"] = lambda x, *a: x.table(a[0] if a and _is_frame(a[0]) else None)
PRIMS["quantile"] = lambda x, probs, method="interpolate", w="_": x.quantile(probs, method)
PRIMS["h2o.hist"] = PRIMS["hist"] = lambda x, breaks="sturges": x.hist(breaks if not isinstance(breaks, float)
                                                                       else int(breaks))
PRIMS["cut"] = lambda x, br, lab=None, lowest=0.0, right=1.0, dig=3.0: x.cut(br, lab or None, bool(lowest),
                                                                            bool(right), int(dig))
def _impute(x, col, method="mean", comb="interpolate", gb=None, *a):
    """AstImpute: imputes the frame IN PLACE (the stored frame too) and
    returns the fill values (the group-by frame of fills with gb columns)."""
    by = [int(g) for g in gb] if isinstance(gb, (list, tuple)) and len(gb) else None
    out = x.impute(int(col), method, comb, by=by)
    src = getattr(x, "_rapids_src", None)
    if src is not None and len(src._vecs) == len(x._vecs):
        for j, v in enumerate(x._vecs):
            if src._vecs[j] is not v:
                src._vecs[j] = v
    return out


PRIMS["h2o.impute"] = lambda x, col, method="mean", comb="interpolate", gb=None, *a: _impute(x, col, method, comb, gb)
PRIMS["h2o.fillna"] = lambda x, method="forward", axis=0.0, maxlen=1.0: x.fillna(method, int(axis), int(maxlen))
PRIMS["pivot"] = lambda x, idx, col, val: x.pivot(idx, col, val)
PRIMS["melt"] = lambda x, ids, vals=None, vn="variable", valn="value", skipna=0.0: x.melt(
    ids, vals or None, vn, valn, bool(skipna))
PRIMS["dropdup"] = lambda x, cols, keep="first": x.drop_duplicates([x.names[int(c)] if not isinstance(c, str) else c
                                                                    for c in cols], keep)
PRIMS["rank_within_groupby"] = lambda x, gb, sc, asc=None, name="New_Rank_column", *a: x.rank_within_group_by(
    [x.names[int(c)] for c in gb], [x.names[int(c)] for c in sc], [bool(v) for v in asc] if asc else None, name)
PRIMS["topn"] = lambda x, col, pct, grab=-1.0: x.topNBottomN(int(col), pct, int(grab))
PRIMS["which"] = lambda x: x.which()
PRIMS["which.max"] = lambda x, na_rm=1.0, axis=0.0: x.idxmax(bool(na_rm), int(axis))
PRIMS["which.min"] = lambda x, na_rm=1.0, axis=0.0: x.idxmin(bool(na_rm), int(axis))
def _match(x, table, nomatch=0.0, *incomparables):
    """AstMatch (match fr table nomatch incomparables): 1 where the value is in
    `table`, else nomatch (NA rows too)."""
    tab = table if isinstance(table, list) else [table]
    pos = x.match(tab, -1.0, 1)
    from .ops_elem import ifelse
    return ifelse(pos > 0, 1.0, float(nomatch))


PRIMS["match"] = lambda x, table, nomatch=0.0, *a: _match(x, table, nomatch, *a)
PRIMS["%in%"] = lambda x, table: x.isin(table)
PRIMS["seq"] = _seq
PRIMS["seq_len"] = lambda n: _seq(1, n)
PRIMS["rep_len"] = lambda x, n: x.rep_len(int(n)) if _is_frame(x) else _F()({"C1": [x] * int(n)})
PRIMS["filterNACols"] = lambda x, frac: [float(i) for i in x.filter_na_cols(frac)]
PRIMS["columnsByType"] = lambda x, t: x.columns_by_type(t)
PRIMS["difflag1"] = lambda x: x.difflag1()
PRIMS["t"] = lambda x: x.transpose()
PRIMS["x"] = lambda a, b: a.mult(b)
PRIMS["distance"] = lambda a, b, measure: a.distance(b, measure)
PRIMS["kfold_column"] = lambda x, n, seed=-1.0: x.kfold_column(int(n), int(seed))
PRIMS["modulo_kfold_column"] = lambda x, n: x.modulo_kfold_column(int(n))
PRIMS["stratified_kfold_column"] = lambda x, n, seed=-1.0: x.stratified_kfold_column(int(n), int(seed))
PRIMS["h2o.random_stratified_split"] = lambda x, frac, seed=-1.0: x.stratified_split(frac, int(seed))
PRIMS["isax"] = lambda x, nw, mc, opt=0.0: x.isax(int(nw), int(mc), bool(opt))
PRIMS["apply"] = _apply
PRIMS["append"] = lambda dst, *pairs: _append(dst, *pairs)
PRIMS[":="] = _assign_cols
PRIMS["ls"] = lambda: _F().from_vecs([__import__("h2o3_amd.core.vec", fromlist=["x"]).make_string(
    np.asarray(sorted(dkv.keys()), dtype=object))], ["key"])   # AstLs: a one-column frame of the keys
PRIMS["mktime"] = lambda *a: _F().mktime(*[x if _is_frame(x) else float(x) for x in a])
PRIMS["as.Date"] = lambda x, fmt: x.as_date(fmt)
PRIMS["getTimeZone"] = lambda: __import__("h2o3_amd.core.timeops", fromlist=["x"]).get_timezone()
PRIMS["setTimeZone"] = lambda tz: __import__("h2o3_amd.core.timeops", fromlist=["x"]).set_timezone(tz)
PRIMS["listTimeZones"] = lambda: __import__("h2o3_amd.core.timeops", fromlist=["x"]).list_timezones()
for _nm in ("year", "month", "day", "hour", "minute", "second", "week", "dayOfWeek"):
    PRIMS[_nm] = _time(_nm)
for _nm, _fn in {"toupper": "toupper", "tolower": "tolower", "trim": "trim", "lstrip": "lstrip", "rstrip": "rstrip",
                 "strlen": "nchar", "countmatches": "countmatches", "entropy": "entropy", "strsplit": "strsplit",
                 "tokenize": "tokenize", "num_valid_substrings": "num_valid_substrings"}.items():
    PRIMS[_nm] = _str(_fn)
PRIMS["substring"] = lambda x, s, e=None: _str("substring")(x, int(s), None if e is None or math.isnan(e) else int(e))
PRIMS["replacefirst"] = lambda x, pat, rep, ic=0.0: _str("sub")(x, pat, rep, bool(ic))
PRIMS["replaceall"] = lambda x, pat, rep, ic=0.0: _str("gsub")(x, pat, rep, bool(ic))
PRIMS["grep"] = lambda x, pat, ic=0.0, inv=0.0, logical=0.0: _str("grep")(x, pat, bool(ic), bool(inv), bool(logical))
PRIMS["strDistance"] = lambda x, y, measure="lv", ce=1.0: _str("strdistance")(x, y, measure, bool(ce))


def pd_series(lv):
    return list(lv)


def _rename(fr, idx, names):
    idx = idx if isinstance(idx, list) else [idx]
    names = names if isinstance(names, list) else [names]
    out = fr  # in place, like AstColNames
    nm = out.names
    for i, n in zip(idx, names):
        nm[int(i)] = n
    out.names = nm
    return out


def _append(dst, *pairs):
    """AstAppend: (append dst (src name)+) -> a NEW frame sharing dst's
    columns plus each src (a one-column frame, number or string) under name."""
    if not pairs or len(pairs) % 2:
        raise RapidsError("append expects dst followed by (src name) pairs")
    out = _F().from_vecs(list(dst._vecs), list(dst.names))
    for src, name in zip(pairs[0::2], pairs[1::2]):
        if _is_frame(src) and src.ncols != 1:
            raise RapidsError("Can only append one column")
        out[str(name)] = src if _is_frame(src) else (src if isinstance(src, str) else float(src))
    return out




# ---- model / utility prims the reference client sends over /99/Rapids
# (water/rapids/ast/prims/models/*, advmath/AstMad, reducers/AstSumAxis,
# time/AstMoment, misc/AstMillis, AstRename, hex/leaderboard AstMakeLeaderboard)
def _frame_of_df(df):
    return _F()(df)


def _names_or_idx(fr, c):
    if isinstance(c, (int, float)):
        return fr.names[int(c)]
    return str(c)


def _perm_varimp(model, frame, metric="AUTO", n_samples=10000, n_repeats=1, features=None, seed=-1):
    feats = None if features in (None, [], "") else [str(f) for f in (features if isinstance(features, list)
                                                                       else [features])]
    out = model.permutation_importance(frame, str(metric), int(n_samples), int(n_repeats), feats, int(seed))
    return _frame_of_df(out.reset_index() if hasattr(out, "reset_index") and "Variable" not in out.columns else out)


def _pva(model, frame, variable, predicted):
    return _frame_of_df(model.predicted_vs_actual_by_variable(frame, predicted, str(variable), use_pandas=True))


def _make_lb(models, lb_frame="", sort_metric="AUTO", extra_columns=None, scoring_data="AUTO"):
    from ..automl.leaderboard import make_leaderboard
    ids = models if isinstance(models, list) else [models]
    objs = [dkv.get(str(m)) if isinstance(m, str) else m for m in ids]
    lbf = dkv.get(lb_frame) if isinstance(lb_frame, str) and lb_frame else (lb_frame if _is_frame(lb_frame) else None)
    ex = [str(e) for e in extra_columns] if isinstance(extra_columns, list) else \
        ([] if extra_columns in (None, "") else [str(extra_columns)])
    return make_leaderboard(objs, lbf, str(sort_metric), ex, str(scoring_data))


def _sum_axis(fr, skipna=1.0, axis=0.0):
    import torch as _t
    from .vec import T_REAL, Vec
    X = _t.stack([fr.vec(c).as_float(_t.float64) for c in fr.names], 1)
    if bool(skipna):
        X = _t.nan_to_num(X, nan=0.0)
    if int(axis) == 1:
        return _F().from_vecs([Vec(X.sum(1).to(_t.float32).contiguous(), T_REAL)], ["sum"])
    from ..parallel import collectives as coll
    s = X.sum(0)
    coll.allreduce_(s)
    return _F()(__import__("pandas").DataFrame({c: [float(v)] for c, v in zip(fr.names, s.tolist())}))


def _reset_threshold(model, threshold):
    """AstModelResetThreshold: the model's binomial threshold becomes
    `threshold`; returns the old one."""
    old = getattr(model, "_threshold_override", None)
    if old is None:
        tm = model._training_metrics
        old = tm.get("max_f1_threshold") if tm is not None else None
    model._threshold_override = float(threshold)
    return _F()(__import__("pandas").DataFrame({"old_threshold": [float("nan") if old is None else float(old)]}))


def _mad(fr, combine="interpolate", const=1.4826):
    import torch as _t
    x = fr.vec(fr.names[0]).as_float(_t.float64)
    x = x[~_t.isnan(x)]
    med = _t.quantile(x, 0.5) if x.numel() else _t.tensor(float("nan"))
    return float(const) * float(_t.quantile((x - med).abs(), 0.5)) if x.numel() else float("nan")


def _mode(fr):
    import torch as _t
    v = fr.vec(fr.names[0])
    d = v.data.to(_t.int64)
    d = d[d >= 0]
    return float(_t.argmax(_t.bincount(d))) if d.numel() else float("nan")


def _rename_key(old, new):
    obj = dkv.get(str(old))
    if obj is None:
        raise RapidsError(f"rename: no key {old}")
    dkv.put(str(new), obj)
    dkv.remove(str(old))
    if hasattr(obj, "frame_id"):
        try:
            obj.frame_id = str(new)
        except AttributeError:
            pass
    return None


def _tf_idf(fr, doc_col, text_col, preprocess=1.0, case_sensitive=1.0):
    from ..information_retrieval import tf_idf
    return tf_idf(fr, _names_or_idx(fr, doc_col), _names_or_idx(fr, text_col), bool(preprocess), bool(case_sensitive))


def _moment(*parts):
    from .frame import H2OFrame
    keys = ("year", "month", "day", "hour", "minute", "second", "msec")
    return H2OFrame.moment(**{k: v for k, v in zip(keys, parts) if v is not None})


PRIMS.update({
    "PermutationVarImp": _perm_varimp,
    "predicted.vs.actual.by.var": _pva,
    "makeLeaderboard": _make_lb,
    "sumaxis": _sum_axis,
    "model.reset.threshold": _reset_threshold,
    "rulefit.predict.rules": lambda m, fr, ids: m.predict_rules(fr, [str(i) for i in (ids if isinstance(ids, list)
                                                                                       else [ids])]),
    "tf-idf": _tf_idf,
    "word2vec.to.frame": lambda m: m.to_frame(),
    "tree.update.weights": lambda m, fr, w: (m.update_tree_weights(fr, str(w)), 0.0)[1],
    "segment_models_as_frame": lambda s: s.as_frame(),
    "transform": lambda m, fr: m.transform_frame(fr),
    "result": lambda m: m.result(),
    "moment": _moment,
    "h2o.mad": _mad,
    "mode": _mode,
    "millis": lambda: float(int(__import__("time").time() * 1000)),
    "rename": _rename_key,
})


def _perfect_auc(probs, actuals):
    """AstPerfectAUC: exact (tie-averaged) AUC of a probability column
    against 0/1 actuals."""
    import torch as _t
    from ..models.metrics import _auc_exact
    p = probs.vec(probs.names[0]).as_float(_t.float64)
    a = actuals.vec(actuals.names[0])
    y = a.data.to(_t.float64) if a.type == "enum" else a.as_float(_t.float64)
    ok = ~_t.isnan(p) & ~_t.isnan(y)
    return float(_auc_exact(p[ok], y[ok], _t.ones_like(p[ok]))[0])


def _ddply(fr, cols, fun):
    """AstDdply: fun applied to the rows of each group of `cols` -> one row
    per group: the group keys, then the function's value(s)."""
    import pandas as pd
    g = fr.gather()
    keys = [g.names[int(c)] if isinstance(c, (int, float)) else str(c) for c in (cols if isinstance(cols, list)
                                                                              else [cols])]
    df = g[keys].as_data_frame()
    out = []
    for kv, idx in df.groupby(keys, sort=True, dropna=False).indices.items():
        sub = g[[int(i) for i in idx], :]
        v = call(fun, [sub])
        vals = v.as_data_frame().iloc[0].tolist() if _is_frame(v) else [float(v)]
        out.append(list(kv if isinstance(kv, tuple) else (kv,)) + vals)
    ncol = max((len(r) for r in out), default=len(keys) + 1)
    return _F()(pd.DataFrame(out, columns=keys + [f"ddply_C{j + 1}" for j in range(ncol - len(keys))]))


PRIMS.update({"perfectAUC": _perfect_auc, "ddply": _ddply})


def _pav(fr):
    """AstPoolAdjacentViolators: frame (y, X, weights) -> the isotonic fit's
    thresholds (y, X) (hex/isotonic/PoolAdjacentViolatorsDriver.runPAV)."""
    import pandas as pd
    from ..models.isotonic import H2OIsotonicRegressionEstimator
    if fr.ncols != 3:
        raise RapidsError("Input frame is expected to have 3 columns: y, X, weights.")
    y, x, w = fr.names
    m = H2OIsotonicRegressionEstimator(weights_column=w)
    m.train(x=[x], y=y, training_frame=fr)
    return _F()(pd.DataFrame({y: m._ty, x: m._tx}))


def _grouped_permute(fr, perm_col, group_by, permute_by, keep_col):
    """AstGroupedPermute: within each group, every row whose permute_by
    level is 0 paired with every row whose level is 1 -> (group keys,
    In = keep value of the first, Out = keep value of the second, InAmnt,
    OutAmnt = their perm_col values)."""
    import pandas as pd
    g = fr.gather().as_data_frame()
    names = list(g.columns)
    gb = [names[int(c)] for c in (group_by if isinstance(group_by, list) else [group_by])]
    pc, pb, kc = names[int(perm_col)], names[int(permute_by)], names[int(keep_col)]
    levels = sorted(g[pb].dropna().unique())
    rows = []
    for key, sub in g.groupby(gb, sort=True):
        a = sub[sub[pb] == levels[0]] if levels else sub.iloc[:0]
        b = sub[sub[pb] == levels[1]] if len(levels) > 1 else sub.iloc[:0]
        for _, ra in a.iterrows():
            for _, rb in b.iterrows():
                rows.append(list(key if isinstance(key, tuple) else (key,)) + [ra[kc], rb[kc], ra[pc], rb[pc]])
    return _F()(pd.DataFrame(rows, columns=gb + ["In", "Out", "InAmnt", "OutAmnt"]))


PRIMS.update({"isotonic.pav": _pav, "grouped_permute": _grouped_permute})
