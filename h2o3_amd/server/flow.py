"""Flow notebooks: the cell language of h2o-web's Flow and a runner for it.

The reference's Flow (h2o-web, the bundled h2o-flow app) keeps notebooks as
``.flow`` JSON documents -- ``{"version": "1.0.0", "cells": [{"type": "cs" |
"md" | "h1".."h6" | "raw", "input": ...}]}`` -- whose ``cs`` cells are
CoffeeScript calls of Flow *routines* (``importFiles``, ``setupParse``,
``parseFiles``, ``splitFrame``, ``buildModel``, ``predict``, ``runAutoML``,
...), each of which drives the /3 REST API.  The reference ships 343 such
notebooks as its Flow test packs (h2o-docs/src/product/flow/packs/*/*.flow)
and saves user notebooks through NodePersistentStorage
(water/api/NodePersistentStorageHandler.java, category ``notebook``).

Here the cell language is parsed in Python (the literal / call subset of
CoffeeScript those notebooks use: implicit calls ``f a, g b`` = ``f(a, g(b))``,
implicit objects ``k: v, k2: v2`` (also one pair per indented line), JSON
arrays / objects, quoted or bare keys, ``#`` comments) and every routine is
run against a transport: ``LocalTransport`` calls the REST handlers of an
in-process app directly (the server's ``POST /flow/cell`` endpoint and the
tests use it), ``HttpTransport`` talks to any running server over HTTP
(``python -m h2o3_amd.server.flow notebook.flow --url http://host:54321``, a
headless notebook runner).  The browser notebook (static/flow.html) keeps the
cell list, renders results and saves notebooks; the cells themselves run
server-side through this module, so the language is implemented once.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from urllib.parse import quote

__all__ = ["FlowSyntaxError", "FlowError", "parse_cell", "Call", "Symbol", "FlowRunner", "LocalTransport",
           "HttpTransport", "load_notebook", "ROUTINES"]


class FlowSyntaxError(ValueError):
    pass


class FlowError(RuntimeError):
    pass


# --------------------------------------------------------------------------- parser
@dataclass
class Call:
    name: str
    args: list = field(default_factory=list)


@dataclass(frozen=True)
class Symbol:
    """A bare name used as a value: a notebook variable, else a routine
    reference (``assist splitFrame, ...``)."""
    name: str


@dataclass
class Assign:
    name: str
    value: object


@dataclass
class BinOp:
    op: str
    left: object
    right: object


@dataclass
class If:
    cond: object
    then: list
    other: list


_LITERALS = {"true": True, "false": False, "yes": True, "no": False, "on": True, "off": False,
             "null": None, "undefined": None}
_NUM = re.compile(r"-?(?:0[xX][0-9a-fA-F]+|(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)")
_IDENT = re.compile(r"[A-Za-z_$][\w$]*")


@dataclass
class _Tok:
    kind: str      # num str ident punct nl eof
    val: object
    space: bool    # whitespace before the token on the same line
    indent: int    # for nl: indentation of the next non-blank line


def _tokenize(src: str) -> list[_Tok]:
    toks: list[_Tok] = []
    i, n, depth, space = 0, len(src), 0, False
    while i < n:
        c = src[i]
        if c in " \t\r":
            i += 1
            space = True
            continue
        if c == "#":                                   # comment to the end of the line
            while i < n and src[i] != "\n":
                i += 1
            continue
        if c == "\n":
            j = i + 1
            while True:                                # skip blank / comment-only lines
                k = j
                while k < n and src[k] in " \t\r":
                    k += 1
                if k < n and src[k] == "#":
                    while k < n and src[k] != "\n":
                        k += 1
                if k < n and src[k] == "\n":
                    j = k + 1
                    continue
                break
            indent = 0
            while j + indent < n and src[j + indent] in " \t":
                indent += 1
            if depth == 0 and (not toks or toks[-1].kind != "nl"):
                toks.append(_Tok("nl", None, False, indent))
            i, space = j + indent, True
            continue
        if c in "\"'":
            q, j, buf = c, i + 1, []
            while j < n and src[j] != q:
                if src[j] == "\\" and j + 1 < n:
                    esc = src[j + 1]
                    if esc == "u" and j + 5 < n:
                        buf.append(chr(int(src[j + 2:j + 6], 16)))
                        j += 6
                        continue
                    buf.append({"n": "\n", "t": "\t", "r": "\r", "b": "\b", "f": "\f", "0": "\0"}.get(esc, esc))
                    j += 2
                    continue
                buf.append(src[j])
                j += 1
            if j >= n:
                raise FlowSyntaxError(f"unterminated string at offset {i}")
            toks.append(_Tok("str", "".join(buf), space, 0))
            i, space = j + 1, False
            continue
        prev_value = toks and (toks[-1].kind in ("num", "str", "ident") or toks[-1].val in (")", "]", "}"))
        m = _NUM.match(src, i)
        if m and (c != "-" or not prev_value or space):
            txt = m.group(0)
            if txt != "-":
                if "x" in txt or "X" in txt:
                    v = int(txt, 16)
                else:
                    v = float(txt) if any(ch in txt for ch in ".eE") else int(txt)
                toks.append(_Tok("num", v, space, 0))
                i, space = m.end(), False
                continue
        m = _IDENT.match(src, i)
        if m:
            toks.append(_Tok("ident", m.group(0), space, 0))
            i, space = m.end(), False
            continue
        if c in "[{(":
            depth += 1
        elif c in "]})":
            depth = max(0, depth - 1)
            if toks and toks[-1].kind == "nl":
                toks.pop()
        if c == ";" and depth > 0:                    # lenient: ';' as a list separator
            c = ","
        if c in "[]{}(),:=+":
            toks.append(_Tok("punct", c, space, 0))
            i, space = i + 1, False
            continue
        raise FlowSyntaxError(f"unexpected character {c!r} at offset {i}")
    while toks and toks[-1].kind == "nl":
        toks.pop()
    toks.append(_Tok("eof", None, True, 0))
    return toks


class _Parser:
    def __init__(self, src: str):
        self.t = _tokenize(src)
        self.i = 0

    def peek(self, k=0) -> _Tok:
        return self.t[min(self.i + k, len(self.t) - 1)]

    def next(self) -> _Tok:
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, p):
        tok = self.next()
        if tok.kind != "punct" or tok.val != p:
            raise FlowSyntaxError(f"expected {p!r}, got {tok.val!r}")
        return tok

    def is_p(self, p, k=0):
        tok = self.peek(k)
        return tok.kind == "punct" and tok.val == p

    def skip_nl(self):
        while self.peek().kind == "nl":
            self.i += 1

    def program(self) -> list:
        self.skip_nl()
        if self.peek().kind == "eof":
            return []
        out = self.block(0)
        self.skip_nl()
        if self.peek().kind != "eof":
            raise FlowSyntaxError(f"unexpected {self.peek().val!r}")
        return out

    def block(self, ind) -> list:
        """Statements at one indentation level."""
        out = []
        while True:
            out.append(self.statement(ind))
            tok = self.peek()
            if tok.kind == "nl" and tok.indent == ind and self.peek(1).kind != "eof" and \
                    not (self.peek(1).kind == "ident" and self.peek(1).val == "else"):
                self.next()
                continue
            if tok.kind == "nl" and tok.indent > ind:
                raise FlowSyntaxError("unexpected indentation")
            return out

    def _body(self, ind):
        tok = self.next()
        if tok.kind != "nl" or tok.indent <= ind:
            raise FlowSyntaxError("expected an indented block")
        return self.block(tok.indent)

    def statement(self, ind):
        tok = self.peek()
        if tok.kind == "ident" and tok.val == "if":
            self.next()
            cond = self.expr()
            then = self._body(ind)
            other = []
            if self.peek().kind == "nl" and self.peek().indent == ind and self.peek(1).val == "else":
                self.i += 2
                other = self._body(ind)
            return If(cond, then, other)
        if tok.kind == "ident" and self.is_p("=", 1):
            self.i += 2
            return Assign(tok.val, self.expr())
        return self.expr(top=True)

    def _starts_pair(self, k=0):
        tok = self.peek(k)
        return tok.kind in ("ident", "str", "num") and self.is_p(":", k + 1)

    def _starts_arg(self, tok):
        return tok.kind in ("num", "str", "ident") or (tok.kind == "punct" and tok.val in "[{")

    def expr(self, top=False):
        left = self.primary(top)
        while self.is_p("+"):
            self.next()
            left = BinOp("+", left, self.primary())
        return left

    def primary(self, top=False):
        tok = self.peek()
        if self._starts_pair():
            return self.implicit_object()
        if tok.kind == "ident":
            self.next()
            if tok.val in _LITERALS:
                return _LITERALS[tok.val]
            nxt = self.peek()
            if nxt.kind == "punct" and nxt.val == "(" and not nxt.space:
                self.next()
                args = []
                self.skip_nl()
                while not self.is_p(")"):
                    args.append(self.expr())
                    self.skip_nl()
                    if self.is_p(","):
                        self.next()
                        self.skip_nl()
                self.expect(")")
                return Call(tok.val, args)
            if self._starts_arg(nxt) and nxt.space:
                return Call(tok.val, self.arglist())
            if nxt.kind == "nl" and nxt.indent > 0 and self._starts_pair(1):
                self.next()                            # routine name, then an indented key: value block
                return Call(tok.val, [self.implicit_object()])
            return Call(tok.val, []) if top else Symbol(tok.val)
        if tok.kind in ("num", "str"):
            self.next()
            return tok.val
        if self.is_p("["):
            return self.array()
        if self.is_p("{"):
            return self.obj()
        raise FlowSyntaxError(f"unexpected {tok.val!r}")

    def arglist(self):
        args = [self.expr()]
        while self.is_p(","):
            self.next()
            self.skip_nl()
            args.append(self.expr())
        return args

    def key(self):
        tok = self.next()
        if tok.kind not in ("ident", "str", "num"):
            raise FlowSyntaxError(f"bad object key {tok.val!r}")
        self.expect(":")
        return str(tok.val)

    def implicit_object(self):
        out = {}
        while True:
            k = self.key()
            if self.peek().kind == "nl" and self._starts_pair(1):
                self.next()                            # key:\n  nested: block
                out[k] = self.implicit_object()
            else:
                out[k] = self.expr()
            if self.is_p(",") and self._starts_pair(1):
                self.next()
                continue
            if self.is_p(",") and self.peek(1).kind == "nl" and self._starts_pair(2):
                self.i += 2
                continue
            if self.peek().kind == "nl" and self._starts_pair(1):
                self.next()
                continue
            return out

    def array(self):
        self.expect("[")
        out = []
        while not self.is_p("]"):
            out.append(self.expr())
            if self.is_p(","):
                self.next()
        self.expect("]")
        return out

    def obj(self):
        self.expect("{")
        out = {}
        while not self.is_p("}"):
            k = self.key()
            out[k] = self.expr()
            if self.is_p(","):
                self.next()
        self.expect("}")
        return out


def parse_cell(src: str) -> list:
    """Parse one ``cs`` cell into a list of statements (Call / literal)."""
    return _Parser(src).program()


def load_notebook(src) -> dict:
    """A .flow document (path, JSON text or dict) -> {"version", "cells"}."""
    if isinstance(src, dict):
        return src
    text = src
    if not str(src).lstrip().startswith("{"):
        with open(src, encoding="utf-8") as f:
            text = f.read()
    doc = json.loads(text)
    if not isinstance(doc.get("cells"), list):
        raise FlowSyntaxError("not a Flow notebook: no cells")
    return doc


# --------------------------------------------------------------------------- transports
class LocalTransport:
    """Calls the REST handlers of an in-process app (rest.create_app) without
    HTTP: the app records (method, path regex, handler) for every route."""

    def __init__(self, app):
        self.routes = app.state.flow_routes

    def __call__(self, method, path, params=None):
        path = path.split("?")[0]
        for m, rx, fn, wrap in self.routes:
            if m != method:
                continue
            hit = rx.fullmatch(path)
            if hit:
                try:
                    return wrap(fn(dict(params or {}), None, **hit.groupdict()))
                except Exception as e:  # noqa: BLE001 - the cell reports it
                    raise FlowError(getattr(e, "msg", None) or str(e)) from e
        raise FlowError(f"no route {method} {path}")


class HttpTransport:
    """JSON over HTTP to a running server (urllib; or any requests/httpx-like
    session with .request(method, url, json=...))."""

    def __init__(self, url="http://127.0.0.1:54321", session=None, auth=None):
        self.url, self.session, self.auth = url.rstrip("/"), session, auth

    def __call__(self, method, path, params=None):
        if self.session is not None:
            kw = {"json": params} if method in ("POST", "PUT") else {"params": _flat(params)}
            r = self.session.request(method, self.url + path, **kw)
            body = r.json() if r.content else {}
            if r.status_code >= 400:
                raise FlowError(body.get("msg") or body.get("exception_msg") or str(body))
            return body
        import base64
        import urllib.error
        import urllib.parse
        import urllib.request
        url = self.url + path
        data = None
        headers = {"Content-Type": "application/json"}
        if method in ("POST", "PUT"):
            data = json.dumps(params or {}).encode()
        elif params:
            url += "?" + urllib.parse.urlencode(_flat(params))
        if self.auth:
            headers["Authorization"] = "Basic " + base64.b64encode(":".join(self.auth).encode()).decode()
        req = urllib.request.Request(url, data=data, method=method, headers=headers)
        try:
            with urllib.request.urlopen(req) as resp:
                raw = resp.read()
        except urllib.error.HTTPError as e:
            raw = e.read()
            try:
                body = json.loads(raw)
            except ValueError:
                body = {"msg": raw.decode("utf-8", "replace")}
            raise FlowError(body.get("msg") or str(body)) from e
        return json.loads(raw) if raw else {}


def _flat(params):
    return {k: (json.dumps(v) if isinstance(v, (list, dict)) else v) for k, v in (params or {}).items()}


# --------------------------------------------------------------------------- routines
def _q(s):
    return quote(str(s), safe="")


def _opts(args, i=0):
    """Trailing options object of a routine call (or {})."""
    return args[i] if len(args) > i and isinstance(args[i], dict) else {}


def _result(kind, data=None, **kw):
    return {"kind": kind, "data": data, **kw}


def _form(routine, args):
    """Calls without their data open a form in Flow (assist / the routine's
    input dialog); headless they are no-ops that say so."""
    return _result("form", None, routine=routine, args=[a.name if isinstance(a, Symbol) else a for a in args])


def _frame_key(x):
    if isinstance(x, dict):
        if x.get("kind") == "frame":
            return x["key"]
        if "name" in x:
            return x["name"]
    return str(x)


_PARSE_KEYS = ("destination_frame", "separator", "column_names", "column_types", "check_header",
               "delete_on_done", "skipped_columns", "na_strings", "single_quotes", "parse_type",
               "number_columns", "chunk_size", "escapechar", "quotechar", "decrypt_tool",
               "custom_non_data_line_markers", "partition_by", "tz_adjust_to_local")


class FlowRunner:
    """Runs Flow cells against a transport.  ``path_map`` rewrites the file
    paths the notebooks import (e.g. the reference packs' ``../smalldata``)."""

    def __init__(self, transport, path_map=None, automl_max_runtime_secs=None):
        self.vars: dict = {}                           # the notebook's shared sandbox
        self.t = transport
        self.path_map = path_map or (lambda p: p)
        self.automl_max_runtime_secs = automl_max_runtime_secs

    # --- evaluation
    def run_cell(self, src: str, ctype: str = "cs"):
        if ctype != "cs":
            return _result("markup", src, cell_type=ctype)
        out = None
        for stmt in parse_cell(src):
            out = self.eval(stmt)
        return out if out is not None else _result("empty")

    def eval(self, node):
        if isinstance(node, Assign):
            self.vars[node.name] = self.eval(node.value)
            return _result("value", self.vars[node.name])
        if isinstance(node, If):
            out = None
            for st in (node.then if self.eval(node.cond) else node.other):
                out = self.eval(st)
            return out
        if isinstance(node, BinOp):
            a, b = self.eval(node.left), self.eval(node.right)
            return (str(a) + str(b)) if isinstance(a, str) or isinstance(b, str) else a + b
        if isinstance(node, Symbol):
            return self.vars.get(node.name, node)
        if isinstance(node, Call) and not node.args and node.name in self.vars:
            return _result("value", self.vars[node.name])
        if isinstance(node, Call):
            fn = ROUTINES.get(node.name)
            if fn is None:
                raise FlowError(f"unknown Flow routine: {node.name}")
            args = [self.eval(a) for a in node.args]
            try:
                return fn(self, args)
            except (IndexError, KeyError, TypeError, ValueError, AttributeError) as e:
                raise FlowError(f"{node.name}: bad arguments ({type(e).__name__}: {e})") from e
        if isinstance(node, list):
            return [self.eval(a) for a in node]
        if isinstance(node, dict):
            return {k: self.eval(v) for k, v in node.items()}
        return node

    def run_notebook(self, nb, stop_on_error=True):
        """Run every cell; -> [(cell index, type, result or exception)]."""
        doc = load_notebook(nb)
        out = []
        for i, cell in enumerate(doc["cells"]):
            try:
                out.append((i, cell.get("type", "cs"), self.run_cell(cell.get("input", ""), cell.get("type", "cs"))))
            except (FlowError, FlowSyntaxError) as e:
                if stop_on_error:
                    raise FlowError(f"cell {i} ({cell.get('input', '')[:80]!r}): {e}") from e
                out.append((i, cell.get("type", "cs"), e))
        return out

    # --- REST helpers
    def get(self, path, params=None):
        return self.t("GET", path, params)

    def post(self, path, params=None):
        return self.t("POST", path, params)

    def delete(self, path):
        return self.t("DELETE", path, None)

    def rapids(self, ast):
        return self.post("/99/Rapids", {"ast": ast})

    def frame_columns(self, key):
        fr = self.get(f"/3/Frames/{_q(key)}", {"row_count": 0})["frames"][0]
        return [c["label"] for c in fr["columns"]]


ROUTINES: dict = {}


def routine(*names):
    def deco(fn):
        for n in names:
            ROUTINES[n] = fn
        return fn
    return deco


# --- help / forms
@routine("assist")
def _assist(r, args):
    return _form("assist", args)


@routine("help")
def _help(r, args):
    return _result("help", sorted(ROUTINES))


@routine("inspect")
def _inspect(r, args):
    """inspect [name,] object: the object's tables (all, or the named one)."""
    if not args:
        return _form("inspect", args)
    obj = args[-1]
    name = args[0] if len(args) > 1 else None
    data = obj.get("data") if isinstance(obj, dict) else obj
    tables = {}

    def walk(x, path=""):
        if isinstance(x, dict):
            if x.get("__meta", {}).get("schema_type") == "TwoDimTable" or "columns" in x and "data" in x \
                    and isinstance(x.get("data"), list) and "name" in x:
                tables[x.get("name") or path] = x
                return
            for k, v in x.items():
                walk(v, k)
        elif isinstance(x, list):
            for v in x:
                walk(v, path)
    walk(data)
    if isinstance(obj, dict) and obj.get("kind") == "prediction" and isinstance(data, dict):
        mm = (data.get("model_metrics") or [{}])[0]
        scal = {k: v for k, v in mm.items() if isinstance(v, (int, float, str)) and not k.startswith("__")}
        tables["Prediction"] = {"__meta": {"schema_type": "TwoDimTable"}, "name": "Prediction",
                                "columns": [{"name": "metric"}, {"name": "value"}],
                                "data": [list(scal), [scal[k] for k in scal]]}
    if name is None:
        return _result("tables", tables, of=obj.get("kind") if isinstance(obj, dict) else None)
    low = {k.lower(): k for k in tables}
    # Flow names inspections "output - Coefficients", "output - training_metrics - Gains/Lift Table"
    cands = [str(name).lower(), str(name).split(" - ")[-1].lower()]
    key = next((low[c] for c in cands if c in low), None) or \
        next((k for c in cands for k in tables if c in k.lower()), None)
    if key is None:
        if str(name).lower() in ("summary", "parameters") and isinstance(data, dict):
            return _result("table", data.get("summary_table") if name == "summary" else data.get("parameters"),
                           name=name)
        raise FlowError(f"inspect: no table {name!r} (have {sorted(tables)})")
    return _result("table", tables[key], name=key)


@routine("grid", "plot")
def _grid(r, args):
    """grid / plot <inspection>: Flow renders it; headless it passes through."""
    return args[0] if args else _form("grid", args)


# --- cloud
@routine("getCloud")
def _get_cloud(r, args):
    return _result("cloud", r.get("/3/Cloud"))


@routine("getTimeline")
def _get_timeline(r, args):
    return _result("timeline", r.get("/3/Timeline"))


@routine("getJobs")
def _get_jobs(r, args):
    return _result("jobs", r.get("/3/Jobs"))


@routine("getJob")
def _get_job(r, args):
    return _result("job", r.get(f"/3/Jobs/{_q(args[0])}"))


@routine("cancelJob")
def _cancel_job(r, args):
    return _result("job", r.post(f"/3/Jobs/{_q(args[0])}/cancel"))


# --- import / parse
@routine("importFiles")
def _import_files(r, args):
    if not args:
        return _form("importFiles", args)
    paths = args[0] if isinstance(args[0], list) else [args[0]]
    out = [r.get("/3/ImportFiles", {"path": r.path_map(p)}) for p in paths]
    return _result("import", out, keys=[k for o in out for k in o["destination_frames"]])


@routine("setupParse")
def _setup_parse(r, args):
    o = _opts(args)
    paths = o.get("paths") or o.get("source_frames")
    if not paths:
        return _form("setupParse", args)
    return _result("parse_setup", r.post("/3/ParseSetup", {"source_frames": [r.path_map(p) for p in paths]}))


@routine("parseFiles")
def _parse_files(r, args):
    o = _opts(args)
    paths = o.get("paths") or o.get("source_frames")
    if not paths:
        return _form("parseFiles", args)
    body = {k: o[k] for k in _PARSE_KEYS if k in o}
    body["source_frames"] = [r.path_map(p) for p in paths]
    out = r.post("/3/Parse", body)
    return _result("frame", out, key=out["destination_frame"]["name"])


@routine("importModel")
def _import_model(r, args):
    o = _opts(args, 1)
    out = r.post("/99/Models.bin/", {"dir": r.path_map(args[0]), "force": o.get("overwrite", True)})
    return _result("model", out)


# --- frames
@routine("getFrames")
def _get_frames(r, args):
    return _result("frames", r.get("/3/Frames"))


@routine("getFrame", "getFrameData")
def _get_frame(r, args):
    key = _frame_key(args[0])
    return _result("frame", r.get(f"/3/Frames/{_q(key)}", {"row_count": 20}), key=key)


@routine("getFrameSummary")
def _get_frame_summary(r, args):
    key = _frame_key(args[0])
    return _result("frame", r.get(f"/3/Frames/{_q(key)}/summary"), key=key)


@routine("getColumnSummary")
def _get_column_summary(r, args):
    key = _frame_key(args[0])
    return _result("column", r.get(f"/3/Frames/{_q(key)}/columns/{_q(args[1])}/summary"), key=key)


@routine("deleteFrame")
def _delete_frame(r, args):
    return _result("deleted", r.delete(f"/3/Frames/{_q(_frame_key(args[0]))}"))


@routine("deleteFrames")
def _delete_frames(r, args):
    return _result("deleted", [r.delete(f"/3/Frames/{_q(_frame_key(k))}") for k in args[0]])


@routine("splitFrame")
def _split_frame(r, args):
    if len(args) < 2:
        return _form("splitFrame", args)
    key = _frame_key(args[0])
    ratios = args[1]
    dests = args[2] if len(args) > 2 and isinstance(args[2], list) else None
    seed = args[3] if len(args) > 3 and not isinstance(args[3], dict) else -1
    body = {"dataset": key, "ratios": ratios, "seed": seed}
    if dests:
        body["destination_frames"] = dests
    out = r.post("/3/SplitFrame", body)
    return _result("split", out, keys=[d["name"] for d in out["destination_frames"]])


@routine("createFrame")
def _create_frame(r, args):
    o = _opts(args)
    if not o:
        return _form("createFrame", args)
    body = dict(o)
    for k in ("rows", "cols", "factors"):
        if isinstance(body.get(k), str):
            body[k] = int(body[k])
    body.pop("seed_for_column_types", None)
    out = r.post("/3/CreateFrame", body)
    return _result("frame", out, key=out["destination_frame"]["name"])


@routine("exportFrame")
def _export_frame(r, args):
    if len(args) < 2:
        return _form("exportFrame", args)
    o = _opts(args, 2)
    out = r.post(f"/3/Frames/{_q(_frame_key(args[0]))}/export",
                 {"path": r.path_map(args[1]), "force": bool(o.get("overwrite", False))})
    return _result("export", out)


@routine("bindFrames")
def _bind_frames(r, args):
    dest, srcs = args[0], args[1]
    out = r.rapids(f"(assign {dest} (cbind {' '.join(_frame_key(s) for s in srcs)}))")
    return _result("frame", out, key=dest)


@routine("changeColumnType")
def _change_column_type(r, args):
    o = _opts(args)
    fr, col, typ = o["frame"], o["column"], str(o["type"]).lower()
    cols = r.frame_columns(fr)
    j = cols.index(col) if not isinstance(col, int) else col
    conv = {"enum": "as.factor", "factor": "as.factor", "numeric": "as.numeric", "real": "as.numeric",
            "int": "as.numeric", "string": "as.character"}[typ]
    out = r.rapids(f"(assign {fr} (:= {fr} ({conv} (cols {fr} {j})) {j} []))")
    return _result("frame", out, key=fr)


@routine("imputeColumn")
def _impute_column(r, args):
    o = _opts(args)
    fr = o["frame"]
    cols = r.frame_columns(fr)
    j = cols.index(o["column"])
    gb = [cols.index(c) for c in (o.get("groupByColumns") or [])]
    method = str(o.get("method", "mean")).lower()
    comb = str(o.get("combineMethod", "interpolate")).lower()
    out = r.rapids(f"(h2o.impute {fr} {j} \"{method}\" \"{comb}\" [{' '.join(map(str, gb))}] _ _)")
    return _result("impute", out, key=fr)


# --- models
def _clean_params(p):
    """Flow's form fills every field; empty strings / lists mean 'unset'."""
    return {k: v for k, v in p.items() if v is not None and v != "" and v != []}


def _grid_values(vals):
    out = []
    for v in vals:
        if v is None:
            continue
        if isinstance(v, str):
            try:
                v = json.loads(v)
            except ValueError:
                pass
        out.append(v)
    return out


@routine("buildModel")
def _build_model(r, args):
    if len(args) < 2 or not isinstance(args[1], dict):
        return _form("buildModel", args)
    algo = args[0].name if isinstance(args[0], Symbol) else str(args[0])
    p = _clean_params(args[1])
    hyper = p.pop("hyper_parameters", None)
    if hyper:
        hyper = {k: _grid_values(v) for k, v in hyper.items()}
        p["hyper_parameters"] = {k: v for k, v in hyper.items() if v}
        p.setdefault("grid_id", p.pop("model_id", None) or f"{algo}_grid")
        p.pop("model_id", None)
        out = r.post(f"/99/Grid/{_q(algo)}", p)
        return _result("grid", out, key=out["grid_id"]["name"])
    out = r.post(f"/3/ModelBuilders/{_q(algo)}", p)
    return _result("model_build", out, key=out["job"]["dest"]["name"])


@routine("getModels")
def _get_models(r, args):
    return _result("models", r.get("/3/Models"))


@routine("getModel")
def _get_model(r, args):
    key = args[0]
    return _result("model", r.get(f"/3/Models/{_q(key)}"), key=key)


@routine("deleteModel")
def _delete_model(r, args):
    return _result("deleted", r.delete(f"/3/Models/{_q(args[0])}"))


@routine("deleteModels")
def _delete_models(r, args):
    return _result("deleted", [r.delete(f"/3/Models/{_q(k)}") for k in args[0]])


@routine("exportModel")
def _export_model(r, args):
    o = _opts(args, 2)
    return _result("export", r.get(f"/99/Models.bin/{_q(args[0])}",
                                   {"dir": r.path_map(args[1]), "force": bool(o.get("overwrite", False))}))


@routine("predict")
def _predict(r, args):
    o = _opts(args)
    if not o.get("model") or not o.get("frame"):
        return _form("predict", args)
    body = {k: v for k, v in o.items() if k not in ("model", "frame")}
    out = r.post(f"/3/Predictions/models/{_q(o['model'])}/frames/{_q(_frame_key(o['frame']))}", body)
    key = (out.get("predictions_frame") or {}).get("name") or o.get("predictions_frame")
    return _result("prediction", out, key=key)


@routine("getPrediction")
def _get_prediction(r, args):
    o = _opts(args)
    out = r.get(f"/3/ModelMetrics/models/{_q(o['model'])}/frames/{_q(_frame_key(o['frame']))}")
    return _result("prediction", out)


# --- grids / automl
@routine("getGrids")
def _get_grids(r, args):
    return _result("grids", r.get("/99/Grids"))


@routine("getGrid")
def _get_grid(r, args):
    o = _opts(args, 1)
    out = r.get(f"/99/Grids/{_q(args[0])}", {k: o[k] for k in ("sort_by", "decreasing") if k in o})
    return _result("grid", out, key=args[0])


@routine("runAutoML")
def _run_automl(r, args):
    if not args or not isinstance(args[0], dict):
        return _form("runAutoML", args)
    spec = json.loads(json.dumps(args[0]))
    if r.automl_max_runtime_secs is not None:
        sc = spec.setdefault("build_control", {}).setdefault("stopping_criteria", {})
        sc["max_runtime_secs"] = r.automl_max_runtime_secs
    out = r.post("/99/AutoMLBuilder", spec)
    return _result("automl", out, key=out["build_control"]["project_name"])


@routine("getLeaderboard")
def _get_leaderboard(r, args):
    key = str(args[0])
    try:
        out = r.get(f"/99/Leaderboards/{_q(key)}")
    except FlowError:
        if "@@" not in key:                            # Leaderboard.idForProject: project@@response
            raise
        out = r.get(f"/99/Leaderboards/{_q(key.split('@@')[0])}")
    return _result("leaderboard", out, key=key)


@routine("getAutoML")
def _get_automl(r, args):
    return _result("automl", r.get(f"/99/AutoML/{_q(str(args[0]).split('@@')[0])}"))


# --------------------------------------------------------------------------- CLI
def main(argv=None):
    """Headless notebook runner: run every cell of .flow files against a
    server and report per-cell status."""
    import argparse
    ap = argparse.ArgumentParser(prog="python -m h2o3_amd.server.flow")
    ap.add_argument("notebooks", nargs="+")
    ap.add_argument("--url", default="http://127.0.0.1:54321")
    ap.add_argument("--user")
    ap.add_argument("--password")
    ap.add_argument("--data-root", help="directory the notebooks' ../smalldata paths resolve against")
    ap.add_argument("--keep-going", action="store_true")
    a = ap.parse_args(argv)
    pm = None
    if a.data_root:
        import os
        root = a.data_root

        def pm(p):
            p = str(p)
            return os.path.join(root, p[3:]) if p.startswith("../") else p
    runner = FlowRunner(HttpTransport(a.url, auth=(a.user, a.password) if a.user else None), path_map=pm)
    bad = 0
    for nb in a.notebooks:
        for i, ctype, res in runner.run_notebook(nb, stop_on_error=not a.keep_going):
            ok = not isinstance(res, Exception)
            bad += not ok
            kind = res.get("kind") if ok and isinstance(res, dict) else type(res).__name__
            print(f"{nb}:{i} [{ctype}] {'ok' if ok else 'FAIL'} {kind}{'' if ok else ': ' + str(res)}")
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
