"""Run the reference's Flow test packs on synthetic data of the declared shape.

The reference ships its Flow regression notebooks under
h2o-docs/src/product/flow/packs/{test-small,test-medium,test-large,examples}
(343 ``.flow`` files).  Their datasets (``../smalldata/...``) are not in the
reference tree, but every ``parseFiles`` cell declares the file's layout:
column names, column types, separator, header and parse type.  This module
writes a synthetic file of exactly that layout for every parsed path
(CSV / ARFF / SVMLight / XLS, gz / zip compressed by extension), shaped so the
models the notebook builds on it are valid (a response used with a
binomial family or bernoulli distribution is 0/1, poisson / tweedie counts
are non-negative, gamma responses positive, weights positive), then runs
every cell through flow.FlowRunner and reports per-cell results.

``python -m h2o3_amd.server.flow_packs [--pack test-small] [--rows 200]``
runs a pack in-process; tests/test_flow.py runs a handful of notebooks.
"""
from __future__ import annotations

import glob
import gzip
import io
import json
import os
import time
import zipfile

import numpy as np

from .flow import Call, FlowRunner, FlowSyntaxError, load_notebook, parse_cell

PACKS = "/root/reference/h2o-docs/src/product/flow/packs"


def _calls(node):
    if isinstance(node, Call):
        yield node
        for a in node.args:
            yield from _calls(a)
    elif isinstance(node, list):
        for a in node:
            yield from _calls(a)
    elif isinstance(node, dict):
        for a in node.values():
            yield from _calls(a)


def scan(nb) -> tuple[list[dict], dict]:
    """-> (parse specs, {column name: response kind}) of a notebook."""
    specs, kinds = [], {}
    for cell in load_notebook(nb)["cells"]:
        if cell.get("type", "cs") != "cs":
            continue
        try:
            stmts = parse_cell(cell.get("input", ""))
        except FlowSyntaxError:
            continue
        for c in _calls(stmts):
            o = c.args[0] if c.args and isinstance(c.args[0], dict) else {}
            if c.name == "parseFiles" and (o.get("paths") or o.get("source_frames")):
                specs.append(o)
            if c.name == "buildModel" and len(c.args) > 1 and isinstance(c.args[1], dict):
                p = c.args[1]
                y = p.get("response_column")
                fam = str(p.get("family") or p.get("distribution") or "").lower()
                algo = str(c.args[0]).lower()
                for w in ("weights_column",):
                    if p.get(w):
                        kinds[p[w]] = "positive"
                if p.get("fold_column"):
                    kinds[p["fold_column"]] = "fold"
                if not y:
                    continue
                if fam in ("binomial", "bernoulli", "quasibinomial", "fractionalbinomial") or \
                        algo in ("naivebayes", "psvm"):
                    kinds[y] = "binary"
                elif fam in ("poisson", "tweedie", "negativebinomial"):
                    kinds.setdefault(y, "count")
                elif fam == "gamma":
                    kinds.setdefault(y, "positive")
                elif fam in ("multinomial", "ordinal"):
                    kinds.setdefault(y, "multiclass")
                elif algo == "coxph":
                    kinds.setdefault(y, "binary")
    return specs, kinds


def _column(rng, n, ctype, kind, signal):
    t = str(ctype).lower()
    if t == "enum":
        k = 2 if kind == "binary" else 3
        if kind in ("binary", "multiclass") and signal is not None:
            codes = np.clip(np.digitize(signal, np.quantile(signal, np.linspace(0, 1, k + 1)[1:-1])), 0, k - 1)
        else:
            codes = rng.integers(0, k, n)
        return [f"L{c}" for c in codes]
    if t == "string":
        return [f"w{int(x)}" for x in rng.integers(0, 50, n)]
    if t == "time":
        return [f"2015-{1 + int(m):02d}-{1 + int(d):02d}" for m, d in zip(rng.integers(0, 12, n),
                                                                           rng.integers(0, 28, n))]
    if t == "uuid":
        return ["%08x-%04x-4%03x-8%03x-%012x" % tuple(int(x) for x in (rng.integers(0, 2**32), rng.integers(0, 2**16),
                                                                         rng.integers(0, 2**12), rng.integers(0, 2**12),
                                                                         rng.integers(0, 2**48))) for _ in range(n)]
    s = signal if signal is not None else rng.normal(size=n)
    if kind == "binary":
        return (s + 0.5 * rng.normal(size=n) > 0).astype(int).tolist()
    if kind == "count":
        return rng.poisson(np.exp(0.3 * s)).tolist()
    if kind == "positive":
        return np.round(np.exp(0.3 * s + 0.2 * rng.normal(size=n)), 4).tolist()
    if kind == "fold":
        return rng.integers(0, 3, n).tolist()
    if kind == "multiclass":
        return np.digitize(s, [-0.5, 0.5]).tolist()
    return np.round(rng.normal(size=n) + 0.5 * s, 4).tolist()


def synth_table(spec, kinds, rows=200, seed=0):
    names = list(spec.get("column_names") or [])
    types = list(spec.get("column_types") or [])
    if not names:
        names = [f"C{i + 1}" for i in range(int(spec.get("number_columns") or len(types) or 4))]
    types += ["Numeric"] * (len(names) - len(types))
    rng = np.random.default_rng(seed)
    signal = rng.normal(size=rows)
    cols = [_column(rng, rows, t, kinds.get(nm), signal) for nm, t in zip(names, types)]
    return names, types, cols


def _encode(spec, names, types, cols, path):
    ptype = str(spec.get("parse_type", "CSV")).upper()
    sep = spec.get("separator", 44)
    sep = chr(sep) if isinstance(sep, int) and 0 < sep < 128 else (sep if isinstance(sep, str) and sep else ",")
    rows = list(zip(*cols))
    buf = io.StringIO()
    if ptype == "ARFF":
        buf.write("@relation synthetic\n")
        for nm, t, col in zip(names, types, cols):
            tl = str(t).lower()
            kind = "{" + ",".join(sorted(set(col))) + "}" if tl == "enum" else \
                ("string" if tl in ("string", "uuid") else 'date "yyyy-MM-dd"' if tl == "time" else "numeric")
            buf.write(f"@attribute '{nm}' {kind}\n")
        buf.write("@data\n")
        for r in rows:
            buf.write(",".join(str(v) for v in r) + "\n")
    elif ptype.startswith("SVML"):
        for r in rows:
            buf.write(str(r[0]) + " " + " ".join(f"{j}:{v}" for j, v in enumerate(r[1:], 1) if v != 0) + "\n")
    else:
        if spec.get("check_header", 1) != -1:
            buf.write(sep.join(f'"{n}"' if sep in n else n for n in names) + "\n")
        for r in rows:
            buf.write(sep.join(str(v) for v in r) + "\n")
    data = buf.getvalue().encode()
    if path.endswith(".gz"):
        data = gzip.compress(data)
    elif path.endswith(".zip"):
        b = io.BytesIO()
        with zipfile.ZipFile(b, "w") as z:
            z.writestr(os.path.basename(path)[:-4] or "data.csv", data)
        data = b.getvalue()
    return data


def _local(root, p):
    p = str(p)
    if "://" in p:                                       # remote datasets: a local stand-in
        p = "remote/" + p.split("://", 1)[1]
    while p.startswith("../"):
        p = p[3:]
    return os.path.join(root, p.lstrip("/"))


def synthesize(nb, root, rows=200, seed=0) -> list[str]:
    """Write the files the notebook parses under root; -> paths written."""
    specs, kinds = scan(nb)
    out = []
    for k, spec in enumerate(specs):
        names, types, cols = synth_table(spec, kinds, rows, seed + k)
        for p in spec.get("paths") or spec.get("source_frames"):
            path = _local(root, p)
            if path.endswith("/") or os.path.isdir(path):
                path = os.path.join(path, "part0.csv")
            if os.path.exists(path):
                continue
            os.makedirs(os.path.dirname(path), exist_ok=True)
            if str(spec.get("parse_type", "CSV")).upper() == "XLS":
                from ..core.excel import write_xls, write_xlsx
                table = [names] + [list(r) for r in zip(*cols)]
                (write_xlsx if path.endswith(".xlsx") else write_xls)(path, table)
                out.append(path)
                continue
            with open(path, "wb") as f:
                f.write(_encode(spec, names, types, cols, path))
            out.append(path)
    return out


def run_pack(notebooks, root, transport, rows=200, automl_secs=20, clear=None, log=None):
    """Run notebooks on synthetic data; -> [{notebook, cells, ok, failed, errors, secs}]."""
    results = []
    for nb in notebooks:
        if clear is not None:
            clear()
        t0 = time.time()
        nb_root = os.path.join(root, os.path.splitext(os.path.basename(nb))[0])   # own data per notebook
        try:
            synthesize(nb, nb_root, rows)
        except NotImplementedError as e:
            rec = {"notebook": os.path.relpath(nb, PACKS) if nb.startswith(PACKS) else nb, "skipped": str(e)}
            results.append(rec)
            if log:
                log(rec)
            continue
        runner = FlowRunner(transport, path_map=lambda p, r=nb_root: _local(r, p), automl_max_runtime_secs=automl_secs)
        res = runner.run_notebook(nb, stop_on_error=False)
        cs = [(i, r) for i, t, r in res if t == "cs"]
        errs = [(i, str(r)) for i, r in cs if isinstance(r, Exception)]
        rec = {"notebook": os.path.relpath(nb, PACKS) if nb.startswith(PACKS) else nb, "cells": len(cs),
               "ok": len(cs) - len(errs), "failed": len(errs), "errors": errs[:5], "secs": round(time.time() - t0, 2)}
        results.append(rec)
        if log:
            log(rec)
    return results


def write_report(res, path, pack, rows):
    """Per-notebook table; failures split into validation errors the
    reference's builders raise as well (``ERRR on field``: the notebook's
    declared column types contradict the requested family) and the rest."""
    ran = [r for r in res if "skipped" not in r]
    full = sum(r["failed"] == 0 for r in ran)
    lines = [f"Flow pack(s) {pack}: {len(ran)} notebooks run on synthetic data ({rows} rows per parsed file, "
             f"layout from each parseFiles cell), in-process server on the CPU",
             f"{full}/{len(ran)} notebooks with every cell ok; {sum(r['ok'] for r in ran)}/"
             f"{sum(r['cells'] for r in ran)} cs cells ok; {len(res) - len(ran)} skipped", ""]
    # classified by the first failing cell (later cells that use the unbuilt model fail with it)
    ref_err = [r for r in ran if r["failed"] and "ERRR on field" in r["errors"][0][1]]
    other = [r for r in ran if r["failed"] and r not in ref_err]
    lines.append(f"notebooks whose first failing cell is a builder validation error the reference raises too "
                 f"(the notebook's declared column types contradict the requested family; {len(ref_err)} notebooks):")
    lines += [f"  {r['notebook']}: cell {r['errors'][0][0]}: {r['errors'][0][1][:150]}" for r in ref_err]
    lines.append(f"other failures ({len(other)} notebooks):")
    lines += [f"  {r['notebook']}: cell {r['errors'][0][0]}: {r['errors'][0][1][:150]}" for r in other]
    lines += ["", "per notebook: ok/cells seconds"]
    lines += [f"  {r['notebook']}: {r['ok']}/{r['cells']} {r['secs']}" if "skipped" not in r else
              f"  {r['notebook']}: skipped ({r['skipped']})" for r in res]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def main(argv=None):
    import argparse
    import tempfile
    ap = argparse.ArgumentParser(prog="python -m h2o3_amd.server.flow_packs")
    ap.add_argument("--pack", default="test-small")
    ap.add_argument("--rows", type=int, default=200)
    ap.add_argument("--limit", type=int, default=0)
    ap.add_argument("--match", default="")
    ap.add_argument("--out", default=None, help="JSON lines of per-notebook results")
    ap.add_argument("--verbose", action="store_true", help="print each notebook before it runs")
    ap.add_argument("--report", default=None, help="text summary (profiles/flow_packs_*.txt)")
    a = ap.parse_args(argv)
    import importlib
    api = importlib.import_module("h2o3_amd.api")
    from .rest import create_app
    from .flow import LocalTransport
    api.init()
    app = create_app(flow_dir=tempfile.mkdtemp(prefix="nps_"))
    t = LocalTransport(app)
    nbs = [n for pack in a.pack.split(",") for n in sorted(glob.glob(os.path.join(PACKS, pack, "*.flow")))]
    nbs = [n for n in nbs if a.match in n][: a.limit or None]
    root = tempfile.mkdtemp(prefix="flowdata_")
    fh = open(a.out, "w") if a.out else None

    def log(rec):
        if "skipped" in rec:
            print(f"{rec['notebook']}: skipped ({rec['skipped']})", flush=True)
            return
        print(f"{rec['notebook']}: {rec['ok']}/{rec['cells']} cells ok, {rec['secs']} s"
              + (f"  first error: cell {rec['errors'][0][0]}: {rec['errors'][0][1][:160]}" if rec["errors"] else ""),
              flush=True)
        if fh:
            fh.write(json.dumps(rec) + "\n")
            fh.flush()
    def clear():
        t("DELETE", "/3/DKV")
    res = []
    for nb in nbs:
        if a.verbose:
            print(f"start {os.path.relpath(nb, PACKS)}", flush=True)
        res += run_pack([nb], root, t, a.rows, clear=clear, log=log)
    if a.report:
        write_report(res, a.report, a.pack, a.rows)
    ran = [r for r in res if "skipped" not in r]
    full = sum(r["failed"] == 0 for r in ran)
    cells = sum(r["cells"] for r in ran)
    ok = sum(r["ok"] for r in ran)
    print(f"SUMMARY {a.pack}: {full}/{len(ran)} notebooks fully ok, {ok}/{cells} cells ok, "
          f"{len(res) - len(ran)} skipped (no synthetic data)")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
