"""Parsing / export.

Reference: water/parser/ParseSetup.java (separator/header/type guessing),
water/parser/CsvParser.java, ParseDataset.java (distributed parse by byte
range), SVMLightParser.java, ARFFParser.java, and h2o-parsers (Parquet,
ORC, Avro).

CSV goes through the native multi-threaded tokenizer in
h2o3_amd/native/csv_parser.cpp (host C++, one pass: split lines across
threads, tokenize, classify each column numeric / categorical / string /
time, emit dense numeric columns + categorical dictionaries), then the
columns are pushed into HBM.  With several ranks each rank parses the byte
range of its row shard.
"""
from __future__ import annotations

import glob
import io
import os
import re

import numpy as np
import torch

from ..parallel import cloud
from .frame import H2OFrame, _local_slice, _vec_from_array
from .vec import T_ENUM, T_INT, T_REAL, T_STR, T_TIME, T_UUID, Vec, make_enum, make_numeric, make_string, make_time

_DEFAULT_NA = {"", "NA", "N/A", "NaN", "nan", "null", "NULL", "?", "-", "na", "n/a"}


def _files(path, pattern=None):
    if isinstance(path, (list, tuple)):
        out = []
        for p in path:
            out += _files(p, pattern)
        return out
    if os.path.isdir(path):
        fs = sorted(os.path.join(path, f) for f in os.listdir(path) if not f.startswith("."))
        if pattern:
            fs = [f for f in fs if re.search(pattern, os.path.basename(f))]
        return fs
    if "://" in str(path):
        from .persist import resolve_all
        return resolve_all(path)
    g = sorted(glob.glob(path))
    from .persist import decompress
    return [decompress(f) for f in g] if g else [path]


def guess_sep(sample: str):
    lines = [l for l in sample.splitlines()[:20] if l.strip()]
    best, score = ",", -1
    for s in [",", "\t", ";", "|", " "]:
        counts = [l.count(s) for l in lines]
        if counts and min(counts) > 0 and len(set(counts)) == 1 and counts[0] > score:
            best, score = s, counts[0]
    if score < 0:
        for s in [",", "\t", ";", "|", " "]:
            if lines and lines[0].count(s) > 0:
                return s
    return best


def parse_setup(path, header=0, sep=None):
    fs = _files(path)
    with open(fs[0], "rb") as f:
        head = f.read(65536).decode("utf-8", "replace")
    s = sep or guess_sep(head)
    return {"separator": s, "source_frames": fs, "header": header}


def import_file(path, destination_frame=None, header=0, sep=None, col_names=None, col_types=None,
                na_strings=None, pattern=None, skipped_columns=None, quotechar=None):
    fs = _files(path, pattern)
    ext = os.path.splitext(fs[0])[1].lower()
    if ext in (".parquet", ".pq"):
        return _import_arrow(fs, "parquet", destination_frame, col_types)
    if ext == ".orc":
        return _import_arrow(fs, "orc", destination_frame, col_types)
    if ext == ".avro":
        from .avro import import_avro
        return import_avro(fs, destination_frame, col_types)
    if ext in (".svm", ".svmlight", ".libsvm"):
        return _import_svmlight(fs, destination_frame)
    if ext == ".arff":
        return _import_arff(fs[0], destination_frame)
    if ext in (".xls", ".xlsx"):
        # first worksheet decoded in-house (core/excel.py, XlsParser.java), then the CSV path's guessing
        from .excel import read_excel_rows, rows_to_csv
        from .persist import _tmpfile
        tmp = _tmpfile(".csv")
        with open(tmp, "w", encoding="utf-8") as f:
            f.write(rows_to_csv(read_excel_rows(fs[0])))
        try:
            return _import_csv([tmp], destination_frame, header, ",", col_names, col_types, na_strings,
                               skipped_columns, '"')
        finally:
            os.remove(tmp)
    return _import_csv(fs, destination_frame, header, sep, col_names, col_types, na_strings, skipped_columns,
                       quotechar)


_UUID_RE = __import__("re").compile(r"^[0-9a-fA-F]{8}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{12}$")


def _guess_string(codes, sample=10000):
    """String-vs-categorical guess (PreviewParseWriter.guessType: a column of
    strings with almost no duplicates -- distinct >= 95% of the non-NA
    values in the preview sample, more than one distinct value -- is T_STR)."""
    c = np.asarray(codes[:sample])
    c = c[c >= 0]
    if c.size < 2:
        return False
    nd = np.unique(c).size
    return nd > 1 and nd >= 0.95 * c.size


def _import_csv(fs, dest, header, sep, col_names, col_types, na_strings, skipped, quotechar):
    from . import native_csv
    res = native_csv.parse_files(fs, sep=sep, header=header, na_strings=na_strings, quotechar=quotechar or '"')
    names, cols = res["names"], res["columns"]
    if col_names:
        names = list(col_names)
    ctypes = {}
    if isinstance(col_types, dict):
        ctypes = col_types
    elif isinstance(col_types, (list, tuple)):
        ctypes = dict(zip(names, col_types))
    n = res["nrows"]
    s, e = _local_slice(n) if cloud.is_distributed() else (0, n)
    vecs, out_names = [], []
    skipped = set(skipped or [])
    for j, (name, col) in enumerate(zip(names, cols)):
        if j in skipped:
            continue
        want = ctypes.get(name)
        kind = col["kind"]
        if want is not None:
            want = {"numeric": "real", "factor": "enum", "categorical": "enum"}.get(want, want)
        if kind == "num" and want in (None, "real", "int", "numeric"):
            v = make_numeric(col["values"][s:e])
            if want == "int":
                v.type = T_INT
        elif kind == "num" and want == "enum":
            v = _vec_from_array(col["values"][s:e].astype(object), "enum",
                                domain=_vec_from_array(col["values"].astype(object), "enum").domain)
        elif kind == "num" and want == "string":
            v = make_string([None if np.isnan(x) else (str(int(x)) if float(x).is_integer() else str(x))
                             for x in col["values"][s:e]])
        elif kind == "cat":
            dom, codes = col["domain"], col["codes"]
            if want is None and dom and all(_UUID_RE.match(d) for d in dom[:1000]):
                want = "uuid"   # ParseSetup guesses T_UUID for 8-4-4-4-12 hex tokens
            if want is None and _guess_string(codes):
                want = "string"
            if want in ("string", "uuid"):
                arr = np.array(dom + [None], dtype=object)[np.where(codes < 0, len(dom), codes)]
                v = make_string(arr[s:e])
                if want == "uuid":
                    v.type = T_UUID
            elif want in ("real", "int", "numeric"):
                vals = []
                for d in dom:
                    try:
                        vals.append(float(d))
                    except ValueError:
                        vals.append(np.nan)
                lut = np.array(vals + [np.nan])
                v = make_numeric(lut[np.where(codes < 0, len(dom), codes)][s:e])
            elif want == "time":
                arr = np.array(dom + [None], dtype=object)[np.where(codes < 0, len(dom), codes)]
                v = _vec_from_array(arr[s:e], "time")
            else:
                # reference sorts the domain; remap codes to sorted order
                from .vec import _sort_domain
                sdom = _sort_domain(dom)
                pos = {d: i for i, d in enumerate(sdom)}
                remap = np.array([pos[d] for d in dom] + [-1], dtype=np.int32)
                v = make_enum(remap[np.where(codes < 0, len(dom), codes)][s:e], sdom)
        elif kind == "time":
            v = make_time(col["values"][s:e])
        else:
            v = make_string(col["values"][s:e])
        vecs.append(v)
        out_names.append(name)
    return H2OFrame.from_vecs(vecs, out_names, frame_id=dest or os.path.basename(fs[0]).replace(".", "_"))


def _import_arrow(fs, fmt, dest, col_types):
    import pandas as pd
    if fmt == "parquet":
        import pyarrow.parquet as pq
        df = pd.concat([pq.read_table(f).to_pandas() for f in fs], ignore_index=True)
    else:
        import pyarrow.orc as orc
        df = pd.concat([orc.read_table(f).to_pandas() for f in fs], ignore_index=True)
    return H2OFrame(df, destination_frame=dest, column_types=col_types)


def _import_svmlight(fs, dest):
    rows, ys, maxf = [], [], 0
    for fn in fs:
        with open(fn) as f:
            for line in f:
                line = line.split("#")[0].strip()
                if not line:
                    continue
                parts = line.split()
                ys.append(float(parts[0]))
                feats = {}
                for kv in parts[1:]:
                    k, v = kv.split(":")
                    k = int(k)
                    feats[k] = float(v)
                    maxf = max(maxf, k)
                rows.append(feats)
    X = np.zeros((len(rows), maxf), dtype=np.float64)
    for i, r in enumerate(rows):
        for k, v in r.items():
            X[i, k - 1] = v
    data = {"C1": np.array(ys)}
    for j in range(maxf):
        data[f"C{j + 2}"] = X[:, j]
    import pandas as pd
    return H2OFrame(pd.DataFrame(data), destination_frame=dest)


def _import_arff(fn, dest):
    import pandas as pd
    names, types, data_lines = [], [], []
    in_data = False
    with open(fn) as f:
        for line in f:
            s = line.strip()
            if not s or s.startswith("%"):
                continue
            if in_data:
                data_lines.append(s)
                continue
            low = s.lower()
            if low.startswith("@attribute"):
                m = re.match(r"@attribute\s+('([^']*)'|\"([^\"]*)\"|(\S+))\s+(.*)", s, re.I)
                nm = m.group(2) or m.group(3) or m.group(4)
                t = m.group(5).strip()
                names.append(nm)
                if t.startswith("{"):
                    types.append("enum")
                elif t.lower() in ("numeric", "real", "integer"):
                    types.append("real")
                elif t.lower().startswith("date"):
                    types.append("time")
                else:
                    types.append("string")
            elif low.startswith("@data"):
                in_data = True
    df = pd.read_csv(io.StringIO("\n".join(data_lines)), header=None, names=names, na_values=["?"],
                     quotechar="'", skipinitialspace=True)
    return H2OFrame(df, destination_frame=dest, column_types=dict(zip(names, types)))


def export_file(frame, path, force=False, sep=",", header=True, format="csv"):
    from .persist import is_remote, upload, _tmpfile
    remote = is_remote(path)
    from ..parallel import collectives as coll
    if not remote and coll.broadcast_object(os.path.exists(path)) and not force:    # rank 0's view
        raise FileExistsError(path)
    df = frame.as_data_frame()
    if cloud.rank() != 0:
        return path
    out = _tmpfile(os.path.splitext(path)[1]) if remote else path
    if format == "parquet" or path.endswith(".parquet"):
        df.to_parquet(out)
    else:
        df.to_csv(out, sep=sep, header=header, index=False, na_rep="")
    if remote:
        upload(out, path)      # s3:// gs:// hdfs:// (core/persist.py)
    return path
