"""Avro object-container-file reader (no avro/fastavro dependency).

Reference: h2o-parsers/h2o-avro-parser (AvroParser.java / AvroParserProvider):
a file of records whose top-level fields are primitives (or unions of a
primitive with null) becomes one column per field: int/long/float/double ->
numeric, boolean -> 0/1, enum -> categorical (domain = the schema symbols),
string/bytes -> categorical or string (the usual guess), null -> NA.  Nested
records, arrays and maps are not flattened, as in the reference (such fields
are skipped).

Format (Avro 1.x spec): magic "Obj\\x01", metadata map (avro.schema JSON,
avro.codec null|deflate), 16-byte sync marker, then blocks of (count, byte
size, data, sync).  Values use zig-zag varints for int/long, little-endian
IEEE for float/double.
"""
from __future__ import annotations

import io
import json
import struct
import zlib

import numpy as np

_MAGIC = b"Obj\x01"


class _Buf:
    __slots__ = ("b", "i")

    def __init__(self, b):
        self.b, self.i = b, 0

    def long(self):
        b, i = self.b, self.i
        shift = acc = 0
        while True:
            c = b[i]
            i += 1
            acc |= (c & 0x7F) << shift
            if not c & 0x80:
                break
            shift += 7
        self.i = i
        return (acc >> 1) ^ -(acc & 1)

    def read(self, n):
        s = self.b[self.i:self.i + n]
        self.i += n
        return s

    def bytes_(self):
        return self.read(self.long())

    def float_(self):
        return struct.unpack("<f", self.read(4))[0]

    def double(self):
        return struct.unpack("<d", self.read(8))[0]


def _reader(schema, named):
    """Compile a schema node into a decode function f(buf) -> python value."""
    if isinstance(schema, str):
        if schema in named:
            return _reader(named[schema], named)
        t = schema
        schema = {"type": t}
    if isinstance(schema, list):
        branches = [_reader(s, named) for s in schema]
        return lambda buf: branches[buf.long()](buf)
    t = schema["type"]
    if isinstance(t, (dict, list)):
        return _reader(t, named)
    if t == "null":
        return lambda buf: None
    if t == "boolean":
        return lambda buf: buf.read(1)[0] != 0
    if t in ("int", "long"):
        return lambda buf: buf.long()
    if t == "float":
        return lambda buf: buf.float_()
    if t == "double":
        return lambda buf: buf.double()
    if t == "bytes":
        return lambda buf: buf.bytes_()
    if t == "string":
        return lambda buf: buf.bytes_().decode("utf-8")
    if t == "fixed":
        named[schema["name"]] = schema
        size = schema["size"]
        return lambda buf: buf.read(size)
    if t == "enum":
        named[schema["name"]] = schema
        syms = schema["symbols"]
        return lambda buf: syms[buf.long()]
    if t == "array":
        item = _reader(schema["items"], named)

        def arr(buf):
            out = []
            while True:
                n = buf.long()
                if n == 0:
                    return out
                if n < 0:
                    n = -n
                    buf.long()
                out.extend(item(buf) for _ in range(n))
        return arr
    if t == "map":
        val = _reader(schema["values"], named)

        def mp(buf):
            out = {}
            while True:
                n = buf.long()
                if n == 0:
                    return out
                if n < 0:
                    n = -n
                    buf.long()
                for _ in range(n):
                    k = buf.bytes_().decode("utf-8")
                    out[k] = val(buf)
        return mp
    if t == "record":
        named[schema["name"]] = schema
        fields = [(f["name"], _reader(f["type"], named)) for f in schema["fields"]]
        return lambda buf: {n: r(buf) for n, r in fields}
    raise ValueError(f"unsupported avro type {t}")


def read_avro(path):
    """Returns (schema, list of record dicts)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != _MAGIC:
        raise ValueError(f"{path} is not an Avro object container file")
    buf = _Buf(data)
    buf.i = 4
    meta = {}
    while True:
        n = buf.long()
        if n == 0:
            break
        if n < 0:
            n = -n
            buf.long()
        for _ in range(n):
            k = buf.bytes_().decode("utf-8")
            meta[k] = buf.bytes_()
    sync = buf.read(16)
    schema = json.loads(meta["avro.schema"].decode("utf-8"))
    codec = meta.get("avro.codec", b"null").decode("utf-8")
    rec = _reader(schema, {})
    rows = []
    while buf.i < len(data):
        count = buf.long()
        size = buf.long()
        block = buf.read(size)
        if codec == "deflate":
            block = zlib.decompress(block, -15)
        elif codec != "null":
            raise ValueError(f"unsupported avro codec {codec}")
        bb = _Buf(block)
        for _ in range(count):
            rows.append(rec(bb))
        if buf.read(16) != sync:
            raise ValueError("avro sync marker mismatch")
    return schema, rows


def _field_kind(t):
    """Column kind of a top-level field type, or None when it is not flat."""
    if isinstance(t, list):
        non_null = [x for x in t if x != "null" and not (isinstance(x, dict) and x.get("type") == "null")]
        return _field_kind(non_null[0]) if len(non_null) == 1 else None
    if isinstance(t, dict):
        tt = t["type"]
        if tt == "enum":
            return ("enum", t["symbols"])
        if tt in ("record", "array", "map", "fixed"):
            return None
        return _field_kind(tt)
    if t in ("int", "long", "float", "double", "boolean"):
        return ("num", None)
    if t in ("string", "bytes"):
        return ("str", None)
    return None


def import_avro(paths, destination_frame=None, col_types=None):
    import pandas as pd
    from .frame import H2OFrame
    cols, kinds = None, None
    data = {}
    for p in paths:
        schema, rows = read_avro(p)
        if schema.get("type") != "record":
            raise ValueError("top-level Avro schema must be a record")
        if cols is None:
            kinds = {f["name"]: _field_kind(f["type"]) for f in schema["fields"]}
            cols = [f["name"] for f in schema["fields"] if kinds[f["name"]] is not None]
            data = {c: [] for c in cols}
        for r in rows:
            for c in cols:
                v = r.get(c)
                if isinstance(v, bytes):
                    v = v.decode("utf-8", "replace")
                data[c].append(v)
    df = pd.DataFrame({c: (pd.Categorical(data[c], categories=kinds[c][1]) if kinds[c][0] == "enum"
                           else (np.array([np.nan if v is None else float(v) for v in data[c]])
                                 if kinds[c][0] == "num" else np.array(data[c], dtype=object)))
                       for c in cols})
    return H2OFrame(df, destination_frame=destination_frame, column_types=col_types)


def write_avro(path, schema, records, codec="null", block_size=1000):
    """Minimal writer (tests / export of flat records)."""
    out = io.BytesIO()

    def long(v):
        v = (v << 1) ^ (v >> 63)
        while True:
            b = v & 0x7F
            v >>= 7
            if v:
                out.write(bytes([b | 0x80]))
            else:
                out.write(bytes([b]))
                return

    def enc_into(o, s, v, named):
        if isinstance(s, str) and s in named:
            s = named[s]
        if isinstance(s, list):
            for i, b in enumerate(s):
                bt = b if isinstance(b, str) else b.get("type")
                if (v is None) == (bt == "null"):
                    o.append(("long", i))
                    enc_into(o, b, v, named)
                    return
            raise ValueError("no union branch")
        t = s if isinstance(s, str) else s["type"]
        if t == "null":
            return
        if t == "boolean":
            o.append(("raw", b"\x01" if v else b"\x00"))
        elif t in ("int", "long"):
            o.append(("long", int(v)))
        elif t == "float":
            o.append(("raw", struct.pack("<f", v)))
        elif t == "double":
            o.append(("raw", struct.pack("<d", v)))
        elif t in ("string", "bytes"):
            b = v.encode("utf-8") if isinstance(v, str) else v
            o.append(("long", len(b)))
            o.append(("raw", b))
        elif t == "enum":
            named[s["name"]] = s
            o.append(("long", s["symbols"].index(v)))
        elif t == "record":
            named[s["name"]] = s
            for f in s["fields"]:
                enc_into(o, f["type"], v.get(f["name"]), named)
        elif t == "array":
            if v:
                o.append(("long", len(v)))
                for it in v:
                    enc_into(o, s["items"], it, named)
            o.append(("long", 0))
        else:
            raise ValueError(t)

    out.write(_MAGIC)
    meta = {"avro.schema": json.dumps(schema).encode(), "avro.codec": codec.encode()}
    long(len(meta))
    for k, v in meta.items():
        long(len(k))
        out.write(k.encode())
        long(len(v))
        out.write(v)
    long(0)
    sync = bytes(range(16))
    out.write(sync)
    for s0 in range(0, len(records), block_size):
        chunk = records[s0:s0 + block_size]
        ops = []
        for r in chunk:
            enc_into(ops, schema, r, {})
        body = io.BytesIO()

        def w_long(v, o=body):
            v = (v << 1) ^ (v >> 63)
            while True:
                b = v & 0x7F
                v >>= 7
                if v:
                    o.write(bytes([b | 0x80]))
                else:
                    o.write(bytes([b]))
                    return
        for kind, v in ops:
            if kind == "long":
                w_long(v)
            else:
                body.write(v)
        blob = body.getvalue()
        if codec == "deflate":
            c = zlib.compressobj(9, zlib.DEFLATED, -15)
            blob = c.compress(blob) + c.flush()
        long(len(chunk))
        long(len(blob))
        out.write(blob)
        out.write(sync)
    with open(path, "wb") as f:
        f.write(out.getvalue())
    return path
