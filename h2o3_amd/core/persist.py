"""Persistence back-ends (where files come from).

Reference: water/persist/{PersistManager, PersistNFS, PersistHTTP,
PersistS3, PersistHdfs, PersistGcs}.java.  Supported here: local paths and
file:// URIs, http(s):// (downloaded to a temporary file), and transparent
decompression of .gz / .bz2 / .zip / .xz inputs before parsing (the
reference's ZipUtil decompression in ParseDataset).  Object stores (s3://,
gs://, hdfs://) raise a clear error: this build has no cloud SDKs and no
egress.
"""
from __future__ import annotations

import bz2
import gzip
import lzma
import os
import shutil
import tempfile
import urllib.parse
import urllib.request
import zipfile

_TMP = []


def _tmpfile(suffix=""):
    fd, p = tempfile.mkstemp(prefix="h2o3_amd_", suffix=suffix)
    os.close(fd)
    _TMP.append(p)
    return p


def resolve(uri: str) -> str:
    """Local path for a URI (downloading / decompressing as needed)."""
    u = urllib.parse.urlparse(uri)
    if u.scheme in ("http", "https"):
        out = _tmpfile(os.path.splitext(u.path)[1])
        with urllib.request.urlopen(uri) as r, open(out, "wb") as f:
            shutil.copyfileobj(r, f)
        return decompress(out)
    if u.scheme in ("s3", "s3a", "s3n", "gs", "hdfs", "maprfs"):
        raise NotImplementedError(f"{u.scheme}:// persistence is not available in this build (no object-store SDK)")
    if u.scheme == "file":
        uri = u.path
    return decompress(uri)


def decompress(path: str) -> str:
    low = path.lower()
    opener = {".gz": gzip.open, ".bz2": bz2.open, ".xz": lzma.open}
    for ext, op in opener.items():
        if low.endswith(ext):
            out = _tmpfile(os.path.splitext(path[: -len(ext)])[1])
            with op(path, "rb") as src, open(out, "wb") as dst:
                shutil.copyfileobj(src, dst)
            return out
    if low.endswith(".zip"):
        with zipfile.ZipFile(path) as z:
            names = [n for n in z.namelist() if not n.endswith("/")]
            if len(names) != 1:
                raise ValueError("zip archives must contain exactly one file to parse")
            out = _tmpfile(os.path.splitext(names[0])[1])
            with z.open(names[0]) as src, open(out, "wb") as dst:
                shutil.copyfileobj(src, dst)
            return out
    return path


def cleanup():
    while _TMP:
        p = _TMP.pop()
        try:
            os.remove(p)
        except OSError:
            pass
