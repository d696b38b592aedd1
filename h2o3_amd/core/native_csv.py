"""ctypes binding of the native CSV parser (h2o3_amd/native/csv_parser.cpp)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ..ops import _native

_DEFAULT_NA = ["NA", "N/A", "NaN", "nan", "null", "NULL", "?", "na", "n/a", "None"]


def _lib():
    lib = _native.get_lib("csv_parser", required=True)
    if not getattr(lib, "_typed", False):
        lib.h2o_csv_parse.restype = ctypes.c_void_p
        lib.h2o_csv_parse.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_char, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_char, ctypes.c_int,
                                      ctypes.c_int]
        for fn in ("h2o_csv_error", "h2o_csv_name", "h2o_csv_domain"):
            getattr(lib, fn).restype = ctypes.c_char_p
        lib.h2o_csv_error.argtypes = [ctypes.c_void_p]
        lib.h2o_csv_name.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.h2o_csv_domain.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        lib.h2o_csv_ncols.argtypes = [ctypes.c_void_p]
        lib.h2o_csv_nrows.argtypes = [ctypes.c_void_p]
        lib.h2o_csv_nrows.restype = ctypes.c_longlong
        lib.h2o_csv_kind.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.h2o_csv_num.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        lib.h2o_csv_codes.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        lib.h2o_csv_domain_size.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.h2o_csv_free.argtypes = [ctypes.c_void_p]
        lib._typed = True
    return lib


def parse_files(paths, sep=None, header=0, na_strings=None, quotechar='"', nthreads=0, sample_rows=1000):
    from .parse import guess_sep
    paths = [os.path.abspath(p) for p in paths]
    if sep is None:
        with open(paths[0], "rb") as f:
            sep = guess_sep(f.read(65536).decode("utf-8", "replace"))
    lib = _lib()
    arr = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])
    nas = list(_DEFAULT_NA)
    if na_strings:
        if isinstance(na_strings, dict):
            for v in na_strings.values():
                nas += list(v if isinstance(v, (list, tuple)) else [v])
        else:
            for v in na_strings:
                if isinstance(v, (list, tuple)):
                    nas += list(v)
                elif v is not None:
                    nas.append(v)
    na_arr = (ctypes.c_char_p * len(nas))(*[str(s).encode() for s in nas])
    h = lib.h2o_csv_parse(arr, len(paths), sep.encode()[:1], int(header), na_arr, len(nas),
                          quotechar.encode()[:1], int(nthreads), int(sample_rows))
    try:
        err = lib.h2o_csv_error(h).decode()
        if err:
            raise IOError(err)
        nc = lib.h2o_csv_ncols(h)
        n = lib.h2o_csv_nrows(h)
        names, cols = [], []
        for j in range(nc):
            names.append(lib.h2o_csv_name(h, j).decode("utf-8", "replace"))
            k = lib.h2o_csv_kind(h, j)
            if k == 1:
                codes = np.empty(n, dtype=np.int32)
                lib.h2o_csv_codes(h, j, codes.ctypes.data)
                dom = [lib.h2o_csv_domain(h, j, i).decode("utf-8", "replace") for i in range(lib.h2o_csv_domain_size(h, j))]
                cols.append({"kind": "cat", "codes": codes, "domain": dom})
            else:
                v = np.empty(n, dtype=np.float64)
                lib.h2o_csv_num(h, j, v.ctypes.data)
                cols.append({"kind": "num" if k == 0 else "time", "values": v})
        return {"names": names, "columns": cols, "nrows": int(n)}
    finally:
        lib.h2o_csv_free(h)
