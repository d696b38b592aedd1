"""Excel import without xlrd/openpyxl (core/excel.py; reference
water/parser/XlsParser.java): BIFF8-in-OLE2 .xls and OOXML .xlsx first
sheets, SST strings continued across CONTINUE records, RK / MULRK numbers,
and the rows going through the CSV type guessing."""
import struct

import numpy as np

from h2o3_amd.core import parse as P
from h2o3_amd.core.excel import _rk, _sst, read_xls, read_xlsx, write_xls, write_xlsx


def _rows(n=2500, seed=0):
    rng = np.random.default_rng(seed)
    head = [["x", "k", "name", "tag"]]
    # many unique strings: the SST spans several CONTINUE records
    return head + [[float(rng.normal()), int(rng.integers(0, 5)), f"name_{i}_{'u' * (i % 13)}", "ü" if i % 2 else None]
                   for i in range(n)]


def test_xls_and_xlsx_round_trip(tmp_path):
    rows = _rows()
    write_xls(tmp_path / "a.xls", rows)
    write_xlsx(tmp_path / "a.xlsx", rows)
    for got in (read_xls(str(tmp_path / "a.xls")), read_xlsx(str(tmp_path / "a.xlsx"))):
        assert len(got) == len(rows)
        assert got[0] == rows[0]
        assert [r[2] for r in got[1:]] == [r[2] for r in rows[1:]]
        np.testing.assert_allclose([r[0] for r in got[1:]], [r[0] for r in rows[1:]])


def test_import_file_types(tmp_path):
    rows = _rows(500, 1)
    for ext, writer in ((".xls", write_xls), (".xlsx", write_xlsx)):
        path = str(tmp_path / f"b{ext}")
        writer(path, rows)
        fr = P.import_file(path)
        assert fr.nrow == 500 and fr.names == ["x", "k", "name", "tag"]
        assert fr.types["x"] == "real" and fr.types["k"] == "int"
        df = fr.as_data_frame()
        np.testing.assert_allclose(df["x"].values, [r[0] for r in rows[1:]], rtol=1e-6)
        assert df["tag"].isna().sum() == 250


def test_sst_string_split_across_continue():
    # "hello" + wide "wörld" split mid-string: the CONTINUE part restarts with an option byte
    first = struct.pack("<II", 2, 2) + struct.pack("<HB", 5, 0) + b"hello" + struct.pack("<HB", 5, 1) + \
        "wö".encode("utf-16-le")
    cont = bytes([0]) + b"rld"
    assert _sst([first, cont]) == ["hello", "wörld"]


def test_rk_numbers():
    assert _rk((123 << 2) | 2) == 123.0
    assert _rk((12345 << 2) | 3) == 123.45
    bits = struct.unpack("<Q", struct.pack("<d", 1.5))[0] >> 32
    assert _rk(bits << 0 & 0xFFFFFFFC) == 1.5
