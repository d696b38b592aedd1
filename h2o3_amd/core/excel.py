"""Excel workbooks without third-party readers: .xls (BIFF8 inside an OLE2
compound file) and .xlsx (Office Open XML zip).

Reference: water/parser/XlsParser.java -- the reference reads the first
worksheet of a BIFF8 workbook out of the OLE2 container (big / small block
depots, the "Workbook" directory entry, SST shared strings with CONTINUE
records, LABELSST / NUMBER / RK / MULRK / LABEL / FORMULA cells) and feeds
the cells to the CSV-style parse pipeline.  Neither xlrd nor openpyxl is in
this image, so both formats are decoded here (stdlib only) into rows, and the
rows go through the same CSV parse + type guessing as text files
(parse.py).  Small writers for both formats exist for tests and synthetic
data (flow_packs.py).
"""
from __future__ import annotations

import io
import math
import re
import struct
import zipfile
import xml.etree.ElementTree as ET

_CFB_MAGIC = b"\xd0\xcf\x11\xe0\xa1\xb1\x1a\xe1"
_END, _FREE, _FATSECT, _NOSTREAM = 0xFFFFFFFE, 0xFFFFFFFF, 0xFFFFFFFD, 0xFFFFFFFF


# ---------------------------------------------------------------- OLE2 / CFB
def _cfb_stream(data: bytes, want=("Workbook", "Book")) -> bytes:
    """The named stream of a compound file (MS-CFB)."""
    if data[:8] != _CFB_MAGIC:
        raise ValueError("not an OLE2 compound file (.xls)")
    ssz = 1 << struct.unpack_from("<H", data, 0x1E)[0]
    mssz = 1 << struct.unpack_from("<H", data, 0x20)[0]
    n_fat, dir_start = struct.unpack_from("<II", data, 0x2C)[0], struct.unpack_from("<I", data, 0x30)[0]
    cutoff, mfat_start, n_mfat, difat_start, n_difat = struct.unpack_from("<IIIII", data, 0x38)

    def sector(i):
        off = (i + 1) * ssz
        return data[off:off + ssz]
    difat = list(struct.unpack_from("<109I", data, 0x4C))
    d, k = difat_start, 0
    while d not in (_END, _FREE) and k < n_difat:
        ent = struct.unpack(f"<{ssz // 4}I", sector(d))
        difat += ent[:-1]
        d, k = ent[-1], k + 1
    fat = []
    for s in difat[:n_fat]:
        fat += struct.unpack(f"<{ssz // 4}I", sector(s))

    def chain(start, table):
        out, s, seen = [], start, 0
        while s not in (_END, _FREE) and s < len(table) and seen <= len(table):
            out.append(s)
            s, seen = table[s], seen + 1
        return out
    dirdata = b"".join(sector(s) for s in chain(dir_start, fat))
    entries = []
    for off in range(0, len(dirdata) - 127, 128):
        nlen = struct.unpack_from("<H", dirdata, off + 0x40)[0]
        name = dirdata[off:off + max(nlen - 2, 0)].decode("utf-16-le", "replace")
        typ = dirdata[off + 0x42]
        start, size = struct.unpack_from("<IQ", dirdata, off + 0x74)
        if ssz == 512:
            size &= 0xFFFFFFFF
        entries.append((name, typ, start, size))
    root = entries[0]
    for name, typ, start, size in entries:
        if typ == 2 and name in want:
            if size < cutoff:
                mfat = []
                for s in chain(mfat_start, fat):
                    mfat += struct.unpack(f"<{ssz // 4}I", sector(s))
                ministream = b"".join(sector(s) for s in chain(root[2], fat))
                return b"".join(ministream[m * mssz:(m + 1) * mssz] for m in chain(start, mfat))[:size]
            return b"".join(sector(s) for s in chain(start, fat))[:size]
    raise ValueError("no Workbook stream in the compound file")


# ---------------------------------------------------------------- BIFF8
def _rk(v: int) -> float:
    if v & 2:
        x = float(v >> 2 if v < 0x80000000 else (v >> 2) - (1 << 30))
    else:
        x = struct.unpack("<d", struct.pack("<Q", (v & 0xFFFFFFFC) << 32))[0]
    return x / 100.0 if v & 1 else x


def _records(wb: bytes):
    off, n = 0, len(wb)
    while off + 4 <= n:
        typ, ln = struct.unpack_from("<HH", wb, off)
        yield typ, wb[off + 4:off + 4 + ln]
        off += 4 + ln


def _sst(parts: list[bytes]) -> list[str]:
    """Shared strings; parts = the SST record body and its CONTINUE bodies
    (a string's characters may continue in the next part behind a fresh
    option byte)."""
    out, pi, buf = [], 0, parts[0]
    pos = 8
    total = struct.unpack_from("<I", buf, 4)[0]

    def need(k):
        nonlocal pi, buf, pos
        if pos + k > len(buf) and pi + 1 < len(parts):
            pi, buf, pos = pi + 1, parts[pi + 1], 0
    while len(out) < total:
        need(3)
        if pos + 3 > len(buf):
            break
        cch, flags = struct.unpack_from("<HB", buf, pos)
        pos += 3
        runs = ext = 0
        if flags & 8:
            runs = struct.unpack_from("<H", buf, pos)[0]
            pos += 2
        if flags & 4:
            ext = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        chars, wide = [], flags & 1
        left = cch
        while left > 0:
            avail = (len(buf) - pos) // (2 if wide else 1)
            if avail <= 0:                       # continue: a new option byte
                pi, buf, pos = pi + 1, parts[pi + 1], 0
                wide = buf[0] & 1
                pos = 1
                continue
            k = min(left, avail)
            raw = buf[pos:pos + k * (2 if wide else 1)]
            chars.append(raw.decode("utf-16-le") if wide else raw.decode("latin-1"))
            pos += len(raw)
            left -= k
        out.append("".join(chars))
        skip = 4 * runs + ext
        while skip > 0:
            k = min(skip, len(buf) - pos)
            pos += k
            skip -= k
            if skip > 0:
                pi, buf, pos = pi + 1, parts[pi + 1], 0
    return out


def _xlstr(b: bytes, pos: int):
    cch, flags = struct.unpack_from("<HB", b, pos)
    pos += 3
    if flags & 1:
        return b[pos:pos + 2 * cch].decode("utf-16-le")
    return b[pos:pos + cch].decode("latin-1")


def read_xls(path_or_bytes) -> list[list]:
    """Cells of the first worksheet as rows (None for empty cells)."""
    data = path_or_bytes if isinstance(path_or_bytes, bytes) else open(path_or_bytes, "rb").read()
    wb = _cfb_stream(data)
    sst: list[str] = []
    cells: dict = {}
    sst_parts, in_sst, sheet, done = [], False, False, False
    pending = None                                         # FORMULA cell awaiting its STRING
    for typ, b in _records(wb):
        if typ == 0x003C and in_sst:                     # CONTINUE of the SST
            sst_parts.append(b)
            continue
        if in_sst:
            sst, in_sst = _sst(sst_parts), False
        if typ == 0x0809:                                # BOF
            if struct.unpack_from("<H", b, 2)[0] == 0x0010:
                if done:
                    break
                sheet = True
            continue
        if typ == 0x000A:                                # EOF
            if sheet:
                done, sheet = True, False
                break
            continue
        if typ == 0x00FC:
            sst_parts, in_sst = [b], True
            continue
        if not sheet:
            continue
        if typ == 0x00FD:                                # LABELSST
            r, c, _, i = struct.unpack_from("<HHHI", b)
            cells[(r, c)] = sst[i] if i < len(sst) else None
        elif typ == 0x0203:                              # NUMBER
            r, c, _, v = struct.unpack_from("<HHHd", b)
            cells[(r, c)] = v
        elif typ == 0x027E:                              # RK
            r, c, _, v = struct.unpack_from("<HHHI", b)
            cells[(r, c)] = _rk(v)
        elif typ == 0x00BD:                              # MULRK
            r, c0 = struct.unpack_from("<HH", b)
            n = (len(b) - 6) // 6
            for k in range(n):
                cells[(r, c0 + k)] = _rk(struct.unpack_from("<I", b, 4 + 6 * k + 2)[0])
        elif typ == 0x0204:                              # LABEL
            r, c, _ = struct.unpack_from("<HHH", b)
            cells[(r, c)] = _xlstr(b, 6)
        elif typ == 0x0205:                              # BOOLERR
            r, c, _, v, err = struct.unpack_from("<HHHBB", b)
            cells[(r, c)] = None if err else float(v)
        elif typ == 0x0006:                              # FORMULA: cached result
            r, c = struct.unpack_from("<HH", b)
            res = b[6:14]
            if res[6:8] == b"\xff\xff":
                kind = res[0]
                cells[(r, c)] = float(res[2]) if kind == 1 else None
                pending = (r, c) if kind == 0 else None
            else:
                cells[(r, c)] = struct.unpack("<d", res)[0]
        elif typ == 0x0207 and pending is not None:      # STRING after a string FORMULA
            cells[pending] = _xlstr(b, 0)
            pending = None
    return _grid(cells)


def _grid(cells: dict) -> list[list]:
    if not cells:
        return []
    nr = max(r for r, _ in cells) + 1
    nc = max(c for _, c in cells) + 1
    rows = [[None] * nc for _ in range(nr)]
    for (r, c), v in cells.items():
        rows[r][c] = v
    return [row for row in rows if any(v is not None and v != "" for v in row)]


# ---------------------------------------------------------------- XLSX
_NS = "{http://schemas.openxmlformats.org/spreadsheetml/2006/main}"
_REL = "{http://schemas.openxmlformats.org/officeDocument/2006/relationships}"


def _col_index(ref: str) -> int:
    k = 0
    for ch in re.match(r"[A-Z]+", ref).group(0):
        k = k * 26 + ord(ch) - 64
    return k - 1


def read_xlsx(path_or_bytes) -> list[list]:
    src = io.BytesIO(path_or_bytes) if isinstance(path_or_bytes, bytes) else path_or_bytes
    with zipfile.ZipFile(src) as z:
        names = set(z.namelist())
        shared = []
        if "xl/sharedStrings.xml" in names:
            for si in ET.fromstring(z.read("xl/sharedStrings.xml")).iter(_NS + "si"):
                shared.append("".join(t.text or "" for t in si.iter(_NS + "t")))
        sheet = None
        try:                                             # the first sheet of the workbook
            wbx = ET.fromstring(z.read("xl/workbook.xml"))
            rid = next(wbx.iter(_NS + "sheet")).get(_REL + "id")
            rels = ET.fromstring(z.read("xl/_rels/workbook.xml.rels"))
            for rel in rels:
                if rel.get("Id") == rid:
                    t = rel.get("Target").lstrip("/")
                    sheet = t if t.startswith("xl/") else "xl/" + t
        except (KeyError, StopIteration):
            pass
        if sheet not in names:
            sheet = sorted(n for n in names if n.startswith("xl/worksheets/sheet"))[0]
        cells = {}
        for r_i, row in enumerate(ET.fromstring(z.read(sheet)).iter(_NS + "row")):
            r = int(row.get("r", r_i + 1)) - 1
            for k, c in enumerate(row.iter(_NS + "c")):
                col = _col_index(c.get("r")) if c.get("r") else k
                t = c.get("t", "n")
                v = c.find(_NS + "v")
                if t == "inlineStr":
                    val = "".join(x.text or "" for x in c.iter(_NS + "t"))
                elif v is None or v.text is None:
                    continue
                elif t == "s":
                    val = shared[int(v.text)]
                elif t in ("str", "e"):
                    val = v.text if t == "str" else None
                elif t == "b":
                    val = float(v.text)
                else:
                    val = float(v.text)
                cells[(r, col)] = val
    return _grid(cells)


def read_excel_rows(path) -> list[list]:
    with open(path, "rb") as f:
        head = f.read(8)
    if head == _CFB_MAGIC:
        return read_xls(path)
    if head[:2] == b"PK":
        return read_xlsx(path)
    raise ValueError(f"{path}: not an Excel workbook")


def rows_to_csv(rows: list[list]) -> str:
    import csv
    buf = io.StringIO()
    w = csv.writer(buf, lineterminator="\n")
    for row in rows:
        w.writerow(["" if v is None else (repr(v) if isinstance(v, float) and not v.is_integer() else
                                          (str(int(v)) if isinstance(v, float) and math.isfinite(v) else v))
                    for v in row])
    return buf.getvalue()


# ---------------------------------------------------------------- writers
def write_xlsx(path, rows: list[list]):
    def ref(r, c):
        s = ""
        c += 1
        while c:
            c, m = divmod(c - 1, 26)
            s = chr(65 + m) + s
        return f"{s}{r + 1}"

    def esc(s):
        return str(s).replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;")
    body = []
    for r, row in enumerate(rows):
        cs = []
        for c, v in enumerate(row):
            if v is None:
                continue
            if isinstance(v, (int, float)) and not isinstance(v, bool):
                cs.append(f'<c r="{ref(r, c)}"><v>{v!r}</v></c>')
            else:
                cs.append(f'<c r="{ref(r, c)}" t="inlineStr"><is><t>{esc(v)}</t></is></c>')
        body.append(f'<row r="{r + 1}">{"".join(cs)}</row>')
    ns = 'xmlns="http://schemas.openxmlformats.org/spreadsheetml/2006/main"'
    with zipfile.ZipFile(path, "w", zipfile.ZIP_DEFLATED) as z:
        z.writestr("[Content_Types].xml",
                   '<?xml version="1.0" encoding="UTF-8"?><Types xmlns="http://schemas.openxmlformats.org/'
                   'package/2006/content-types"><Default Extension="rels" ContentType="application/vnd.'
                   'openxmlformats-package.relationships+xml"/><Default Extension="xml" ContentType='
                   '"application/xml"/><Override PartName="/xl/workbook.xml" ContentType="application/vnd.'
                   'openxmlformats-officedocument.spreadsheetml.sheet.main+xml"/><Override PartName='
                   '"/xl/worksheets/sheet1.xml" ContentType="application/vnd.openxmlformats-officedocument.'
                   'spreadsheetml.worksheet+xml"/></Types>')
        z.writestr("_rels/.rels", '<?xml version="1.0" encoding="UTF-8"?><Relationships xmlns="http://schemas.'
                   'openxmlformats.org/package/2006/relationships"><Relationship Id="rId1" Type="http://schemas.'
                   'openxmlformats.org/officeDocument/2006/relationships/officeDocument" Target="xl/workbook.xml"/>'
                   '</Relationships>')
        z.writestr("xl/workbook.xml", f'<?xml version="1.0" encoding="UTF-8"?><workbook {ns} xmlns:r="http://'
                   'schemas.openxmlformats.org/officeDocument/2006/relationships"><sheets><sheet name="Sheet1" '
                   'sheetId="1" r:id="rId1"/></sheets></workbook>')
        z.writestr("xl/_rels/workbook.xml.rels", '<?xml version="1.0" encoding="UTF-8"?><Relationships xmlns='
                   '"http://schemas.openxmlformats.org/package/2006/relationships"><Relationship Id="rId1" Type='
                   '"http://schemas.openxmlformats.org/officeDocument/2006/relationships/worksheet" Target='
                   '"worksheets/sheet1.xml"/></Relationships>')
        z.writestr("xl/worksheets/sheet1.xml", f'<?xml version="1.0" encoding="UTF-8"?><worksheet {ns}>'
                   f'<sheetData>{"".join(body)}</sheetData></worksheet>')


def _rec(typ, body=b""):
    return struct.pack("<HH", typ, len(body)) + body


def write_xls(path, rows: list[list]):
    """A BIFF8 workbook with one sheet (strings through the SST, numbers as
    NUMBER records) in a version-3 compound file."""
    strings, index = [], {}
    for row in rows:
        for v in row:
            if isinstance(v, str) and v not in index:
                index[v] = len(strings)
                strings.append(v)
    n_refs = sum(isinstance(v, str) for row in rows for v in row)
    sst, cur = [], struct.pack("<II", n_refs, len(strings))
    for s in strings:
        enc = s.encode("utf-16-le")
        item = struct.pack("<HB", len(s), 1) + enc
        if len(cur) + len(item) > 8224:
            sst.append(cur)
            cur = b""
        cur += item
    sst.append(cur)
    wb = _rec(0x0809, struct.pack("<HHHHII", 0x0600, 0x0005, 0, 0, 0, 0))
    wb += _rec(0x00FC, sst[0]) + b"".join(_rec(0x003C, p) for p in sst[1:])
    wb += _rec(0x000A)
    wb += _rec(0x0809, struct.pack("<HHHHII", 0x0600, 0x0010, 0, 0, 0, 0))
    for r, row in enumerate(rows):
        for c, v in enumerate(row):
            if v is None:
                continue
            if isinstance(v, str):
                wb += _rec(0x00FD, struct.pack("<HHHI", r, c, 15, index[v]))
            else:
                wb += _rec(0x0203, struct.pack("<HHHd", r, c, 15, float(v)))
    wb += _rec(0x000A)
    wb += b"\0" * max(0, 4096 - len(wb))                 # above the mini-stream cutoff
    ssz = 512
    k = (len(wb) + ssz - 1) // ssz
    wb += b"\0" * (k * ssz - len(wb))
    nfat = 1
    while nfat * 128 < nfat + 1 + k:
        nfat += 1
    if nfat > 109:
        raise ValueError("workbook too large for the minimal writer")
    fat = [_FATSECT] * nfat + [_END]                     # FAT sectors, then the directory sector
    first = nfat + 1
    fat += [first + i + 1 for i in range(k - 1)] + [_END]
    fat += [_FREE] * (nfat * 128 - len(fat))
    hdr = bytearray(512)
    hdr[:8] = _CFB_MAGIC
    struct.pack_into("<HHHH", hdr, 0x18, 0x3E, 3, 0xFFFE, 9)
    struct.pack_into("<H", hdr, 0x20, 6)
    struct.pack_into("<IIII", hdr, 0x2C, nfat, nfat, 0, 4096)
    struct.pack_into("<IIII", hdr, 0x3C, _END, 0, _END, 0)
    difat = list(range(nfat)) + [_FREE] * (109 - nfat)
    struct.pack_into("<109I", hdr, 0x4C, *difat)

    def dirent(name, typ, start, size, child=_NOSTREAM):
        e = bytearray(128)
        enc = (name + "\0").encode("utf-16-le") if name else b""
        e[:len(enc)] = enc
        struct.pack_into("<HBB", e, 0x40, len(enc), typ, 1)
        struct.pack_into("<III", e, 0x44, _NOSTREAM, _NOSTREAM, child)
        struct.pack_into("<IQ", e, 0x74, start, size)
        return bytes(e)
    dirsec = dirent("Root Entry", 5, _END, 0, child=1) + dirent("Workbook", 2, first, k * ssz) + \
        dirent("", 0, 0, 0) + dirent("", 0, 0, 0)
    with open(path, "wb") as f:
        f.write(bytes(hdr))
        f.write(struct.pack(f"<{nfat * 128}I", *fat))
        f.write(dirsec)
        f.write(wb)
