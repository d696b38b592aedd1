"""Time prims (reference: water/rapids/ast/prims/time/*).

Time columns are float64 milliseconds since the epoch in HBM; calendar
fields are computed on the host via numpy datetime64 (vectorized) in the
cloud time zone (UTC by default, like a fresh reference cluster).
"""
from __future__ import annotations

import numpy as np
import torch

from .vec import T_INT, T_TIME, Vec

_TZ = {"tz": "UTC"}


def get_timezone():
    return _TZ["tz"]


def set_timezone(tz):
    _TZ["tz"] = tz


def list_timezones():
    try:
        import zoneinfo
        return sorted(zoneinfo.available_timezones())
    except Exception:
        return ["UTC"]


def _field(fr, fn):
    from .frame import H2OFrame
    import pandas as pd
    out = []
    for v in fr._vecs:
        ms = v.as_float(torch.float64).cpu().numpy()
        s = pd.to_datetime(pd.Series(ms), unit="ms", utc=True)
        if _TZ["tz"] != "UTC":
            s = s.dt.tz_convert(_TZ["tz"])
        vals = fn(s).astype("float64").values
        vals[np.isnan(ms)] = np.nan
        out.append(Vec(torch.tensor(vals, dtype=torch.float32, device=v.data.device), T_INT))
    return H2OFrame.from_vecs(out, fr.names)


def year(fr): return _field(fr, lambda s: s.dt.year)
def month(fr): return _field(fr, lambda s: s.dt.month)
def day(fr): return _field(fr, lambda s: s.dt.day)
def hour(fr): return _field(fr, lambda s: s.dt.hour)
def minute(fr): return _field(fr, lambda s: s.dt.minute)
def second(fr): return _field(fr, lambda s: s.dt.second)
def week(fr): return _field(fr, lambda s: s.dt.isocalendar().week)


def dayOfWeek(fr):
    from .frame import H2OFrame
    from .vec import T_ENUM
    r = _field(fr, lambda s: s.dt.dayofweek)
    v = r._vecs[0]
    codes = torch.nan_to_num(v.data, nan=-1).to(torch.int32)
    return H2OFrame.from_vecs([Vec(codes, T_ENUM, ["Mon", "Tue", "Wed", "Thu", "Fri", "Sat", "Sun"])], fr.names[:1])


def as_date(fr, format):
    from .frame import H2OFrame
    import pandas as pd
    fmt = format.replace("%y", "%y")
    out = []
    for v in fr._vecs:
        arr = v.to_numpy()
        s = pd.to_datetime(pd.Series(arr, dtype=object), format=fmt, errors="coerce", utc=True)
        ms = (s.astype("int64") // 10 ** 6).astype("float64").values
        ms[s.isna().values] = np.nan
        out.append(Vec(torch.tensor(ms, dtype=torch.float64, device=_dev()), T_TIME))
    return H2OFrame.from_vecs(out, fr.names)


def _dev():
    from ..parallel import cloud
    return cloud.device()


def moment(year=None, month=None, day=None, hour=None, minute=None, second=None, msec=None, date=None, time=None):
    """Time column from its parts (water/rapids/ast/prims/time/AstMoment.java): every
    part is a number or a single-column frame; scalar-only arguments give a 1x1
    frame, otherwise one row per frame row; invalid dates (Feb 30) and NA parts
    are NA.  `date` / `time` take Python date/datetime/time objects (h2o-py
    H2OFrame.moment).  Computed in UTC (ISOChronology.getInstanceUTC)."""
    import datetime as _dt
    import pandas as pd
    from .frame import H2OFrame
    if date is not None:
        if isinstance(date, _dt.datetime):
            if any(v is not None for v in (year, month, day, hour, minute, second, msec, time)):
                raise ValueError("moment(date=datetime) takes no other arguments")
            year, month, day = date.year, date.month, date.day
            hour, minute, second, msec = date.hour, date.minute, date.second, date.microsecond // 1000
        else:
            if any(v is not None for v in (year, month, day)):
                raise ValueError("moment: give either date or (year, month, day)")
            year, month, day = date.year, date.month, date.day
    if time is not None:
        if any(v is not None for v in (hour, minute, second, msec)):
            raise ValueError("moment: give either time or (hour, minute, second, msec)")
        hour, minute, second, msec = time.hour, time.minute, time.second, time.microsecond // 1000
    if year is None or month is None or day is None:
        raise ValueError("moment needs the date part: year, month and day (or date)")
    parts = [year, month, day, hour or 0, minute or 0, second or 0, msec or 0]
    n = None
    vals = []
    for i, p in enumerate(parts):
        if isinstance(p, H2OFrame):
            if p.ncol != 1:
                raise ValueError(f"Argument {i} is a frame with {p.ncol} columns")
            a = p._vecs[0].as_float(torch.float64).cpu().numpy()
            if a.size == 0:
                raise ValueError(f"Column {i} has 0 rows")
            if a.size > 1:
                if n is not None and a.size != n:
                    raise ValueError(f"Incompatible vec {i} having {a.size} rows, whereas other vecs have {n} rows.")
                n = a.size
            vals.append(a)
        else:
            vals.append(np.asarray([float(p)]))
    m = n or 1
    cols = [np.broadcast_to(v if v.size > 1 else v.reshape(1), (m,)) for v in vals]
    na = np.zeros(m, dtype=bool)
    for c in cols:
        na |= np.isnan(c)
    ic = [np.where(np.isnan(c), 1, np.trunc(c)).astype(np.int64) for c in cols]
    df = pd.DataFrame({"year": ic[0], "month": ic[1], "day": ic[2], "hour": ic[3], "minute": ic[4],
                       "second": ic[5]})
    ts = pd.to_datetime(df, errors="coerce", utc=True)
    ms = (ts.astype("int64") // 10 ** 6).astype("float64").values + ic[6]
    bad = na | ts.isna().values
    ms[bad] = np.nan
    return H2OFrame.from_vecs([Vec(torch.tensor(ms, dtype=torch.float64, device=_dev()), T_TIME)], ["time"])
