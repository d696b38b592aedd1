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
    import pandas as pd
    from .frame import H2OFrame
    ts = pd.Timestamp(year=year or 1970, month=month or 1, day=day or 1, hour=hour or 0, minute=minute or 0,
                      second=second or 0, tz="UTC")
    ms = ts.value // 10 ** 6 + (msec or 0)
    return H2OFrame.from_vecs([Vec(torch.tensor([float(ms)], dtype=torch.float64, device=_dev()), T_TIME)], ["time"])
