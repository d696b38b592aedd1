"""H2OFrame: the columnar, HBM-resident, row-sharded data frame.

Reference: water/fvec/Frame.java (storage), h2o-py/h2o/frame.py (client API)
and the Rapids primitives in water/rapids/ast/prims/* (operators, math,
reducers, mungers).  In the reference the Python H2OFrame is a lazy
expression builder shipped to the JVM as Rapids text; here the frame *is*
the data (torch tensors on the rank's GPU) and operations execute eagerly as
GPU kernels, so there is no AST round-trip.

Distribution: each rank holds rows [row_offset, row_offset + nlocal) of
every column.  Column-wise ops are shard-local; reductions all-reduce;
order-dependent ops (sort, merge, group-by, row indexing by global number)
gather what they need with collectives.
"""
from __future__ import annotations

import math
import numbers

import numpy as np
import torch

from ..parallel import cloud
from ..parallel import collectives as coll
from . import dkv
from .vec import (NUMERIC_TYPES, T_ENUM, T_INT, T_REAL, T_STR, T_TIME, T_UUID, Vec, make_enum,
                  make_enum_from_strings, make_numeric, make_string, make_time)  # noqa: F401

_TYPE_ALIASES = {"numeric": T_REAL, "real": T_REAL, "float": T_REAL, "double": T_REAL, "int": T_INT,
                 "integer": T_INT, "enum": T_ENUM, "factor": T_ENUM, "categorical": T_ENUM,
                 "string": T_STR, "str": T_STR, "time": T_TIME, "date": T_TIME, "uuid": T_UUID}


def _dev():
    return cloud.device()
from .groupsum import index_add as _ia


def _local_slice(n_global: int):
    """Row range owned by this rank for a frame of n_global rows."""
    w, r = cloud.world(), cloud.rank()
    per = n_global // w
    extra = n_global % w
    start = r * per + min(r, extra)
    end = start + per + (1 if r < extra else 0)
    return start, end


def _vec_from_array(arr, want_type=None, domain=None):
    """Build a Vec from a numpy/pandas 1-D array (full or local)."""
    want = _TYPE_ALIASES.get(want_type, want_type) if want_type else None
    a = np.asarray(arr)
    if want == T_STR or want == T_UUID:
        v = make_string(a)
        v.type = want
        return v
    if want == T_TIME or np.issubdtype(a.dtype, np.datetime64):
        if np.issubdtype(a.dtype, np.datetime64):
            ms = a.astype("datetime64[ms]").astype(np.int64).astype(np.float64)
            ms[np.isnat(a)] = np.nan
        else:
            ms = _parse_times(a)
        return make_time(ms)
    if want == T_ENUM:
        if domain is not None and np.issubdtype(a.dtype, np.integer):
            return make_enum(a.astype(np.int32), domain)
        vals = [None if _is_na(x) else _fmt_level(x) for x in a]
        return make_enum_from_strings(vals, domain=domain)
    if a.dtype == bool:
        return make_numeric(a.astype(np.float32))
    if np.issubdtype(a.dtype, np.number):
        return make_numeric(a.astype(np.float64) if a.dtype.kind in "iu" else a)
    # object: try numeric
    num = np.empty(len(a), dtype=np.float64)
    ok = True
    for i, x in enumerate(a):
        if _is_na(x):
            num[i] = np.nan
            continue
        try:
            num[i] = float(x)
        except (TypeError, ValueError):
            ok = False
            break
    if ok and want is None:
        return make_numeric(num)
    if ok and want in NUMERIC_TYPES:
        return make_numeric(num)
    if want in NUMERIC_TYPES:
        raise ValueError("column is not numeric")
    return make_enum_from_strings([None if _is_na(x) else str(x) for x in a], domain=domain)


def _fmt_level(x):
    if isinstance(x, float) and float(x).is_integer():
        return str(int(x))
    return str(x)


def _is_na(x):
    if x is None:
        return True
    if isinstance(x, float) and math.isnan(x):
        return True
    try:
        import pandas as pd
        if x is pd.NaT or (not isinstance(x, str) and pd.isna(x)):
            return True
    except Exception:
        pass
    return False


def _parse_times(a):
    import pandas as pd
    s = pd.to_datetime(pd.Series(a), errors="coerce")
    ms = s.values.astype("datetime64[ms]").astype(np.int64).astype(np.float64)
    ms[s.isna().values] = np.nan
    return ms


class H2OFrame:
    """Columnar frame of Vecs; API mirrors h2o-py's H2OFrame."""

    def __init__(self, python_obj=None, destination_frame=None, header=0, separator=",",
                 column_names=None, column_types=None, na_strings=None, skipped_columns=None,
                 _vecs=None, _names=None, _local=False):
        self._vecs: list[Vec] = []
        self._names: list[str] = []
        self.frame_id = destination_frame or dkv.make_key("py_frame")
        if _vecs is not None:
            self._vecs = list(_vecs)
            self._names = list(_names) if _names is not None else [f"C{i+1}" for i in range(len(_vecs))]
        elif python_obj is not None:
            self._init_from_python(python_obj, column_names, column_types, na_strings, skipped_columns,
                                   header, local=_local)
        dkv.put(self.frame_id, self, weak=True)

    # ------------------------------------------------------------ construction
    def _init_from_python(self, obj, column_names, column_types, na_strings, skipped, header, local=False):
        import pandas as pd
        if isinstance(obj, H2OFrame):
            self._vecs = [v.copy() for v in obj._vecs]
            self._names = list(obj._names)
            return
        if isinstance(obj, pd.DataFrame):
            df = obj
        elif isinstance(obj, pd.Series):
            df = obj.to_frame()
        elif isinstance(obj, dict):
            df = pd.DataFrame({k: (v if isinstance(v, (list, tuple, np.ndarray)) else [v]) for k, v in obj.items()})
        elif isinstance(obj, np.ndarray):
            df = pd.DataFrame(obj if obj.ndim == 2 else obj.reshape(-1, 1))
            df.columns = [f"C{i+1}" for i in range(df.shape[1])]
        elif isinstance(obj, (list, tuple)):
            if len(obj) and isinstance(obj[0], (list, tuple)):
                rows = [list(r) for r in obj]
                if header == 1 or (header == 0 and column_names is None and all(isinstance(x, str) for x in rows[0])
                                   and len(rows) > 1 and not all(isinstance(x, str) for x in rows[1])):
                    cols, rows = rows[0], rows[1:]
                else:
                    cols = [f"C{i+1}" for i in range(len(rows[0]))]
                df = pd.DataFrame(rows, columns=cols)
            else:
                df = pd.DataFrame({"C1": list(obj)})
        else:
            df = pd.DataFrame({"C1": [obj]})
        if column_names is not None:
            df.columns = list(column_names)
        if skipped:
            keep = [c for i, c in enumerate(df.columns) if i not in set(skipped)]
            df = df[keep]
        if na_strings:
            df = df.replace(list(na_strings) if isinstance(na_strings, (list, tuple)) else [na_strings], np.nan)
        ctypes = {}
        if isinstance(column_types, dict):
            ctypes = column_types
        elif isinstance(column_types, (list, tuple)):
            ctypes = dict(zip(df.columns, column_types))
        n = len(df)
        if cloud.is_distributed() and not local:
            s, e = _local_slice(n)
        else:
            s, e = 0, n
        for c in df.columns:
            col = df[c]
            want = ctypes.get(c)
            if want is None and isinstance(col.dtype, pd.CategoricalDtype):
                want = T_ENUM
                dom = [str(x) for x in col.cat.categories]
                codes = col.cat.codes.values.astype(np.int32)
                self._vecs.append(make_enum(codes[s:e], dom))
                self._names.append(str(c))
                continue
            if want is None and col.dtype == object:
                # H2O's parse guesser: all-numeric -> numeric, else categorical
                want = None
            full = col.values
            if want in (None,) and col.dtype == object:
                v = _vec_from_array(full, None)
                if v.type == T_ENUM and (s, e) != (0, n):
                    v = _vec_from_array(full[s:e], T_ENUM, domain=v.domain)
                elif (s, e) != (0, n):
                    v = _vec_from_array(full[s:e], v.type)
            else:
                if _TYPE_ALIASES.get(want, want) == T_ENUM and (s, e) != (0, n):
                    dom = _vec_from_array(full, T_ENUM).domain
                    v = _vec_from_array(full[s:e], T_ENUM, domain=dom)
                else:
                    v = _vec_from_array(full[s:e], want)
            if _TYPE_ALIASES.get(want, want) == T_INT and v.is_numeric:
                v.type = T_INT
            self._vecs.append(v)
            self._names.append(str(c))

    @classmethod
    def from_vecs(cls, vecs, names=None, frame_id=None):
        return cls(_vecs=vecs, _names=names, destination_frame=frame_id)

    @classmethod
    def from_tensor(cls, t: torch.Tensor, names=None, local=True):
        """Wrap a local [n, p] tensor (this rank's shard) as numeric columns."""
        if t.dim() == 1:
            t = t.reshape(-1, 1)
        vecs = []
        for j in range(t.shape[1]):
            col = t[:, j].contiguous()
            if not col.is_floating_point():
                col = col.to(torch.float32)
            vecs.append(Vec(col.to(_dev()), T_REAL))
        return cls.from_vecs(vecs, names or [f"C{i+1}" for i in range(t.shape[1])])

    # ------------------------------------------------------------ properties
    @property
    def names(self):
        return list(self._names)

    @names.setter
    def names(self, v):
        self.set_names(v)

    columns = names

    @property
    def col_names(self):
        return self.names

    def set_names(self, names):
        assert len(names) == len(self._vecs)
        self._names = [str(n) for n in names]
        return self

    def set_name(self, col=None, name=None):
        idx = self._col_index(col if col is not None else 0)
        self._names[idx] = name
        return self

    def rename(self, columns=None):
        for k, v in (columns or {}).items():
            self._names[self._col_index(k)] = v
        return self

    @property
    def nrows(self):
        if not self._vecs:
            return 0
        return self._vecs[0].nrow()

    nrow = nrows

    @property
    def nlocal(self):
        return self._vecs[0].nlocal if self._vecs else 0

    @property
    def ncols(self):
        return len(self._vecs)

    ncol = ncols

    @property
    def shape(self):
        return (self.nrows, self.ncols)

    @property
    def dim(self):
        return [self.nrows, self.ncols]

    def __len__(self):
        return self.nrows

    def __bool__(self):
        # truthiness must not be a collective: `frame or other` on one rank
        # only would split the SPMD collective sequence
        return True

    @property
    def types(self):
        return {n: v.type for n, v in zip(self._names, self._vecs)}

    @property
    def dtypes(self):
        return [v.type for v in self._vecs]

    def type(self, col):
        return self._vecs[self._col_index(col)].type

    @property
    def key(self):
        return self.frame_id

    def vec(self, col) -> Vec:
        return self._vecs[self._col_index(col)]

    def vecs(self):
        return list(self._vecs)

    def _col_index(self, c):
        if isinstance(c, str):
            try:
                return self._names.index(c)
            except ValueError:
                raise KeyError(f"column '{c}' not found in frame {self._names[:20]}...")
        c = int(c)
        if c < 0:
            c += len(self._vecs)
        if not 0 <= c < len(self._vecs):
            raise IndexError(c)
        return c

    def row_offset(self):
        """Global index of this rank's first row."""
        if not cloud.is_distributed():
            return 0
        n = torch.tensor([self.nlocal], dtype=torch.int64, device=_dev())
        alln = coll.all_gather_dim0(n).tolist()
        return int(sum(alln[: cloud.rank()]))

    # ------------------------------------------------------------ conversion
    def as_data_frame(self, use_pandas=True, header=True, use_multi_thread=False, local=False):
        """pandas view of the whole frame (gathered on every rank), or of this
        rank's row shard only (local=True: per-rank host scoring)."""
        import pandas as pd
        data = {}
        for n, v in zip(self._names, self._vecs if local else self._gathered_vecs()):
            if v.type == T_TIME:
                a = v.data.cpu().numpy()
                data[n] = pd.to_datetime(pd.Series(a), unit="ms")
            elif v.type == T_ENUM:
                data[n] = pd.Series(v.to_numpy(), dtype=object)
            elif v.type == T_INT:
                a = v.data.cpu().numpy()
                data[n] = a.astype(np.int64) if not np.isnan(a).any() else a
            else:
                data[n] = v.to_numpy()
        df = pd.DataFrame(data, columns=self._names)
        if not use_pandas:
            rows = df.values.tolist()
            return [self._names] + rows if header else rows
        return df

    def _gathered_vecs(self):
        """Full columns on every rank (for small-data host conversions)."""
        if not cloud.is_distributed():
            return self._vecs
        out = []
        for v in self._vecs:
            if v.replicated:
                out.append(v)
                continue
            if v.on_host:
                parts = coll.all_gather_object(list(v.data))
                nv = Vec(np.array(sum(parts, []), dtype=object), v.type)
            else:
                nv = Vec(coll.all_gather_var(v.data), v.type, v.domain)
            nv.replicated = True
            out.append(nv)
        return out

    def gather(self):
        """Return a non-sharded copy of the frame (identical on all ranks)."""
        if not cloud.is_distributed():
            return self
        return H2OFrame.from_vecs(self._gathered_vecs(), self._names)

    def to_tensor(self, cols=None, dtype=torch.float32) -> torch.Tensor:
        cols = self._names if cols is None else cols
        return torch.stack([self.vec(c).as_float(dtype) for c in cols], 1) if cols else \
            torch.empty((self.nlocal, 0), dtype=dtype, device=_dev())

    def as_matrix(self):
        return self.to_tensor().cpu().numpy()

    def get_frame_data(self):
        return self.as_data_frame().to_csv(index=False)

    # ------------------------------------------------------------ display
    def head(self, rows=10, cols=200):
        return self[: min(rows, self.nrows), : min(cols, self.ncols)]

    def tail(self, rows=10, cols=200):
        n = self.nrows
        return self[max(0, n - rows): n, : min(cols, self.ncols)]

    def __repr__(self):
        try:
            df = self.head(10).as_data_frame()
            return f"H2OFrame {self.frame_id} [{self.nrows} rows x {self.ncols} cols]\n{df}"
        except Exception as e:  # pragma: no cover
            return f"H2OFrame {self.frame_id} [{self.ncols} cols] ({e})"

    def show(self, *a, **k):
        print(repr(self))

    def describe(self, chunk_summary=False):
        print(f"Rows:{self.nrows}\nCols:{self.ncols}")
        print(self.summary(return_data=True))

    def summary(self, return_data=False):
        out = {}
        from ..ops import frame_ops
        frame_ops.rollups_many(self._vecs)          # every numeric device column in one batched pass
        for n, v in zip(self._names, self._vecs):
            r = v.rollups()
            out[n] = {"type": v.type, "mins": r["min"], "maxs": r["max"], "mean": r["mean"], "sigma": r["sigma"],
                      "zeros": r["zeros"], "missing_count": r["nacnt"],
                      "domain": v.domain if v.domain is not None and len(v.domain) <= 100 else None}
        if return_data:
            return out
        print(out)
        return out

    # ------------------------------------------------------------ indexing
    def _select_cols(self, item):
        if isinstance(item, slice):
            idx = list(range(self.ncols))[item]
        elif isinstance(item, (list, tuple)):
            if len(item) and isinstance(item[0], (bool, np.bool_)):
                idx = [i for i, b in enumerate(item) if b]
            else:
                idx = [self._col_index(c) for c in item]
        else:
            idx = [self._col_index(item)]
        return idx

    def _row_mask_or_index(self, item):
        """Return ('mask', bool tensor local) or ('index', global idx list) or ('slice', s)."""
        if isinstance(item, H2OFrame):
            v = item._vecs[0]
            m = v.as_float()
            return "mask", (m != 0) & ~torch.isnan(m)
        if isinstance(item, slice):
            return "slice", item
        if isinstance(item, numbers.Integral):
            n = self.nrows
            i = int(item) + (n if item < 0 else 0)
            return "index", [i]
        if isinstance(item, torch.Tensor):
            if item.dtype == torch.bool:
                return "mask", item.to(_dev())
            return "index", item.tolist()
        if isinstance(item, (list, tuple, np.ndarray, range)):
            lst = list(item)
            if len(lst) and isinstance(lst[0], (bool, np.bool_)):
                return "mask", torch.tensor(lst, dtype=torch.bool, device=_dev())
            n = self.nrows
            return "index", [int(i) + (n if i < 0 else 0) for i in lst]
        raise TypeError(f"bad row selector {type(item)}")

    def _take_rows_local(self, vecs, sel_kind, sel):
        out = []
        if sel_kind == "mask":
            midx = torch.nonzero(sel, as_tuple=False).flatten()
            for v in vecs:
                out.append(_take(v, midx))
            return out
        if sel_kind == "slice":
            n = self.nrows
            s, e, st = sel.indices(n)
            off = self.row_offset()
            gidx = torch.arange(s, e, st, device=_dev())
            lidx = gidx - off
            lidx = lidx[(lidx >= 0) & (lidx < self.nlocal)]
            for v in vecs:
                out.append(_take(v, lidx))
            return out
        # global index list: every rank contributes the rows it owns, then
        # rows are re-sharded in request order
        gidx = torch.tensor(sel, dtype=torch.int64, device=_dev())
        if not cloud.is_distributed():
            for v in vecs:
                out.append(_take(v, gidx))
            return out
        g = self.gather()
        res = H2OFrame.from_vecs([_take(v, gidx) for v in g._vecs], g._names)
        s, e = _local_slice(len(sel))
        return [_take(v, torch.arange(s, e, device=_dev())) for v in res._vecs]

    def __getitem__(self, item):
        if isinstance(item, tuple) and len(item) == 2:
            rows, cols = item
            cidx = self._select_cols(cols) if not (isinstance(cols, slice) and cols == slice(None)) else list(range(self.ncols))
            vecs = [self._vecs[i] for i in cidx]
            names = [self._names[i] for i in cidx]
            if isinstance(rows, slice) and rows == slice(None):
                return H2OFrame.from_vecs(vecs, names)
            kind, sel = self._row_mask_or_index(rows)
            nv = self._take_rows_local(vecs, kind, sel)
            fr = H2OFrame.from_vecs(nv, names)
            if isinstance(rows, numbers.Integral) and isinstance(cols, (numbers.Integral, str)):
                return fr.flatten()
            return fr
        if isinstance(item, H2OFrame) or (isinstance(item, torch.Tensor) and item.dtype == torch.bool):
            kind, sel = self._row_mask_or_index(item)
            return H2OFrame.from_vecs(self._take_rows_local(self._vecs, kind, sel), self._names)
        cidx = self._select_cols(item)
        return H2OFrame.from_vecs([self._vecs[i] for i in cidx], [self._names[i] for i in cidx])

    def flatten(self):
        v = self._gathered_vecs()[0]
        if len(v) == 0:
            return None
        x = v.to_numpy()[0]
        if v.type == T_ENUM or v.on_host:
            return x
        x = float(x)
        return x

    def __setitem__(self, key, value):
        rows = None
        if isinstance(key, tuple):
            rows, key = key
        if isinstance(key, (list, tuple)) and not isinstance(key, str):
            for k in key:
                self.__setitem__((rows, k) if rows is not None else k, value)
            return
        newvec = self._coerce_value_vec(value)
        if isinstance(key, str) and key not in self._names:
            if rows is not None:
                base = Vec(torch.full((self.nlocal,), float("nan"), device=_dev()), T_REAL)
                self._vecs.append(base)
                self._names.append(key)
            else:
                self._vecs.append(newvec)
                self._names.append(key)
                return
        idx = self._col_index(key)
        if rows is None:
            self._vecs[idx] = newvec
            return
        kind, sel = self._row_mask_or_index(rows)
        old = self._vecs[idx]
        if kind == "mask":
            m = sel
        else:
            m = torch.zeros(self.nlocal, dtype=torch.bool, device=_dev())
            off = self.row_offset()
            if kind == "slice":
                s, e, st = sel.indices(self.nrows)
                g = torch.arange(s, e, st, device=_dev())
            else:
                g = torch.tensor(sel, dtype=torch.int64, device=_dev())
            l = g - off
            l = l[(l >= 0) & (l < self.nlocal)]
            m[l] = True
        self._vecs[idx] = _where_vec(m, newvec, old)

    def _coerce_value_vec(self, value):
        n = self.nlocal
        if isinstance(value, H2OFrame):
            return value._vecs[0]
        if isinstance(value, Vec):
            return value
        if isinstance(value, str):
            return make_enum(np.zeros(n, dtype=np.int32), [value])
        if value is None:
            return Vec(torch.full((n,), float("nan"), device=_dev()), T_REAL)
        if isinstance(value, (list, np.ndarray)):
            return _vec_from_array(np.asarray(value)[slice(*_local_slice(len(value)))] if cloud.is_distributed() else np.asarray(value))
        return make_numeric(torch.full((n,), float(value), dtype=torch.float64))

    def pop(self, i):
        idx = self._col_index(i)
        fr = H2OFrame.from_vecs([self._vecs[idx]], [self._names[idx]])
        del self._vecs[idx]
        del self._names[idx]
        return fr

    def drop(self, index, axis=1):
        if axis == 1:
            idx = set(self._select_cols(index if isinstance(index, (list, tuple)) else [index]))
            keep = [i for i in range(self.ncols) if i not in idx]
            return H2OFrame.from_vecs([self._vecs[i] for i in keep], [self._names[i] for i in keep])
        rows = index if isinstance(index, (list, tuple)) else [index]
        keep = sorted(set(range(self.nrows)) - set(rows))
        return self[keep, :]

    def __contains__(self, name):
        return name in self._names

    def __iter__(self):
        return iter(self._names)

    # ------------------------------------------------------------ cbind/rbind
    def cbind(self, data):
        others = data if isinstance(data, (list, tuple)) else [data]
        vecs, names = list(self._vecs), list(self._names)
        for o in others:
            if not isinstance(o, H2OFrame):
                o = H2OFrame(o)
            for n, v in zip(o._names, o._vecs):
                nn = n
                k = 0
                while nn in names:
                    k += 1
                    nn = f"{n}{k}"
                names.append(nn)
                vecs.append(v)
        return H2OFrame.from_vecs(vecs, names)

    def rbind(self, data):
        from .munging import rbind
        return rbind([self] + (list(data) if isinstance(data, (list, tuple)) else [data]))

    # ------------------------------------------------------------ type conversions
    def asfactor(self):
        vecs = [_to_enum(v) for v in self._vecs]
        return H2OFrame.from_vecs(vecs, self._names)

    as_factor = asfactor

    def asnumeric(self):
        out = []
        for v in self._vecs:
            if v.type == T_ENUM:
                # H2O's as.numeric on a factor returns the level index; on
                # numeric-looking levels as_numeric of the labels is common
                out.append(Vec(v.as_float(), T_INT))
            elif v.on_host:
                arr = np.array([float(x) if x is not None and _try_float(x) else np.nan for x in v.data])
                out.append(make_numeric(arr))
            else:
                out.append(Vec(v.data.clone(), v.type if v.type != T_TIME else T_REAL))
        return H2OFrame.from_vecs(out, self._names)

    as_numeric = asnumeric

    def ascharacter(self):
        out = []
        for v in self._vecs:
            arr = v.to_numpy()
            out.append(make_string([None if _is_na(x) else (_fmt_level(x) if not isinstance(x, str) else x) for x in arr]))
        return H2OFrame.from_vecs(out, self._names)

    def isfactor(self):
        return [v.type == T_ENUM for v in self._vecs]

    def isnumeric(self):
        return [v.type in NUMERIC_TYPES for v in self._vecs]

    def isstring(self):
        return [v.type == T_STR for v in self._vecs]

    def ischaracter(self):
        return self.isstring()

    def levels(self):
        return [list(v.domain) if v.domain is not None else [] for v in self._vecs]

    def nlevels(self):
        return [len(v.domain) if v.domain is not None else 0 for v in self._vecs]

    def set_levels(self, levels):
        v = self._vecs[0]
        assert v.type == T_ENUM and len(levels) == len(v.domain)
        self._vecs[0] = Vec(v.data, T_ENUM, list(levels))
        return self

    def relevel(self, y):
        v = self._vecs[0]
        dom = list(v.domain)
        i = dom.index(y)
        newdom = [y] + dom[:i] + dom[i + 1:]
        remap = torch.tensor([newdom.index(d) for d in dom], dtype=torch.int32, device=_dev())
        codes = torch.where(v.data < 0, v.data, remap[v.data.clamp(min=0).long()])
        return H2OFrame.from_vecs([Vec(codes, T_ENUM, newdom)], self._names[:1])

    def columns_by_type(self, coltype="numeric"):
        m = {"numeric": lambda v: v.type in NUMERIC_TYPES, "categorical": lambda v: v.type == T_ENUM,
             "string": lambda v: v.type == T_STR, "time": lambda v: v.type == T_TIME,
             "uuid": lambda v: v.type == T_UUID, "bad": lambda v: v.type == "bad"}[coltype]
        return [float(i) for i, v in enumerate(self._vecs) if m(v)]

    # ------------------------------------------------------------ elementwise math
    def _binop(self, other, op, rev=False):
        from .ops_elem import binop
        return binop(self, other, op, rev)

    def __add__(self, o): return self._binop(o, "+")
    def __radd__(self, o): return self._binop(o, "+", True)
    def __sub__(self, o): return self._binop(o, "-")
    def __rsub__(self, o): return self._binop(o, "-", True)
    def __mul__(self, o): return self._binop(o, "*")
    def __rmul__(self, o): return self._binop(o, "*", True)
    def __truediv__(self, o): return self._binop(o, "/")
    def __rtruediv__(self, o): return self._binop(o, "/", True)
    def __floordiv__(self, o): return self._binop(o, "//")
    def __rfloordiv__(self, o): return self._binop(o, "//", True)
    def __mod__(self, o): return self._binop(o, "%")
    def __rmod__(self, o): return self._binop(o, "%", True)
    def __pow__(self, o): return self._binop(o, "**")
    def __rpow__(self, o): return self._binop(o, "**", True)
    def __eq__(self, o): return self._binop(o, "==")
    def __ne__(self, o): return self._binop(o, "!=")
    def __lt__(self, o): return self._binop(o, "<")
    def __le__(self, o): return self._binop(o, "<=")
    def __gt__(self, o): return self._binop(o, ">")
    def __ge__(self, o): return self._binop(o, ">=")
    def __and__(self, o): return self._binop(o, "&")
    def __rand__(self, o): return self._binop(o, "&", True)
    def __or__(self, o): return self._binop(o, "|")
    def __ror__(self, o): return self._binop(o, "|", True)

    def __neg__(self):
        return self._unop(lambda x: -x)

    def __invert__(self):
        return self._unop(lambda x: torch.where(torch.isnan(x), x, (x == 0).to(x.dtype)))

    def __abs__(self):
        return self.abs()

    __hash__ = object.__hash__

    def _unop(self, fn, keep_int=False):
        out = []
        for v in self._vecs:
            x = v.as_float(torch.float64 if v.data.dtype == torch.float64 else torch.float32)
            r = fn(x)
            out.append(Vec(r, T_INT if keep_int and v.type == T_INT else T_REAL))
        return H2OFrame.from_vecs(out, self._names)

    def abs(self): return self._unop(torch.abs, True)
    def sqrt(self): return self._unop(torch.sqrt)
    def exp(self): return self._unop(torch.exp)
    def expm1(self): return self._unop(torch.expm1)
    def log(self): return self._unop(torch.log)
    def log10(self): return self._unop(torch.log10)
    def log2(self): return self._unop(torch.log2)
    def log1p(self): return self._unop(torch.log1p)
    def sin(self): return self._unop(torch.sin)
    def cos(self): return self._unop(torch.cos)
    def tan(self): return self._unop(torch.tan)
    def asin(self): return self._unop(torch.asin)
    def acos(self): return self._unop(torch.acos)
    def atan(self): return self._unop(torch.atan)
    def sinh(self): return self._unop(torch.sinh)
    def cosh(self): return self._unop(torch.cosh)
    def tanh(self): return self._unop(torch.tanh)
    def asinh(self): return self._unop(torch.asinh)
    def acosh(self): return self._unop(torch.acosh)
    def atanh(self): return self._unop(torch.atanh)
    def sinpi(self): return self._unop(lambda x: torch.sin(math.pi * x))
    def cospi(self): return self._unop(lambda x: torch.cos(math.pi * x))
    def tanpi(self): return self._unop(lambda x: torch.tan(math.pi * x))
    def ceil(self): return self._unop(torch.ceil)
    def floor(self): return self._unop(torch.floor)
    def trunc(self): return self._unop(torch.trunc)
    def sign(self): return self._unop(torch.sign)
    def gamma(self): return self._unop(lambda x: torch.exp(torch.lgamma(x)))
    def lgamma(self): return self._unop(torch.lgamma)
    def digamma(self): return self._unop(torch.digamma)
    def trigamma(self): return self._unop(lambda x: torch.polygamma(1, x))

    def round(self, digits=0):
        f = 10.0 ** digits
        return self._unop(lambda x: torch.round(x * f) / f)

    def signif(self, digits=6):
        def fn(x):
            mag = torch.floor(torch.log10(torch.abs(x)))
            sc = 10.0 ** (digits - 1 - mag)
            r = torch.round(x * sc) / sc
            return torch.where(x == 0, x, r)
        return self._unop(fn)

    def logical_negation(self):
        return ~self

    def isna(self):
        out = [Vec(v.isna().to(torch.float32), T_INT) for v in self._vecs]
        return H2OFrame.from_vecs(out, [f"isNA({n})" for n in self._names])

    def isnan(self):
        return self.isna()

    def ifelse(self, yes, no):
        from .ops_elem import ifelse
        return ifelse(self, yes, no)

    # ------------------------------------------------------------ reducers
    def _num_data(self, na_rm=True):
        return [v.as_float(torch.float64) for v in self._vecs if not v.on_host]

    def sum(self, skipna=True, axis=0, return_frame=False):
        if axis == 1:
            x = self.to_tensor(dtype=torch.float64)
            r = torch.nansum(x, 1) if skipna else x.sum(1)
            return H2OFrame.from_vecs([Vec(r, T_REAL)], ["sum"])
        res = []
        for v in self._vecs:
            x = v.as_float(torch.float64)
            s = torch.nansum(x) if skipna else x.sum()
            res.append(coll.allreduce_scalar(float(s)))
        return res[0] if len(res) == 1 and not return_frame else res

    def mean(self, skipna=True, axis=0, return_frame=False):
        if axis == 1:
            x = self.to_tensor(dtype=torch.float64)
            r = torch.nanmean(x, 1) if skipna else x.mean(1)
            return H2OFrame.from_vecs([Vec(r, T_REAL)], ["mean"])
        res = []
        from ..ops import frame_ops
        frame_ops.rollups_many(self._vecs)
        for v in self._vecs:
            r = v.rollups()
            if not skipna and r["nacnt"] > 0:
                res.append(float("nan"))
            else:
                res.append(r["mean"])
        if return_frame:
            return H2OFrame({n: [m] for n, m in zip(self._names, res)})
        return res[0] if len(res) == 1 else res

    def min(self):
        return min(v.min() for v in self._vecs)

    def max(self):
        return max(v.max() for v in self._vecs)

    def sd(self, na_rm=True):
        r = [v.sigma() for v in self._vecs]
        return r if len(r) > 1 else r

    def var(self, y=None, na_rm=True, use=None):
        if y is None and self.ncols == 1:
            return self._vecs[0].sigma() ** 2
        from .munging import cov
        return cov(self, y)

    def cor(self, y=None, na_rm=False, use=None, method="Pearson"):
        from .munging import cor
        if use is None:
            use = "complete.obs" if na_rm else "everything"
        return cor(self, y, method=method, use=use)

    def median(self, na_rm=True):
        from .munging import quantile_values
        return [quantile_values(v, [0.5])[0] for v in self._vecs]

    def prod(self, na_rm=False):
        x = self._vecs[0].as_float(torch.float64)
        p = torch.prod(x[~torch.isnan(x)]) if na_rm else torch.prod(x)
        return float(p)

    def all(self):
        x = self._vecs[0].as_float()
        return bool(coll.allreduce_scalar(float(((x != 0) | torch.isnan(x)).logical_not().sum()))) is False

    def any(self):
        x = self._vecs[0].as_float()
        return coll.allreduce_scalar(float(((x != 0) & ~torch.isnan(x)).sum())) > 0

    def any_na_strict(self):
        return any(v.nacnt() > 0 for v in self._vecs)

    def nacnt(self):
        return [v.nacnt() for v in self._vecs]

    def cumsum(self, axis=0):
        return self._cum(torch.cumsum)

    def cumprod(self, axis=0):
        return self._cum(torch.cumprod)

    def cummax(self, axis=0):
        return self._cum(lambda x, d: torch.cummax(x, d).values)

    def cummin(self, axis=0):
        return self._cum(lambda x, d: torch.cummin(x, d).values)

    def _cum(self, fn):
        g = self.gather()
        out = [Vec(fn(v.as_float(torch.float64), 0), T_REAL) for v in g._vecs]
        return _reshard(H2OFrame.from_vecs(out, self._names))

    def quantile(self, prob=None, combine_method="interpolate", weights_column=None):
        from .munging import quantile
        return quantile(self, prob, combine_method, weights_column)

    def unique(self, include_nas=False):
        from .munging import unique
        return unique(self, include_nas)

    def table(self, data2=None, dense=True):
        from .munging import table
        return table(self, data2, dense)

    def hist(self, breaks="sturges", plot=False, **kw):
        from .munging import hist
        return hist(self, breaks)

    def impute(self, column=-1, method="mean", combine_method="interpolate", by=None, group_by_frame=None, values=None):
        from .munging import impute
        return impute(self, column, method, combine_method, by, values)

    def fillna(self, method="forward", axis=0, maxlen=1):
        from .munging import fillna
        return fillna(self, method, axis, maxlen)

    def scale(self, center=True, scale=True, inplace=False):
        from .munging import scale_frame
        return scale_frame(self, center, scale)

    def cut(self, breaks, labels=None, include_lowest=False, right=True, dig_lab=3):
        from .munging import cut
        return cut(self, breaks, labels, include_lowest, right, dig_lab)

    def group_by(self, by):
        from .munging import GroupBy
        return GroupBy(self, by)

    def merge(self, other, all_x=False, all_y=False, by_x=None, by_y=None, method="auto"):
        from .munging import merge
        return merge(self, other, all_x, all_y, by_x, by_y)

    def sort(self, by, ascending=True):
        from .munging import sort
        return sort(self, by, ascending)

    def split_frame(self, ratios=None, destination_frames=None, seed=None):
        from .munging import split_frame
        return split_frame(self, ratios or [0.75], seed)

    def runif(self, seed=None):
        from .munging import runif
        return runif(self, seed)

    def kfold_column(self, n_folds=3, seed=-1):
        from .munging import kfold_column
        return kfold_column(self, n_folds, seed)

    def modulo_kfold_column(self, n_folds=3):
        from .munging import modulo_kfold_column
        return modulo_kfold_column(self, n_folds)

    def stratified_kfold_column(self, n_folds=3, seed=-1):
        from .munging import stratified_kfold_column
        return stratified_kfold_column(self, n_folds, seed)

    def stratified_split(self, test_frac=0.2, seed=-1):
        from .munging import stratified_split
        return stratified_split(self, test_frac, seed)

    def apply(self, fun=None, axis=0):
        from .munging import apply
        return apply(self, fun, axis)

    def na_omit(self):
        m = torch.ones(self.nlocal, dtype=torch.bool, device=_dev())
        for v in self._vecs:
            m &= ~v.isna()
        return self[m]

    def drop_duplicates(self, columns=None, keep="first"):
        from .munging import drop_duplicates
        return drop_duplicates(self, columns, keep)

    def pivot(self, index, column, value):
        from .munging import pivot
        return pivot(self, index, column, value)

    def melt(self, id_vars, value_vars=None, var_name="variable", value_name="value", skipna=False):
        from .munging import melt
        return melt(self, id_vars, value_vars, var_name, value_name, skipna)

    def rank_within_group_by(self, group_by_cols, sort_cols, ascending=None, new_col_name="New_Rank_column", sort_cols_sorted=False):
        from .munging import rank_within_group_by
        return rank_within_group_by(self, group_by_cols, sort_cols, ascending, new_col_name, sort_cols_sorted)

    def topN(self, column=0, nPercent=10, grabTopN=1):
        """Top nPercent% of a numeric column (h2o-py frame.py:4022 -> topn, grabTopN = 1)."""
        from .munging import topn
        return topn(self, column, nPercent, grabTopN)

    def difflag1(self):
        g = self.gather()
        x = g._vecs[0].as_float(torch.float64)
        d = torch.cat([torch.tensor([float("nan")], dtype=x.dtype, device=x.device), x[1:] - x[:-1]])
        return _reshard(H2OFrame.from_vecs([Vec(d, T_REAL)], self._names[:1]))

    def transpose(self):
        x = self.gather().to_tensor(dtype=torch.float64).T.contiguous()
        return _reshard(H2OFrame.from_tensor(x))

    def mult(self, matrix):
        a = self.gather().to_tensor(dtype=torch.float64)
        b = matrix.gather().to_tensor(dtype=torch.float64)
        return _reshard(H2OFrame.from_tensor(a @ b))

    def distance(self, y, measure="l2"):
        from .munging import distance
        return distance(self, y, measure)

    def entropy(self):
        from .strings import entropy
        return entropy(self)

    # ------------------------------------------------------------ misc Rapids prims (h2o-py/h2o/frame.py parity)
    @property
    def dtype(self):
        """numpy dtype of the first column (h2o-py/h2o/frame.py:370)."""
        v = self._vecs[0]
        if v.type in (T_STR, T_UUID, T_ENUM):
            return np.dtype(object)
        if v.type == T_TIME:
            return np.dtype("datetime64[ms]")
        return np.dtype(np.int64) if v.type == T_INT and v.nacnt() == 0 else np.dtype(np.float64)

    def any_na_rm(self):
        """True if any value of any column is non-zero, NAs ignored (AstAnyNa/AstAny)."""
        hit = 0.0
        for v in self._vecs:
            if v.on_host:
                hit += float(sum(1 for x in v.data if x not in (None, "")))
                continue
            x = v.as_float()
            hit += float(((x != 0) & ~torch.isnan(x)).sum())
        return coll.allreduce_scalar(hit) > 0

    def anyfactor(self):
        """mungers/AstAnyFactor.java"""
        return any(v.type == T_ENUM for v in self._vecs)

    def categories(self):
        """Levels of a single categorical column."""
        if self.ncols != 1 or self._vecs[0].type != T_ENUM:
            raise ValueError("categories() requires a single categorical column")
        return list(self._vecs[0].domain)

    def append_levels(self, levels):
        """Append levels to the domain of every categorical column (mungers/AstAppendLevels.java)."""
        out = []
        for v in self._vecs:
            if v.type != T_ENUM:
                raise ValueError("append_levels applies to categorical columns only")
            dom = list(v.domain) + [str(l) for l in levels if str(l) not in v.domain]
            out.append(Vec(v.data, T_ENUM, dom))
        return H2OFrame.from_vecs(out, self._names)

    def set_level(self, level):
        """Set every value of a categorical column to `level` (mungers/AstSetLevel.java)."""
        out = []
        for v in self._vecs:
            if v.type != T_ENUM or level not in v.domain:
                raise ValueError(f"level '{level}' not in the column domain")
            out.append(Vec(torch.full_like(v.data, v.domain.index(level)), T_ENUM, list(v.domain)))
        return H2OFrame.from_vecs(out, self._names)

    def relevel_by_frequency(self, weights_column=None, top_n=-1):
        """Most frequent level first (mungers/AstRelevelByFreq.java): ascending stable
        sort of level weights, read back to front; with top_n only the top_n levels move."""
        if top_n != -1 and (top_n <= 0 or int(top_n) != top_n):
            raise ValueError(f"TopN argument needs to be a positive integer number, got: {top_n}")
        w = self.vec(weights_column).as_float(torch.float64) if weights_column is not None else None
        out = []
        for v in self._vecs:
            if v.type != T_ENUM:
                out.append(v)
                continue
            k = len(v.domain)
            ok = v.data >= 0
            ww = torch.ones_like(v.data, dtype=torch.float64) if w is None else torch.nan_to_num(w)
            lw = torch.zeros(k, dtype=torch.float64, device=v.data.device)
            _ia(lw, v.data[ok].long(), ww[ok])
            lw = coll.allreduce_(lw).cpu().numpy()
            order = list(np.argsort(lw, kind="stable"))
            if top_n != -1 and top_n < k - 1:
                top = [order[k - 1 - i] for i in range(top_n)]
                new_order = [0] * k
                for i, t in enumerate(top):
                    new_order[k - 1 - i] = t
                pos = k - top_n - 1
                tops = set(top)
                for i in range(k):
                    if i in tops:
                        continue
                    new_order[pos] = i
                    pos -= 1
                order = new_order
            newdom = [v.domain[order[k - 1 - i]] for i in range(k)]
            remap = torch.empty(k, dtype=torch.int32)
            for i, lvl in enumerate(order):
                remap[lvl] = k - 1 - i
            remap = remap.to(v.data.device)
            codes = torch.where(ok, remap[v.data.clamp(min=0).long()], v.data)
            out.append(Vec(codes, T_ENUM, newdom))
        return H2OFrame.from_vecs(out, self._names)

    def concat(self, frames, axis=1):
        """cbind (axis=1) or rbind (axis=0) of this frame with `frames`."""
        frames = list(frames) if isinstance(frames, (list, tuple)) else [frames]
        if axis == 1:
            out = self
            for f in frames:
                out = out.cbind(f)
            return out
        return self.rbind(frames)

    def detach(self):
        """Drop the DKV registration of this frame (the data stays with the object)."""
        dkv.remove(self.frame_id)

    @staticmethod
    def get_frame(frame_id, **kw):
        return dkv.get(frame_id)

    @staticmethod
    def from_python(python_obj, destination_frame=None, header=0, separator=",", column_names=None,
                    column_types=None, na_strings=None, skipped_columns=None, **kw):
        return H2OFrame(python_obj, destination_frame=destination_frame, header=header, separator=separator,
                        column_names=column_names, column_types=column_types, na_strings=na_strings,
                        skipped_columns=skipped_columns)

    def get_summary(self):
        return self.summary(return_data=True)

    def show_summary(self):
        self.summary()

    def filter_na_cols(self, frac=0.2):
        """Indices of the columns whose NA count is < frac * nrows (mungers/AstFilterNaCols.java)."""
        lim = self.nrows * frac
        return [i for i, v in enumerate(self._vecs) if v.nacnt() < lim]

    def getrow(self):
        """The single row of a 1-row frame as a list (mungers/AstGetrow.java)."""
        if self.nrows != 1:
            raise ValueError("getrow() requires a frame with exactly one row")
        row = []
        for v in self._gathered_vecs():
            x = v.to_numpy()[0]
            row.append(None if _is_na(x) else (float(x) if v.type in NUMERIC_TYPES else x))
        return row

    def _idx_extreme(self, skipna, axis, largest):
        if axis == 1:
            x = self.to_tensor(dtype=torch.float64)
            nan = torch.isnan(x)
            fill = -math.inf if largest else math.inf
            xf = torch.where(nan, torch.full_like(x, fill), x)
            r = (xf.argmax(1) if largest else xf.argmin(1)).to(torch.float64)
            if not skipna:
                r = torch.where(nan.any(1), torch.full_like(r, float("nan")), r)
            return H2OFrame.from_vecs([Vec(r, T_INT)], ["which.max" if largest else "which.min"])
        off = self.row_offset()
        res = []
        for v in self._vecs:
            x = v.as_float(torch.float64)
            nan = torch.isnan(x)
            if not skipna and coll.allreduce_scalar(float(nan.sum())) > 0:
                res.append(float("nan"))
                continue
            fill = -math.inf if largest else math.inf
            xf = torch.where(nan, torch.full_like(x, fill), x)
            if xf.numel():
                i = int(xf.argmax() if largest else xf.argmin())
                val, gi = float(xf[i]), float(i + off)
            else:
                val, gi = fill, float("nan")
            if cloud.is_distributed():
                cands = coll.all_gather_object((val, gi))
                best = max(cands, key=lambda c: (c[0], -c[1])) if largest else min(cands, key=lambda c: (c[0], c[1]))
                val, gi = best
            res.append(gi if math.isfinite(val) else float("nan"))
        return H2OFrame({n: [r] for n, r in zip(self._names, res)})

    def idxmax(self, skipna=True, axis=0):
        """Row index of the max per column (axis=0) or column index per row (axis=1) (AstWhichMax)."""
        return self._idx_extreme(skipna, axis, True)

    def idxmin(self, skipna=True, axis=0):
        return self._idx_extreme(skipna, axis, False)

    def which(self):
        """Global row indices of the non-zero entries of a single column (AstWhich)."""
        x = self._vecs[0].as_float()
        idx = torch.nonzero((x != 0) & ~torch.isnan(x)).flatten().to(torch.float64) + self.row_offset()
        return H2OFrame.from_vecs([Vec(idx, T_INT)], ["which"])

    def isin(self, item):
        """Elementwise membership test against a scalar or list of values."""
        items = list(item) if isinstance(item, (list, tuple, set)) else [item]
        out = []
        for v in self._vecs:
            if v.type == T_ENUM:
                codes = [v.domain.index(str(i)) for i in items if str(i) in v.domain]
                t = torch.tensor(codes or [-2], dtype=v.data.dtype, device=v.data.device)
                m = torch.isin(v.data, t)
            elif v.on_host:
                s = set(str(i) for i in items)
                m = torch.tensor([x is not None and str(x) in s for x in v.data], device=_dev())
            else:
                nums = [float(i) for i in items if _try_float(i)]
                t = torch.tensor(nums or [float("nan")], dtype=torch.float64, device=v.data.device)
                m = torch.isin(v.as_float(torch.float64), t)
            out.append(Vec(m.to(torch.float32), T_INT))
        return H2OFrame.from_vecs(out, self._names)

    def match(self, table, nomatch=0, start_index=1):
        """Position (start_index-based) of each value in `table`, else `nomatch` (AstMatch)."""
        table = list(table) if isinstance(table, (list, tuple)) else [table]
        out = []
        for v in self._vecs:
            if v.type == T_ENUM:
                lut = [float(table.index(d) + start_index) if d in table else
                       (float(table.index(_num_or(d)) + start_index) if _num_or(d) in table else float(nomatch))
                       for d in v.domain] or [float(nomatch)]
                lt = torch.tensor(lut, dtype=torch.float64, device=v.data.device)
                r = torch.where(v.data >= 0, lt[v.data.clamp(min=0).long()],
                                torch.full(v.data.shape, float(nomatch), dtype=torch.float64, device=v.data.device))
            elif v.on_host:
                pos = {str(t): i + start_index for i, t in reversed(list(enumerate(table)))}
                r = torch.tensor([float(pos.get(str(x), nomatch)) if x is not None else float(nomatch)
                                  for x in v.data], dtype=torch.float64, device=_dev())
            else:
                x = v.as_float(torch.float64)
                r = torch.full_like(x, float(nomatch))
                for i in reversed(range(len(table))):
                    if _try_float(table[i]):
                        r = torch.where(x == float(table[i]), torch.full_like(x, float(i + start_index)), r)
            out.append(Vec(r, T_INT))
        return H2OFrame.from_vecs(out, self._names)

    def _moment(self, k, na_rm):
        res = []
        for v in self._vecs:
            if not v.is_numeric or self.nrows == 0 or (not na_rm and v.nacnt() > 0):
                res.append(float("nan"))
                continue
            x = v.as_float(torch.float64)
            x = x[~torch.isnan(x)]
            mu = v.mean()
            d = x - mu
            ss = coll.allreduce_scalar(float((d * d).sum()))
            sk = coll.allreduce_scalar(float((d ** k).sum()))
            n = self.nrows  # reference divides by the full length (AstHist.third/fourth_moment)
            m2 = ss / n
            res.append((sk / n) / (m2 ** (k / 2.0)) if m2 > 0 else float("nan"))
        return res

    def skewness(self, na_rm=False):
        """Per-column skewness m3/m2^1.5 (advmath/AstSkewness.java)."""
        return self._moment(3, na_rm)

    def kurtosis(self, na_rm=False):
        """Per-column (non-excess) kurtosis m4/m2^2 (advmath/AstKurtosis.java)."""
        return self._moment(4, na_rm)

    def insert_missing_values(self, fraction=0.1, seed=None):
        """Replace ~fraction of all values with NA, in place (hex/MissingInserter.java)."""
        gen = torch.Generator(device="cpu").manual_seed(int(seed if seed is not None and seed >= 0 else
                                                            np.random.randint(1 << 30)) + cloud.rank())
        for i, v in enumerate(self._vecs):
            m = torch.rand(v.nlocal, generator=gen) < fraction
            if v.on_host:
                arr = np.array(v.data, dtype=object)
                arr[m.numpy()] = None
                nv = Vec(arr, v.type)
            elif v.type == T_ENUM:
                nv = Vec(torch.where(m.to(v.data.device), torch.full_like(v.data, -1), v.data), T_ENUM, v.domain)
            else:
                d = v.data if v.data.is_floating_point() else v.data.to(torch.float32)
                nv = Vec(torch.where(m.to(d.device), torch.full_like(d, float("nan")), d), v.type)
            self._vecs[i] = nv
        return self

    def interaction(self, factors, pairwise, max_factors, min_occurrence, destination_frame=None):
        from .munging import interaction
        return interaction(self, factors, pairwise, max_factors, min_occurrence)

    def rep_len(self, length_out):
        """Repeat rows (or the single column's values) cyclically to length_out (AstRepLen)."""
        g = self.gather()
        n = g.nrows
        if self.ncols > 1 and n == 1:
            # reference: replicate the columns of a one-row frame
            k = length_out
            vecs = [g._vecs[j % self.ncols] for j in range(k)]
            return H2OFrame.from_vecs(vecs, [f"C{j + 1}" for j in range(k)])
        idx = torch.arange(length_out, device=_dev()) % max(n, 1)
        return _reshard(H2OFrame.from_vecs([_take(v, idx) for v in g._vecs], self._names))

    def topNBottomN(self, column=0, nPercent=10, grabTopN=-1):
        from .munging import topn
        return topn(self, column, nPercent, grabTopN)

    def bottomN(self, column=0, nPercent=10):
        return self.topNBottomN(column, nPercent, -1)

    def isax(self, num_words, max_cardinality, optimize_card=False, **kwargs):
        """iSAX index of row-wise time series (timeseries/AstIsax.java): PAA word means
        z-scored by the series mean/std, bucketed at the N(0,1) quantiles."""
        from scipy.stats import norm
        if num_words <= 0 or max_cardinality <= 0:
            raise ValueError("num_words and max_cardinality must be > 0")
        x = self.to_tensor(dtype=torch.float64)
        step = max(self.ncols // num_words, 1)
        words, sums, cnt, sse = [], 0.0, 0, 0.0
        for w in range(num_words):
            seg = x[:, w * step: (w + 1) * step]
            if seg.shape[1] == 0:
                break
            m = seg.mean(1)
            words.append(m)
            sums = sums + seg.sum(1)
            cnt += seg.shape[1]
            # Welford inside a word, the reference's quirk
            sse = sse + ((seg - m[:, None]) ** 2).sum(1)
        mu = sums / cnt
        sd = torch.sqrt(sse / (cnt - 1))
        bounds = torch.tensor([norm.ppf(i / max_cardinality) for i in range(1, max_cardinality)],
                              dtype=torch.float64, device=x.device)
        toks = [torch.searchsorted(bounds, ((wm - mu) / sd).contiguous(), right=False).clamp(max=max_cardinality - 1)
                for wm in words]
        cards = [max_cardinality] * len(toks)
        if optimize_card:
            for i, t in enumerate(toks):
                u = torch.unique(coll.all_gather_var(t) if cloud.is_distributed() else t)
                cards[i] = int(u.numel())
                if cards[i] < max_cardinality:
                    toks[i] = torch.searchsorted(u, t)
        tok_np = [t.cpu().numpy() for t in toks]
        strs = ["_".join(f"{int(tok_np[w][r])}^{cards[w]}" for w in range(len(toks))) for r in range(x.shape[0])]
        vecs = [make_string(strs)] + [Vec(t.to(torch.float64), T_INT) for t in toks]
        return H2OFrame.from_vecs(vecs, ["iSax_index"] + [f"c{i}" for i in range(len(toks))])

    @staticmethod
    def mktime(year=1970, month=0, day=0, hour=0, minute=0, second=0, msec=0):
        """Epoch milliseconds from calendar fields; month and day are 0-based like the
        reference (time/AstMktime.java).  Arguments are scalars or single-column frames."""
        import pandas as pd
        parts = [year, month, day, hour, minute, second, msec]
        n = max((p.nlocal for p in parts if isinstance(p, H2OFrame)), default=1)
        cols = []
        for p in parts:
            if isinstance(p, H2OFrame):
                cols.append(p._vecs[0].as_float(torch.float64).cpu().numpy())
            else:
                cols.append(np.full(n, float(p)))
        y, mo, d, h, mi, s, ms = cols
        bad = np.zeros(n, dtype=bool)
        for c in cols:
            bad |= np.isnan(c)
        cl = [np.nan_to_num(c).astype(np.int64) for c in cols]
        ts = pd.to_datetime(pd.DataFrame({"year": cl[0], "month": cl[1] + 1, "day": cl[2] + 1, "hour": cl[3],
                                          "minute": cl[4], "second": cl[5]}), utc=True)
        out = (ts.astype("int64") // 10 ** 6).values.astype(np.float64) + cl[6]
        out[bad] = np.nan
        return H2OFrame.from_vecs([make_time(out)], ["mktime"])

    def save(self, path, force=True):
        """Binary frame export (h2o.save_frame / Frame export): see core/frame_io.py."""
        from .frame_io import save_frame
        return save_frame(self, path, force=force)

    def convert_H2OFrame_2_DMatrix(self, predictors, yresp, h2oXGBoostModel=None, in_place=False):
        """Dense (X, y) numpy export; returns an xgboost.DMatrix when xgboost is importable."""
        X = self.gather().to_tensor(predictors, dtype=torch.float32).cpu().numpy()
        y = self.gather().vec(yresp).as_float(torch.float32).cpu().numpy()
        try:
            import xgboost
            return xgboost.DMatrix(X, label=y)
        except ImportError:
            return X, y

    def save_to_hive(self, jdbc_url, table_name, format="csv", table_path=None, tmp_path=None):
        raise NotImplementedError("Hive export needs a JDBC/Hive stack, which this platform does not ship")

    # strings & time (delegated)
    @staticmethod
    def moment(year=None, month=None, day=None, hour=None, minute=None, second=None, msec=None, date=None,
               time=None):
        """Time column from its parts (h2o-py frame.py H2OFrame.moment, a staticmethod)."""
        from . import timeops
        return timeops.moment(year=year, month=month, day=day, hour=hour, minute=minute, second=second, msec=msec,
                              date=date, time=time)

    def __getattr__(self, name):
        from . import strings, timeops
        if name.startswith("__"):
            raise AttributeError(name)
        for mod in (strings, timeops):
            fn = getattr(mod, name, None)
            if fn is not None and callable(fn) and not name.startswith("_"):
                return lambda *a, **k: fn(self, *a, **k)
        raise AttributeError(name)

    def refresh(self):
        return self

    def structure(self):
        print(self.types)

    def frame_id_(self):
        return self.frame_id

    def deep_copy(self, xid=None):
        fr = H2OFrame.from_vecs([v.copy() for v in self._vecs], self._names, frame_id=xid)
        return fr


# ---------------------------------------------------------------- helpers
def _num_or(s):
    try:
        f = float(s)
        return int(f) if f.is_integer() else f
    except (TypeError, ValueError):
        return s


def _try_float(x):
    try:
        float(x)
        return True
    except (TypeError, ValueError):
        return False


def _take(v: Vec, idx: torch.Tensor) -> Vec:
    if v.on_host:
        return Vec(v.data[idx.cpu().numpy()], v.type)
    return Vec(v.data[idx], v.type, v.domain)


def _where_vec(mask, new: Vec, old: Vec) -> Vec:
    if old.type == T_ENUM and new.type == T_ENUM:
        dom = list(old.domain)
        for d in new.domain:
            if d not in dom:
                dom.append(d)
        remap = torch.tensor([dom.index(d) for d in new.domain] or [0], dtype=torch.int32, device=_dev())
        nd = torch.where(new.data < 0, new.data, remap[new.data.clamp(min=0).long()])
        nd = nd.expand_as(old.data) if nd.numel() == 1 else nd
        return Vec(torch.where(mask, nd, old.data), T_ENUM, dom)
    if old.on_host or new.on_host:
        o = np.array(old.to_numpy(), dtype=object)
        nn = np.array(new.to_numpy(), dtype=object)
        m = mask.cpu().numpy()
        o[m] = nn[m] if len(nn) == len(o) else nn[0]
        return Vec(o, T_STR)
    a = new.as_float(torch.float64)
    b = old.as_float(torch.float64)
    if a.numel() == 1:
        a = a.expand_as(b)
    r = torch.where(mask, a, b)
    t = T_INT if (old.type == T_INT and new.type == T_INT) else T_REAL
    return Vec(r.to(old.data.dtype if old.data.is_floating_point() else torch.float32), t)


def _to_enum(v: Vec) -> Vec:
    if v.type == T_ENUM:
        return v
    if v.on_host:
        return make_enum_from_strings(list(v.data))
    x = v.as_float(torch.float64)
    nan = torch.isnan(x)
    uniq = torch.unique(x[~nan])
    if cloud.is_distributed():
        uniq = torch.unique(coll.all_gather_var(uniq))
    vals = uniq.tolist()
    dom = [_fmt_level(u) for u in vals]
    codes = torch.searchsorted(uniq, torch.where(nan, torch.zeros_like(x), x)).to(torch.int32)
    codes = torch.where(nan, torch.full_like(codes, -1), codes)
    return Vec(codes, T_ENUM, dom)


def _reshard(fr: H2OFrame) -> H2OFrame:
    """Turn a frame that is replicated on every rank back into row shards."""
    if not cloud.is_distributed():
        return fr
    s, e = _local_slice(fr.nlocal)
    idx = torch.arange(s, e, device=_dev())
    out = []
    for v in fr._vecs:
        nv = _take(v, idx)
        nv.replicated = False
        out.append(nv)
    return H2OFrame.from_vecs(out, fr._names)
