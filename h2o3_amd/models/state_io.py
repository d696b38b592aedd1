"""Full estimator state archives for binary save / load.

Reference: hex/Model.exportBinaryModel / importBinaryModel write the whole
Java model object, so a loaded model is the same model -- it scores, it
keeps its outputs and metrics, and it can be a checkpoint to continue
training.  Here the estimator's attribute tree is flattened into plain
containers (dict / list / tuple / str / numbers / None) plus a list of
tensors and written with torch.save; loading uses torch.load(weights_only=True),
which executes nothing from the file, and re-creates only classes of this
package (module names are checked against the h2o3_amd prefix).

Training-only state is dropped: the training / validation frames referenced
by the parameters and the TrainSpec, IRLS drivers, jobs, RNG objects and
anything that is not data (functions, streams, graphs).
"""
from __future__ import annotations

import importlib
import io

import numpy as np
import torch

_PREFIX = "h2o3_amd."
_SKIP_ATTRS = {"_job", "_drv", "_lg", "_lg_key", "_pen_cache", "_graph", "_ea"}
# estimator attributes holding per-rank ROW SHARDS as plain tensors (dim 0 =
# this rank's rows): cross-validation holdout predictions, the GLRM row
# representation X
_SHARDED_ATTRS = {"_cv_holdout", "_X"}


class _Packer:
    """gather=True (multi-rank save, called on EVERY rank in the same order):
    row-sharded state -- non-replicated Vecs and the _SHARDED_ATTRS tensors of
    estimators -- is all-gathered into whole-frame arrays marked "sharded", so
    the archive holds every row; loading re-shards them to the loading cloud."""

    def __init__(self, gather=False):
        self.tensors = []
        self.memo = {}
        self.gather = gather

    def t(self, x):
        self.tensors.append(x.detach().to("cpu").contiguous().clone())
        return len(self.tensors) - 1

    def pack(self, obj, depth=0):
        if depth > 200:
            return {"__skip": "depth"}
        if obj is None or type(obj) in (bool, int, float, str):
            return obj
        if isinstance(obj, np.generic):
            return self.pack(obj.item(), depth + 1)
        for base in (bool, int, float, str):          # subclasses (enums, numpy floats)
            if isinstance(obj, base):
                return base(obj)
        if isinstance(obj, torch.Tensor):
            return {"__t": self.t(obj), "dev": obj.device.type}
        if isinstance(obj, np.ndarray):
            if obj.dtype == object or obj.dtype.kind in "USV":
                return {"__nplist": self.pack(obj.tolist(), depth + 1), "shape": list(obj.shape),
                        "dtype": "object" if obj.dtype == object else str(obj.dtype)}
            return {"__np": self.t(torch.from_numpy(np.ascontiguousarray(obj)))}
        if isinstance(obj, list):
            return [self.pack(x, depth + 1) for x in obj]
        if isinstance(obj, tuple):
            return {"__tuple": [self.pack(x, depth + 1) for x in obj]}
        if isinstance(obj, (set, frozenset)):
            return {"__set": [self.pack(x, depth + 1) for x in obj]}
        if isinstance(obj, dict):
            if all(isinstance(k, str) for k in obj):
                return {"__dict": {k: self.pack(v, depth + 1) for k, v in obj.items()}}
            return {"__kvs": [[self.pack(k, depth + 1), self.pack(v, depth + 1)] for k, v in obj.items()]}
        import pandas as pd
        if isinstance(obj, pd.DataFrame):
            return {"__df": {str(c): self.pack(obj[c].to_numpy(), depth + 1) for c in obj.columns},
                    "cols": [str(c) for c in obj.columns]}
        if isinstance(obj, pd.Series):
            return {"__series": self.pack(obj.to_numpy(), depth + 1), "name": str(obj.name),
                    "index": self.pack(obj.index.to_numpy(), depth + 1)}
        from ..core.vec import Vec
        if isinstance(obj, Vec):
            if self.gather and not obj.replicated:
                from ..parallel import collectives as coll
                if obj.on_host:
                    data = np.array(sum(coll.all_gather_object(list(obj.data)), []), dtype=object)
                else:
                    data = coll.all_gather_var(obj.data)
                return {"__vec": {"data": self.pack(data, depth + 1), "type": obj.type,
                                  "domain": self.pack(obj.domain, depth + 1), "replicated": False,
                                  "sharded": True}}
            return {"__vec": {"data": self.pack(obj.data, depth + 1), "type": obj.type,
                              "domain": self.pack(obj.domain, depth + 1), "replicated": bool(obj.replicated)}}
        cls = type(obj)
        mod = cls.__module__ or ""
        if not (mod.startswith(_PREFIX) and hasattr(obj, "__dict__")):
            return {"__skip": f"{mod}.{cls.__qualname__}"}
        key = id(obj)
        if key in self.memo:
            return {"__ref": self.memo[key]}
        ref = len(self.memo)
        self.memo[key] = ref
        state = dict(obj.__dict__)
        from .base import TrainSpec, H2OEstimator
        from ..core.frame import H2OFrame
        if isinstance(obj, TrainSpec):
            state["frame"] = None
            state["valid"] = None
        if isinstance(obj, H2OEstimator):
            parms = {}
            for k, v in state.get("_parms", {}).items():
                parms[k] = None if isinstance(v, H2OFrame) else v
            state["_parms"] = parms
        for k in _SKIP_ATTRS:
            state.pop(k, None)
        packed = {}
        for k, v in state.items():
            if self.gather and k in _SHARDED_ATTRS and isinstance(obj, H2OEstimator) and \
                    isinstance(v, torch.Tensor) and v.dim() >= 1:
                from ..parallel import collectives as coll
                packed[k] = {"__t": self.t(coll.all_gather_var(v.detach().contiguous())), "dev": v.device.type,
                             "sharded": True}
            else:
                packed[k] = self.pack(v, depth + 1)
        return {"__obj": f"{mod}:{cls.__qualname__}", "id": ref, "state": {"__dict": packed}}


class _Unpacker:
    def __init__(self, tensors, device):
        self.tensors = tensors
        self.device = device
        self.memo = {}

    def unpack(self, x):
        if x is None or isinstance(x, (bool, int, float, str)):
            return x
        if isinstance(x, list):
            return [self.unpack(v) for v in x]
        if not isinstance(x, dict):
            return x
        if "__t" in x:
            t = self.tensors[x["__t"]]
            if x.get("sharded"):
                t = self._local(t)
            return t.to(self.device) if x.get("dev") == "cuda" and self.device.type == "cuda" else t
        if "__np" in x:
            return self.tensors[x["__np"]].numpy()
        if "__nplist" in x:
            vals = self.unpack(x["__nplist"])
            return np.array(vals, dtype=object if x.get("dtype") == "object" else x.get("dtype"))
        if "__tuple" in x:
            return tuple(self.unpack(v) for v in x["__tuple"])
        if "__set" in x:
            return set(self.unpack(v) for v in x["__set"])
        if "__dict" in x:
            return {k: self.unpack(v) for k, v in x["__dict"].items()}
        if "__kvs" in x:
            return {self._hashable(self.unpack(k)): self.unpack(v) for k, v in x["__kvs"]}
        if "__df" in x:
            import pandas as pd
            cols = x["cols"]
            return pd.DataFrame({c: self.unpack(x["__df"][c]) for c in cols}, columns=cols)
        if "__series" in x:
            import pandas as pd
            return pd.Series(self.unpack(x["__series"]), name=x["name"], index=self.unpack(x["index"]))
        if "__vec" in x:
            from ..core.vec import Vec
            d = x["__vec"]
            data = self.unpack(d["data"])
            if d.get("sharded"):
                data = self._local(data)
            v = Vec(data, d["type"], self.unpack(d["domain"]))
            v.replicated = d["replicated"]
            return v
        if "__skip" in x:
            return None
        if "__ref" in x:
            return self.memo.get(x["__ref"])
        if "__obj" in x:
            mod, qual = x["__obj"].split(":", 1)
            if not mod.startswith(_PREFIX):
                raise ValueError(f"refusing to restore a class outside the package: {mod}")
            cls = importlib.import_module(mod)
            for part in qual.split("."):
                cls = getattr(cls, part)
            if not isinstance(cls, type) or not (cls.__module__ or "").startswith(_PREFIX):
                raise ValueError(f"refusing to restore a class outside the package: {x['__obj']}")
            inst = cls.__new__(cls)
            self.memo[x["id"]] = inst
            inst.__dict__.update(self.unpack(x["state"]))
            return inst
        return {k: self.unpack(v) for k, v in x.items()}

    @staticmethod
    def _local(t):
        """This rank's row shard of a whole-frame array saved by a gathering
        pack (the frame layout of core/frame._local_slice)."""
        from ..core.frame import _local_slice
        a, b = _local_slice(len(t))
        return t[a:b]

    @staticmethod
    def _hashable(k):
        if isinstance(k, list):
            return tuple(_Unpacker._hashable(v) for v in k)
        return k


def dumps(est, gather=False) -> bytes:
    """gather=True: multi-rank save, a collective -- every rank must call it."""
    p = _Packer(gather)
    tree = p.pack(est)
    buf = io.BytesIO()
    torch.save({"format": 1, "tree": tree, "tensors": p.tensors}, buf)
    return buf.getvalue()


def loads(data: bytes):
    from ..parallel import cloud
    blob = torch.load(io.BytesIO(data), map_location="cpu", weights_only=True)
    if blob.get("format") != 1:
        raise ValueError("unknown model state format")
    return _Unpacker(blob["tensors"], cloud.device()).unpack(blob["tree"])
