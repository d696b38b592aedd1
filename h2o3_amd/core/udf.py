"""User-defined metric and distribution functions.

Reference: `h2o.upload_custom_metric` / `h2o.upload_custom_distribution`
(h2o-py/h2o/h2o.py:2130, :2232) ship Python source as a jar to the cluster,
where Jython runs it behind the `water.udf.CMetricFunc` /
`CDistributionFunc` interfaces (h2o-core/src/main/java/water/udf/*).  Here the
cluster is this process group, so the class is registered directly in a
key -> class table; the returned reference string has the same
`python:<key>=<module>.<Class>Wrapper` shape the estimators accept.

Metric classes implement map(pred, act, w, o, model) -> list, reduce(l, r)
-> list and metric(l) -> float, evaluated per row like the reference.  An
optional vectorised `map_tensor(pred, act, w, o)` returning an [n, k] tensor
whose column sums are the reduced state is used on the GPU when present.

Distribution classes implement link() -> str, init(w, o, y) -> [num, den],
gradient(y, f) -> float, gamma(w, y, z, f) -> [num, den]; they are first
called with whole device tensors (most user formulas are plain arithmetic and
vectorise as-is) and fall back to a per-row loop if that fails.
"""
from __future__ import annotations

import inspect
import textwrap

import numpy as np
import torch

from . import dkv

_REGISTRY: dict[str, type] = {}


def _register(func, func_file, func_name, class_name, kind, methods):
    if not (inspect.isclass(func) or isinstance(func, str)):
        raise TypeError("func needs to be a class or a string with the class source")
    if not func_file.endswith(".py"):
        raise ValueError("func_file needs to end with '.py'")
    module = func_file[:-3]
    if isinstance(func, str):
        if not class_name:
            raise ValueError("class_name is required when func is given as a string")
        ns: dict = {}
        exec(compile(textwrap.dedent(func), f"<{func_file}>", "exec"), ns)  # user-supplied UDF source
        cls = ns[class_name]
    else:
        if class_name is not None:
            raise ValueError("class_name must be None when func is a class")
        cls = func
        class_name = func.__name__
    for m in methods:
        if not hasattr(cls, m):
            raise ValueError(f"the {kind} class needs to define method `{m}`")
    key = func_name or f"{kind}s_{class_name}"
    _REGISTRY[key] = cls
    dkv.put(key, cls)
    return f"python:{key}={module}.{class_name}Wrapper"


def upload_custom_metric(func, func_file="metrics.py", func_name=None, class_name=None, source_provider=None):
    return _register(func, func_file, func_name, class_name, "metric", ("map", "reduce", "metric"))


def upload_custom_distribution(func, func_file="distributions.py", func_name=None, class_name=None,
                               source_provider=None):
    return _register(func, func_file, func_name, class_name, "distribution",
                     ("link", "init", "gradient", "gamma"))


def resolve(ref):
    """Instance of the class behind a `python:key=module.ClassWrapper` reference
    (a class or an instance is also accepted)."""
    if ref is None:
        return None
    if inspect.isclass(ref):
        return ref()
    if not isinstance(ref, str):
        return ref
    body = ref[len("python:"):] if ref.startswith("python:") else ref
    key = body.split("=", 1)[0]
    if key not in _REGISTRY:
        raise KeyError(f"custom function '{key}' has not been uploaded")
    return _REGISTRY[key]()


def metric_name(ref):
    if isinstance(ref, str):
        body = ref[len("python:"):] if ref.startswith("python:") else ref
        return body.split("=", 1)[0]
    return type(ref).__name__ if not inspect.isclass(ref) else ref.__name__


def custom_metric_value(ref, pred: torch.Tensor, act: torch.Tensor, w=None, o=None, model=None,
                        domain=None) -> float:
    """Evaluate a custom metric.  `pred` rows follow the reference's layout:
    regression [value]; classification [label, p0, p1, ...]."""
    from ..parallel import cloud
    from ..parallel import collectives as coll
    fn = resolve(ref)
    n = pred.shape[0]
    if hasattr(fn, "map_tensor"):
        wt = torch.ones(n, dtype=torch.float64, device=pred.device) if w is None else w.to(torch.float64)
        ot = torch.zeros(n, dtype=torch.float64, device=pred.device) if o is None else o.to(torch.float64)
        st = fn.map_tensor(pred.to(torch.float64), act.to(torch.float64).view(n, -1), wt, ot)
        state = coll.allreduce_(st.sum(0).to(torch.float64)).cpu().tolist()
        return float(fn.metric(state))
    P = pred.detach().to(torch.float64).cpu().numpy()
    A = act.detach().to(torch.float64).cpu().numpy().reshape(n, -1)
    W = np.ones(n) if w is None else w.detach().to(torch.float64).cpu().numpy()
    O = np.zeros(n) if o is None else o.detach().to(torch.float64).cpu().numpy()
    state = None
    for i in range(n):
        if np.isnan(A[i, 0]):
            continue
        r = fn.map(P[i].tolist(), A[i].tolist(), float(W[i]), float(O[i]), model)
        state = r if state is None else fn.reduce(state, r)
    if cloud.is_distributed():
        parts = [s for s in coll.all_gather_object(state) if s is not None]
        state = None
        for s in parts:
            state = s if state is None else fn.reduce(state, s)
    return float(fn.metric(state)) if state is not None else float("nan")


class CustomDistribution:
    """Adapter exposing a user CDistributionFunc through the Distribution API
    used by the boosting drivers (models/distributions.py)."""
    family = "custom"

    def __init__(self, ref, **kw):
        self.fn = resolve(ref)
        self.link = str(self.fn.link()).lower()
        self.tweedie_power = kw.get("tweedie_power", 1.5)
        self.quantile_alpha = kw.get("quantile_alpha", 0.5)
        self.huber_alpha = kw.get("huber_alpha", 0.9)
        self.huber_delta = None

    @property
    def is_classification(self):
        return self.link == "logit"

    def _call(self, name, *args):
        f = getattr(self.fn, name)
        try:
            r = f(*args)
            if isinstance(r, (list, tuple)):
                r = [x if isinstance(x, torch.Tensor) else torch.full_like(args[0], float(x)) for x in r]
                if all(x.shape == args[0].shape for x in r):
                    return r
            elif isinstance(r, torch.Tensor) and r.shape == args[0].shape:
                return r
        except Exception:
            pass
        cols = [a.detach().to(torch.float64).cpu().numpy() for a in args]
        out = [f(*[float(c[i]) for c in cols]) for i in range(len(cols[0]))]
        dev, dt = args[0].device, args[0].dtype
        if out and isinstance(out[0], (list, tuple)):
            return [torch.tensor([o[k] for o in out], dtype=dt, device=dev) for k in range(len(out[0]))]
        return torch.tensor(out, dtype=dt, device=dev)

    def link_fn(self, mu):
        import math
        if self.link == "logit":
            mu = min(max(mu, 1e-15), 1 - 1e-15)
            return math.log(mu / (1 - mu))
        if self.link == "log":
            return math.log(max(mu, 1e-300))
        if self.link == "inverse":
            return 1.0 / mu
        return mu

    def linkinv(self, f):
        if self.link == "logit":
            return torch.sigmoid(f)
        if self.link == "log":
            return torch.exp(torch.clamp(f, max=88.0))
        if self.link == "inverse":
            return 1.0 / f
        return f

    def init_f(self, y, w, offset=None):
        from ..parallel import collectives as coll
        o = torch.zeros_like(y) if offset is None else offset.to(y.dtype)
        num, den = self._call("init", w.to(y.dtype), o, y)
        num = coll.allreduce_scalar(float(num.sum()))
        den = coll.allreduce_scalar(float(den.sum()))
        return self.link_fn(num / den if den != 0 else 0.0)

    def neg_half_gradient(self, y, f):
        return self._call("gradient", y, f)

    def gamma_num(self, w, y, z, f):
        return self._call("gamma", w, y, z, f)[0]

    def gamma_denom(self, w, y, z, f):
        return self._call("gamma", w, y, z, f)[1]

    def gamma(self, num, den):
        return num / den if den != 0 else 0.0

    def deviance(self, w, y, mu):
        return w * (y - mu) ** 2

    def grad_hess(self, y, f):
        return -self.neg_half_gradient(y, f), torch.ones_like(f)
