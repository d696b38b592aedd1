"""Binomial metric sketch at 6.7M rows: torch index_add path vs the
wave-aggregated HIP kernel, for constant / few-distinct / continuous scores."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.models import metrics as mm  # noqa: E402
from h2o3_amd.ops import metrics_ops  # noqa: E402

n, nb = 6_700_000, mm._NB_BIN
g = torch.Generator(device="cuda").manual_seed(1)
y = (torch.rand(n, generator=g, device="cuda") < 0.4).float()
cases = {"constant": torch.full((n,), 0.4, device="cuda"),
         "few64": torch.sigmoid(torch.randint(-32, 32, (n,), generator=g, device="cuda").float() / 8),
         "continuous": torch.rand(n, generator=g, device="cuda")}


def old(y, p):
    ok = ~torch.isnan(y) & ~torch.isnan(p)
    yy, pp = y[ok].double(), p[ok].double()
    w = torch.ones_like(yy)
    pc = pp.clamp(1e-15, 1 - 1e-15)
    s = torch.stack([w.sum(), -(w * (yy * pc.log() + (1 - yy) * (1 - pc).log())).sum(), (w * (yy - pp) ** 2).sum()])
    return mm._binomial_sketch(yy, pp, w), s


def new(y, p):
    return metrics_ops.logit_hist(y, p, None, nb)


for name, p in cases.items():
    for fn_name, fn in (("hip", new), ("torch", old)):
        # the torch path on constant scores serialises millions of f64
        # atomics on one address: time it on a 1/100 (constant) or 1/10 slice, once
        m = (n // 100 if name == "constant" else n // 10) if (fn_name == "torch" and name != "continuous") else n
        reps = 1 if fn_name == "torch" else 10
        fn(y[:m], p[:m])
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn(y[:m], p[:m])
        torch.cuda.synchronize()
        print(f"{name:11s} {fn_name:6s} rows {m:9d} {(time.perf_counter() - t) / reps * 1e3:10.3f} ms", flush=True)
t = time.perf_counter()
for _ in range(10):
    mm.binomial_metrics(y, cases["few64"], gainslift=False)
torch.cuda.synchronize()
print(f"binomial_metrics(few64, lite) {(time.perf_counter() - t) / 10 * 1e3:8.3f} ms", flush=True)
