"""Micro-benchmark of the GLM IRLS kernels at the bench shape (100M x 100 -> Pp 128)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.ops import linalg_ops  # noqa: E402

N = int(os.environ.get("N", 100_000_000))
P, Pp = 100, 128
torch.manual_seed(0)
X = torch.zeros((N, Pp), device="cuda")
X[:, :P].normal_()
beta = torch.zeros(Pp, device="cuda")
beta[:P] = 0.01 * torch.randn(P, device="cuda")
y = (torch.rand(N, device="cuda") < 0.5).float()
W = torch.rand(N, device="cuda")


def t(name, f, reps=5):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    gb = N * Pp * 4 / 1e9
    print(f"{name:28s} {ms:8.2f} ms  {gb / ms:6.2f} TB/s eff", flush=True)


t("fused binomial", lambda: linalg_ops.glm_irls(X, aug=P, beta=beta, b0=0.1, y=y, codes=(1, 1)))
t("external W,z", lambda: linalg_ops.glm_irls(X, aug=P, W=W, z=y))
t("gram W only", lambda: linalg_ops.glm_irls(X, W=W))
t("torch X@beta", lambda: X @ beta)
t("torch X.sum(0)", lambda: X.sum(0))
if os.environ.get("DBG_SWEEP"):
    import ctypes
    for d in ("1", "2", "3"):
        os.environ["H2O3_GI_DBG"] = d
        # the library caches the env on first use -> run in a subprocess
        import subprocess
        code = ("import os,sys,time,torch;sys.path.insert(0,'.');from h2o3_amd.ops import linalg_ops as l;"
                f"N={N};X=torch.zeros((N,128),device='cuda');W=torch.rand(N,device='cuda');"
                "l.glm_irls(X,aug=100,W=W,z=W);torch.cuda.synchronize();t=time.perf_counter();"
                "[l.glm_irls(X,aug=100,W=W,z=W) for _ in range(5)];torch.cuda.synchronize();"
                "print('dbg', os.environ['H2O3_GI_DBG'], (time.perf_counter()-t)/5*1e3, 'ms', flush=True)")
        subprocess.run([sys.executable, "-c", code], check=True, env=dict(os.environ))
