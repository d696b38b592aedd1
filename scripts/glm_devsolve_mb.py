"""Microbenchmark: the (P+1)^2 IRLS system on the device vs the host.

Times, at P + 1 = 1001 (the wide GLM bench), the pieces of one IRLS step's
host work -- f64 Cholesky, triangular solves, a 1-norm condition estimate --
with torch on the GPU (rocSOLVER / rocBLAS f64) and with numpy / scipy
LAPACK on the box's CPU share, plus the 8 MB device -> host copy the host
path needs."""
import sys
import time

import numpy as np
import torch

P = int(sys.argv[1]) if len(sys.argv) > 1 else 1001
dev = torch.device("cuda")
A = torch.randn(20000, P, dtype=torch.float64, device=dev)
G = (A.T @ A) / 20000
b = torch.randn(P, dtype=torch.float64, device=dev)


def tdev(f, n=10):
    f()
    torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - s) / n * 1e3


def thost(f, n=5):
    f()
    s = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - s) / n * 1e3


def hager(L, n):
    x = torch.full((n, 1), 1.0 / n, dtype=L.dtype, device=L.device)
    est = 0.0
    for k in range(5):
        y = torch.cholesky_solve(x, L)
        est = float(y.abs().sum())
        z = torch.cholesky_solve(torch.sign(y), L)
        za = z.abs()
        j = int(za.argmax())
        if k > 0 and float(za[j]) <= float((z * x).sum()):
            break
        x = torch.zeros_like(x)
        x[j] = 1.0
    return est


L = torch.linalg.cholesky(G)
print(f"P={P}")
print(f"dev cholesky        {tdev(lambda: torch.linalg.cholesky(G)):8.3f} ms")
print(f"dev cholesky_ex     {tdev(lambda: torch.linalg.cholesky_ex(G)):8.3f} ms")
print(f"dev cholesky_solve  {tdev(lambda: torch.cholesky_solve(b.view(-1, 1), L)):8.3f} ms")
G32 = G.float()
print(f"dev cholesky f32    {tdev(lambda: torch.linalg.cholesky_ex(G32)):8.3f} ms")
L32 = torch.linalg.cholesky(G32)
print(f"dev chol_solve f32  {tdev(lambda: torch.cholesky_solve(b.float().view(-1, 1), L32)):8.3f} ms")
print(f"dev inverse f64     {tdev(lambda: torch.cholesky_inverse(L)):8.3f} ms")
print(f"dev hager estimate  {tdev(lambda: hager(L, P)):8.3f} ms")
print(f"dev gemv            {tdev(lambda: G @ b):8.3f} ms")
print(f"dev->host copy      {tdev(lambda: G.cpu()):8.3f} ms")
Gh, bh = G.cpu().numpy(), b.cpu().numpy()
import scipy.linalg as sla
from scipy.linalg import lapack
print(f"host cho_factor+solve {thost(lambda: sla.cho_solve(sla.cho_factor(Gh, lower=True, check_finite=False), bh, check_finite=False)):8.3f} ms")
print(f"host dpotrf           {thost(lambda: lapack.dpotrf(np.asfortranarray(Gh), lower=1, clean=0, overwrite_a=1)):8.3f} ms")
c, _ = lapack.dpotrf(np.asfortranarray(Gh), lower=1, clean=0)
anorm = float(np.abs(Gh).sum(0).max())
rc, _ = lapack.dpocon(c, anorm, uplo="L")
print(f"kappa dpocon {1 / rc:.4g}  hager {hager(L, P) * anorm:.4g}")
