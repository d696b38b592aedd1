"""Microbenchmark for PMC / timing: one K-Means split-path Lloyd pass at
N x 100, k = 128 (assignment kernel + sums kernel) and the DL GEMM shapes of a
hidden=[1024, 1024] batch-1024 step.  Usage: python scripts/km_dl_mb.py [N]."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.ops import cluster_ops, dl_ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn((N, 100), generator=g, device=dev)
C = X[:128].double() + 0.01
a = torch.full((N,), -1, dtype=torch.int32, device=dev)
xa = cluster_ops.abs_bound(X)
for _ in range(2):
    cluster_ops.lloyd_pass(X, C, None, a, xabs_max=xa)
torch.cuda.synchronize()
t0 = time.perf_counter()
R = 5
for _ in range(R):
    cluster_ops.lloyd_pass(X, C, None, a, xabs_max=xa)
torch.cuda.synchronize()
print(f"kmeans k=128 N={N}: {(time.perf_counter() - t0) / R * 1e3:.3f} ms/pass", flush=True)
del X
B, H, F = 1024, 1024, 100
A0 = torch.randn((B, F), device=dev)
W1 = torch.randn((H, F), device=dev)
A1 = torch.randn((B, H), device=dev)
W2 = torch.randn((H, H), device=dev)
Wo = torch.randn((2, H), device=dev)
dZ2 = torch.randn((B, H), device=dev)
dZo = torch.randn((B, 2), device=dev)
shapes = {
    "Z1=A0 W1^T": lambda: dl_ops.gemm(A0, W1.t()),
    "Z2=A1 W2^T": lambda: dl_ops.gemm(A1, W2.t()),
    "Zo=A2 Wo^T": lambda: dl_ops.gemm(A1, Wo.t()),
    "dWo=dZo^T A2": lambda: dl_ops.gemm(dZo.t(), A1),
    "dA2=dZo Wo": lambda: dl_ops.gemm(dZo, Wo),
    "dW2=dZ2^T A1": lambda: dl_ops.gemm(dZ2.t(), A1),
    "dA1=dZ2 W2": lambda: dl_ops.gemm(dZ2, W2),
    "dW1=dZ1^T A0": lambda: dl_ops.gemm(dZ2.t(), A0),
}
for name, f in shapes.items():
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        f()
    torch.cuda.synchronize()
    print(f"gemm {name}: {(time.perf_counter() - t0) / 50 * 1e6:.1f} us", flush=True)
