"""f64 weighted Gram of [X | 1] at 1M x 711 (RuleFit's rule-matrix width):
f64-MFMA kernel vs the torch f64 GEMM path it replaces."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.ops import linalg_ops  # noqa: E402

N, P = int(os.environ.get("ROWS", 1_000_000)), int(os.environ.get("COLS", 711))
g = torch.Generator(device="cuda").manual_seed(0)
LD = int(os.environ.get("LDX", -(-P // 4) * 4))       # row pitch (16-byte rows: vector loads)
Xs = (torch.rand((N, LD), generator=g, device="cuda") > 0.7).float()
X = Xs[:, :P]
W = torch.rand(N, generator=g, device="cuda", dtype=torch.float64)
print(f"N={N} P={P} ldx={LD}")


def torch_path():
    Xa = torch.cat([X.double(), torch.ones((N, 1), dtype=torch.float64, device="cuda")], 1)
    return (Xa * W.view(-1, 1)).T @ Xa


def mfma_path():
    return linalg_ops.gram_f64_aug(X, P, W)


for name, fn in (("mfma_f64", mfma_path), ("torch_f64", torch_path)):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        G = fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 5 * 1e3
    fl = 2.0 * N * (P + 1) ** 2
    print(f"{name:10s} {ms:8.2f} ms  {fl / ms / 1e9:7.1f} TFLOP/s (full square)", flush=True)
print("max rel diff", float(((mfma_path() - torch_path()).abs() / torch_path().abs().clamp_min(1e-300)).max()))
