"""Weighted Gram X'WX for wide GLMs (P = 1024): HIP 32x32 tile-pair kernel vs
rocBLAS/hipBLASLt fp32 GEMM vs bf16x3 split GEMM (hi/lo) with fp32 output."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.ops import linalg_ops  # noqa: E402

N = int(os.environ.get("N", 12_500_000))
P = int(os.environ.get("P", 1024))
X = torch.randn(N, P, device="cuda")
w = torch.rand(N, device="cuda")
ref = None


def timeit(name, fn, reps=3):
    global ref
    g = fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g = fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    g = g.to(torch.float64)
    if ref is None:
        ref = g
    err = float((g - ref).abs().max() / ref.abs().max())
    print(f"{name:34s} {ms:9.2f} ms  {2 * N * P * P / ms / 1e9:8.1f} TFLOP/s  rel.err {err:.2e}", flush=True)


def hip():
    return linalg_ops.weighted_gram(X, w)


def fp32():
    Xs = X * w.sqrt().view(-1, 1)
    return Xs.T @ Xs


def bf16x3():
    Xs = X * w.sqrt().view(-1, 1)
    hi = Xs.to(torch.bfloat16)
    lo = (Xs - hi.float()).to(torch.bfloat16)
    kc = 1 << 18
    B = N // kc
    h3, l3 = hi[: B * kc].view(B, kc, P), lo[: B * kc].view(B, kc, P)
    G = torch.zeros(P, P, device="cuda", dtype=torch.float32)
    for a, b in ((h3, h3), (h3, l3), (l3, h3)):
        G += torch.bmm(a.transpose(1, 2), b).float().sum(0)
    return G


def bf16x3_out32():
    Xs = X * w.sqrt().view(-1, 1)
    hi = Xs.to(torch.bfloat16)
    lo = (Xs - hi.float()).to(torch.bfloat16)
    G = torch.mm(hi.T, hi, out_dtype=torch.float32)
    G += torch.mm(hi.T, lo, out_dtype=torch.float32)
    G += torch.mm(lo.T, hi, out_dtype=torch.float32)
    return G


def bf3_split():
    return linalg_ops.gram_aug_bf3(X, w, None, P - 2)[: P - 2, : P - 2]


def fp32_aug():
    return fp32()[: P - 2, : P - 2]


timeit("fp32 GEMM (aug width)", fp32_aug)
timeit("bf16 hi|lo split + 1 GEMM (HIP+hipBLASLt)", bf3_split)
ref = None
timeit("fp64 ref (X'WX via fp32 GEMM)", fp32)
timeit("HIP weighted_gram (32x32 tiles)", hip)
try:
    timeit("bf16x3 mm out_dtype=fp32", bf16x3_out32)
except Exception as e:  # noqa: BLE001
    print("out_dtype not supported:", repr(e)[:200])
timeit("bf16x3 bmm (k-chunked, bf16 out)", bf16x3)
