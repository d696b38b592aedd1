"""bf16 [hi | lo] Gram GEMM for wide GLMs (P = 1024, the per-GPU share of the
100M x 1000 config): one GEMM per 512K-row chunk (current) vs batched GEMMs
over g chunks (more output tiles in flight) -- time and accuracy."""
import os
import sys
import time

import torch

N = int(os.environ.get("N", 12_500_000))
Pa = 1024
st = 1 << 19
nch = -(-N // st)
torch.manual_seed(0)
# one bf16 [hi | lo] buffer for all rows (51 GB at 12.5M x 2048)
HL = torch.empty((nch * st, 2 * Pa), dtype=torch.bfloat16, device="cuda")
for a in range(0, nch * st, 1 << 20):
    x = torch.randn(min(1 << 20, nch * st - a), Pa, device="cuda")
    hi = x.to(torch.bfloat16)
    HL[a:a + x.shape[0], :Pa] = hi
    HL[a:a + x.shape[0], Pa:] = (x - hi.float()).to(torch.bfloat16)
HL[N:] = 0


def per_chunk():
    G = torch.zeros((Pa, 2 * Pa), dtype=torch.float64, device="cuda")
    for i in range(nch):
        H = HL[i * st:(i + 1) * st]
        G += torch.mm(H[:, :Pa].T, H, out_dtype=torch.float32).to(torch.float64)
    return G


def batched(g):
    def f():
        G = torch.zeros((Pa, 2 * Pa), dtype=torch.float64, device="cuda")
        for b in range(0, nch, g):
            e = min(nch, b + g)
            H3 = HL[b * st:e * st].view(e - b, st, 2 * Pa)
            C = torch.bmm(H3[:, :, :Pa].transpose(1, 2), H3, out_dtype=torch.float32)
            G += C.to(torch.float64).sum(0)
        return G
    return f


ref = None
for name, fn in [("per-chunk mm", per_chunk), ("bmm g=4", batched(4)), ("bmm g=8", batched(8)),
                 ("bmm g=all", batched(nch))]:
    try:
        G = fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            G = fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 3 * 1e3
    except Exception as e:  # noqa: BLE001
        print(f"{name}: failed {type(e).__name__}: {e}", flush=True)
        continue
    if ref is None:
        ref = G
    err = float((G - ref).abs().max() / ref.abs().max())
    tf = 2 * N * Pa * 2 * Pa / ms / 1e9
    print(f"{name:14s} {ms:8.2f} ms  {tf:7.1f} TFLOP/s  diff vs per-chunk {err:.1e}", flush=True)
