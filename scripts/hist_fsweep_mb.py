"""Histogram cost vs feature count and group width: is the quad kernel bound
per feature-group pass (loads/issue) or by LDS atomics?  F = 96 / 100 / 128 at
Fp = 128, FG = 32 / 64, root level (contiguous) and a scattered depth-3 level."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.models.tree.binning import BinnedData  # noqa: E402
from h2o3_amd.ops import tree_ops  # noqa: E402

N = int(os.environ.get("N", 100_000_000))
Fp, Bs = 128, 256
dev = "cuda"
codes = torch.randint(0, 254, (N, Fp), dtype=torch.uint8, device=dev)
va = torch.randn(N, device=dev)
vmax = tree_ops.channel_max(va, None, 0)
ident = torch.arange(N, dtype=torch.int32, device=dev)
g = torch.Generator(device=dev).manual_seed(3)
nid = torch.randint(0, 8, (N,), generator=g, device=dev)
order = torch.argsort(nid, stable=True).to(torch.int32)
cnt = torch.bincount(nid, minlength=8).cpu().tolist()
st = [0]
for c in cnt[:-1]:
    st.append(st[-1] + c)


def run(name, bd, ridx, starts, counts, reps=5):
    kw = dict(vmax=vmax, unit_w=True, posv=True, want_wyy=True)
    tree_ops.hist_build(bd, ridx, va, None, 0, starts, counts, len(starts), **kw)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        tree_ops.hist_build(bd, ridx, va, None, 0, starts, counts, len(starts), **kw)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    rows = sum(counts)
    print(f"{name:44s} {ms:7.2f} ms  {rows * bd.F / ms / 1e9:6.3f} G row-feat/ms", flush=True)


for F in (96, 100, 128):
    bd = BinnedData()
    bd.codes = codes
    bd.F, bd.Fp, bd.Bs, bd.code_bytes, bd.nrows_local = F, Fp, Bs, 1, N
    for kern in os.environ.get("KERNELS", "row,quad").split(","):
        os.environ["H2O3_HIST_KERNEL"] = kern
        run(f"F={F} {kern} root", bd, ident, [0], [N])
        b = [0, 2, 4, 6]
        run(f"F={F} {kern} depth3 4 scattered nodes", bd, order, [st[i] for i in b], [cnt[i] for i in b])
