"""Micro-benchmark: histogram build cost vs row scattering and node count
(100M x 100 uint8 codes, like the GBM bench's deep levels)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.models.tree.binning import BinnedData  # noqa: E402
from h2o3_amd.ops import tree_ops  # noqa: E402

N = int(os.environ.get("N", 100_000_000))
F, Fp, Bs = 100, int(os.environ.get('FP', 128)), 256
dev = "cuda"
bd = BinnedData()
bd.codes = torch.randint(0, 254, (N, Fp), dtype=torch.uint8, device=dev)
bd.F, bd.Fp, bd.Bs, bd.code_bytes, bd.nrows_local = F, Fp, Bs, 1, N
va = torch.randn(N, device=dev)
vb = torch.ones(N, device=dev)
vmax = tree_ops.channel_max(va, vb, 0)


def run(name, ridx, starts, counts, reps=5, **kw):
    tree_ops.hist_build(bd, ridx, va, vb, 0, starts, counts, len(starts), vmax=vmax, **kw)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        tree_ops.hist_build(bd, ridx, va, vb, 0, starts, counts, len(starts), vmax=vmax, **kw)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    rows = sum(counts)
    print(f"{name:40s} {ms:7.2f} ms  {rows / ms / 1e6:6.2f} Grows/s", flush=True)


ident = torch.arange(N, dtype=torch.int32, device=dev)
for fg in ("16", "32", "64"):
    os.environ["H2O3_HIST_FG"] = fg
    run(f"L0 all rows contiguous FG={fg}", ident, [0], [N], unit_w=True)
os.environ["H2O3_HIST_FG"] = "16"
run("L0 all rows contiguous", ident, [0], [N], unit_w=True)
run("L0 all rows contiguous (no pack)", ident, [0], [N], unit_w=False)
half = N // 2
run("half rows contiguous, 1 node", ident, [0], [half], unit_w=True)
for d in (1, 3, 5, 7):
    nodes = 2 ** d
    # rows of a depth-d node: a sorted random 1/2^d subset; build half of the nodes
    g = torch.Generator(device=dev).manual_seed(d)
    nid = torch.randint(0, nodes, (N,), generator=g, device=dev)
    order = torch.argsort(nid, stable=True).to(torch.int32)
    cnt = torch.bincount(nid, minlength=nodes).cpu().tolist()
    st = [0]
    for c in cnt[:-1]:
        st.append(st[-1] + c)
    b = list(range(0, nodes, 2))
    run(f"depth {d}: {len(b)} scattered nodes", order, [st[i] for i in b], [cnt[i] for i in b], unit_w=True)
    run(f"depth {d}: {len(b)} scattered nodes (no pack)", order, [st[i] for i in b], [cnt[i] for i in b],
        unit_w=False)
# same row count, contiguous rows but many segments
seg = N // 128
run("64 contiguous segments", ident, [2 * i * seg for i in range(64)], [seg] * 64, unit_w=True)
