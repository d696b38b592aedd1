"""Root + depth-5 histogram time for one H2O3_HIST_TB setting."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.models.tree.binning import BinnedData  # noqa: E402
from h2o3_amd.ops import tree_ops  # noqa: E402

N = int(os.environ.get("N", 100_000_000))
F, Fp, Bs = 100, 128, 256
bd = BinnedData()
bd.codes = torch.randint(0, 254, (N, Fp), dtype=torch.uint8, device="cuda")
bd.F, bd.Fp, bd.Bs, bd.code_bytes, bd.nrows_local = F, Fp, Bs, 1, N
va = torch.randn(N, device="cuda")
vmax = tree_ops.channel_max(va, None, 0)


def run(ridx, starts, counts, reps=5):
    tree_ops.hist_build(bd, ridx, va, None, 0, starts, counts, len(starts), vmax=vmax, unit_w=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        tree_ops.hist_build(bd, ridx, va, None, 0, starts, counts, len(starts), vmax=vmax, unit_w=True)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


ident = torch.arange(N, dtype=torch.int32, device="cuda")
r0 = run(ident, [0], [N])
g = torch.Generator(device="cuda").manual_seed(5)
nid = torch.randint(0, 32, (N,), generator=g, device="cuda")
order = torch.argsort(nid, stable=True).to(torch.int32)
cnt = torch.bincount(nid, minlength=32).cpu().tolist()
st = [0]
for c in cnt[:-1]:
    st.append(st[-1] + c)
b = list(range(0, 32, 2))
r5 = run(order, [st[i] for i in b], [cnt[i] for i in b])
print(f"N={N} TB={os.environ.get('H2O3_HIST_TB')}: root {r0:.3f} ms, depth5 (16 nodes, half rows) {r5:.3f} ms",
      flush=True)
