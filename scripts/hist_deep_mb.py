"""Root or deep-level (16 nodes, half the rows, sorted scattered row ids)
histogram pass over 100M x 100 uint8 codes, packed path, for rocprofv3 --pmc
passes and feature-group-width A/B: LEVEL=root|deep N=... H2O3_HIST_FGW=..."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.models.tree.binning import BinnedData  # noqa: E402
from h2o3_amd.ops import tree_ops  # noqa: E402

N = int(os.environ.get("N", 100_000_000))
LEVEL = os.environ.get("LEVEL", "deep")
F, Fp, Bs = 100, 128, 256
bd = BinnedData()
bd.codes = torch.randint(0, 254, (N, Fp), dtype=torch.uint8, device="cuda")
bd.F, bd.Fp, bd.Bs, bd.code_bytes, bd.nrows_local = F, Fp, Bs, 1, N
va = torch.randn(N, device="cuda")
vmax = tree_ops.channel_max(va, None, 0)
if LEVEL == "root":
    ridx = torch.arange(N, dtype=torch.int32, device="cuda")
    starts, counts = [0], [N]
else:
    g = torch.Generator(device="cuda").manual_seed(5)
    nid = torch.randint(0, 32, (N,), generator=g, device="cuda")
    ridx = torch.argsort(nid, stable=True).to(torch.int32)
    cnt = torch.bincount(nid, minlength=32).cpu().tolist()
    st = [0]
    for c in cnt[:-1]:
        st.append(st[-1] + c)
    starts, counts = [st[i] for i in range(0, 32, 2)], [cnt[i] for i in range(0, 32, 2)]
    del nid
vp = va[ridx.long()].contiguous()      # position-ordered payload, as in the tree
reps = int(os.environ.get("REPS", 5))
tree_ops.hist_build(bd, ridx, vp, None, 0, starts, counts, len(starts), vmax=vmax, unit_w=True, posv=True)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(reps):
    tree_ops.hist_build(bd, ridx, vp, None, 0, starts, counts, len(starts), vmax=vmax, unit_w=True, posv=True)
torch.cuda.synchronize()
ms = (time.perf_counter() - t) / reps * 1e3
print(f"N={N} level={LEVEL} fgw={os.environ.get('H2O3_HIST_FGW', 'auto')} "
      f"groups={tree_ops.quad_groups(F, Fp, Bs, True)}: {ms:.3f} ms", flush=True)
