"""One histogram configuration (root level, 100M x F uint8 codes, packed
path) for rocprofv3 --pmc passes: KERNEL=row|quad F=100 N=..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.models.tree.binning import BinnedData  # noqa: E402
from h2o3_amd.ops import tree_ops  # noqa: E402

N = int(os.environ.get("N", 50_000_000))
F = int(os.environ.get("F", 100))
os.environ["H2O3_HIST_KERNEL"] = os.environ.get("KERNEL", "row")
bd = BinnedData()
bd.codes = torch.randint(0, 254, (N, 128), dtype=torch.uint8, device="cuda")
bd.F, bd.Fp, bd.Bs, bd.code_bytes, bd.nrows_local = F, 128, 256, 1, N
va = torch.randn(N, device="cuda")
vmax = tree_ops.channel_max(va, None, 0)
ridx = torch.arange(N, dtype=torch.int32, device="cuda")
for _ in range(3):
    tree_ops.hist_build(bd, ridx, va, None, 0, [0], [N], 1, vmax=vmax, unit_w=True, posv=True)
torch.cuda.synchronize()
print("done", os.environ["H2O3_HIST_KERNEL"], F, N)
