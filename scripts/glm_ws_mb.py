"""Microbenchmark of one fused IRLS pass (glm_irls_ws_kernel), 100M x 100
binomial, narrow rows (ldx = 100, logical width 128).  Env: H2O3_GLM_BF3,
H2O3_GI_DBG (bit0 skip MFMA, bit1 skip HBM loads), H2O3_MB_GRAD (0: no
gradient channel, 1: f32 products, 2: f64 products)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.ops import linalg_ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
ldx = int(sys.argv[2]) if len(sys.argv) > 2 else 100
P = 100
X = torch.randn(n, ldx, device="cuda")
beta = torch.zeros(128, device="cuda")
beta[:P] = 0.01 * torch.randn(P, device="cuda")
y = (torch.rand(n, device="cuda") < 0.5).float()
codes = linalg_ops.glm_fused_codes("binomial", "logit")
gm = int(os.environ.get("H2O3_MB_GRAD", "0"))
kw = dict(grad=gm > 0, grad_f64=gm == 2)
for _ in range(2):
    linalg_ops.glm_irls(X, aug=P, beta=beta, b0=0.1, y=y, codes=codes, width=128, **kw)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
K = 10
for _ in range(K):
    linalg_ops.glm_irls(X, aug=P, beta=beta, b0=0.1, y=y, codes=codes, width=128, **kw)
ev1.record()
torch.cuda.synchronize()
ms = ev0.elapsed_time(ev1) / K
gb = n * (ldx * 4 + 4) / 1e9
print(f"bf3={os.environ.get('H2O3_GLM_BF3', '1')} dbg={os.environ.get('H2O3_GI_DBG', '0')} grad={gm} ldx={ldx}: "
      f"{ms:.2f} ms/pass  {gb / ms:.2f} TB/s")
