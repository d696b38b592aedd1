"""Wide GLM IRLS pass at 12.5M x 1000 (binomial): the fused pass (eta kernel
+ hand-written MFMA Gram, glm_wide_gram_kernel) against the split + library
GEMM pass, time per pass and the Gram difference between the two."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.ops import linalg_ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
P = 1000
X = torch.randn(N, P, device="cuda")
beta = 0.01 * torch.randn(P, device="cuda")
y = (torch.rand(N, device="cuda") < 0.5).float()
w = torch.ones(N, device="cuda")
out = {}
for fused in (True, False):
    f = lambda: linalg_ops.glm_wide_irls(X, P, beta, 0.1, y, w, None, (1, 1), fused=fused)  # noqa: E731
    G, _, _ = f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        G, _, _ = f()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 3 * 1e3
    out[fused] = G[:P + 1, :P + 1]
    print(f"fused={fused}: {ms:7.2f} ms/pass", flush=True)
d = (out[True] - out[False]).abs().max() / out[False].abs().max()
print(f"max |G_fused - G_split| / max |G| = {float(d):.2e}", flush=True)
