"""glm_wide_irls row-chunk size sweep at 12.5M x 1000 (binomial)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.ops import linalg_ops  # noqa: E402

N, P = 12_500_000, 1000
X = torch.randn(N, 1024, device="cuda")
X[:, P:] = 0
beta = 0.01 * torch.randn(P, device="cuda")
y = (torch.rand(N, device="cuda") < 0.5).float()
w = torch.ones(N, device="cuda")
ref = None
for step in (1 << 18, 1 << 19, 1 << 20, 1 << 21):
    f = lambda: linalg_ops.glm_wide_irls(X, P, beta, 0.1, y, w, None, (1, 1), step=step)  # noqa: E731
    G, _ = f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        G, _ = f()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 3 * 1e3
    if ref is None:
        ref = G
    print(f"step {step:8d}: {ms:7.2f} ms/pass  max rel diff vs step 2^18 {float((G - ref).abs().max() / ref.abs().max()):.2e}",
          flush=True)
