"""Host cost of the GLM condition estimate (dpotrf + dpocon) at P = 1001 for
a few BLAS thread counts (threadpoolctl)."""
import os
import sys
import time

import numpy as np
from threadpoolctl import threadpool_limits

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.models.glm.glm import GLMDriver  # noqa: E402

A = np.random.default_rng(0).standard_normal((20000, 1001))
G = A.T @ A
GLMDriver._scaled_cond(G)
for nt in (1, 4, 8, 16, None):
    with threadpool_limits(limits=nt):
        t = time.perf_counter()
        for _ in range(3):
            GLMDriver._scaled_cond(G)
        print(f"threads={nt}: {(time.perf_counter() - t) / 3 * 1e3:.1f} ms", flush=True)
