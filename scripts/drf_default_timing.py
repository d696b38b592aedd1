"""Default-parameter DRF (AutoML's DRF_1 step: max_depth 20, mtries sqrt(P))
on synthetic ROWS x COLS binomial data: per-tree time and phase profile."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("H2O3_PROFILE", "1")
import h2o3_amd as h2o  # noqa: E402
from h2o3_amd.core.frame import H2OFrame  # noqa: E402
from h2o3_amd.core.vec import Vec, T_REAL, T_ENUM  # noqa: E402
from h2o3_amd.estimators import H2ORandomForestEstimator  # noqa: E402
from h2o3_amd.utils import timer  # noqa: E402

N = int(os.environ.get("ROWS", 2_000_000))
P = int(os.environ.get("COLS", 50))
h2o.init(verbose=False)
g = torch.Generator(device="cuda").manual_seed(7)
X = torch.randn((N, P), generator=g, device="cuda")
beta = torch.randn(P, generator=g, device="cuda") / P ** 0.5
y = (torch.rand(N, generator=g, device="cuda") < torch.sigmoid(X @ beta)).to(torch.int32)
fr = H2OFrame.from_vecs([Vec(X[:, j].contiguous(), T_REAL) for j in range(P)] + [Vec(y, T_ENUM, ["0", "1"])],
                        [f"x{j}" for j in range(P)] + ["y"])
for nt in (2, 10):
    t0 = time.time()
    m = H2ORandomForestEstimator(ntrees=nt, seed=1)
    m.train(y="y", training_frame=fr)
    torch.cuda.synchronize()
    print(f"ntrees={nt}: {time.time() - t0:.2f} s", flush=True)
print(timer.report() if hasattr(timer, "report") else "", flush=True)
