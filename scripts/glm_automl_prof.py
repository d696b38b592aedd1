"""Where the AutoML GLM step's time goes at 10M x 200 (binomial, lambda
search over the alpha grid 0 .. 1, nfolds 3): cProfile."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("H2O3_PROFILE", "0")
import h2o3_amd as h2o  # noqa: E402
from h2o3_amd.core.frame import H2OFrame  # noqa: E402
from h2o3_amd.core.vec import T_ENUM, T_REAL, Vec  # noqa: E402
from h2o3_amd.estimators import H2OGeneralizedLinearEstimator  # noqa: E402

N = int(os.environ.get("ROWS", 10_000_000))
P = int(os.environ.get("COLS", 200))
h2o.init(verbose=False)
DEV = "cuda" if torch.cuda.is_available() else "cpu"
g = torch.Generator(device=DEV).manual_seed(7)
X = torch.randn((N, P), generator=g, device=DEV)
beta = torch.randn(P, generator=g, device=DEV) / P ** 0.5
logit = X @ beta + 0.5 * X[:, 0] * X[:, 1] - 0.3 * X[:, 2].abs()
y = (torch.rand(N, generator=g, device=DEV) < torch.sigmoid(logit)).to(torch.int32)
fr = H2OFrame.from_vecs([Vec(X[:, j].contiguous(), T_REAL) for j in range(P)] + [Vec(y, T_ENUM, ["0", "1"])],
                        [f"x{j}" for j in range(P)] + ["y"])
del X, logit
m = H2OGeneralizedLinearEstimator(family="binomial", lambda_search=True, alpha=[0.0, 0.2, 0.4, 0.6, 0.8, 1.0],
                                  nfolds=int(os.environ.get("NFOLDS", 3)), seed=1,
                                  keep_cross_validation_predictions=True)
pr = cProfile.Profile()
t0 = time.time()
pr.enable()
m.train(y="y", training_frame=fr)
pr.disable()
print(f"train {time.time() - t0:.2f} s", flush=True)
from h2o3_amd.utils import timer  # noqa: E402
print("phases:", timer.report(), flush=True)
st = pstats.Stats(pr); st.sort_stats("cumulative").print_stats(45); st.sort_stats("tottime").print_stats(20)
