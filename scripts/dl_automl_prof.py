"""Where an AutoML DeepLearning grid model's time goes at 10M x 200 (hidden
[50], RectifierWithDropout, 10 epochs, adaptive rate, nfolds 3): cProfile."""
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
from h2o3_amd.estimators import H2ODeepLearningEstimator  # noqa: E402

N = int(os.environ.get("ROWS", 10_000_000))
P = int(os.environ.get("COLS", 200))
h2o.init(verbose=False)
g = torch.Generator(device="cuda").manual_seed(7)
X = torch.randn((N, P), generator=g, device="cuda")
beta = torch.randn(P, generator=g, device="cuda") / P ** 0.5
logit = X @ beta + 0.5 * X[:, 0] * X[:, 1] - 0.3 * X[:, 2].abs()
y = (torch.rand(N, generator=g, device="cuda") < torch.sigmoid(logit)).to(torch.int32)
fr = H2OFrame.from_vecs([Vec(X[:, j].contiguous(), T_REAL) for j in range(P)] + [Vec(y, T_ENUM, ["0", "1"])],
                        [f"x{j}" for j in range(P)] + ["y"])
del X, logit
m = H2ODeepLearningEstimator(epochs=10, adaptive_rate=True, activation="RectifierWithDropout", hidden=[50],
                             hidden_dropout_ratios=[0.1], rho=0.95, epsilon=1e-8, input_dropout_ratio=0.05,
                             nfolds=int(os.environ.get("NFOLDS", 3)), seed=1, keep_cross_validation_predictions=True)
pr = cProfile.Profile()
t0 = time.time()
pr.enable()
m.train(y="y", training_frame=fr)
pr.disable()
print(f"train {time.time() - t0:.2f} s", flush=True)
from h2o3_amd.utils import timer  # noqa: E402
print("phases:", timer.report(), flush=True)
pstats.Stats(pr).sort_stats("cumulative").print_stats(45)
