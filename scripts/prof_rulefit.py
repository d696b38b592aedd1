"""cProfile of one RuleFit training (1M x 10, GPU) -- top functions by own time."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import h2o3_amd as h2o  # noqa: E402
from h2o3_amd.core.frame import H2OFrame  # noqa: E402
from h2o3_amd.core.vec import Vec, T_REAL, T_ENUM  # noqa: E402
from h2o3_amd import estimators as E  # noqa: E402

h2o.init(verbose=False)
n = int(os.environ.get("ROWS", 1_000_000))
dev = "cuda" if torch.cuda.is_available() else "cpu"
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn((n, 10), generator=g, device=dev)
y = (torch.rand(n, generator=g, device=dev) < torch.sigmoid(X[:, 0] - X[:, 1])).to(torch.int32)
fr = H2OFrame.from_vecs([Vec(X[:, j].contiguous(), T_REAL) for j in range(10)] + [Vec(y, T_ENUM, ["0", "1"])],
                        [f"x{j}" for j in range(10)] + ["y"])
algo = os.environ.get("ALGO", "rulefit")
mk = {"rulefit": lambda: E.H2ORuleFitEstimator(max_num_rules=50, seed=1),
      "aggregator": lambda: E.H2OAggregatorEstimator(),
      "infogram": lambda: E.H2OInfogram()}[algo]
m = mk()
pr = cProfile.Profile()
t0 = time.time()
pr.enable()
if algo == "aggregator":
    m.train(x=[f"x{j}" for j in range(10)], training_frame=fr)
else:
    m.train(x=[f"x{j}" for j in range(10)], y="y", training_frame=fr)
if dev == "cuda":
    torch.cuda.synchronize()
pr.disable()
print(f"{algo} train_s {time.time() - t0:.2f}", flush=True)
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
