"""Wall time of one default-parameter training per estimator on 2M x 50
synthetic binomial data (GPU), to spot algorithms whose per-model cost is out
of line.  Prints one JSON line per estimator."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import h2o3_amd as h2o  # noqa: E402
from h2o3_amd.core.frame import H2OFrame  # noqa: E402
from h2o3_amd.core.vec import Vec, T_REAL, T_ENUM  # noqa: E402
from h2o3_amd import estimators as E  # noqa: E402

N = int(os.environ.get("ROWS", 2_000_000))
P = int(os.environ.get("COLS", 50))
h2o.init(verbose=False)
g = torch.Generator(device="cuda").manual_seed(7)
X = torch.randn((N, P), generator=g, device="cuda")
beta = torch.randn(P, generator=g, device="cuda") / P ** 0.5
y = (torch.rand(N, generator=g, device="cuda") < torch.sigmoid(X @ beta)).to(torch.int32)
names = [f"x{j}" for j in range(P)]
fr = H2OFrame.from_vecs([Vec(X[:, j].contiguous(), T_REAL) for j in range(P)] + [Vec(y, T_ENUM, ["0", "1"])],
                        names + ["y"])
cases = [
    ("gbm", lambda: E.H2OGradientBoostingEstimator(ntrees=50, seed=1), True),
    ("xgboost", lambda: E.H2OXGBoostEstimator(ntrees=50, seed=1), True),
    ("drf", lambda: E.H2ORandomForestEstimator(ntrees=50, seed=1), True),
    ("glm", lambda: E.H2OGeneralizedLinearEstimator(family="binomial"), True),
    ("deeplearning", lambda: E.H2ODeepLearningEstimator(epochs=1, seed=1), True),
    ("naivebayes", lambda: E.H2ONaiveBayesEstimator(), True),
    ("kmeans", lambda: E.H2OKMeansEstimator(k=8, seed=1), False),
    ("pca", lambda: E.H2OPrincipalComponentAnalysisEstimator(k=5), False),
    ("isolationforest", lambda: E.H2OIsolationForestEstimator(ntrees=50, seed=1), False),
    ("extendedisolationforest", lambda: E.H2OExtendedIsolationForestEstimator(ntrees=50, seed=1), False),
]
only = os.environ.get("ONLY")
for name, mk, sup in cases:
    if only and name not in only.split(","):
        continue
    m = mk()
    t0 = time.time()
    try:
        if sup:
            m.train(x=names, y="y", training_frame=fr)
        else:
            m.train(x=names, training_frame=fr)
        torch.cuda.synchronize()
        el = time.time() - t0
        auc = None
        try:
            auc = round(float(m.model_performance(fr).auc()), 4) if sup else None
        except Exception:
            pass
        print(json.dumps({"algo": name, "rows": N, "cols": P, "train_s": round(el, 2), "train_auc": auc}), flush=True)
        from h2o3_amd.utils import timer
        if timer.ENABLED:
            print("  phases(ms,count):", timer.report(), flush=True)
    except Exception as e:  # keep surveying the rest
        print(json.dumps({"algo": name, "error": repr(e)[:300]}), flush=True)
