"""Wall time of one training per remaining estimator (the ones
scripts/algo_survey.py does not cover) on synthetic GPU data: 1M x 20
numeric + 2 categorical columns (PSVM on 100K rows), to spot algorithms
whose cost is out of line.  One JSON line per estimator."""
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

N = int(os.environ.get("ROWS", 1_000_000))
P = int(os.environ.get("COLS", 20))
h2o.init(verbose=False)
DEV = "cuda" if torch.cuda.is_available() else "cpu"
g = torch.Generator(device=DEV).manual_seed(7)


def frame(n):
    X = torch.randn((n, P), generator=g, device=DEV)
    beta = torch.randn(P, generator=g, device=DEV) / P ** 0.5
    eta = X @ beta
    y = (torch.rand(n, generator=g, device=DEV) < torch.sigmoid(eta)).to(torch.int32)
    c1 = torch.randint(0, 10, (n,), generator=g, device=DEV).to(torch.int32)
    c2 = torch.randint(0, 100, (n,), generator=g, device=DEV).to(torch.int32)
    tr = torch.randint(0, 2, (n,), generator=g, device=DEV).to(torch.int32)
    t = torch.exp(-eta + 0.3 * torch.randn(n, generator=g, device=DEV))
    names = [f"x{j}" for j in range(P)]
    vecs = [Vec(X[:, j].contiguous(), T_REAL) for j in range(P)]
    vecs += [Vec(c1, T_ENUM, [f"a{i}" for i in range(10)]), Vec(c2, T_ENUM, [f"b{i}" for i in range(100)]),
             Vec(y, T_ENUM, ["0", "1"]), Vec(tr, T_ENUM, ["control", "treatment"]), Vec(t.float(), T_REAL),
             Vec(eta.float().contiguous(), T_REAL)]
    return H2OFrame.from_vecs(vecs, names + ["c1", "c2", "y", "treat", "time", "yr"]), names


fr, xs = frame(N)
small, _ = frame(100_000)
x = xs + ["c1", "c2"]
cases = [
    ("glrm", lambda: E.H2OGeneralizedLowRankEstimator(k=5, seed=1, max_iterations=50), dict(x=xs), fr),
    ("svd", lambda: E.H2OSingularValueDecompositionEstimator(nv=5), dict(x=xs), fr),
    ("gam", lambda: E.H2OGeneralizedAdditiveEstimator(family="binomial", gam_columns=["x0", "x1"]),
     dict(x=xs[2:], y="y"), fr),
    ("rulefit", lambda: E.H2ORuleFitEstimator(max_num_rules=50, seed=1), dict(x=xs[:10], y="y"), fr),
    ("coxph", lambda: E.H2OCoxProportionalHazardsEstimator(stop_column="time"), dict(x=xs[:10], y="y"), fr),
    ("psvm", lambda: E.H2OSupportVectorMachineEstimator(seed=1), dict(x=xs, y="y"), small),
    ("aggregator", lambda: E.H2OAggregatorEstimator(), dict(x=xs), fr),
    ("anovaglm", lambda: E.H2OANOVAGLMEstimator(family="binomial"), dict(x=["x0", "x1", "c1"], y="y"), fr),
    ("modelselection", lambda: E.H2OModelSelectionEstimator(mode="maxr", max_predictor_number=3),
     dict(x=xs, y="yr"), fr),
    ("isotonic", lambda: E.H2OIsotonicRegressionEstimator(), dict(x=["x0"], y="yr"), fr),
    ("targetencoder", lambda: E.H2OTargetEncoderEstimator(), dict(x=["c1", "c2"], y="y"), fr),
    ("infogram", lambda: E.H2OInfogram(), dict(x=xs[:10], y="y"), fr),
    ("upliftdrf", lambda: E.H2OUpliftRandomForestEstimator(ntrees=20, treatment_column="treat", seed=1),
     dict(x=xs[:10], y="y"), fr),
    ("gbm_cv_se", None, None, fr),
    ("glm_lambda_search", lambda: E.H2OGeneralizedLinearEstimator(family="binomial", lambda_search=True,
                                                                 nlambdas=20), dict(x=x, y="y"), fr),
    ("xgboost_dart", lambda: E.H2OXGBoostEstimator(ntrees=30, booster="dart", seed=1), dict(x=x, y="y"), fr),
    ("kmeans_estimate_k", lambda: E.H2OKMeansEstimator(k=20, estimate_k=True, seed=1), dict(x=xs), fr),
]
import signal  # noqa: E402


def _alarm(signum, frame):
    raise TimeoutError("case exceeded 150 s")


signal.signal(signal.SIGALRM, _alarm)
only = os.environ.get("ONLY")
for name, mk, kw, data in cases:
    if only and name not in only.split(","):
        continue
    t0 = time.time()
    signal.alarm(150)
    try:
        if name == "gbm_cv_se":
            b1 = E.H2OGradientBoostingEstimator(ntrees=20, nfolds=3, keep_cross_validation_predictions=True, seed=1)
            b1.train(x=x, y="y", training_frame=data)
            b2 = E.H2OGeneralizedLinearEstimator(family="binomial", nfolds=3, keep_cross_validation_predictions=True,
                                                 seed=1)
            b2.train(x=x, y="y", training_frame=data)
            m = E.H2OStackedEnsembleEstimator(base_models=[b1, b2])
            m.train(x=x, y="y", training_frame=data)
        else:
            m = mk()
            m.train(training_frame=data, **kw)
        if DEV == "cuda":
            torch.cuda.synchronize()
        print(json.dumps({"algo": name, "rows": data.nrows, "train_s": round(time.time() - t0, 2)}), flush=True)
    except Exception as e:  # keep surveying the rest
        print(json.dumps({"algo": name, "error": repr(e)[:300], "after_s": round(time.time() - t0, 2)}), flush=True)
    finally:
        signal.alarm(0)
