"""AutoML at the BASELINE shape: 10M x 200 binomial synthetic data on the
device, the default modeling plan restricted to the BASELINE's algorithms
(GBM + XGBoost + GLM + DeepLearning + StackedEnsemble), a max_runtime_secs
budget, then the leader's MOJO export in the reference (h2o-genmodel) layout
-- timed -- and a standalone (numpy, no torch) scoring of 100k rows that must
equal leader.predict.  Writes the leaderboard, the event log and a JSON
summary into OUT (default gpurun_out/automl).

Reference: h2o-automl/src/main/java/ai/h2o/automl/AutoML.java:49."""
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import h2o3_amd as h2o  # noqa: E402
from h2o3_amd.automl import H2OAutoML  # noqa: E402
from h2o3_amd.core.frame import H2OFrame  # noqa: E402
from h2o3_amd.core.vec import T_ENUM, T_REAL, Vec  # noqa: E402

N = int(os.environ.get("ROWS", 10_000_000))
P = int(os.environ.get("COLS", 200))
BUDGET = int(os.environ.get("BUDGET", 900))
OUT = os.environ.get("OUT", "gpurun_out/automl")
NSCORE = int(os.environ.get("NSCORE", 100_000))
os.makedirs(OUT, exist_ok=True)
h2o.init(verbose=False)
t0 = time.time()


def _beat():
    while True:
        time.sleep(30)
        print(f"[{time.time() - t0:6.0f} s] running", flush=True)


threading.Thread(target=_beat, daemon=True).start()
DEV = "cuda" if torch.cuda.is_available() else "cpu"
g = torch.Generator(device=DEV).manual_seed(7)
X = torch.randn((N, P), generator=g, device=DEV)
beta = torch.randn(P, generator=g, device=DEV) / P ** 0.5
logit = X @ beta + 0.5 * X[:, 0] * X[:, 1] - 0.3 * X[:, 2].abs()
y = (torch.rand(N, generator=g, device=DEV) < torch.sigmoid(logit)).to(torch.int32)
vecs = [Vec(X[:, j].contiguous(), T_REAL) for j in range(P)] + [Vec(y, T_ENUM, ["0", "1"])]
names = [f"x{j}" for j in range(P)] + ["y"]
del X, logit
fr = H2OFrame.from_vecs(vecs, names)
print(f"data {N}x{P} ready in {time.time() - t0:.1f} s", flush=True)
t1 = time.time()
aml = H2OAutoML(max_runtime_secs=BUDGET, seed=1, nfolds=3, verbosity="info",
                include_algos=["GBM", "XGBoost", "GLM", "DeepLearning", "StackedEnsemble"])
aml.train(y="y", training_frame=fr)
wall = time.time() - t1
lb = aml.get_leaderboard("ALL").as_data_frame()
lb.to_csv(os.path.join(OUT, "leaderboard.csv"), index=False)
with open(os.path.join(OUT, "event_log.txt"), "w") as f:
    ev = aml.event_log
    f.write(ev.as_data_frame().to_string() if hasattr(ev, "as_data_frame") else str(ev))
print(lb.head(30).to_string(), flush=True)
leader = aml.leader
import tempfile  # noqa: E402
mdir = tempfile.mkdtemp(prefix="automl_mojo_")
t2 = time.time()
p_h2o = leader.download_mojo(mdir, format="h2o")
export_s = time.time() - t2
mojo_mb = os.path.getsize(p_h2o) / 2 ** 20
print(f"leader MOJO (reference layout) {mojo_mb:.1f} MB in {export_s:.1f} s", flush=True)
# standalone scoring of NSCORE rows vs leader.predict on the same rows
sub = fr[:NSCORE, :]
t3 = time.time()
pm = leader.predict(sub).as_data_frame()
pred_s = time.time() - t3
from h2o3_amd.mojo.genmodel import MojoModel  # noqa: E402
df = sub.as_data_frame()
t4 = time.time()
mj = MojoModel.load(p_h2o)
pj = mj.predict(df[[f"x{j}" for j in range(P)]])
mojo_score_s = time.time() - t4
a = pm.iloc[:, -1].to_numpy(dtype=np.float64)
b = pj.iloc[:, -1].to_numpy(dtype=np.float64)
maxdiff = float(np.abs(a - b).max())
labels_equal = float((pm.iloc[:, 0].astype(str).to_numpy() == pj.iloc[:, 0].astype(str).to_numpy()).mean())
summary = {"rows": N, "cols": P, "budget_s": BUDGET, "automl_wall_s": round(wall, 1), "n_models": int(len(lb)),
           "algos": sorted(set(lb["algo"])) if "algo" in lb else None,
           "leader": leader.model_id, "leader_auc": float(lb.iloc[0]["auc"]),
           "mojo_layout": "h2o-genmodel", "mojo_mb": round(mojo_mb, 2), "mojo_export_s": round(export_s, 2),
           "score_rows": NSCORE, "leader_predict_s": round(pred_s, 2), "mojo_standalone_score_s": round(mojo_score_s, 2),
           "mojo_vs_leader_max_abs_p1_diff": maxdiff, "mojo_vs_leader_label_agreement": labels_equal}
with open(os.path.join(OUT, "summary.json"), "w") as f:
    json.dump(summary, f, indent=1)
print(json.dumps(summary), flush=True)
