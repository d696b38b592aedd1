"""AutoML on the GPU (the BASELINE AutoML config at reduced size and budget):
synthetic ROWS x COLS binomial data built on the device, AutoML with a
max_runtime_secs budget (GBM, XGBoost, GLM, DRF, DL, grids, Stacked
Ensembles), leaderboard + per-model training times, leader MOJO export
(native and reference layout) and a re-score of the exported leader."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import h2o3_amd as h2o  # noqa: E402
from h2o3_amd.automl import H2OAutoML  # noqa: E402
from h2o3_amd.core.frame import H2OFrame  # noqa: E402
from h2o3_amd.core.vec import Vec, T_REAL, T_ENUM  # noqa: E402

N = int(os.environ.get("ROWS", 2_000_000))
P = int(os.environ.get("COLS", 50))
BUDGET = int(os.environ.get("BUDGET", 240))
h2o.init(verbose=False)
g = torch.Generator(device="cuda").manual_seed(7)
X = torch.randn((N, P), generator=g, device="cuda")
beta = torch.randn(P, generator=g, device="cuda") / P ** 0.5
logit = X @ beta + 0.5 * X[:, 0] * X[:, 1] - 0.3 * X[:, 2].abs()
y = (torch.rand(N, generator=g, device="cuda") < torch.sigmoid(logit)).to(torch.int32)
vecs = [Vec(X[:, j].contiguous(), T_REAL) for j in range(P)] + [Vec(y, T_ENUM, ["0", "1"])]
names = [f"x{j}" for j in range(P)] + ["y"]
fr = H2OFrame.from_vecs(vecs, names)
t0 = time.time()


def _beat():
    while True:
        time.sleep(30)
        print(f"[{time.time() - t0:6.0f} s] automl running", flush=True)


import threading  # noqa: E402
threading.Thread(target=_beat, daemon=True).start()
aml = H2OAutoML(max_runtime_secs=BUDGET, seed=1, nfolds=3, verbosity="info")
aml.train(y="y", training_frame=fr)
wall = time.time() - t0
lb = aml.leaderboard.as_data_frame() if hasattr(aml.leaderboard, "as_data_frame") else aml.leaderboard
print(lb.head(25).to_string(), flush=True)
leader = aml.leader
# MOJOs go to local scratch (an ensemble over deep forests is GBs: not for gpurun_out/)
import tempfile  # noqa: E402
mdir = tempfile.mkdtemp(prefix="automl_mojo_")
t1 = time.time()
p_native = leader.download_mojo(mdir)
mojo_s = time.time() - t1
mojo_mb = os.path.getsize(p_native) / 2 ** 20
try:
    p_h2o = leader.download_mojo(os.path.join(mdir, "h2o"), format="h2o")
except NotImplementedError as e:
    p_h2o = f"not exported: {e}"
print(json.dumps({"rows": N, "cols": P, "budget_s": BUDGET, "wall_s": round(wall, 1),
                  "n_models": len(lb), "leader": leader.model_id, "leader_auc": float(lb.iloc[0]["auc"]),
                  "mojo": os.path.basename(p_native), "mojo_mb": round(mojo_mb, 1), "mojo_s": round(mojo_s, 1),
                  "mojo_h2o": p_h2o if p_h2o.startswith("not") else os.path.basename(p_h2o)}), flush=True)
