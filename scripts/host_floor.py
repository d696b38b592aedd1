"""Host-overhead floor of the GBM tree step: bench shape at few rows (GPU work
negligible), cProfile of the timed steps -> gpurun_out/host_floor.txt."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import h2o3_amd  # noqa: E402
import bench  # noqa: E402
from h2o3_amd.models.base import TrainSpec  # noqa: E402
from h2o3_amd.models.tree.gbm import GBMDriver, H2OGradientBoostingEstimator  # noqa: E402

h2o3_amd.init(verbose=False)
rows = int(os.environ.get("ROWS", 200000))


class A:
    cols, cat_cols, cat_card = 100, 0, 1000


fr, names, y = bench.make_frame(A, torch.device("cuda"), 0, rows)
est = H2OGradientBoostingEstimator(ntrees=500, max_depth=8, seed=42, ignore_const_cols=False)
spec = TrainSpec(fr, names, "y")
est._spec = spec
drv = GBMDriver(est, spec)
for _ in range(5):
    drv.step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(30):
    drv.step()
torch.cuda.synchronize()
print(f"rows={rows}: {(time.perf_counter() - t) / 30 * 1e3:.3f} ms/tree (host floor)")
pr = cProfile.Profile()
pr.enable()
for _ in range(30):
    drv.step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
