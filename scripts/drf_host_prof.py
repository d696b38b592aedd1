"""Host-side cProfile of DRF trees at the BASELINE DRF per-GPU shape
(6.25M x 500, 100 categoricals of cardinality 1000, depth 20): where the
level loop's host time goes between kernels."""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6_250_000)
    ap.add_argument("--trees", type=int, default=4)
    a = ap.parse_args()
    import torch
    import h2o3_amd
    import bench
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.models.tree.drf import DRFDriver, H2ORandomForestEstimator
    h2o3_amd.init(verbose=False)
    args = argparse.Namespace(cols=500, cat_cols=100, cat_card=1000)
    fr, names, y = bench.make_frame(args, torch.device("cuda"), 0, a.rows)
    est = H2ORandomForestEstimator(ntrees=1000, max_depth=20, seed=42, histogram_type="QuantilesGlobal", nbins=255,
                                   ignore_const_cols=False)
    spec = TrainSpec(fr, names, "y")
    est._spec = spec
    drv = DRFDriver(est, spec)
    for _ in range(2):
        drv.step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.trees):
        drv.step()
    torch.cuda.synchronize()
    pr.disable()
    print(f"drf ms/tree={1000 * (time.perf_counter() - t0) / a.trees:.2f}", flush=True)
    pstats.Stats(pr).sort_stats("tottime").print_stats(40)


if __name__ == "__main__":
    main()
