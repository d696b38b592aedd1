"""Grow GBM trees on the bench frame for a kernel trace: warm-up trees, a
200 ms idle gap (scripts/prof_summary.py --after-gap-ms cuts there), then the
traced trees.  usage: python scripts/devtree_trace.py --rows R --trees K"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=12_500_000)
    ap.add_argument("--cols", type=int, default=100)
    ap.add_argument("--trees", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--max-depth", type=int, default=8)
    a = ap.parse_args()
    import torch
    import h2o3_amd
    import bench
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.models.tree.gbm import GBMDriver, H2OGradientBoostingEstimator
    h2o3_amd.init(verbose=False)
    args = argparse.Namespace(cols=a.cols, cat_cols=0, cat_card=1000)
    fr, names, y = bench.make_frame(args, torch.device("cuda"), 0, a.rows)
    est = H2OGradientBoostingEstimator(ntrees=500, max_depth=a.max_depth, seed=42, histogram_type="QuantilesGlobal",
                                       nbins=255, ignore_const_cols=False)
    spec = TrainSpec(fr, names, "y")
    est._spec = spec
    drv = GBMDriver(est, spec)
    for _ in range(a.warmup):
        drv.step()
    torch.cuda.synchronize()
    time.sleep(0.2)
    t0 = time.perf_counter()
    for _ in range(a.trees):
        drv.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"devtree={getattr(drv, '_devtree', None) is not None} trees={a.trees} ms/tree={1000 * el / a.trees:.3f}")


if __name__ == "__main__":
    main()
