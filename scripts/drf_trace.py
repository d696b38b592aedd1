"""Grow DRF trees of the BASELINE DRF shape for a kernel trace: warm-up trees,
a 200 ms idle gap (prof_summary.py --after-gap-ms cuts there), then the
traced trees.  usage: python scripts/drf_trace.py --rows R --trees K"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6_250_000)
    ap.add_argument("--cols", type=int, default=500)
    ap.add_argument("--cat-cols", type=int, default=100)
    ap.add_argument("--trees", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    import torch
    import h2o3_amd
    import bench
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.models.tree.drf import DRFDriver, H2ORandomForestEstimator
    h2o3_amd.init(verbose=False)
    args = argparse.Namespace(cols=a.cols, cat_cols=a.cat_cols, cat_card=1000)
    fr, names, y = bench.make_frame(args, torch.device("cuda"), 0, a.rows)
    est = H2ORandomForestEstimator(ntrees=1000, max_depth=20, seed=42, histogram_type="QuantilesGlobal", nbins=255,
                                   ignore_const_cols=False)
    spec = TrainSpec(fr, names, "y")
    est._spec = spec
    drv = DRFDriver(est, spec)
    for _ in range(a.warmup):
        drv.step()
    torch.cuda.synchronize()
    time.sleep(0.2)
    t0 = time.perf_counter()
    for _ in range(a.trees):
        drv.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"drf trees={a.trees} ms/tree={1000 * el / a.trees:.3f}")


if __name__ == "__main__":
    main()
