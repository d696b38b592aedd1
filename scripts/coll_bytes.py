"""Collective bytes per tree level of the multi-rank tree builders.

Run under torch.distributed.run (one rank per GPU, or 8 gloo ranks on one
GPU as a rehearsal): grows a few trees of the bench's GBM (100M x 100) or
DRF (50M x 500, 100 categoricals of cardinality 1000) configuration and
writes, per tree and level, the payload bytes this rank handed to each
collective (parallel/collectives.bytes_report, tagged tree.L<level> by the
tree engine), plus the per-tree totals.

  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
      scripts/coll_bytes.py --algo drf --rows 50000000 --cols 500 --cat-cols 100 --trees 2 \
      --out gpurun_out/coll_bytes_drf.json
"""
import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="gbm", choices=["gbm", "drf"])
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--cols", type=int, default=100)
    ap.add_argument("--cat-cols", type=int, default=0)
    ap.add_argument("--cat-card", type=int, default=1000)
    ap.add_argument("--trees", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/coll_bytes.json")
    a = ap.parse_args()
    import bench
    import h2o3_amd
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.parallel import cloud
    from h2o3_amd.parallel import collectives as coll
    h2o3_amd.init(verbose=False)
    W, r = cloud.world(), cloud.rank()
    dev = cloud.device()
    rows_local = a.rows // W + (1 if r < a.rows % W else 0)
    args = SimpleNamespace(cols=a.cols, cat_cols=a.cat_cols, cat_card=a.cat_card)
    fr, names, _ = bench.make_frame(args, dev, r, rows_local)
    if r == 0:
        print(f"frame ready: {rows_local} local rows x {a.cols} cols on {W} ranks", flush=True)
    if a.algo == "gbm":
        from h2o3_amd.models.tree.gbm import GBMDriver, H2OGradientBoostingEstimator
        est = H2OGradientBoostingEstimator(ntrees=500, max_depth=8, seed=42, histogram_type="QuantilesGlobal",
                                           nbins=255, ignore_const_cols=False)
        spec = TrainSpec(fr, names, "y")
        est._spec = spec
        drv = GBMDriver(est, spec)
    else:
        from h2o3_amd.models.tree.drf import DRFDriver, H2ORandomForestEstimator
        est = H2ORandomForestEstimator(ntrees=1000, max_depth=20, seed=42, histogram_type="QuantilesGlobal",
                                       nbins=255, ignore_const_cols=False)
        spec = TrainSpec(fr, names, "y")
        est._spec = spec
        drv = DRFDriver(est, spec)
    if r == 0:
        print("binned; growing trees", flush=True)
    trees = []
    for t in range(a.trees):
        coll.reset_bytes()
        t0 = time.time()
        drv.step()
        cloud.barrier()
        rep = coll.bytes_report()
        levels = {}
        for (tag, op), b in rep.items():
            levels.setdefault(tag, {})[op] = b
        tot = sum(rep.values())
        trees.append({"tree": t, "seconds": round(time.time() - t0, 3), "bytes_total": tot,
                      "levels": dict(sorted(levels.items(), key=lambda kv: (len(kv[0]), kv[0])))})
        if r == 0:
            print(f"tree {t}: {tot / 1e6:.1f} MB handed to collectives by rank 0", flush=True)
            for lv, ops in trees[-1]["levels"].items():
                print(f"  {lv}: " + ", ".join(f"{op} {b / 1e6:.2f} MB" for op, b in ops.items()), flush=True)
            # partial results survive a later failure
            os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
            with open(a.out + ".partial", "w") as f:
                json.dump({"algo": a.algo, "world": W, "trees": trees}, f, indent=1)
    allr = coll.all_gather_object([tr["bytes_total"] for tr in trees])
    if r == 0:
        res = {"algo": a.algo, "rows": a.rows, "cols": a.cols, "cat_cols": a.cat_cols, "cat_card": a.cat_card,
               "world": W, "backend": cloud.info().get("backend") if hasattr(cloud, "info") else None,
               "per_rank_tree_bytes": allr, "trees": trees,
               "note": "payload bytes one rank hands to each collective (reduce_scatter / all_reduce: the full "
                       "buffer; all_gather: its slice; all_to_all: its send buffer), per tree level"}
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps({"algo": a.algo, "world": W, "MB_per_tree_rank0": [round(tr["bytes_total"] / 1e6, 1)
                                                                             for tr in trees]}))
    cloud.barrier()


if __name__ == "__main__":
    main()
