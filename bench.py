#!/usr/bin/env python
"""Headline benchmark: GBM binomial trees/sec on 100M x 100 synthetic data.

BASELINE.json metric: "GBM trees/sec + GLM iters/sec on 100M x 100
synthetic at 1/2/4/8 MI355X"; config "GBM binomial, 100M rows x 100 num
cols, ntrees=500 max_depth=8".

One step = one boosting iteration = one tree (binomial), including the
residual computation, histogram build for every level, split search,
partition, gamma (leaf value) pass and prediction update — nothing skipped.
The total data size is fixed (strong scaling): with N GPUs every rank holds
100M/N rows and histograms are reduce-scattered over RCCL.

The GLM half of the headline metric (GLM binomial IRLSM iterations/s on the
same frame) is measured after the GBM steps and reported as extra keys
(glm_iters_per_sec, glm_ms_per_iter) of the same JSON line; --no-glm skips it.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--algo gbm|glm|drf] [--no-glm]
       [--cols C] [--cat-cols K --cat-card L]   (DRF config: --algo drf --rows 50000000 --cols 500 --cat-cols 100)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


_HESSIAN = {
    "bf16": "one bf16 MFMA per product (hi*hi), f32 accumulate, f64 across row slices (kappa < 32 tier)",
    "bf3": "bf16x3 split operands (hi*hi + hi*lo + lo*hi) on MFMA, f32 accumulate, f64 across row blocks",
    "f32": "f32 MFMA products, f64 across row blocks",
    "f64": "fp64 GEMMs",
}


def _glm_precision(tier):
    """The config's precision statement for the Hessian tier the run ended on
    (glm.py _TIER_LIMITS: chosen from the scaled condition number)."""
    return (f"Hessian X'WX: {_HESSIAN.get(tier or 'bf3', tier)}; gradient X'(w (y - mu)): f32 VALU products, f64 "
            "sums, in the same pass; Newton step beta + H^-1 g, so the converged coefficients are those of the "
            "exact gradient whatever the Hessian tier (scripts/glm_precision.py)")


_GLM_PRECISION = _glm_precision("bf3")


def make_frame(args, dev, rank, rows_local):
    """Synthetic data of the benchmark shape (random, generated on device):
    args.cols features (the last args.cat_cols categorical), binomial y."""
    import torch
    F = args.cols
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    gb = torch.Generator(device="cpu").manual_seed(42)
    beta = torch.zeros(F)
    beta[: min(10, F)] = torch.randn(min(10, F), generator=gb)
    cols = []
    logit = torch.zeros(rows_local, device=dev)
    n_cat = min(args.cat_cols, F)
    cat_eff = torch.randn(args.cat_card, generator=gb) * 0.5
    for j in range(F):
        if j >= F - n_cat:
            c = torch.randint(0, args.cat_card, (rows_local,), generator=g, device=dev, dtype=torch.int32)
            if j == F - n_cat:
                logit += cat_eff.to(dev)[c.long()]
            cols.append(c)
            continue
        c = torch.randn(rows_local, generator=g, device=dev)
        if beta[j] != 0:
            logit += float(beta[j]) * c
        cols.append(c)
    logit += 0.5 * torch.sin(3 * cols[0]) * cols[1]
    y = (torch.rand(rows_local, generator=g, device=dev) < torch.sigmoid(logit)).to(torch.int32)
    del logit
    from h2o3_amd.core.frame import H2OFrame
    from h2o3_amd.core.vec import Vec, T_REAL, T_ENUM
    names = [f"x{j}" for j in range(F)]
    dom = [f"L{i}" for i in range(args.cat_card)]
    vecs = [Vec(c, T_ENUM, dom) if c.dtype == torch.int32 else Vec(c, T_REAL) for c in cols] + \
        [Vec(y, T_ENUM, ["0", "1"])]
    fr = H2OFrame.from_vecs(vecs, names + ["y"])
    return fr, names, y


def _launch(n):
    """Run this script on n ranks (one process per GPU) under
    torch.distributed.run on 127.0.0.1 and return its exit status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--cols", type=int, default=100)
    ap.add_argument("--max-depth", type=int, default=8)
    ap.add_argument("--algo", default="gbm", choices=["gbm", "glm", "drf", "kmeans", "dl", "pca"])
    ap.add_argument("--hidden", default="200,200", help="DL hidden layers (--algo dl)")
    ap.add_argument("--batch", type=int, default=1024, help="DL mini-batch rows (--algo dl)")
    ap.add_argument("--glm-lambda", type=float, default=0.0,
                    help="GLM lambda (--algo glm); > 0 with --glm-alpha > 0 measures the l1 (COD) path")
    ap.add_argument("--glm-alpha", type=float, default=0.5, help="GLM elastic-net alpha (used when lambda > 0)")
    ap.add_argument("--k", type=int, default=16, help="K-Means clusters (--algo kmeans)")
    ap.add_argument("--cat-cols", type=int, default=0,
                    help="replace this many of the --cols columns by categoricals (DRF config: mixed num/cat)")
    ap.add_argument("--cat-card", type=int, default=1000, help="cardinality of the categorical columns")
    ap.add_argument("--histogram-type", default="QuantilesGlobal")
    ap.add_argument("--nbins", type=int, default=255)
    ap.add_argument("--no-glm", action="store_true",
                    help="--algo gbm: skip the companion GLM measurement (the headline metric is GBM trees/s + "
                         "GLM iters/s on the same 100M x 100 frame; the GLM figure is reported as extra keys)")
    args = ap.parse_args()

    ws = os.environ.get("WORLD_SIZE")
    if ws is None and args.gpus > 1:
        # self-launch: one rank per GPU as child processes of torch.distributed.run,
        # started before this process touches the GPU
        return _launch(args.gpus)
    if ws is not None and int(ws) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
        return 2

    import torch
    import torch.distributed as dist
    import h2o3_amd
    from h2o3_amd.parallel import cloud

    h2o3_amd.init(verbose=False)
    world, rank = cloud.world(), cloud.rank()
    dev = cloud.device()
    rows_local = args.rows // world + (1 if rank < args.rows % world else 0)
    F = args.cols

    fr, names, y = make_frame(args, dev, rank, rows_local)
    from h2o3_amd.models.base import TrainSpec

    extra_cfg = {}
    if args.algo == "gbm":
        from h2o3_amd.models.tree.gbm import GBMDriver, H2OGradientBoostingEstimator
        est = H2OGradientBoostingEstimator(ntrees=500, max_depth=args.max_depth, seed=42,
                                           histogram_type=args.histogram_type, nbins=args.nbins,
                                           ignore_const_cols=False)
        spec = TrainSpec(fr, names, "y")
        est._spec = spec
        drv = GBMDriver(est, spec)
        step = drv.step
        metric = "gbm_trees_per_sec"
        unit = "trees/s"
        model = f"GBM binomial {args.rows / 1e6:g}Mx{F} ntrees=500 max_depth={args.max_depth}"
    elif args.algo == "drf":
        from h2o3_amd.models.tree.drf import DRFDriver, H2ORandomForestEstimator
        est = H2ORandomForestEstimator(ntrees=1000, max_depth=args.max_depth if args.max_depth != 8 else 20,
                                       seed=42, histogram_type=args.histogram_type, nbins=args.nbins,
                                       ignore_const_cols=False)
        spec = TrainSpec(fr, names, "y")
        est._spec = spec
        drv = DRFDriver(est, spec)
        step = drv.step
        metric = "drf_trees_per_sec"
        unit = "trees/s"
        model = f"DRF binomial {args.rows // 1_000_000}Mx{F} ({args.cat_cols} cat, card {args.cat_card}) ntrees=1000"
    elif args.algo == "kmeans":
        # one step = one Lloyd iteration: fused HIP pass (distances, arg-min,
        # per-cluster sums) + all-reduce + center update
        from h2o3_amd.models.kmeans import H2OKMeansEstimator
        from h2o3_amd.ops import cluster_ops
        from h2o3_amd.parallel import collectives as coll
        est = H2OKMeansEstimator(k=args.k, seed=42, standardize=False)
        spec = TrainSpec(fr, names, None)
        from h2o3_amd.models.datainfo import DataInfo
        est._dinfo = DataInfo(fr, names, standardize=False, use_all_factor_levels=True, pad_to=4)
        Xk, _ = est._design(fr)
        del fr
        C = [est._init_centers(Xk, None, args.k, __import__("numpy").random.RandomState(1))]
        asg = torch.full((Xk.shape[0],), -1, dtype=torch.int32, device=dev)
        xabs = cluster_ops.abs_bound(Xk)

        def step():
            st = cluster_ops.lloyd_pass(Xk, C[0], None, asg, xabs_max=xabs)
            coll.allreduce_(st.vec)
            C[0] = torch.where(st.weights.view(-1, 1) > 0, st.sums / st.weights.clamp_min(1e-300).view(-1, 1), C[0])
        metric = "kmeans_iters_per_sec"
        unit = "iters/s"
        model = f"KMeans k={args.k} {args.rows / 1e6:g}Mx{F}"
        extra_cfg = {"distance_precision": "f32 MFMA (v_mfma_f32_16x16x4_f32), f64 cross-workgroup sums"}
    elif args.algo == "pca":
        # one step = one PCA fit of rank k (pca_method="Randomized") + the
        # projection of every row: the MFMA Gram pass (gram.hip) and the
        # covariance, the subspace iterations on the P x P covariance, then
        # X V on the skinny MFMA kernel (kmeans.hip, cluster_ops.xv)
        from h2o3_amd.models.datainfo import DataInfo
        from h2o3_amd.models.clustering import _top_eig
        from h2o3_amd.ops import cluster_ops, linalg_ops
        from h2o3_amd.parallel import collectives as coll
        from h2o3_amd.models.clustering import gram_and_mean
        # pad_to=32 as the PCA model's expansion (clustering._transform_info):
        # the Gram kernel's column tiling; one padding column carries the 1s
        di = DataInfo(fr, names, standardize=False, use_all_factor_levels=True, pad_to=32)
        Xp, _ = di.expand(fr)
        del fr
        P = di.P
        kk = args.k

        def step():
            G, mu, nrow = gram_and_mean(Xp, P)
            cov = (G - nrow * torch.outer(mu, mu)) / max(nrow - 1, 1)
            ev, V = _top_eig(cov, kk, "randomized", 30, 1)
            Vp = torch.zeros((Xp.shape[1], V.shape[1]), dtype=torch.float64)
            Vp[:P] = V
            cluster_ops.xv(Xp, Vp, min_rows=0)
        metric = "pca_fits_per_sec"
        unit = "fits/s"
        model = f"PCA Randomized k={args.k} {args.rows / 1e6:g}Mx{F} (Gram pass + subspace iterations + projections)"
        extra_cfg = {"gram": "gram.hip MFMA, f64 across row blocks", "projection": "kmeans.hip skinny MFMA (f32)"}
    elif args.algo == "dl":
        # one step = one mini-batch training step of the MLP (forward, backward,
        # per-row ADADELTA update); value = training samples / s
        from h2o3_amd.models.deeplearning import H2ODeepLearningEstimator
        from h2o3_amd.models.datainfo import DataInfo
        hidden = [int(h) for h in args.hidden.split(",")]
        est = H2ODeepLearningEstimator(hidden=hidden, activation="RectifierWithDropout", seed=42,
                                       input_dropout_ratio=0.1)
        est._dinfo = DataInfo(fr, names, standardize=True, use_all_factor_levels=True, pad_to=0)
        Xd, _ = est._dinfo.expand(fr, pad=False)
        Yd = y.long()
        del fr
        est._layers = est._build(Xd.shape[1], 2, True)
        est._processed = 0.0
        hp = dict(K=2, ae=False, bs=args.batch, ada=True, rate0=0.005, anneal=1e-6, decay=1.0, mom_start=0.0,
                  mom_ramp=1e6, mom_stable=0.0, has_mom=False, l1=0.0, l2=0.0, max_w2=3.4e38, sparsity=0.0)
        gdl = torch.Generator(device=dev).manual_seed(7)
        nloc = Xd.shape[0]
        gstep = est._step_graph(Xd, Yd, None, hp, None) if est._graph_ok(Xd, hp, None) else None

        def step():
            idx = torch.randint(0, nloc, (args.batch,), generator=gdl, device=dev)
            if gstep is not None:
                gstep["idx"].copy_(idx)
                gstep["g"].replay()
            else:
                est._train_step(Xd.index_select(0, idx), Yd.index_select(0, idx), None, 1000, hp)
        metric = "dl_samples_per_sec"
        unit = "samples/s"
        model = f"DeepLearning MLP {args.cols}-{args.hidden}-2 RectifierWithDropout, batch {args.batch}"
        extra_cfg = {"hidden": hidden, "batch": args.batch, "hip_graph": gstep is not None}
    else:
        from h2o3_amd.models.glm.glm import GLMDriver, H2OGeneralizedLinearEstimator
        kw = {"lambda_": args.glm_lambda}
        if args.glm_lambda > 0:
            kw["alpha"] = args.glm_alpha
        est = H2OGeneralizedLinearEstimator(family="binomial", solver="IRLSM", **kw)
        spec = TrainSpec(fr, names, "y")
        est._spec = spec
        drv = GLMDriver(est, spec)
        step = drv.step
        metric = "glm_iters_per_sec"
        unit = "iters/s"
        model = f"GLM binomial IRLSM {args.rows / 1e6:g}Mx{F}" + \
            (f" lambda={args.glm_lambda:g} alpha={args.glm_alpha:g}" if args.glm_lambda > 0 else "")
        extra_cfg = {"gram_precision": _GLM_PRECISION, "lambda": args.glm_lambda,
                     "alpha": args.glm_alpha if args.glm_lambda > 0 else None}

    def sync():
        torch.cuda.synchronize() if dev.type == "cuda" else None
        if world > 1:
            cloud.barrier()

    for _ in range(args.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    value = args.steps / el
    if args.algo == "dl":
        value = args.steps * args.batch * world / el
    extra = {}
    if args.algo == "gbm":
        # training-quality sanity (not timed): logloss of the boosted model so far
        import math
        p = drv.predictions().clamp(1e-7, 1 - 1e-7)
        yy = (y == 1).to(torch.float32)
        ll = float(-(yy * torch.log(p) + (1 - yy) * torch.log(1 - p)).mean())
        extra["train_logloss_after"] = round(ll, 5)
        extra["trees_built"] = len(drv.forest)
    if args.algo == "glm":
        # convergence sanity (not timed): deviance of the last iteration and the
        # final coefficient step
        extra["train_deviance_per_row"] = round(float(drv.last_dev) / float(drv.wsum), 6)
        extra["iters"] = int(drv.iter)
        extra["hessian_tier"] = getattr(drv, "_hprec", None) or ("f64" if dev.type == "cpu" else None)
        extra_cfg["gram_precision"] = _glm_precision(extra["hessian_tier"])
        k_ = getattr(drv, "hessian_kappa", None)
        extra["hessian_kappa"] = None if k_ is None else round(float(k_), 3)
    if args.algo == "gbm" and not args.no_glm:
        # companion half of the headline metric: GLM binomial IRLSM iterations/s
        # on the SAME frame, timed separately with the same barrier + sync
        # discipline (the GBM value / ms_per_step above are not affected)
        from h2o3_amd.models.glm.glm import GLMDriver, H2OGeneralizedLinearEstimator
        gest = H2OGeneralizedLinearEstimator(family="binomial", solver="IRLSM", lambda_=0.0)
        gspec = TrainSpec(fr, names, "y")
        gest._spec = gspec
        gdrv = GLMDriver(gest, gspec)
        for _ in range(args.warmup):
            gdrv.step()
        sync()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            gdrv.step()
        sync()
        gel = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([gel], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            gel = float(t.item())
        extra["glm_iters_per_sec"] = round(args.steps / gel, 4)
        extra["glm_ms_per_iter"] = round(1000 * gel / args.steps, 3)
        extra["glm_model"] = f"GLM binomial IRLSM {args.rows / 1e6:g}Mx{F} (same frame, {args.steps} timed iterations)"
        extra["glm_hessian_tier"] = getattr(gdrv, "_hprec", None) or ("f64" if dev.type == "cpu" else None)
        extra["glm_precision"] = _glm_precision(extra["glm_hessian_tier"])
    from h2o3_amd.utils import timer
    if timer.ENABLED and rank == 0:
        print("phases(ms,count):", timer.report(), file=sys.stderr)
    if rank == 0:
        out = {"metric": metric, "value": round(value, 4), "unit": unit, "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(1000 * el / args.steps, 3), "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
               "data": "synthetic (random normal features, logistic label), generated on device",
               "config": {"model": model, "rows": args.rows, "cols": F,
                          **({} if args.algo in ("glm", "kmeans", "dl", "pca") else {"max_depth": est._parms.get("max_depth"),
                                                            "histogram_type": args.histogram_type,
                                                            "nbins": args.nbins}),
                          "global_batch": args.rows, "seq_len": None, "parallelism": f"dp{world}", **extra_cfg},
               **extra}
        print(json.dumps(out))


if __name__ == "__main__":
    sys.exit(main() or 0)
