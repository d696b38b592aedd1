"""GLM coefficient parity at the bench scale.

Fits the bench's binomial IRLSM problem (100M x 100, synthetic, standardized
design) to convergence three times -- bf16x3 Hessian with the exact f32/f64
gradient channel (default), bf16x3 Gram with its own X'Wz right-hand side
(H2O3_GLM_EXACT_GRAD=0) and f32 MFMA (H2O3_GLM_BF3=0) -- then runs an independent fp64 IRLS on the
very same device design matrix (f32 values are exact in f64; Gram, X'Wz,
solve all in fp64) and reports per-iteration time of both MFMA paths and the
coefficient differences against the fp64 solution.

Usage: python scripts/glm_precision.py [--rows 100000000] [--out gpurun_out/glm_precision.json]
"""
import argparse
import json
import os
import statistics
import sys
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--cols", type=int, default=100)
    ap.add_argument("--out", default="gpurun_out/glm_precision.json")
    a = ap.parse_args()
    import torch
    import bench
    import h2o3_amd
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.models.glm.glm import GLMDriver, H2OGeneralizedLinearEstimator
    from h2o3_amd.parallel import cloud
    h2o3_amd.init(verbose=False)
    dev = cloud.device()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    args = SimpleNamespace(rows=a.rows, cols=a.cols, cat_cols=0, cat_card=2)
    fr, names, _ = bench.make_frame(args, dev, 0, a.rows)
    spec = TrainSpec(fr, names, "y")
    est = H2OGeneralizedLinearEstimator(family="binomial", solver="IRLSM", lambda_=0.0)
    est._spec = spec
    res = {"rows": a.rows, "cols": a.cols, "model": "GLM binomial IRLSM, lambda=0, standardized design"}
    drv = None
    # (H2O3_GLM_BF3, H2O3_GLM_EXACT_GRAD, H2O3_GLM_BF16): the default tier ladder
    # (one-MFMA bf16 Hessian while kappa < 32), bf16x3 pinned, the round-4
    # Gram right-hand side, f32 MFMA
    modes = {"default_tiers": ("1", "1", "1"), "bf16x3_exact_grad": ("1", "1", "0"),
             "bf16x3_gram_rhs": ("1", "0", "0"), "f32": ("0", "1", "0")}
    for name, (bf3, exact, bf16) in modes.items():
        os.environ["H2O3_GLM_BF3"] = bf3
        os.environ["H2O3_GLM_EXACT_GRAD"] = exact
        os.environ["H2O3_GLM_BF16"] = bf16
        drv = GLMDriver(est, spec)
        times = []
        while not drv.converged and drv.iter < 25:
            sync()
            t0 = time.time()
            drv.step()
            sync()
            times.append(time.time() - t0)
        res[name] = {
            "iterations": drv.iter, "ms_per_iter_median": 1000 * statistics.median(times),
            "ms_per_iter_all": [round(1000 * t, 3) for t in times], "beta_std": drv.beta.tolist(),
            "hessian_tier": getattr(drv, "_hprec", None), "hessian_kappa": getattr(drv, "hessian_kappa", None)}
        print(name, drv.iter, 1000 * statistics.median(times), flush=True)
    # independent fp64 IRLS on the same design (drv.X holds the standardized f32 rows)
    X, y, w = drv.X, drv.y, drv.w
    P = drv.P
    beta = torch.as_tensor(drv._init_beta, dtype=torch.float64, device=dev)
    chunk = 1 << 22
    t0 = time.time()
    it64 = 0
    for it64 in range(1, 26):
        G = torch.zeros((P + 1, P + 1), dtype=torch.float64, device=dev)
        b = torch.zeros(P + 1, dtype=torch.float64, device=dev)
        for s in range(0, X.shape[0], chunk):
            Xc = X[s:s + chunk, :P].to(torch.float64)
            Xa = torch.cat([Xc, torch.ones((Xc.shape[0], 1), dtype=torch.float64, device=dev)], 1)
            del Xc
            eta = Xa @ beta
            mu = torch.sigmoid(eta).clamp(1e-10, 1 - 1e-10)
            wi = mu * (1 - mu) * w[s:s + chunk]
            z = eta + (y[s:s + chunk] - mu) / (mu * (1 - mu))
            G += Xa.T @ (Xa * wi.view(-1, 1))
            b += Xa.T @ (wi * z)
            del Xa
        new = torch.linalg.solve(G, b)
        diff = float((new - beta).abs().max())
        beta = new
        print("fp64", it64, diff, flush=True)
        if diff < 1e-12:
            break
    sync()
    b64 = beta.cpu().tolist()
    res["fp64"] = {"iterations": it64, "seconds": time.time() - t0, "beta_std": b64}
    import numpy as np
    ref = np.array(b64)
    scale = max(float(np.abs(ref).max()), 1e-300)
    for k in modes:
        bb = np.array(res[k]["beta_std"])
        res[k]["max_abs_diff_vs_fp64"] = float(np.abs(bb - ref).max())
        res[k]["max_rel_diff_vs_fp64"] = float((np.abs(bb - ref) / np.maximum(np.abs(ref), 1e-3)).max())
        res[k]["max_diff_over_max_coef"] = float(np.abs(bb - ref).max() / scale)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk not in ("beta_std", "ms_per_iter_all")}
                      for k, v in res.items() if isinstance(v, dict)}, indent=1))


if __name__ == "__main__":
    main()
