"""GLM binomial IRLSM with lambda search on the wide config shape (the per-GPU
share of 100M x 1000 at 8 GPUs by default: 12.5M x 1000), timed end to end.
Usage: python scripts/glm_lambda_search.py [rows] [cols] [nlambdas]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    import h2o3_amd
    from h2o3_amd.parallel import cloud
    from h2o3_amd.models.glm.glm import H2OGeneralizedLinearEstimator
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
    cols = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    nl = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    h2o3_amd.init(verbose=False)
    args = argparse.Namespace(cols=cols, cat_cols=0, cat_card=2)
    fr, names, _ = bench.make_frame(args, cloud.device(), cloud.rank(), rows // cloud.world())
    est = H2OGeneralizedLinearEstimator(family="binomial", solver="IRLSM", lambda_search=True, nlambdas=nl)
    t0 = time.perf_counter()
    est.train(x=names, y="y", training_frame=fr)
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    el = time.perf_counter() - t0
    path = est._output.get("regularization_path") or {}
    lams = path.get("lambdas") if isinstance(path, dict) else None
    it = len(getattr(est, "_scoring_history", []) or [])
    nz = sum(1 for k, v in est.coef().items() if v != 0 and k != "Intercept")
    print(json.dumps({"rows": rows, "cols": cols, "nlambdas": nl, "seconds": round(el, 2), "iterations": it,
                      "lambdas_fit": len(lams) if lams is not None else None, "nonzero_coefs": nz,
                      "lambda_best": est._output.get("lambda_best"),
                      "ms_per_iteration": round(1000 * el / max(1, int(it or 1)), 1)}))
    from h2o3_amd.utils import timer
    if timer.ENABLED:
        print("phases(ms,count):", timer.report())


if __name__ == "__main__":
    main()
