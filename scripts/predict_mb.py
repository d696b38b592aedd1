"""Forest scoring throughput: a GBM of T trees (depth D) trained on a small
synthetic frame, then Forest.predict (the HIP scoring kernel,
tree_predict.hip) over N rows x F float32 features already on the device.
Prints rows/s and row-trees/s.  argv: N T D (default 10M 100 8)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    D = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    F = 100
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(0)
    n0 = 200_000
    Xs = rng.standard_normal((n0, F)).astype(np.float32)
    y = (Xs[:, :10].sum(1) + 0.5 * rng.standard_normal(n0) > 0).astype(int)
    df = pd.DataFrame(Xs, columns=[f"x{j}" for j in range(F)])
    df["y"] = np.where(y == 1, "a", "b")
    fr = h2o.H2OFrame(df)
    m = H2OGradientBoostingEstimator(ntrees=T, max_depth=D, seed=1, min_rows=1, learn_rate=0.05)
    m.train(y="y", training_frame=fr)
    forest = m._forest
    nodes = sum(t.n_nodes for t in forest.trees)
    X = torch.randn(F, N, device="cuda")
    out = forest.predict(X, 1)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        out = forest.predict(X, 1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    # check a slice against the torch reference walk
    P = forest.pack(X.device)
    ref = forest._predict_torch(X[:, :20000], 1, P)
    err = float((ref - out[:20000]).abs().max())
    print(f"N={N} T={len(forest.trees)} depth={D} nodes={nodes}: {dt * 1e3:.2f} ms/predict, "
          f"{N / dt / 1e6:.1f} M rows/s, {N * len(forest.trees) / dt / 1e9:.2f} G row-trees/s, max err {err:.2e}",
          flush=True)


if __name__ == "__main__":
    main()
