"""K-Means Lloyd kernel microbenchmark: per-phase cost via skip flags
(h2o_kmeans_set_debug) at 100M x 100, plus grid-size sweep."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from h2o3_amd.ops import cluster_ops

N, P, k = int(os.environ.get("N", 100_000_000)), int(os.environ.get("P", 100)), int(os.environ.get("K", 16))
X = torch.randn((N, P), device="cuda")
C = X[:k].double()
a = torch.full((N,), -1, dtype=torch.int32, device="cuda")
lib = cluster_ops._lib()
lib.h2o_kmeans_set_debug.argtypes = [cluster_ops._ci]


XA = cluster_ops.abs_bound(X) if os.environ.get("FX", "1") == "1" else None


def run(flags, G=None, reps=5):
    lib.h2o_kmeans_set_debug(flags)
    cluster_ops.lloyd_pass(X, C, None, a, n_groups=G, xabs_max=XA)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        cluster_ops.lloyd_pass(X, C, None, a, n_groups=G, xabs_max=XA)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


lib.h2o_kmeans_resident_per_cu.argtypes = [cluster_ops._ci] * 3 + [cluster_ops._cf]
print("resident/CU", lib.h2o_kmeans_resident_per_cu(k, P, 1, 1.0 if XA else 0.0), "fixed-point sums", XA is not None,
      flush=True)
for f, name in [(0, "full"), (1, "no mfma"), (2, "no sums"), (4, "no rowstats"), (8, "no global loads"),
                (16, "no lds staging"), (2 | 4, "no sums+rows"), (1 | 2 | 4, "loads+staging only"),
                (1 | 2 | 4 | 16, "loads only"), (1 | 2 | 4 | 8 | 16, "empty loop")]:
    print(f"{name:22s} {run(f):8.2f} ms", flush=True)
for G in (256, 512, 768, 1024, 2048):
    print(f"G={G:5d} full {run(0, G):8.2f} ms", flush=True)
lib.h2o_kmeans_set_debug(0)

# baseline: the same Lloyd pass as plain torch ops (library GEMM + argmin +
# one-hot GEMM for the sums) on the first 10M rows, scaled to N
NB = min(N, 10_000_000)


def torch_pass():
    cn = (C.float() ** 2).sum(1)
    out_s = torch.zeros((k, P), device="cuda", dtype=torch.float64)
    for i in range(0, NB, 1 << 22):
        Xc = X[i:min(i + (1 << 22), NB)]
        d = cn.view(1, -1) - 2.0 * (Xc @ C.float().T)
        idx = d.argmin(1)
        oh = torch.nn.functional.one_hot(idx, k).float()
        out_s += (oh.T @ Xc).double()
    return out_s


torch_pass()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    torch_pass()
torch.cuda.synchronize()
print(f"torch ops baseline     {(time.perf_counter() - t) / 3 * 1e3 * N / NB:8.2f} ms (scaled from {NB} rows)",
      flush=True)
