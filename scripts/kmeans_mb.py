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


def run(flags, G=None, reps=5):
    lib.h2o_kmeans_set_debug(flags)
    cluster_ops.lloyd_pass(X, C, None, a, n_groups=G)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        cluster_ops.lloyd_pass(X, C, None, a, n_groups=G)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


print("resident/CU", lib.h2o_kmeans_resident_per_cu(k, P, 1), flush=True)
for f, name in [(0, "full"), (1, "no mfma"), (2, "no sums"), (4, "no rowstats"), (8, "no global loads"),
                (16, "no lds staging"), (2 | 4, "no sums+rows"), (1 | 2 | 4, "loads+staging only"),
                (1 | 2 | 4 | 16, "loads only"), (1 | 2 | 4 | 8 | 16, "empty loop")]:
    print(f"{name:22s} {run(f):8.2f} ms", flush=True)
for G in (256, 512, 768, 1024, 2048):
    print(f"G={G:5d} full {run(0, G):8.2f} ms", flush=True)
lib.h2o_kmeans_set_debug(0)

# baseline: the same Lloyd pass as plain torch ops (library GEMM + argmin + index_add)
def torch_pass():
    cn = (C.float() ** 2).sum(1)
    out_s = torch.zeros((k, P), device="cuda", dtype=torch.float64)
    for i in range(0, N, 1 << 24):
        Xc = X[i:i + (1 << 24)]
        d = cn.view(1, -1) - 2.0 * (Xc @ C.float().T)
        idx = d.argmin(1)
        out_s.index_add_(0, idx, Xc.double())
    return out_s


torch_pass()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    torch_pass()
torch.cuda.synchronize()
print(f"torch ops baseline     {(time.perf_counter() - t) / 3 * 1e3:8.2f} ms", flush=True)
