"""Frame kernels alone (ops/csrc/frame.hip): batched rollups (two passes)
and the model-matrix expansion for N rows x C float32 columns.
argv: N C (default 12.5M 1000)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    import h2o3_amd
    from h2o3_amd.core.vec import Vec, T_REAL
    from h2o3_amd.ops import frame_ops
    h2o3_amd.init(verbose=False)
    cols = [torch.randn(N, device="cuda") for _ in range(C)]
    X = torch.empty((N, -(-(C + 2) // 32) * 32), device="cuda")
    for rep in range(3):
        vs = [Vec(c, T_REAL) for c in cols]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        frame_ops.rollups_many(vs)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        frame_ops.expand_numeric(cols, [0.0] * C, [0.0] * C, [1.0] * C, X, 0)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    gb = N * C * 4 / 1e9
    print(f"N={N} C={C}: rollups {1e3 * (t1 - t0):.1f} ms ({2 * gb / (t1 - t0) / 1e3:.2f} TB/s over 2 passes), "
          f"expand {1e3 * (t2 - t1):.1f} ms ({2 * gb / (t2 - t1) / 1e3:.2f} TB/s read+write)", flush=True)


if __name__ == "__main__":
    main()
