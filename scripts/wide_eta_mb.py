"""Wide GLM eta / weight / gradient pass alone (glm_wide_split_kernel in
weight-only mode) at 12.5M x P: ms per pass and the X read rate for
workgroup counts given on the command line (the rows-in-flight variant is
picked by H2O3_WIDE_RW, read once per process)."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.ops import linalg_ops  # noqa: E402

N, P = 12_500_000, int(os.environ.get("MB_P", "1000"))
ldx = int(os.environ.get("MB_LDX", str(P)))
X = torch.randn(N, ldx, device="cuda")
Pa = -(-(P + 2) // 64) * 64
beta = 0.01 * torch.randn(P, device="cuda")
y = (torch.rand(N, device="cuda") < 0.5).float()
wr = torch.empty(N, device="cuda")
lib = linalg_ops._lib()
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
rw = os.environ.get("H2O3_WIDE_RW", "1")
for blocks in [int(b) for b in sys.argv[1:]] or [0]:
    blocks = blocks or linalg_ops._wide_split_grid(lib, Pa)   # 0: whole resident rounds
    dev = torch.zeros(blocks, dtype=torch.float64, device="cuda")
    g = torch.zeros((blocks, Pa), dtype=torch.float64, device="cuda")

    def run():
        rc = lib.h2o_glm_wide_split(ctypes.c_void_p(X.data_ptr()), ldx, P, Pa, N, ctypes.c_void_p(beta.data_ptr()),
                                    0.1, ctypes.c_void_p(y.data_ptr()), None, None, 1, 1, 0.0, 0.0, None,
                                    ctypes.c_void_p(dev.data_ptr()), blocks, ctypes.c_void_p(g.data_ptr()),
                                    ctypes.c_void_p(wr.data_ptr()), stream)
        assert rc == 0, rc
    run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 10 * 1e3
    print(f"P={P} ldx={ldx} RW={rw} blocks={blocks:5d}: {ms:6.2f} ms  {N * P * 4 / ms / 1e9:5.2f} TB/s", flush=True)
