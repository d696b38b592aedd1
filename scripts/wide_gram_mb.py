"""Fused wide Gram kernels alone at 12.5M x 1000: time per launch of the
256 x 256-tile kernel (bf16x3 default, and the one-MFMA bf16 Hessian) and the
128 x 128 one, plus timing-only arms
whose X loads are dropped by the buffer range check (dbg=1: MFMA + LDS +
conversion cost without HBM/L2 traffic).  argv: rows (default 12.5M)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.ops import linalg_ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
P = 1000
lib = linalg_ops._lib()
X = torch.randn(N, P, device="cuda")
w = torch.zeros(-(-N // 64) * 64, device="cuda")   # weights zero-padded to whole 64-row chunks
w[:N] = torch.rand(N, device="cuda")
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
arms = ((256, 25, 0, 1), (256, 25, 1, 1), (256, 25, 0, 0), (256, 25, 1, 0), (128, 14, 0, 1))
if os.environ.get("MB_ARMS") == "bf16":
    arms = ((256, 25, 0, 0), (256, 25, 1, 0))
for T, S, dbg, bf3 in arms:
    NB = -(-(P + 1) // T)
    npairs = NB * (NB + 1) // 2
    part = torch.zeros((npairs * S, T, T), dtype=torch.float64, device="cuda")
    args = [ctypes.c_void_p(X.data_ptr()), P, P, N, ctypes.c_void_p(w.data_ptr()), S, 1024,
            ctypes.c_void_p(part.data_ptr()), dbg] + ([bf3] if T == 256 else []) + [stream]
    fn = lib.h2o_glm_wide_gram256 if T == 256 else lib.h2o_glm_wide_gram
    f = lambda: fn(*args)  # noqa: E731
    assert f() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    kr = 32 if bf3 or os.environ.get("H2O3_WIDE_KR") == "32" else 64
    print(f"T={T} S={S:3d} dbg={dbg} bf3={bf3} KR={kr}: {ms:7.2f} ms/launch", flush=True)
