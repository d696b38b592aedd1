"""Micro-benchmark of the bin-major histogram kernel by level shape and phase
(h2o_hist_bm_set_debug: 1 = no flush, 2 = no LDS atomics, 3 = loads only)."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2o3_amd.models.tree.binning import BinnedData  # noqa: E402
from h2o3_amd.ops import tree_ops  # noqa: E402

lib = tree_ops._lib()
lib.h2o_hist_bm_set_debug.argtypes = [ctypes.c_int]
for N in (12_500_000, 100_000_000):
    F, Fp, Bs = 100, 128, 256
    dev = "cuda"
    bd = BinnedData()
    bd.codes = torch.randint(0, 254, (N, Fp), dtype=torch.uint8, device=dev)
    bd.F, bd.Fp, bd.Bs, bd.code_bytes, bd.nrows_local = F, Fp, Bs, 1, N
    va = torch.randn(N, device=dev)
    vmax = tree_ops.channel_max(va, None, 0)
    shapes = [("root", torch.arange(N, dtype=torch.int32, device=dev), [0], [N])]
    for d in (3, 7):
        nodes = 2 ** d
        g = torch.Generator(device=dev).manual_seed(d)
        nid = torch.randint(0, nodes, (N,), generator=g, device=dev)
        order = torch.argsort(nid, stable=True).to(torch.int32)
        cnt = torch.bincount(nid, minlength=nodes).cpu().tolist()
        st = [0]
        for c in cnt[:-1]:
            st.append(st[-1] + c)
        b = list(range(0, nodes, 2))
        shapes.append((f"depth {d} ({len(b)} nodes, half rows)", order, [st[i] for i in b], [cnt[i] for i in b]))
    for (name, ridx, starts, counts), tb in [(sh, tb) for sh in shapes
                                             for tb in os.environ.get("TBS", "default").split(",")]:
        if tb == "default":
            os.environ.pop("H2O3_HIST_TB", None)
            os.environ.pop("H2O3_HIST_CHUNK", None)
        elif tb.startswith("c"):
            os.environ.pop("H2O3_HIST_TB", None)
            os.environ["H2O3_HIST_CHUNK"] = tb[1:]
        else:
            os.environ["H2O3_HIST_TB"] = tb
        name = f"{name} TB={tb}"
        line = []
        for flag in (0, 1, 2, 3, 5):
            os.environ["H2O3_HIST_BM_RED"] = "0" if flag == 5 else "1"
            lib.h2o_hist_bm_set_debug(0 if flag == 5 else flag)
            tree_ops.hist_build(bd, ridx, va, None, 0, starts, counts, len(starts), vmax=vmax, unit_w=True, posv=True)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(5):
                tree_ops.hist_build(bd, ridx, va, None, 0, starts, counts, len(starts), vmax=vmax, unit_w=True,
                                    posv=True)
            torch.cuda.synchronize()
            line.append((time.perf_counter() - t) / 5 * 1e3)
        lib.h2o_hist_bm_set_debug(0)
        print(f"N={N/1e6:g}M {name:44s} full {line[0]:7.3f}  no-flush {line[1]:7.3f}  no-atomics {line[2]:7.3f}  "
              f"loads-only {line[3]:7.3f}  atomic-flush {line[4]:7.3f} ms", flush=True)
    del bd, va, shapes
    torch.cuda.empty_cache()
