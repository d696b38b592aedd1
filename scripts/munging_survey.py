"""Frame munging at scale on the GPU (ROWS rows, default 20M): wall time of
each H2OFrame op (sort, group_by, merge, quantile, table, unique, cut,
ifelse, cumsum, rbind, split, impute, isin, apply, kfold, fillna, ...).
One JSON line per op; ops over 5 s are flagged."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import h2o3_amd as h2o  # noqa: E402
from h2o3_amd.core.frame import H2OFrame  # noqa: E402
from h2o3_amd.core.vec import Vec, T_REAL, T_ENUM, T_INT  # noqa: E402

N = int(os.environ.get("ROWS", 20_000_000))
h2o.init(verbose=False)
from h2o3_amd.parallel import cloud  # noqa: E402
dev = cloud.device()
g = torch.Generator(device=dev).manual_seed(3)
a = torch.randn(N, generator=g, device=dev)
a[::97] = float("nan")
b = torch.randn(N, generator=g, device=dev) * 10
k = torch.randint(0, 1000, (N,), generator=g, device=dev, dtype=torch.int32)
ik = torch.randint(0, 100000, (N,), generator=g, device=dev).to(torch.float32)
fr = H2OFrame.from_vecs([Vec(a, T_REAL), Vec(b, T_REAL), Vec(k, T_ENUM, [f"L{i}" for i in range(1000)]),
                         Vec(ik, T_INT)], ["a", "b", "k", "ik"])
small = H2OFrame.from_vecs([Vec(torch.arange(1000, dtype=torch.int32, device=dev), T_ENUM,
                                [f"L{i}" for i in range(1000)]),
                            Vec(torch.rand(1000, device=dev), T_REAL)], ["k", "z"])
small_i = H2OFrame.from_vecs([Vec(torch.arange(100000, device=dev).to(torch.float32), T_INT),
                              Vec(torch.rand(100000, device=dev), T_REAL)], ["ik", "w"])


def run(name, f):
    torch.cuda.synchronize() if dev.type == "cuda" else None
    t0 = time.perf_counter()
    try:
        r = f()
        torch.cuda.synchronize() if dev.type == "cuda" else None
        dt = time.perf_counter() - t0
        shape = getattr(r, "shape", None)
        print(json.dumps({"op": name, "rows": N, "s": round(dt, 3), "shape": list(shape) if shape else None,
                          "slow": dt > 5}), flush=True)
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"op": name, "error": f"{type(e).__name__}: {e}"[:300]}), flush=True)


run("sort_num", lambda: fr.sort("b"))
run("sort_enum_num", lambda: fr.sort(["k", "b"]))
run("group_by_mean", lambda: fr.group_by("k").mean("b").count().get_frame())
run("group_by_int_sum", lambda: fr.group_by("ik").sum("b").get_frame())
run("merge_enum_1k", lambda: fr.merge(small))
run("merge_int_100k", lambda: fr.merge(small_i))
run("quantile", lambda: fr[["a", "b"]].quantile([0.1, 0.5, 0.9]))
run("table_enum", lambda: fr["k"].table())
run("unique_int", lambda: fr["ik"].unique())
run("cut", lambda: fr["b"].cut([-100, -10, 0, 10, 100]))
run("ifelse", lambda: (fr["b"] > 0).ifelse(fr["a"], fr["b"]))
run("cumsum", lambda: fr["b"].cumsum())
run("rbind", lambda: fr.rbind(fr))
run("split_frame", lambda: fr.split_frame([0.7], seed=1)[0])
run("impute_mean", lambda: fr.deep_copy("imp").impute("a", method="mean"))
run("isin", lambda: fr["k"].isin(["L1", "L2", "L3"]))
run("apply_mean", lambda: fr[["a", "b"]].apply(lambda x: x.mean(), axis=0))
run("kfold", lambda: fr.kfold_column(5, 1))
run("fillna", lambda: fr[["a"]].fillna("forward", 0, 10))
run("na_omit", lambda: fr.na_omit())
run("scale", lambda: fr[["a", "b"]].scale())
run("hist", lambda: fr["b"].hist(breaks=50, plot=False))
run("cor", lambda: fr[["a", "b"]].cor(na_rm=True))
run("asfactor_int", lambda: fr["ik"].asfactor())
run("as_data_frame_1M", lambda: fr[0:1000000, :].as_data_frame())
run("rows_filter", lambda: fr[fr["b"] > 5, :])
run("strings_1M", lambda: fr[0:1000000, "k"].ascharacter().toupper())
