"""Frame kernels (ops/csrc/frame.hip) vs their torch paths: batched rollups
against Vec.rollups, the tiled numeric expansion against DataInfo.expand's
per-column loop (bitwise: the same f64 arithmetic)."""
import math

import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _init():
    import h2o3_amd as h2o
    h2o.init(device="cuda:0", verbose=False)


def _frame(n=50_003, seed=0):
    import h2o3_amd as h2o
    g = np.random.default_rng(seed)
    a = g.standard_normal(n).astype(np.float32) * 3 + 7
    b = g.standard_normal(n)
    b[::7] = np.nan
    b[5] = np.inf
    b[9] = -np.inf
    c = g.integers(-5, 6, n).astype(np.float64)
    c[3] = 0.0
    d = np.full(n, 2.5)
    e = np.full(n, np.nan)
    f = (1e8 + g.standard_normal(n)).astype(np.float64)        # large offset: variance stability
    df = pd.DataFrame({"a": a, "b": b, "c": c, "d": d, "e": e, "f": f, "k": np.where(a > 7, "x", "y")})
    return h2o.H2OFrame(df)


def test_rollups_many_matches_vec_rollups():
    from h2o3_amd.ops import frame_ops
    fr1, fr2 = _frame(), _frame()
    cols = ["a", "b", "c", "d", "e", "f"]
    assert all(frame_ops.batchable(fr1.vec(c)) for c in cols)
    assert frame_ops.rollups_many([fr1.vec(c) for c in cols + ["k"]]) == len(cols)
    from h2o3_amd.core.vec import Vec
    for c in cols:
        got = fr1.vec(c)._rollups
        v2 = fr2.vec(c)
        want = Vec(v2.data.cpu(), v2.type).rollups()            # the torch path (host tensors)
        assert fr2.vec(c).rollups()["nacnt"] == want["nacnt"]    # Vec.rollups on the device: the kernel
        for k in ("nacnt", "zeros", "isInt", "nrow", "pinfs", "ninfs"):
            assert got[k] == want[k], (c, k, got[k], want[k])
        for k in ("min", "max", "mean", "sigma"):
            if math.isnan(want[k]):
                assert math.isnan(got[k]), (c, k)
            else:
                assert got[k] == pytest.approx(want[k], rel=1e-12, abs=1e-12), (c, k, got[k], want[k])


@pytest.mark.parametrize("standardize", [True, False])
def test_expand_numeric_kernel_matches_torch_loop(standardize, monkeypatch):
    from h2o3_amd.models.datainfo import DataInfo
    fr = _frame(20_011, seed=3)
    x = ["a", "b", "c", "f", "k"]
    di = DataInfo(fr, x, standardize=standardize)
    X1, ok1 = di.expand(fr)
    monkeypatch.setattr(DataInfo, "_expand_numeric_fast", lambda *a, **k: False)
    X2, ok2 = di.expand(fr)
    assert torch.equal(ok1, ok2)
    assert torch.equal(X1, X2)
    assert (X1 != 0).any()
