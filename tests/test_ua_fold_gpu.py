"""UniformAdaptive fold on the device (tree_split.hip ua_range_kernel /
ua_fold_kernel) against the torch chain it replaces (engine._adapt_hist,
H2O3_UA_FOLD=torch), kernel level and model level.

Reference: DHistogram.java:366-386 (per-node uniform re-binning over the
node's observed range), DTree.java:337 (the parent's range for the children).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_fold(H, first, last, nb, isnum):
    Fl, n, Bs, C = H.shape
    B = Bs - 1
    Hn = H[:, :, :B]
    idx = torch.arange(B, device=H.device)
    L = (last - first + 1).clamp(min=1)
    inr = (idx >= first) & (idx <= last)
    coarse = torch.div((idx - first).clamp(min=0) * nb, L, rounding_mode="floor")
    nxt = torch.div((idx + 1 - first).clamp(min=0) * nb, L, rounding_mode="floor")
    is_end = inr & ((coarse != nxt) | (idx == last))
    is_end = is_end | (inr & (L <= nb))
    is_end = is_end | ~isnum.view(Fl, 1, 1)
    cs = torch.cumsum(Hn, 2)
    E = torch.where(is_end, idx, -1)
    pe_incl = torch.cummax(E, 2).values
    pe = torch.cat([torch.full_like(pe_incl[:, :, :1], -1), pe_incl[:, :, :-1]], 2)
    base = torch.where((pe >= 0).unsqueeze(-1), torch.gather(cs, 2, pe.clamp(min=0).unsqueeze(-1).expand(-1, -1, -1, C)),
                       torch.zeros_like(cs))
    Hf = torch.where(is_end.unsqueeze(-1), cs - base, torch.zeros_like(cs))
    Hf = torch.where(isnum.view(Fl, 1, 1, 1), Hf, Hn)
    return torch.cat([Hf, H[:, :, B:]], 2)


def _lib():
    from h2o3_amd.ops import _native
    lib = _native.get_lib("tree_split")
    assert lib is not None, "libtree_split.so not loaded"
    cv, ci = ctypes.c_void_p, ctypes.c_int
    lib.h2o_ua_range.argtypes = [cv, ci, ci, ci, cv, cv, cv]
    lib.h2o_ua_fold.argtypes = [cv, ci, ci, ci, ci, cv, cv, ci, cv, cv, cv]
    return lib


@pytest.mark.parametrize("B,C,nb", [(1024, 2, 20), (1024, 3, 512), (255, 2, 64), (20, 2, 20), (1000, 4, 37)])
def test_ua_kernels_match_torch_chain(B, C, nb):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(B + C + nb)
    Fl, n, Bs = 7, 13, B + 1
    H = torch.rand((Fl, n, Bs, C), generator=g, dtype=torch.float64) * 100
    # occupied ranges of different widths, a few empty rows
    lo = torch.randint(0, B, (Fl, n), generator=g)
    wd = torch.randint(0, B, (Fl, n), generator=g)
    hi = torch.minimum(lo + wd, torch.full_like(lo, B - 1))
    idx = torch.arange(B)
    keep = (idx.view(1, 1, -1) >= lo.unsqueeze(-1)) & (idx.view(1, 1, -1) <= hi.unsqueeze(-1))
    keep &= torch.rand((Fl, n, B), generator=g) > 0.3
    H[:, :, :B] *= keep.unsqueeze(-1)
    H[2, 5, :B] = 0
    H = H.cuda()
    isnum = torch.ones(Fl, dtype=torch.bool, device="cuda")
    isnum[3] = False
    rows = Fl * n
    fl = torch.empty(2 * rows, dtype=torch.int32, device="cuda")
    assert lib.h2o_ua_range(ctypes.c_void_p(H.data_ptr()), rows, Bs, C, ctypes.c_void_p(fl.data_ptr()),
                            ctypes.c_void_p(fl.data_ptr() + 4 * rows), torch.cuda.current_stream().cuda_stream) == 0
    occ = (H[:, :, :B] != 0).any(-1)
    ii = torch.arange(B, device="cuda")
    f_ref = torch.where(occ, ii, B).amin(-1)
    l_ref = torch.where(occ, ii, -1).amax(-1)
    torch.cuda.synchronize()
    assert torch.equal(fl[:rows].view(Fl, n).long(), f_ref)
    assert torch.equal(fl[rows:].view(Fl, n).long(), l_ref)
    # widen some ranges (a parent's range covers the child's)
    first = (f_ref - (torch.arange(rows, device="cuda").view(Fl, n) % 3)).clamp(min=0)
    last = l_ref.clone()
    out = torch.empty_like(H)
    f32, l32 = first.to(torch.int32).contiguous(), last.to(torch.int32).contiguous()
    isn = isnum.to(torch.uint8)
    assert lib.h2o_ua_fold(ctypes.c_void_p(H.data_ptr()), Fl, n, Bs, C, ctypes.c_void_p(f32.data_ptr()),
                           ctypes.c_void_p(l32.data_ptr()), nb, ctypes.c_void_p(isn.data_ptr()),
                           ctypes.c_void_p(out.data_ptr()), torch.cuda.current_stream().cuda_stream) == 0
    ref = _torch_fold(H, first.unsqueeze(-1), last.unsqueeze(-1), nb, isnum)
    torch.cuda.synchronize()
    # same run ends; sums differ only by f64 summation order
    assert torch.equal(out != 0, ref != 0)
    torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-9)


def test_uniform_adaptive_gbm_kernel_vs_torch_fold(monkeypatch):
    """A UniformAdaptive GBM grows the same trees with the device fold as with
    the torch chain (model level, 1024 top-level cells, depth 6)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pandas as pd
    import h2o3_amd
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    from h2o3_amd.ops import _native
    h2o3_amd.init(verbose=False)
    rng = np.random.RandomState(5)
    n = 20000
    X = rng.randn(n, 6).astype(np.float32)
    X[:, 2] = np.round(X[:, 2] * 3)         # few distinct values: narrow ranges
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(6)])
    df["c"] = rng.choice(list("abcde"), n)
    df["y"] = np.where(X[:, 0] + np.sin(3 * X[:, 1]) + 0.3 * rng.randn(n) > 0, "yes", "no")
    fr = h2o3_amd.H2OFrame(df)
    preds = {}
    for mode in ("torch", "hip"):
        monkeypatch.setenv("H2O3_UA_FOLD", mode)
        m = H2OGradientBoostingEstimator(ntrees=5, max_depth=6, seed=3, histogram_type="UniformAdaptive")
        m.train(y="y", training_frame=fr)
        preds[mode] = m.predict(fr).as_data_frame()["yes"].values
    np.testing.assert_allclose(preds["hip"], preds["torch"], rtol=1e-6, atol=1e-7)
    assert "libtree_split.so" in " ".join(_native.loaded_libs())


def test_uniform_adaptive_packed_wide_histogram(monkeypatch):
    """1024-cell (2-byte code) histograms with the packed single-atomic kernel
    (h2o_hist_build_pk) grow the same model as the two-channel kernel."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pandas as pd
    import h2o3_amd
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    h2o3_amd.init(verbose=False)
    rng = np.random.RandomState(9)
    n = 30000
    X = rng.randn(n, 40).astype(np.float32)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(40)])
    df["y"] = np.where(X[:, 0] - X[:, 3] * X[:, 5] + 0.3 * rng.randn(n) > 0, "yes", "no")
    fr = h2o3_amd.H2OFrame(df)
    preds = {}
    for pk in ("0", "1"):
        monkeypatch.setenv("H2O3_HIST_PACK", pk)
        m = H2OGradientBoostingEstimator(ntrees=4, max_depth=5, seed=3, histogram_type="UniformAdaptive")
        m.train(y="y", training_frame=fr)
        preds[pk] = m.predict(fr).as_data_frame()["yes"].values
    np.testing.assert_allclose(preds["1"], preds["0"], rtol=1e-5, atol=1e-6)
