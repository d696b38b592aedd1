"""HIP tree kernels vs the PyTorch fp32 reference of the same op."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _binned(n=20000, F=13, nbins=255, seed=0, cats=True):
    from h2o3_amd.models.tree.binning import bin_frame_tensors
    g = torch.Generator(device="cuda").manual_seed(seed)
    feats, is_cat, cards = [], [], []
    for j in range(F):
        if cats and j % 5 == 4:
            c = torch.randint(-1, 7, (n,), generator=g, device="cuda").to(torch.int32)
            feats.append(c); is_cat.append(True); cards.append(7)
        else:
            x = torch.randn(n, generator=g, device="cuda")
            x[torch.rand(n, generator=g, device="cuda") < 0.05] = float("nan")
            feats.append(x); is_cat.append(False); cards.append(0)
    bd = bin_frame_tensors(feats, is_cat, cards, [f"f{j}" for j in range(F)], hist_type="QuantilesGlobal",
                           nbins=nbins)
    return bd, feats


@pytest.mark.parametrize("nbins,mode", [(255, 0), (255, 1), (255, 2), (20, 0), (1000, 0), (1000, 1)])
@pytest.mark.parametrize("kernel", ["quad", "old"])
def test_hist_build_matches_reference(nbins, mode, kernel, monkeypatch):
    _need_gpu()
    monkeypatch.setenv("H2O3_HIST_KERNEL", kernel)
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(nbins=nbins)
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(1)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    vb = torch.rand(n, generator=g, device="cuda")
    starts, counts = [0, 5000, 12000], [5000, 7000, 8000]
    h_gpu = tree_ops.hist_build(bd, ridx, va, vb, mode, starts, counts, 3, use_native=True)
    h_ref = tree_ops.hist_build(bd, ridx, va, vb, mode, starts, counts, 3, use_native=False)
    assert h_gpu.shape == h_ref.shape
    torch.testing.assert_close(h_gpu, h_ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("impl", ["ballot", "old"])
def test_partition_matches_reference(impl, monkeypatch):
    _need_gpu()
    monkeypatch.setenv("H2O3_PART", impl)
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(n=50000)
    n = bd.nrows_local
    ridx = torch.arange(n, dtype=torch.int32, device="cuda")
    starts, counts = [0, 20000, 45000], [20000, 25000, 5000]
    if impl == "ballot":
        starts, counts = [0, 20003, 45001], [19999, 24998, 4999]   # unaligned segments
    feats = [0, 4, 7]
    masks = (torch.rand((3, bd.Bs), device="cuda") < 0.5).to(torch.uint8)
    out_g = ridx.clone()
    out_r = ridx.clone()
    nl_g = tree_ops.partition(bd, ridx, out_g, feats, masks, starts, counts, use_native=True, chunk=4096)
    nl_r = tree_ops.partition(bd, ridx, out_r, feats, masks, starts, counts, use_native=False)
    assert nl_g == nl_r
    assert torch.equal(out_g, out_r)


@pytest.mark.parametrize("items", ["dev", "host"])
def test_partition_async_matches_reference(items, monkeypatch):
    """Sync-free partition (device-side offset scan, all-ones mask = node kept
    in place, work items built on the device or the host, an empty segment)
    against the torch reference, with a position-ordered payload."""
    _need_gpu()
    monkeypatch.setenv("H2O3_PART_ITEMS", items)
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(n=50000)
    n = bd.nrows_local
    ridx = torch.randperm(n, device="cuda").to(torch.int32)
    starts, counts = [0, 20003, 30000, 30000, 45001], [19999, 9997, 0, 15001, 4999]
    feats = [0, 4, 1, 2, 7]
    masks = (torch.rand((5, bd.Bs), device="cuda") < 0.5).to(torch.uint8)
    masks[3] = 1   # a node that does not split: rows stay where they are
    pay = torch.randn(n, device="cuda")
    out_g, pay_g = ridx.clone(), pay.clone()
    out_r = ridx.clone()
    nl_g = tree_ops.partition_async(bd, ridx, out_g, torch.tensor(feats, device="cuda"), masks, starts, counts,
                                    chunk=4096, payload=(pay, None, pay_g, None))
    nl_r = tree_ops.partition(bd, ridx, out_r, feats, masks, starts, counts, use_native=False)
    assert nl_g.cpu().tolist() == nl_r
    assert torch.equal(out_g, out_r)
    # payload moved with the rows: pay is position ordered
    pos_of = torch.empty(n, dtype=torch.long, device="cuda")
    pos_of[ridx.long()] = torch.arange(n, device="cuda")
    seg = torch.zeros(n, dtype=torch.bool, device="cuda")
    for s, c in zip(starts, counts):
        seg[s:s + c] = True
    assert torch.equal(pay_g[seg], pay[pos_of[out_g.long()]][seg])


@pytest.mark.parametrize("mode,clamp", [(0, 0b1), (1, 0b0), (3, 0b1111)])
def test_hist_sibling_matches_torch(mode, clamp):
    _need_gpu()
    from h2o3_amd.ops import tree_ops
    C = tree_ops.channels(mode)
    g = torch.Generator(device="cuda").manual_seed(3)
    F, npar, Bs = 7, 5, 33
    Hp = torch.rand((F, npar, Bs, C), generator=g, device="cuda", dtype=torch.float64)
    Hb = torch.rand((F, npar, Bs, C), generator=g, device="cuda", dtype=torch.float64) * 0.7
    bs, ds, ps = [0, 3, 4, 7, 9], [1, 2, 5, 6, 8], [0, 1, 2, 3, 4]
    wb = torch.rand(5, generator=g, device="cuda", dtype=torch.float64)
    wp = torch.rand(5, generator=g, device="cuda", dtype=torch.float64) + 1
    H, wyy = tree_ops.hist_sibling(Hb, Hp, bs, ds, ps, 10, clamp, wyy_b=wb, wyy_prev=wp)
    ref = torch.empty((F, 10, Bs, C), dtype=torch.float64, device="cuda")
    ref[:, bs] = Hb
    d = Hp[:, ps] - Hb
    for c in range(C):
        if (clamp >> c) & 1:
            d[..., c] = d[..., c].clamp_min(0)
    ref[:, ds] = d
    torch.testing.assert_close(H, ref)
    wr = torch.empty(10, dtype=torch.float64, device="cuda")
    wr[bs] = wb
    wr[ds] = wp[ps] - wb
    torch.testing.assert_close(wyy, wr)


def test_grow_async_matches_sync(monkeypatch):
    """The sync-free level loop grows the same tree as the two-sync loop."""
    _need_gpu()
    from h2o3_amd.models.tree.engine import GrowParams, TreeGrower
    bd, feats = _binned(n=60000, cats=False)
    g = torch.Generator(device="cuda").manual_seed(5)
    y = (feats[0].nan_to_num() + 0.3 * torch.randn(60000, generator=g, device="cuda")).contiguous()
    w = torch.ones(60000, device="cuda")
    trees = []
    for flag in ("1", "0"):
        monkeypatch.setenv("H2O3_ASYNC_PART", flag)
        gr = TreeGrower(bd, GrowParams(max_depth=6, min_rows=10))
        tree, nid, leaves, tot = gr.grow(y, w, 0)
        trees.append((tree, nid.cpu(), tot))
    (ta, na, sa), (tb, nb, sb) = trees
    assert list(ta.feat) == list(tb.feat) and list(ta.left) == list(tb.left) and \
        list(ta.split_code) == list(tb.split_code)
    assert torch.equal(na, nb)
    torch.testing.assert_close(sa, sb)


def test_forest_predict_matches_host():
    _need_gpu()
    import pandas as pd
    import h2o3_amd
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    rng = np.random.RandomState(0)
    n = 3000
    X = rng.randn(n, 4)
    X[rng.rand(n) < 0.1, 1] = np.nan
    cat = rng.choice(list("abcde"), n)
    y = X[:, 0] + (cat == "c") * 2 + np.nan_to_num(X[:, 1])
    df = pd.DataFrame(X, columns=list("pqrs"))
    df["cat"] = cat
    df["y"] = y
    fr = h2o3_amd.H2OFrame(df)
    m = H2OGradientBoostingEstimator(ntrees=5, max_depth=4)
    m.train(y="y", training_frame=fr)
    Xs = m._score_matrix(fr)
    gpu = m._forest.predict(Xs, 1)
    from h2o3_amd.models.tree.shared import Forest
    ref = Forest._predict_torch(Xs, 1, m._forest.pack(Xs.device))
    torch.testing.assert_close(gpu, ref, rtol=1e-5, atol=1e-5)
    # training predictions (segment based) agree with scoring (traversal)
    f_train = m._train_f[:, 0]
    f_score = gpu[:, 0] + m._init_f[0]
    torch.testing.assert_close(f_train, f_score, rtol=1e-4, atol=1e-4)


def test_forest_predict_multiclass_and_leaf_ids_match_host():
    """Packed-node scoring kernel, K > 1 (per-class sums into out[r, k]) and
    the leaf-id output, against the torch walk; categorical + NA splits."""
    _need_gpu()
    import pandas as pd
    import h2o3_amd
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    from h2o3_amd.models.tree.shared import Forest
    rng = np.random.RandomState(1)
    n = 4000
    X = rng.randn(n, 4)
    X[rng.rand(n) < 0.1, 2] = np.nan
    cat = rng.choice(list("abcdefg"), n)
    yk = np.where(X[:, 0] + (cat == "b") > 0.5, "u", np.where(np.nan_to_num(X[:, 2]) > 0, "v", "w"))
    df = pd.DataFrame(X, columns=list("pqrs"))
    df["cat"] = cat
    df["y"] = yk
    fr = h2o3_amd.H2OFrame(df)
    m = H2OGradientBoostingEstimator(ntrees=4, max_depth=5, seed=3)
    m.train(y="y", training_frame=fr)
    Xs = m._score_matrix(fr)
    K = m._n_tree_classes()
    assert K == 3
    P = m._forest.pack(Xs.device)
    torch.testing.assert_close(m._forest.predict(Xs, K), Forest._predict_torch(Xs, K, P), rtol=1e-5, atol=1e-5)
    assert torch.equal(m._forest.predict(Xs, K, leaf=True), Forest._predict_torch(Xs, K, P, leaf=True))


def test_gbm_gpu_end_to_end_quality():
    _need_gpu()
    import pandas as pd
    import h2o3_amd
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    from h2o3_amd.ops import _native
    rng = np.random.RandomState(1)
    n = 100000
    X = rng.randn(n, 10)
    logit = X[:, 0] * 2 - X[:, 1] + X[:, 2] * X[:, 3]
    y = (rng.rand(n) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(10)])
    df["y"] = np.where(y == 1, "yes", "no")
    fr = h2o3_amd.H2OFrame(df)
    m = H2OGradientBoostingEstimator(ntrees=30, max_depth=5, seed=3)
    m.train(y="y", training_frame=fr)
    assert m.auc() > 0.85
    assert any("tree_hist" in p for p in _native.loaded_libs())


@pytest.mark.parametrize("crit", ["se", "xgb"])
def test_split_kernel_matches_torch(crit):
    _need_gpu()
    from h2o3_amd.models.tree.engine import GrowParams, TreeGrower
    bd, _ = _binned(n=30000, cats=False)
    p = GrowParams(criterion=crit, min_rows=5.0, max_depth=6)
    gr = TreeGrower(bd, p)
    n = 5
    g = torch.Generator(device="cuda").manual_seed(3)
    H = torch.rand((bd.F, n, bd.Bs, 2), generator=g, device="cuda", dtype=torch.float64) * 50
    if crit == "se":
        H[..., 1] = (torch.rand(H[..., 1].shape, generator=g, device="cuda", dtype=torch.float64) - 0.3) * H[..., 0]
    H[:, :, 200:bd.Bs - 1] = 0  # empty upper bins
    wyy = H[0].sum(1)[:, 0] * 10.0
    cm = torch.ones((n, bd.F), dtype=torch.bool)
    cm[1, 3] = False
    a = gr._find_splits_native(H, cm, wyy)
    b = gr._find_splits_torch(H, cm, wyy)
    torch.testing.assert_close(a["gain"], b["gain"], rtol=1e-9, atol=1e-9)
    assert torch.equal(a["feat"].cpu(), b["feat"].cpu())
    assert torch.equal(a["t"].cpu(), b["t"].cpu())
    assert torch.equal(a["opt"].cpu(), b["opt"].cpu())
    assert torch.equal(a["mask"].cpu(), b["mask"].cpu())
    torch.testing.assert_close(a["L"], b["L"].to(a["L"].dtype), rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("crit", ["se", "xgb"])
@pytest.mark.parametrize("use_bounds", [True, False])
def test_split_kernel_monotone_bounds_match_torch(crit, use_bounds):
    """Node prediction bounds (monotone constraints) inside the HIP split
    kernel equal the torch path: each column's best split clamped (gain
    penalty) or vetoed, then the best column per node."""
    _need_gpu()
    from h2o3_amd.models.tree.engine import GrowParams, TreeGrower
    bd, _ = _binned(n=30000, cats=False)
    mono = np.zeros(bd.F)
    mono[[0, 2]] = [1.0, -1.0]
    p = GrowParams(criterion=crit, min_rows=5.0, max_depth=6, monotone=mono, use_bounds=use_bounds)
    gr = TreeGrower(bd, p)
    n = 6
    g = torch.Generator(device="cuda").manual_seed(5)
    H = torch.rand((bd.F, n, bd.Bs, 2), generator=g, device="cuda", dtype=torch.float64) * 50
    if crit == "se":
        H[..., 1] = (torch.rand(H[..., 1].shape, generator=g, device="cuda", dtype=torch.float64) - 0.3) * H[..., 0]
    H[:, :, 200:bd.Bs - 1] = 0
    wyy = H[0].sum(1)[:, 0] * 10.0
    cm = torch.ones((n, bd.F), dtype=torch.bool)
    lo = torch.tensor([-np.inf, -0.1, 0.05, -np.inf, -1.0, 0.2], dtype=torch.float64)
    hi = torch.tensor([np.inf, 0.1, np.inf, 0.02, 1.0, 0.3], dtype=torch.float64)
    gr._bnd, gr._bnd_off = torch.stack([lo, hi], 1).cuda(), 0
    a = gr._find_splits_native(H, cm, wyy)
    b = gr._find_splits_torch(H, cm, wyy)
    torch.testing.assert_close(a["gain"], b["gain"], rtol=1e-9, atol=1e-9)
    ok = torch.isfinite(b["gain"])
    assert torch.equal(a["feat"].cpu()[ok.cpu()], b["feat"].cpu()[ok.cpu()])
    assert torch.equal(a["t"].cpu()[ok.cpu()], b["t"].cpu()[ok.cpu()])


@pytest.mark.parametrize("weights", [None, "binary"])
def test_hist_packed_single_atomic(weights):
    """Packed (count | biased fixed-point response) 64-bit atomics vs fp64 torch."""
    _need_gpu()
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(nbins=255)
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(3)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    vb = None if weights is None else (torch.rand(n, generator=g, device="cuda") < 0.6).to(torch.float32)
    starts, counts = [0, 7000], [7000, 13000]
    vmax = tree_ops.channel_max(va, vb, 0)
    h_gpu = tree_ops.hist_build(bd, ridx, va, vb, 0, starts, counts, 2, use_native=True, unit_w=True, vmax=vmax)
    h_ref = tree_ops.hist_build(bd, ridx, va, vb, 0, starts, counts, 2, use_native=False)
    torch.testing.assert_close(h_gpu[..., 0], h_ref[..., 0], rtol=0, atol=1e-9)   # counts exact
    torch.testing.assert_close(h_gpu[..., 1], h_ref[..., 1], rtol=1e-5, atol=1e-4)


def test_gbm_position_leaf_path_matches_nid_path(monkeypatch):
    """Leaf sums from the position-ordered payload + segment f-update give the
    same boosted model as the per-row leaf-id path."""
    _need_gpu()
    import numpy as np
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    h2o.init(device="cuda:0", verbose=False)
    rng = np.random.RandomState(0)
    n = 50000
    X = rng.randn(n, 6).astype(np.float32)
    y = (X[:, 0] + 0.5 * X[:, 1] ** 2 + 0.3 * rng.randn(n) > 0.4).astype(int)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(6)])
    df["y"] = np.where(y == 1, "a", "b")
    fr = h2o.H2OFrame(df)
    preds = []
    for flag in ("1", "0"):
        monkeypatch.setenv("H2O3_POS_LEAF", flag)
        m = H2OGradientBoostingEstimator(ntrees=8, max_depth=5, seed=3)
        m.train(y="y", training_frame=fr)
        preds.append(m.predict(fr).as_data_frame()["a"].values)
    np.testing.assert_allclose(preds[0], preds[1], atol=2e-5)


@pytest.mark.parametrize("crit", ["se", "xgb"])
def test_cat_pair_splits_match_dense_torch(crit):
    """Pair-based categorical scoring == dense torch scoring on the eligible features."""
    _need_gpu()
    from h2o3_amd.models.tree.engine import GrowParams, TreeGrower
    bd, _ = _binned(n=20000, F=13, cats=True)
    gr = TreeGrower(bd, GrowParams(criterion=crit, min_rows=5))
    g = torch.Generator(device="cuda").manual_seed(11)
    n, Bs = 9, bd.Bs
    H = torch.rand((gr.Fpad, n, Bs, 2), generator=g, device="cuda", dtype=torch.float64) * 50
    if crit == "se":
        H[..., 1] = (torch.rand(H[..., 1].shape, generator=g, device="cuda", dtype=torch.float64) - 0.3) * H[..., 0]
    cm = torch.rand((n, gr.Fpad), generator=torch.Generator().manual_seed(2)) < 0.6
    wyy = torch.full((n,), 1e6, dtype=torch.float64, device="cuda")
    cat_local = [j for j in range(gr.Fpad) if j < bd.F and bd.is_cat[j]]
    a = gr._cat_splits_pairs(H, cm, cat_local, wyy)
    b = gr._find_splits_torch(H, cm, wyy, merge=False, sub=cat_local)
    fin = torch.isfinite(b["gain"])
    assert torch.equal(torch.isfinite(a["gain"]), fin)
    torch.testing.assert_close(a["gain"][fin], b["gain"][fin])
    assert torch.equal(a["feat"][fin], b["feat"][fin])
    assert torch.equal(a["mask"][fin], b["mask"][fin])
    torch.testing.assert_close(a["L"][fin], b["L"][fin])


@pytest.mark.parametrize("fgw", ["4", "12", "36", "64"])
@pytest.mark.parametrize("lw", ["1", "2"])
def test_packed_hist_group_widths_match_reference(fgw, lw, monkeypatch):
    """Packed single-atomic histogram at forced group widths (idle lanes when
    64 % lanes-per-row != 0, partial last group) vs the torch reference.
    H2O3_HIST_LW is read once per process; both values give correct results."""
    _need_gpu()
    monkeypatch.setenv("H2O3_HIST_BM", "0")     # the grouped-lane kernel's widths
    monkeypatch.setenv("H2O3_HIST_FGW", fgw)
    monkeypatch.setenv("H2O3_HIST_LW", lw)
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(n=40000, F=37, nbins=255, cats=False)
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(4)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    vb = (torch.rand(n, generator=g, device="cuda") < 0.7).to(torch.float32)
    starts, counts = [0, 11000, 30000], [11000, 19000, 10000]
    h_gpu = tree_ops.hist_build(bd, ridx, va, vb, 0, starts, counts, 3, use_native=True, unit_w=True)
    h_ref = tree_ops.hist_build(bd, ridx, va, vb, 0, starts, counts, 3, use_native=False)
    torch.testing.assert_close(h_gpu, h_ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("crit", ["se", "xgb"])
@pytest.mark.parametrize("nb", [200, 1000, 3000])
def test_cat_pair_kernel_matches_torch_gains(crit, nb, sparse):
    """HIP cat_pair_kernel (bitonic sort of the occupied (key, bin) levels +
    f64 scan + 3 NA options) == the torch pair path's arg-max, numeric and
    categorical pairs, monotone constraints, empty levels and NA bins; sparse:
    deep-node shapes where ~97% of the levels are empty."""
    _need_gpu()
    from h2o3_amd.models.tree.engine import GrowParams, TreeGrower
    bd, _ = _binned(n=5000, F=6, cats=True)
    gr = TreeGrower(bd, GrowParams(criterion=crit, min_rows=3, min_split_improvement=1e-7))
    g = torch.Generator(device="cuda").manual_seed(nb)
    n, Bs, F = 40, nb + 1, 5
    H = torch.rand((F, n, Bs, 2), generator=g, device="cuda", dtype=torch.float64) * 20
    if crit == "se":
        H[..., 1] = (torch.rand(H[..., 1].shape, generator=g, device="cuda", dtype=torch.float64) - 0.4) * H[..., 0]
    H[..., : nb // 7, :] *= (torch.rand((F, n, nb // 7, 1), generator=g, device="cuda") < 0.5)  # empty levels
    if sparse:
        H[..., :nb, :] *= (torch.rand((F, n, nb, 1), generator=g, device="cuda") < 0.03)
    H[1, :, -1] = 0                                    # feature 1: no NAs
    P = 150
    fslot = torch.randint(0, F, (P,), generator=g, device="cuda")
    node = torch.randint(0, n, (P,), generator=g, device="cuda")
    pcat = torch.rand(P, generator=g, device="cuda") < 0.7
    mono = torch.randint(-1, 2, (P,), generator=g, device="cuda").to(torch.float64)
    mono[pcat] = 0
    wyy = H[0].sum(1)[:, 1] ** 2 / H[0].sum(1)[:, 0] * 3 + 50
    best, k = gr._pairs_native(H, fslot, node, pcat, mono, wyy)
    st = gr._pair_stats(H[fslot, node], pcat)
    allg = gr._pair_gains(st, mono.view(-1, 1), wyy, node)
    bt, kt = allg.max(1)
    fin = torch.isfinite(bt)
    assert torch.equal(torch.isfinite(best), fin)
    torch.testing.assert_close(best[fin], bt[fin], rtol=1e-9, atol=1e-9)
    if not sparse:
        assert torch.equal(k[fin], kt[fin])
    else:
        # thresholds on both sides of an empty level are the same split; their
        # gains tie up to the prefix sums' rounding, so the kernel's k only
        # has to be an arg-max of the torch gains
        gk = allg.gather(1, k.view(-1, 1).clamp_min(0)).view(-1)
        torch.testing.assert_close(gk[fin], bt[fin], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("nbins", [255, 1000])
@pytest.mark.parametrize("kernel", ["quad", "old"])
def test_hist_need_mask_skips_groups(nbins, kernel, monkeypatch):
    """need_mask (DRF mtries): groups holding a needed feature match the
    unmasked native histogram exactly; groups with none stay zero."""
    _need_gpu()
    monkeypatch.setenv("H2O3_HIST_KERNEL", kernel)
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(F=40, nbins=nbins, cats=False)
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(3)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    vb = torch.rand(n, generator=g, device="cuda")
    starts, counts = [0, 6000, 13000], [6000, 7000, 7000]
    need = torch.zeros((3, bd.F), dtype=torch.bool, device="cuda")
    need[0, [0, 3]] = True
    need[1, [0, 37]] = True
    need[2, [0, 20, 21]] = True
    full = tree_ops.hist_build(bd, ridx, va, vb, 1, starts, counts, 3, use_native=True)
    part = tree_ops.hist_build(bd, ridx, va, vb, 1, starts, counts, 3, use_native=True, need_mask=need)
    for s in range(3):
        for f in torch.nonzero(need[s]).flatten().tolist():
            torch.testing.assert_close(part[f, s], full[f, s], rtol=0, atol=0)
    # features far from every needed one (group size <= 16) are skipped
    # every other (feature, slot) histogram is either the full one (same
    # group as a needed feature) or skipped (all zero); some must be skipped
    skipped = 0
    for s in range(3):
        for f in range(bd.F):
            if float(part[f, s].abs().sum()) == 0.0 and float(full[f, s].abs().sum()) > 0.0:
                skipped += 1
            else:
                torch.testing.assert_close(part[f, s], full[f, s], rtol=0, atol=0)
    assert skipped > 0


@pytest.mark.parametrize("F", [48, 64])
def test_drf_chunked_need_mask_same_model(F, monkeypatch):
    """Deep chunked DRF levels with the need mask grow the same trees as
    with full histograms (F = 64: the packed single-atomic path)."""
    _need_gpu()
    import pandas as pd
    import h2o3_amd
    from h2o3_amd.estimators import H2ORandomForestEstimator
    h2o3_amd.init(device="cuda:0", verbose=False)
    rng = np.random.RandomState(0)
    n = 20000
    X = rng.randn(n, F).astype(np.float32)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(F)])
    df["y"] = X[:, 0] + X[:, 7] * X[:, 30] + 0.1 * rng.randn(n)
    fr = h2o3_amd.H2OFrame(df)
    monkeypatch.setenv("H2O3_HIST_BUDGET", str(1 << 20))   # force the chunked path
    monkeypatch.setenv("H2O3_PAIR_DIRECT", "0")             # the node-batched level histograms
    preds = []
    for flag in ("0", "1"):
        monkeypatch.setenv("H2O3_HIST_NEED", flag)
        m = H2ORandomForestEstimator(ntrees=3, max_depth=12, seed=7, mtries=6)
        m.train(y="y", training_frame=fr)
        preds.append(m.predict(fr).as_data_frame().values[:, 0])
    np.testing.assert_allclose(preds[0], preds[1], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("kernel,fg", [("quad", "8"), ("quad", "36"), ("quad", "64"), ("old", "0"), ("bm", "64")])
@pytest.mark.parametrize("F", [64, 100])
def test_packed_need_mask_matches_full(kernel, fg, F, monkeypatch):
    """Packed single-atomic path (mode 0, 0/1 weights) with a need mask: the
    host-side group count must match the kernel's; needed features equal the
    unmasked histogram exactly, and the result matches fp64 torch."""
    _need_gpu()
    monkeypatch.setenv("H2O3_HIST_KERNEL", "quad" if kernel == "bm" else kernel)
    monkeypatch.setenv("H2O3_HIST_BM", "1" if kernel == "bm" else "0")
    if kernel == "quad":
        monkeypatch.setenv("H2O3_HIST_FGW", fg)
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(n=30000, F=F, nbins=255, cats=False)
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(5)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    vb = (torch.rand(n, generator=g, device="cuda") < 0.8).to(torch.float32)
    starts, counts = [0, 9000, 21000], [9000, 12000, 9000]
    need = torch.zeros((3, bd.F), dtype=torch.bool, device="cuda")
    need[0, [1, F - 1]] = True
    need[1, [33]] = True
    need[2, [0, 40, F - 2]] = True
    vmax = tree_ops.channel_max(va, vb, 0)
    full = tree_ops.hist_build(bd, ridx, va, vb, 0, starts, counts, 3, use_native=True, unit_w=True, vmax=vmax)
    part = tree_ops.hist_build(bd, ridx, va, vb, 0, starts, counts, 3, use_native=True, unit_w=True, vmax=vmax,
                               need_mask=need)
    ref = tree_ops.hist_build(bd, ridx, va, vb, 0, starts, counts, 3, use_native=False)
    torch.testing.assert_close(full[..., 0], ref[..., 0], rtol=0, atol=1e-9)
    torch.testing.assert_close(full[..., 1], ref[..., 1], rtol=1e-5, atol=1e-4)
    for s in range(3):
        for f in torch.nonzero(need[s]).flatten().tolist():
            torch.testing.assert_close(part[f, s], full[f, s], rtol=0, atol=0)
    if kernel in ("quad", "bm") and F > int(fg):   # more than one group: some (slot, group) blocks were skipped
        assert float(part.abs().sum()) < float(full.abs().sum())


@pytest.mark.parametrize("F", [1, 3, 5, 37, 100, 130])
def test_quad_kernel_feature_groups(F):
    """Quad kernel at the default group choice: uneven last group, partial
    last dword, one-feature frames; packed and two-entry layouts."""
    _need_gpu()
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(n=12000, F=F, nbins=255, cats=False)
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(F)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    starts, counts = [0, 2500], [2500, 9500]
    for unit_w in (True, False):
        h = tree_ops.hist_build(bd, ridx, va, None, 0, starts, counts, 2, use_native=True, unit_w=unit_w)
        r = tree_ops.hist_build(bd, ridx, va, None, 0, starts, counts, 2, use_native=False)
        torch.testing.assert_close(h, r, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("dist", ["bernoulli", "gaussian"])
def test_lookahead_levels_same_model(dist, monkeypatch):
    """Next-level histograms built from the device-side work list before the
    host sync (engine._maybe_lookahead) grow the same trees as the host-built
    path; H2O3_LA_CHECK asserts the device pair slots equal the host's."""
    _need_gpu()
    import pandas as pd
    import h2o3_amd
    from h2o3_amd.estimators import H2OGradientBoostingEstimator, H2OXGBoostEstimator
    h2o3_amd.init(device="cuda:0", verbose=False)
    rng = np.random.RandomState(4)
    n = 60000
    X = rng.randn(n, 12).astype(np.float32)
    X[rng.rand(n) < 0.05, 3] = np.nan
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(12)])
    df["c"] = rng.choice(list("abcdefg"), n)
    lin = X[:, 0] + np.nan_to_num(X[:, 3]) * X[:, 1] + (df["c"] == "b") * 0.8
    df["y"] = np.where(rng.rand(n) < 1 / (1 + np.exp(-lin)), "p", "q") if dist == "bernoulli" else lin
    fr = h2o3_amd.H2OFrame(df)
    monkeypatch.setenv("H2O3_LA_CHECK", "1")
    preds = []
    for flag in ("1", "0"):
        monkeypatch.setenv("H2O3_LOOKAHEAD", flag)
        m = H2OGradientBoostingEstimator(ntrees=6, max_depth=7, seed=3, distribution=dist)
        m.train(y="y", training_frame=fr)
        preds.append(m.predict(fr).as_data_frame().values[:, -1].astype(float))
    np.testing.assert_allclose(preds[0], preds[1], rtol=1e-6, atol=1e-6)
    preds = []
    for flag in ("1", "0"):
        monkeypatch.setenv("H2O3_LOOKAHEAD", flag)
        m = H2OXGBoostEstimator(ntrees=4, max_depth=6, seed=3)
        m.train(y="y", training_frame=fr)
        preds.append(m.predict(fr).as_data_frame().values[:, -1].astype(float))
    np.testing.assert_allclose(preds[0], preds[1], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("nbins", [255, 1000])
@pytest.mark.parametrize("mode,weights,posv", [(0, False, False), (0, True, False), (0, False, True), (1, True, False)])
@pytest.mark.parametrize("chunk", [16384, 700])
def test_pair_hist_matches_reference(nbins, mode, weights, posv, chunk):
    """Row-direct pair histograms (pair_hist_kernel, 1- and 2-byte codes,
    single-item stores and multi-item atomics) vs the index_add reference."""
    _need_gpu()
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(nbins=nbins)
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(3)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    if mode == 0 and not weights:
        va[torch.rand(n, generator=g, device="cuda") < 0.1] = float("nan")   # zero-weight rows
    vb = torch.rand(n, generator=g, device="cuda") if weights else None
    st, ct = [0, 3000, 3100, 9000], [3000, 100, 5900, 11000]
    pn = [0, 0, 1, 2, 2, 2, 3, 3]
    pf = [1, 4, 0, 2, 4, 12, 3, 9]
    kw = dict(posv=posv, want_wyy=True, chunk=chunk)
    Hg, wg = tree_ops.pair_hist(bd, ridx, va, vb, mode, st, ct, pn, pf, use_native=True, **kw)
    Hr, wr = tree_ops.pair_hist(bd, ridx, va, vb, mode, st, ct, pn, pf, use_native=False, **kw)
    torch.testing.assert_close(Hg, Hr, rtol=1e-5, atol=1e-4)
    if mode == 0:
        torch.testing.assert_close(wg, wr, rtol=1e-5, atol=1e-3)
    # every pair of a node sums to the node totals
    tot = Hg.sum(1)
    torch.testing.assert_close(tot[0], tot[1])
    torch.testing.assert_close(tot[3], tot[5])


@pytest.mark.parametrize("cats", [False, True])
def test_drf_direct_pairs_same_model(cats, monkeypatch):
    """DRF with mtries grown from row-direct pair histograms at every level
    gives the same forest as the level-histogram path."""
    _need_gpu()
    import pandas as pd
    import h2o3_amd
    from h2o3_amd.estimators import H2ORandomForestEstimator
    h2o3_amd.init(device="cuda:0", verbose=False)
    rng = np.random.RandomState(0)
    n, F = 20000, 40
    X = rng.randn(n, F).astype(np.float32)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(F)])
    if cats:
        df["c"] = pd.Categorical([f"L{v}" for v in rng.randint(0, 300, n)])
    df["y"] = X[:, 0] + X[:, 7] * X[:, 30] + 0.1 * rng.randn(n)
    fr = h2o3_amd.H2OFrame(df)
    preds = []
    for flag in ("0", "1"):
        monkeypatch.setenv("H2O3_PAIR_DIRECT", flag)
        m = H2ORandomForestEstimator(ntrees=3, max_depth=14, seed=7, mtries=6)
        m.train(y="y", training_frame=fr)
        preds.append(m.predict(fr).as_data_frame().values[:, 0])
    np.testing.assert_allclose(preds[0], preds[1], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("nbins", [255, 1000])
@pytest.mark.parametrize("weights", [False, True])
def test_pair_hist_dev_grouped_matches_reference(nbins, weights, monkeypatch):
    """Device-pair histograms with 4 pairs of a node per workgroup
    (pair_hist_multi_kernel, incl. a partial group and multi-item nodes) equal
    the one-pair-per-workgroup kernel and the index_add reference."""
    _need_gpu()
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(nbins=nbins)
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(5)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    vb = torch.rand(n, generator=g, device="cuda") if weights else None
    if not weights:
        va[torch.rand(n, generator=g, device="cuda") < 0.1] = float("nan")
    st, ct = [0, 3000, 3100, 9000], [3000, 100, 5900, 11000]
    sel = torch.stack([torch.randperm(bd.F, generator=g, device="cuda")[:6].sort().values for _ in range(4)])
    vmax = tree_ops.channel_max(va, vb, 0)
    out = {}
    for kp in (1, 4):
        monkeypatch.setattr(tree_ops, "_PAIR_KP", kp)
        out[kp] = tree_ops.pair_hist_dev(bd, ridx, va, vb, 0, st, ct, sel, vmax, chunk=2048)
    torch.testing.assert_close(out[4][0], out[1][0], rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(out[4][1], out[1][1], rtol=1e-12, atol=1e-9)
    pn = np.repeat(np.arange(4), 6)
    pf = sel.cpu().numpy().reshape(-1)
    Hr, wr = tree_ops.pair_hist(bd, ridx, va, vb, 0, st, ct, pn, pf, want_wyy=True, use_native=False)
    torch.testing.assert_close(out[4][0], Hr, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(out[4][1], wr, rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
def test_fill_nid_tiled_matches_reference():
    """Device searchsorted + scatter leaf ids (segments tiling the row
    permutation, incl. empty leaves and unsorted segment order) equal the
    per-segment torch reference; non-tiling segments fall back."""
    import numpy as np
    import torch
    from h2o3_amd.ops import tree_ops
    dev = torch.device("cuda")
    rng = np.random.RandomState(3)
    N = 200_003
    cuts = np.sort(rng.choice(np.arange(1, N), 5000, replace=False))
    st = np.concatenate([[0], cuts])
    ct = np.diff(np.concatenate([st, [N]]))
    st = np.concatenate([st, [N // 2]])          # an empty leaf
    ct = np.concatenate([ct, [0]])
    perm = rng.permutation(len(st))
    st, ct = st[perm], ct[perm]
    lids = np.arange(len(st))
    ridx = torch.as_tensor(rng.permutation(N).astype(np.int32), device=dev)
    ref = tree_ops.fill_nid(ridx.cpu(), list(lids), st.tolist(), ct.tolist(), N, use_native=False)
    got = tree_ops.fill_nid(ridx, lids, st, ct, N)
    assert torch.equal(got.cpu(), ref)
    # a gap in the tiling -> reference path (rows outside every leaf keep -1)
    got2 = tree_ops.fill_nid(ridx, lids[1:], st[1:], ct[1:], N)
    ref2 = tree_ops.fill_nid(ridx.cpu(), list(lids[1:]), st[1:].tolist(), ct[1:].tolist(), N, use_native=False)
    assert torch.equal(got2.cpu(), ref2)


@pytest.mark.gpu
def test_gbm_leaf_scatter_update_matches_rmw(monkeypatch):
    """The write-only leaf scatter (per-row leaf values folded into f by the
    next residual pass) trains the same model as the in-place f[ridx[p]] += v
    update, with and without row sampling (sampled-out rows are NaN-masked
    but still tiled into leaves)."""
    import numpy as np
    import torch
    import h2o3_amd as h2o
    from h2o3_amd.core.frame import H2OFrame
    from h2o3_amd.core.vec import Vec, T_REAL, T_ENUM
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    h2o.init(verbose=False)
    g = torch.Generator(device="cuda").manual_seed(5)
    N, P = 300_000, 16
    X = torch.randn((N, P), generator=g, device="cuda")
    y = (torch.rand(N, generator=g, device="cuda") < torch.sigmoid(X[:, 0] - X[:, 1])).to(torch.int32)
    fr = H2OFrame.from_vecs([Vec(X[:, j].contiguous(), T_REAL) for j in range(P)] + [Vec(y, T_ENUM, ["0", "1"])],
                            [f"x{j}" for j in range(P)] + ["y"])
    for sr in (1.0, 0.7):
        preds = []
        for flag in ("1", "0"):
            monkeypatch.setenv("H2O3_LEAF_SCATTER", flag)
            m = H2OGradientBoostingEstimator(ntrees=6, max_depth=5, seed=3, sample_rate=sr)
            m.train(y="y", training_frame=fr)
            preds.append(m.predict(fr).as_data_frame()["p1"].values)
        np.testing.assert_allclose(preds[0], preds[1], rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_col_sample_kernel_uniform_sorted_distinct():
    """Per-node selection sampling: every row holds k distinct eligible ids in
    ascending order; inclusion frequencies are uniform (k / m each) and the
    pair co-occurrence matches sampling without replacement."""
    import numpy as np
    import torch
    from h2o3_amd.ops import tree_ops
    elig = np.array([0, 2, 3, 5, 8, 9, 11, 14, 15, 20], dtype=np.int64)
    n, k, m = 200_000, 3, len(elig)
    out = tree_ops.col_sample(n, torch.as_tensor(elig, device="cuda"), k, 12345).cpu().numpy()
    assert out.shape == (n, k)
    assert np.all(np.diff(out, axis=1) > 0)
    assert np.isin(out, elig).all()
    freq = np.array([(out == e).sum() for e in elig]) / n
    np.testing.assert_allclose(freq, k / m, atol=0.006)
    both = ((out == elig[0]).any(1) & (out == elig[1]).any(1)).mean()
    assert abs(both - k * (k - 1) / (m * (m - 1))) < 0.004
    out2 = tree_ops.col_sample(n, torch.as_tensor(elig, device="cuda"), k, 12345).cpu().numpy()
    assert np.array_equal(out, out2)


@pytest.mark.parametrize("F", [13, 37, 64, 100])
@pytest.mark.parametrize("mode,pack", [(0, True), (0, False), (1, False), (2, False)])
@pytest.mark.parametrize("posv", [False, True])
def test_hist_bm_kernel_matches_reference(F, mode, pack, posv, monkeypatch):
    """Bank-conflict-free bin-major kernel (hist_bm_kernel, G = 64 / 32 / 16
    feature slots per bin row, rotated code bytes per row) vs the fp64 torch
    reference, for the packed, two-channel and count layouts, row- and
    position-ordered payloads, partial last groups."""
    _need_gpu()
    monkeypatch.setenv("H2O3_HIST_BM", "1")
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(n=30000, F=F, nbins=255, cats=F < 50)
    bm = tree_ops.bm_groups(bd.F, bd.Fp, bd.Bs, pack or mode == 2)
    assert bm is not None
    if F == 100:
        assert bm == ((2, 64) if (pack or mode == 2) else (4, 32))
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(F + mode)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    if pack:
        vb = (torch.rand(n, generator=g, device="cuda") < 0.7).to(torch.float32)
    else:
        vb = torch.rand(n, generator=g, device="cuda")
    starts, counts = [0, 9000, 21000], [9000, 12000, 9000]
    vmax = tree_ops.channel_max(va, vb, mode)
    h_gpu, w_gpu = tree_ops.hist_build(bd, ridx, va, vb, mode, starts, counts, 3, use_native=True, unit_w=pack,
                                       vmax=vmax, posv=posv, want_wyy=True)
    h_ref, w_ref = tree_ops.hist_build(bd, ridx, va, vb, mode, starts, counts, 3, use_native=False, posv=posv,
                                       want_wyy=True)
    torch.testing.assert_close(h_gpu, h_ref, rtol=1e-5, atol=1e-4)
    if mode == 0:
        torch.testing.assert_close(w_gpu, w_ref, rtol=1e-5, atol=1e-3)
    # the grouped-lane kernel gives the same histograms
    monkeypatch.setenv("H2O3_HIST_BM", "0")
    h_q = tree_ops.hist_build(bd, ridx, va, vb, mode, starts, counts, 3, use_native=True, unit_w=pack, vmax=vmax,
                              posv=posv)
    torch.testing.assert_close(h_gpu, h_q, rtol=1e-5, atol=1e-4)


def test_gbm_same_model_bm_and_quad(monkeypatch):
    """GBM grown with the bin-major histogram kernel vs the grouped-lane kernel:
    same trees (the fixed-point sums only differ in the last bits)."""
    _need_gpu()
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    h2o.init(device="cuda:0", verbose=False)
    rng = np.random.RandomState(7)
    n, F = 60000, 70
    X = rng.randn(n, F).astype(np.float32)
    y = (X[:, 0] - X[:, 3] + 0.5 * X[:, 5] * X[:, 6] + 0.3 * rng.randn(n) > 0).astype(int)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(F)])
    df["y"] = np.where(y == 1, "a", "b")
    fr = h2o.H2OFrame(df)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("H2O3_HIST_BM", flag)
        m = H2OGradientBoostingEstimator(ntrees=6, max_depth=6, seed=3)
        m.train(y="y", training_frame=fr)
        out[flag] = (m.logloss(), [list(t.feat) for t in m._forest.trees])
    assert abs(out["1"][0] - out["0"][0]) < 1e-5
    assert out["1"][1] == out["0"][1]


@pytest.mark.parametrize("nbins", [2, 4, 6, 12])
@pytest.mark.parametrize("mode,pack", [(0, True), (0, False), (2, False)])
def test_hist_bm_few_bins_matches_reference(nbins, mode, pack, monkeypatch):
    """Few-bin frames give a bin stride Bs that is not a multiple of 16 (8 for
    <= 7 bins): the two-pass reduce must cover the partial 16-bin tile."""
    _need_gpu()
    monkeypatch.setenv("H2O3_HIST_BM", "1")
    from h2o3_amd.ops import tree_ops
    bd, _ = _binned(n=30000, F=40, nbins=nbins, cats=False)
    assert bd.Bs % 4 == 0
    n = bd.nrows_local
    g = torch.Generator(device="cuda").manual_seed(nbins)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    va = torch.randn(n, generator=g, device="cuda")
    vb = (torch.rand(n, generator=g, device="cuda") < 0.7).to(torch.float32) if pack else \
        torch.rand(n, generator=g, device="cuda")
    starts, counts = [0, 9000, 21000], [9000, 12000, 9000]
    vmax = tree_ops.channel_max(va, vb, mode)
    h_gpu = tree_ops.hist_build(bd, ridx, va, vb, mode, starts, counts, 3, use_native=True, unit_w=pack, vmax=vmax)
    h_ref = tree_ops.hist_build(bd, ridx, va, vb, mode, starts, counts, 3, use_native=False)
    torch.testing.assert_close(h_gpu, h_ref, rtol=1e-5, atol=1e-4)


def test_gbm_all_binary_frame_gpu_matches_cpu():
    """GBM on a frame of 0/1 features only (Bs = 8): the GPU model equals the
    CPU (torch reference) model."""
    _need_gpu()
    import pandas as pd
    import h2o3_amd as h2o
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    rng = np.random.RandomState(11)
    n, F = 40000, 24
    X = (rng.rand(n, F) < 0.4).astype(np.float32)
    y = ((X[:, 0] + X[:, 1] * X[:, 2] + 0.3 * rng.randn(n)) > 0.6).astype(int)
    df = pd.DataFrame(X, columns=[f"b{i}" for i in range(F)])
    df["y"] = np.where(y == 1, "a", "b")
    from h2o3_amd.parallel import cloud
    out = {}
    for dev in ("cuda:0", "cpu"):
        cloud.shutdown()
        h2o.init(device=dev, verbose=False)
        fr = h2o.H2OFrame(df)
        m = H2OGradientBoostingEstimator(ntrees=5, max_depth=5, seed=3)
        m.train(y="y", training_frame=fr)
        out[dev] = (m.logloss(), [list(t.feat) for t in m._forest.trees])
    cloud.shutdown()
    h2o.init(device="cuda:0", verbose=False)
    assert out["cuda:0"][1] == out["cpu"][1]
    assert abs(out["cuda:0"][0] - out["cpu"][0]) < 1e-5


@pytest.mark.parametrize("classify", [False, True])
def test_drf_pair_path_narrow_scoring_and_posv_same_trees(classify, monkeypatch):
    """DRF on the row-direct pair path with a 1000-level categorical (1025-bin
    histograms) and numeric columns of <= 255 bins: scoring the narrow pairs
    with the 256-wide kernel instance (H2O3_PAIR_NARROW) and carrying the
    response as the position-ordered payload (H2O3_DRF_POSV) grow exactly the
    trees of the reference configuration."""
    _need_gpu()
    import pandas as pd
    import h2o3_amd
    from h2o3_amd.estimators import H2ORandomForestEstimator
    h2o3_amd.init(device="cuda:0", verbose=False)
    rng = np.random.RandomState(3)
    n = 30000
    F = 24
    X = rng.randn(n, F).astype(np.float32)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(F)])
    df.loc[::11, "x3"] = np.nan
    lv = rng.randint(0, 1000, n)
    df["c"] = pd.Categorical([f"L{v}" for v in lv])
    eff = rng.randn(1000)
    yv = X[:, 0] + X[:, 5] * X[:, 9] + eff[lv] + 0.3 * rng.randn(n)
    df["y"] = np.where(yv > 0.3, "a", "b") if classify else yv
    fr = h2o3_amd.H2OFrame(df)
    if classify:
        fr["y"] = fr["y"].asfactor()
    out = []
    for narrow, posv in (("0", "0"), ("1", "1")):
        monkeypatch.setenv("H2O3_PAIR_NARROW", narrow)
        monkeypatch.setenv("H2O3_DRF_POSV", posv)
        m = H2ORandomForestEstimator(ntrees=3, max_depth=14, seed=11, mtries=5)
        m.train(y="y", training_frame=fr)
        out.append(m)
    for t0, t1 in zip(out[0]._forest.trees, out[1]._forest.trees):
        assert t0.n_nodes == t1.n_nodes
        np.testing.assert_array_equal(np.asarray(t0.feat), np.asarray(t1.feat))
        np.testing.assert_array_equal(np.asarray(t0.thr), np.asarray(t1.thr))
        np.testing.assert_allclose(np.asarray(t0.value), np.asarray(t1.value), rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("weighted", [False, True])
def test_pair_narrow_scoring_matches_torch_reference(weighted):
    """The DRF device pair path with narrow bins (h2o_pair_hist4b leaves each
    pair's bins past its feature's own codes unwritten; cat_pair_kernel and
    pair_select2 scan only [0, nbins_f) + NA) picks, per node, the gain,
    feature and threshold of the torch split search (_find_splits_torch) run
    on the fp64 torch pair histograms of the same rows -- a 1000-level
    categorical makes Bs = 1025 while the numeric columns have <= 255 bins or
    a dozen integer levels."""
    _need_gpu()
    from h2o3_amd.models.tree.binning import bin_frame_tensors
    from h2o3_amd.models.tree.engine import GrowParams, TreeGrower
    from h2o3_amd.ops import tree_ops
    g = torch.Generator(device="cuda").manual_seed(21)
    n = 24000
    feats, is_cat, cards = [], [], []
    for j in range(7):
        x = torch.randn(n, generator=g, device="cuda")
        if j == 2:
            x = torch.randint(0, 12, (n,), generator=g, device="cuda").float()     # 12 integer levels
        x[torch.rand(n, generator=g, device="cuda") < 0.04] = float("nan")
        feats.append(x), is_cat.append(False), cards.append(0)
    c = torch.randint(-1, 1000, (n,), generator=g, device="cuda").to(torch.int32)
    feats.append(c), is_cat.append(True), cards.append(1000)
    bd = bin_frame_tensors(feats, is_cat, cards, [f"f{j}" for j in range(8)], hist_type="QuantilesGlobal",
                           nbins=255)
    assert bd.Bs - 1 > 256
    eff = torch.randn(1000, generator=g, device="cuda")
    y = feats[0].nan_to_num(0) + 0.5 * feats[2].nan_to_num(0) + eff[c.clamp_min(0).long()] + \
        0.3 * torch.randn(n, generator=g, device="cuda")
    mode = 0
    va, vb = y, (torch.rand(n, generator=g, device="cuda") + 0.5 if weighted else None)
    gr = TreeGrower(bd, GrowParams(min_rows=5, seed=3))
    assert gr._narrow_bins() is not None
    gr._vmax = tree_ops.channel_max(va, vb, mode)
    ridx = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
    st, ct = np.array([0, 9000, 9400]), np.array([9000, 400, 14600])
    k = 4
    sel = torch.stack([torch.tensor(s, device="cuda") for s in ([0, 2, 5, 7], [1, 2, 3, 7], [2, 4, 6, 7])])
    res = gr._pair_direct_dev(ridx, va, vb, mode, st, ct, sel)
    pn = np.repeat(np.arange(3), k)
    pf = sel.cpu().numpy().reshape(-1)
    Hr, wr = tree_ops.pair_hist(bd, ridx, va, vb, mode, st, ct, pn, pf, want_wyy=mode == 0, use_native=False)
    F = bd.F
    H = torch.zeros((gr.Fpad, 3, bd.Bs, 2), dtype=torch.float64, device="cuda")
    allowed = torch.zeros((3, gr.Fpad), dtype=torch.bool, device="cuda")
    for p_, (i, f) in enumerate(zip(pn, pf)):
        H[f, i] = Hr[p_]
        allowed[i, f] = True
    ref = gr._find_splits_torch(H[:F], allowed[:, :F], node_wyy=wr)
    assert bool(torch.isfinite(ref["gain"]).all())
    torch.testing.assert_close(res["gain"].cpu(), ref["gain"].cpu().to(torch.float64), rtol=1e-6, atol=1e-6)
    assert res["feat"].cpu().tolist() == ref["feat"].cpu().tolist()
    num = res["feat"].cpu() != 7                       # numeric winners: the same threshold bin
    assert res["t"].cpu()[num].tolist() == ref["t"].cpu()[num].tolist()
