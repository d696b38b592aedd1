"""Reference histogram semantics of the tree engine (binning.py +
engine.TreeGrower._adapt_hist) and monotone node bounds inside the split
search (engine._bound_cost, tree_split.hip split_kernel).

Reference: hex/tree/DHistogram.java:226-233 (RoundRobin), :366-386 (bins of a
node over its own range), DTree.java:337 (adj_nbins = max(nbins_prev >> 1,
nbins)), SharedTreeModel.java:55-72 (nbins 20, nbins_top_level 1024),
GlobalQuantilesCalc, DTree.java:1386-1445 + Constraints.java (node bounds).
"""
import numpy as np
import pandas as pd
import pytest
import torch

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OGradientBoostingEstimator
from h2o3_amd.models.tree.binning import bin_frame_tensors


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2o.init(verbose=False)


def _step_frame(n=20000, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.random(n)
    y = 3.0 * (x > 0.1) + 2.0 * (x > 0.95) + 0.5 * (x > 0.5317) + 0.01 * rng.normal(size=n)
    return pd.DataFrame({"x": x, "y": y})


def _coarse_ends(first, last, nb):
    """Allowed split codes: the coarse boundaries of nb uniform bins over the
    fine-code range [first, last] (every code when the range is narrower)."""
    L = last - first + 1
    b = np.arange(first, last + 1)
    coarse = np.floor((b - first) * nb / L)
    nxt = np.floor((b + 1 - first) * nb / L)
    return set(b[(coarse != nxt) | (b == last)].tolist()) if L > nb else set(b.tolist())


def test_uniform_adaptive_child_splits_on_its_coarse_grid():
    """Reference UniformAdaptive schedule (DTree.java:337-372, with the bin
    counts the reference fixture's splits show): the root and its children
    use the nbins_top_level grid, a depth-2 node max(nbins_top_level >> 1,
    nbins) uniform bins over its PARENT's range of the column, cut at the
    parent's split."""
    df = _step_frame()
    fr = h2o.H2OFrame(df)
    kw = dict(ntrees=1, max_depth=3, learn_rate=1.0, min_rows=1, seed=1, nbins=20, nbins_top_level=128,
              distribution="gaussian")
    m = H2OGradientBoostingEstimator(histogram_type="UniformAdaptive", **kw)
    m.train(x=["x"], y="y", training_frame=fr)
    t = m._forest.trees[0]
    assert abs(t.thr[0] - 0.1) < 1.5 / 128                      # root: the 128-cell top-level grid
    r = t.right[0]
    assert abs(t.thr[r] - 0.95) < 1.5 / 128                     # depth 1: still the full grid
    rl = t.left[r]
    assert t.left[rl] >= 0, "the depth-2 node [0.1, 0.95) must split"
    # its range: the parent's fine codes (root split + 1 .. last) cut at the parent's split
    first, last = int(t.split_code[0]) + 1, int(t.split_code[r])
    allowed = _coarse_ends(first, last, max(128 >> 1, 20))
    assert len(allowed) < last - first + 1                       # the grid really is coarser here
    assert int(t.split_code[rl]) in allowed
    assert abs(t.thr[rl] - 0.5317) < 2.5 / 128
    # the same data with the global quantile grid is not restricted this way
    q = H2OGradientBoostingEstimator(histogram_type="QuantilesGlobal", **dict(kw, nbins=1000))
    q.train(x=["x"], y="y", training_frame=fr)
    qt = q._forest.trees[0]
    assert abs(qt.thr[qt.left[qt.right[0]]] - 0.5317) < 0.003


def test_quantiles_global_cuts_are_exact_order_statistics():
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.exponential(size=30000), np.full(5000, 0.7)]).astype(np.float32)
    bd = bin_frame_tensors([torch.tensor(x)], [False], [0], ["x"], hist_type="QuantilesGlobal", nbins=50)
    xs = np.sort(x.astype(np.float64))
    ks = np.round(np.linspace(0, 1, 51)[1:-1] * (len(xs) - 1)).astype(int)
    ref = np.unique(xs[ks])
    ref = ref[ref > xs[0]]
    np.testing.assert_array_equal(bd.cuts[0], ref.astype(np.float32).astype(np.float64))


def test_uniform_grid_uses_exact_range_and_integer_cells():
    rng = np.random.default_rng(4)
    x = rng.normal(size=50000).astype(np.float32)
    x[123] = 40.0                                                 # one far value sets the range
    k = rng.integers(3, 60, 50000).astype(np.float32)
    bd = bin_frame_tensors([torch.tensor(x), torch.tensor(k)], [False, False], [0, 0], ["x", "k"],
                           hist_type="UniformAdaptive", nbins=20, nbins_top_level=1024)
    assert bd.cuts[0][-1] > 39.0 and bd.nbins[0] == 1024
    np.testing.assert_allclose(bd.cuts[1], np.arange(3.5, 59.0, 1.0))     # one cell per integer
    assert bd.nbins[1] == 57


def test_round_robin_cycles_tree_types_and_random_redraws():
    df = _step_frame(4000)
    fr = h2o.H2OFrame(df)
    m = H2OGradientBoostingEstimator(ntrees=4, max_depth=3, histogram_type="RoundRobin", seed=5, nbins=20,
                                     nbins_top_level=64)
    m.train(x=["x"], y="y", training_frame=fr)
    from h2o3_amd.models.tree.engine import TreeGrower
    seq = [TreeGrower._RR_TYPES[(5 + t) % 4] for t in range(4)]
    assert set(seq) == {"uniformadaptive", "random", "quantilesglobal"}
    # Random: a node's folded histogram keeps about nb - 1 of its boundaries
    from h2o3_amd.models.tree.engine import GrowParams
    bd = bin_frame_tensors([torch.tensor(df.x.values.astype(np.float32))], [False], [0], ["x"],
                           hist_type="Random", nbins=20, nbins_top_level=1024)
    g = TreeGrower(bd, GrowParams(seed=7))
    g._tree_no, g._depth = 0, 4                                   # nb = max(1024 >> (4 - 1), 20) = 128
    H = torch.zeros((1, 2, bd.Bs, 2), dtype=torch.float64)
    H[0, :, : bd.nbins[0], 0] = 1.0
    H[0, :, : bd.nbins[0], 1] = torch.arange(bd.nbins[0], dtype=torch.float64)
    Hf = g._adapt_hist(H)
    kept = (Hf[0, :, : bd.nbins[0], 0] != 0).sum(1)
    assert torch.all((kept > 90) & (kept < 170)), kept
    assert not torch.equal(Hf[0, 0], Hf[0, 1])                   # redrawn per node
    torch.testing.assert_close(Hf[..., :bd.nbins[0], :].sum(2), H[..., :bd.nbins[0], :].sum(2))


def test_monotone_bounds_in_split_search():
    """A node bounded to [lo, hi]: a split whose child means leave the bounds
    loses w (c - mean)^2 per clamped child (use_bounds), or is vetoed."""
    from h2o3_amd.models.tree.engine import GrowParams, TreeGrower
    x = torch.arange(16, dtype=torch.float32)
    bd = bin_frame_tensors([x], [False], [0], ["x"], hist_type="QuantilesGlobal", nbins=16)
    Bs = bd.Bs
    H = torch.zeros((1, 1, Bs, 2), dtype=torch.float64)
    y = torch.tensor([0.0] * 8 + [10.0] * 8, dtype=torch.float64)
    H[0, 0, :16, 0] = 1.0
    H[0, 0, :16, 1] = y
    wyy = (y * y).sum().view(1)
    res = {}
    for ub in (True, False):
        g = TreeGrower(bd, GrowParams(min_rows=1, monotone=np.array([1.0]), use_bounds=ub))
        g._bnd, g._bnd_off = torch.tensor([[2.0, 8.0]], dtype=torch.float64), 0
        res[ub] = g._find_splits_torch(H, torch.ones((1, 1), dtype=torch.bool), wyy)
        g._bnd = None
        free = g._find_splits_torch(H, torch.ones((1, 1), dtype=torch.bool), wyy)
    # unbounded best: means 0 | 10 at t = 7, gain 400; clamped to 2 | 8: 400 - 8*4 - 8*4
    assert float(free["gain"][0]) == pytest.approx(400.0)
    assert float(res[True]["gain"][0]) == pytest.approx(400.0 - 64.0)
    assert not np.isfinite(float(res[False]["gain"][0]))


def test_uniform_adaptive_gbm_matches_reference_mojo_top_splits():
    """Pinned against the reference's own GBM MOJO fixture
    (h2o-genmodel/src/test/resources/hex/genmodel/algos/gbm/
    gbm_variable_importance.zip: prostate, CAPSULE ~ AGE..GLEASON, 50 trees,
    reference defaults -- deterministic: sample_rate 1, col_sample_rate 1).
    With histogram_type UniformAdaptive (the reference AUTO) our first two
    trees split the root and both depth-1 children exactly as the reference
    (GLEASON < 6.5 with NAs left, DPROS < 2.5, PSA < 14.7301: the depth-1
    node bins its parent's PSA range on the top-level grid), and tree 0 has
    the reference's 23 internal nodes.  Deeper thresholds differ slightly:
    the reference re-bins each node over the parent's exact float min / max
    (DTree.java:337-351), ours folds the fixed top-level grid over the
    parent's occupied code range, so its cut points stay on that grid."""
    import os
    R = "/root/reference/h2o-genmodel/src/test/resources/hex/genmodel/algos/gbm/gbm_variable_importance.zip"
    D = "/root/reference/h2o-core/src/main/resources/extdata/prostate.csv"
    if not (os.path.exists(R) and os.path.exists(D)):
        pytest.skip("reference fixture not present")
    import pandas as pd
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    from h2o3_amd.mojo import h2o_mojo
    from h2o3_amd.tree import H2OTree
    cols = ["AGE", "RACE", "DPROS", "DCAPS", "PSA", "VOL", "GLEASON"]
    ref = h2o_mojo.load(R)
    df = pd.read_csv(D)
    fr = h2o.H2OFrame(df)
    fr["CAPSULE"] = fr["CAPSULE"].asfactor()
    g = H2OGradientBoostingEstimator(ntrees=2, seed=1, histogram_type="UniformAdaptive")
    g.train(x=cols, y="CAPSULE", training_frame=fr)
    psa = df.loc[df.GLEASON >= 6.5, "PSA"]
    cell = (psa.max() - psa.min()) / 20
    for t in range(2):
        rt = ref.trees[0][t]
        ot = H2OTree(g, t)
        assert ot.features[0] == cols[rt.col[0]] == "GLEASON"
        assert ot.thresholds[0] == pytest.approx(rt.split[0]) == 6.5
        assert (ot.nas[0] == "LEFT") == bool(rt.na_left[0])
        lo, ro = ot.left_children[0], ot.right_children[0]
        lr, rr = rt.left[0], rt.right[0]
        assert ot.features[lo] == cols[rt.col[lr]] == "DPROS"
        assert ot.thresholds[lo] == pytest.approx(rt.split[lr])
        assert ot.features[ro] == cols[rt.col[rr]] == "PSA"
        assert ot.thresholds[ro] == pytest.approx(rt.split[rr], abs=1e-4)
        assert abs(ot.thresholds[ro] - rt.split[rr]) < cell
    n_internal = sum(1 for f in H2OTree(g, 0).features if f is not None)
    assert n_internal == len(ref.trees[0][0].col) == 23


def test_uniform_adaptive_50_tree_fixture_parity_numbers():
    """The whole 50-tree reference fixture (gbm_variable_importance.zip, the
    reference AUTO = UniformAdaptive, defaults) against our UniformAdaptive
    GBM on the same prostate frame.  Splits are pinned exactly down to depth
    1 (test above); deeper, our fold snaps cut points to the top-level grid
    while the reference re-bins over each parent's exact float range, so
    parity is UNPINNED beyond depth 1 and the whole-model distance is stated
    instead (measured: max |p - p_ref| 0.124, mean 0.026 over the 380 rows;
    training AUC 0.97986 vs the fixture's 0.98016, logloss 0.2718 vs
    0.2676)."""
    import os
    R = "/root/reference/h2o-genmodel/src/test/resources/hex/genmodel/algos/gbm/gbm_variable_importance.zip"
    D = "/root/reference/h2o-core/src/main/resources/extdata/prostate.csv"
    if not (os.path.exists(R) and os.path.exists(D)):
        pytest.skip("reference fixture not present")
    import pandas as pd
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    from h2o3_amd.mojo.genmodel import MojoModel
    cols = ["AGE", "RACE", "DPROS", "DCAPS", "PSA", "VOL", "GLEASON"]
    df = pd.read_csv(D)
    fr = h2o.H2OFrame(df)
    fr["CAPSULE"] = fr["CAPSULE"].asfactor()
    p_ref = MojoModel.load(R).predict(df[cols])["p1"].values
    g = H2OGradientBoostingEstimator(ntrees=50, seed=1, histogram_type="UniformAdaptive")
    g.train(x=cols, y="CAPSULE", training_frame=fr)
    p = g.predict(fr).as_data_frame()["p1"].values
    d = np.abs(p - p_ref)
    assert d.max() < 0.13 and d.mean() < 0.03, (d.max(), d.mean())
    assert g.auc() == pytest.approx(0.9801618150931445, abs=1e-3)
    assert g.logloss() == pytest.approx(0.2675723908575812, rel=0.03)
