"""Device-resident GBM tree (models/tree/devtree.py) vs the level loop.

The whole tree runs as one captured hipGraph (residual, histograms, split
search, partition, leaf values, per-row scatter) with ONE host read of the
tree record per tree.  It must grow the trees of the level loop
(engine.TreeGrower, H2O3_DEV_TREE=0): same splits, thresholds, NA
directions and leaf values, and the same predictions.  Reference:
hex/tree/SharedTree.java:481-516, GBM.java:464.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _frame(n, F, family, seed=0, na=0.0):
    import h2o3_amd
    from h2o3_amd.core.frame import H2OFrame
    h2o3_amd.init(verbose=False)
    g = np.random.default_rng(seed)
    X = g.standard_normal((n, F)).astype(np.float32)
    if na:
        X[g.random((n, F)) < na] = np.nan
    Xz = np.nan_to_num(X)
    eta = Xz[:, 0] - 0.7 * Xz[:, 1] + 0.5 * np.sin(2 * Xz[:, 2]) * Xz[:, 3]
    cols = {f"x{j}": X[:, j] for j in range(F)}
    if family == "bernoulli":
        cols["y"] = (g.random(n) < 1 / (1 + np.exp(-eta))).astype(int)
    else:
        cols["y"] = eta + 0.3 * g.standard_normal(n)
    fr = H2OFrame(cols)
    if family == "bernoulli":
        fr["y"] = fr["y"].asfactor()
    return fr, [f"x{j}" for j in range(F)]


def _fit(monkeypatch, fr, names, dev_tree, ntrees=6, **kw):
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.models.tree.gbm import GBMDriver, H2OGradientBoostingEstimator
    monkeypatch.setenv("H2O3_DEV_TREE", "1" if dev_tree else "0")
    est = H2OGradientBoostingEstimator(ntrees=ntrees, seed=7, ignore_const_cols=False, histogram_type="QuantilesGlobal",
                                       nbins=255, **kw)
    spec = TrainSpec(fr, names, "y")
    est._spec = spec
    drv = GBMDriver(est, spec)
    for _ in range(ntrees):
        drv.step()
    forest = drv.forest
    return drv, forest, drv.predictions().detach().cpu().numpy()


def _same_trees(fa, fb):
    assert len(fa.trees) == len(fb.trees)
    for ta, tb in zip(fa.trees, fb.trees):
        assert ta.n_nodes == tb.n_nodes
        np.testing.assert_array_equal(np.asarray(ta.feat), np.asarray(tb.feat))
        np.testing.assert_array_equal(np.asarray(ta.left), np.asarray(tb.left))
        np.testing.assert_array_equal(np.asarray(ta.right), np.asarray(tb.right))
        np.testing.assert_array_equal(np.asarray(ta.na_left), np.asarray(tb.na_left))
        np.testing.assert_allclose(np.asarray(ta.thr), np.asarray(tb.thr))
        np.testing.assert_allclose(np.asarray(ta.value), np.asarray(tb.value), rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(np.asarray(ta.weight), np.asarray(tb.weight), rtol=1e-9)


@pytest.mark.parametrize("family,na,depth", [("bernoulli", 0.0, 6), ("bernoulli", 0.03, 5), ("gaussian", 0.0, 4)])
def test_devtree_matches_level_loop(monkeypatch, family, na, depth):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fr, names = _frame(400_000, 32, family, na=na)
    d1, f1, p1 = _fit(monkeypatch, fr, names, True, max_depth=depth)
    assert getattr(d1, "_devtree", None) is not None, getattr(d1, "_devtree_why", None)
    if family == "bernoulli":
        assert d1._devtree.graph is not None          # trees 2.. replayed from the captured graph
    d0, f0, p0 = _fit(monkeypatch, fr, names, False, max_depth=depth)
    assert getattr(d0, "_devtree", None) is None
    _same_trees(f1, f0)
    np.testing.assert_allclose(p1, p0, rtol=1e-5, atol=1e-6)


def test_devtree_tree_column_sample_and_min_rows(monkeypatch):
    """col_sample_rate_per_tree (the split kernels' eligibility mask is
    rewritten outside the graph per tree) and a large min_rows (early leaves:
    absent heap nodes and leaves above the last level)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fr, names = _frame(200_000, 32, "bernoulli", seed=3)
    kw = dict(max_depth=7, col_sample_rate_per_tree=0.5, min_rows=4000.0)
    d1, f1, p1 = _fit(monkeypatch, fr, names, True, ntrees=5, **kw)
    assert getattr(d1, "_devtree", None) is not None
    d0, f0, p0 = _fit(monkeypatch, fr, names, False, ntrees=5, **kw)
    # early leaves shrink the level loop's frontier, so its histogram chunks
    # (fixed-point scales) may differ in the last bits: same structure, values close
    for ta, tb in zip(f1.trees, f0.trees):
        np.testing.assert_array_equal(np.asarray(ta.feat), np.asarray(tb.feat))
        np.testing.assert_array_equal(np.asarray(ta.left), np.asarray(tb.left))
        np.testing.assert_allclose(np.asarray(ta.value), np.asarray(tb.value), rtol=1e-5, atol=1e-8)
    assert any(np.asarray(t.depth)[np.asarray(t.left) < 0].min() < 7 for t in f1.trees)
    np.testing.assert_allclose(p1, p0, rtol=1e-5, atol=1e-6)


def test_devtree_model_predicts_like_training_state(monkeypatch):
    """A full estimator train on the device-resident path: the decoded host
    trees score (forest kernel) to the driver's running predictions."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from h2o3_amd.models.tree.gbm import H2OGradientBoostingEstimator
    monkeypatch.setenv("H2O3_DEV_TREE", "1")
    fr, names = _frame(100_000, 16, "bernoulli", seed=5)
    m = H2OGradientBoostingEstimator(ntrees=10, max_depth=5, seed=1)
    m.train(x=names, y="y", training_frame=fr)
    p = m.predict(fr).as_data_frame()["p1"].values
    assert m.auc() > 0.7
    assert np.isfinite(p).all() and p.min() >= 0 and p.max() <= 1


@pytest.mark.parametrize("kw", [dict(sample_rate=0.7), dict(col_sample_rate=0.6),
                                dict(sample_rate=0.8, col_sample_rate=0.8, col_sample_rate_per_tree=0.8,
                                     col_sample_rate_change_per_level=0.9)])
def test_devtree_row_and_column_sampling(monkeypatch, kw):
    """AutoML's GBM sampling settings on the device-resident tree: row sampling
    as the residual pass's 0/1 weights (NaN = out of sample), per-node column
    samples built on the device with the level loop's per-node draws -- the
    same trees as the level loop."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fr, names = _frame(200_000, 32, "bernoulli", seed=11)
    d1, f1, p1 = _fit(monkeypatch, fr, names, True, ntrees=5, max_depth=6, **kw)
    assert getattr(d1, "_devtree", None) is not None, getattr(d1, "_devtree_why", None)
    d0, f0, p0 = _fit(monkeypatch, fr, names, False, ntrees=5, max_depth=6, **kw)
    for ta, tb in zip(f1.trees, f0.trees):
        np.testing.assert_array_equal(np.asarray(ta.feat), np.asarray(tb.feat))
        np.testing.assert_array_equal(np.asarray(ta.left), np.asarray(tb.left))
        np.testing.assert_allclose(np.asarray(ta.thr), np.asarray(tb.thr))
        np.testing.assert_allclose(np.asarray(ta.value), np.asarray(tb.value), rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(p1, p0, rtol=1e-5, atol=1e-6)


# draws from AutoML's GBM grid space (automl/_grid_space) with max_depth in
# the device tree's range: the device tree must grow the level loop's trees
# for every sampling / min_rows / min_split_improvement combination it takes
_GRID_DRAWS = [dict(max_depth=3, min_rows=100, sample_rate=0.5, col_sample_rate=0.4, col_sample_rate_per_tree=0.4,
                    min_split_improvement=1e-4),
               dict(max_depth=7, min_rows=30, sample_rate=1.0, col_sample_rate=1.0, col_sample_rate_per_tree=0.4,
                    min_split_improvement=1e-5),
               dict(max_depth=11, min_rows=1, sample_rate=0.9, col_sample_rate=0.7, col_sample_rate_per_tree=1.0,
                    min_split_improvement=1e-4),
               dict(max_depth=5, min_rows=15, sample_rate=0.6, col_sample_rate=0.4, col_sample_rate_per_tree=0.7,
                    min_split_improvement=1e-5)]


@pytest.mark.parametrize("hp", _GRID_DRAWS, ids=[f"d{h['max_depth']}" for h in _GRID_DRAWS])
def test_devtree_matches_level_loop_on_automl_grid_draws(monkeypatch, hp):
    fr, names = _frame(300_000, 48, "bernoulli", seed=4)
    d1, f1, p1 = _fit(monkeypatch, fr, names, True, **hp)
    assert getattr(d1, "_devtree", None) is not None, getattr(d1, "_devtree_why", None)
    d0, f0, p0 = _fit(monkeypatch, fr, names, False, **hp)
    _same_trees(f1, f0)
    np.testing.assert_allclose(p1, p0, rtol=1e-5, atol=1e-6)


def test_devtree_full_train_with_early_stopping(monkeypatch):
    """The estimator path (scoring every 5 trees, early stopping, validation
    scoring) gives the level loop's model and a sound AUC."""
    from h2o3_amd.estimators import H2OGradientBoostingEstimator
    fr, names = _frame(200_000, 48, "bernoulli", seed=5)
    va, _ = _frame(50_000, 48, "bernoulli", seed=6)
    out = {}
    for dev in (True, False):
        monkeypatch.setenv("H2O3_DEV_TREE", "1" if dev else "0")
        m = H2OGradientBoostingEstimator(ntrees=60, score_tree_interval=5, stopping_rounds=3, seed=3,
                                         **_GRID_DRAWS[0])
        m.train(x=names, y="y", training_frame=fr, validation_frame=va)
        out[dev] = (len(m._forest), m.auc(valid=True),
                    m.predict(va).as_data_frame().iloc[:, -1].to_numpy())
    assert out[True][0] == out[False][0]
    assert out[True][1] > 0.7, out[True][1]
    np.testing.assert_allclose(out[True][2], out[False][2], rtol=1e-5, atol=1e-6)
