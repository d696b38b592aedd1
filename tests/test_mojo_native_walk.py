"""The standalone MOJO reader's native tree walks (native/mojo_forest.cpp)
give bit-equal outputs to its numpy level walk -- GBM (binomial, regression,
multinomial), DRF and XGBoost (gbtree, DART) MOJOs in the reference layout,
with NAs, categoricals and unseen levels."""
import os
import tempfile

import numpy as np
import pandas as pd
import pytest

import h2o3_amd
from h2o3_amd.estimators import H2OGradientBoostingEstimator, H2ORandomForestEstimator, H2OXGBoostEstimator
from h2o3_amd.mojo import h2o_mojo
from h2o3_amd.mojo.genmodel import MojoModel


def _set_native(on):
    os.environ["H2O3_MOJO_NATIVE"] = "1" if on else "0"
    h2o_mojo._FOREST[0] = False
    h2o_mojo._FOREST[1] = None


@pytest.fixture(scope="module")
def data():
    h2o3_amd.init(verbose=False)
    rng = np.random.RandomState(0)
    n = 3000
    X = rng.randn(n, 5).astype(np.float32).astype(np.float64)
    X[rng.rand(n, 5) < 0.05] = np.nan
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(5)])
    df["c"] = rng.choice(list("abcdefghijklmnopqrstuvwxyz0123456789"), n)
    df["y"] = np.where(np.nan_to_num(X[:, 0]) + (df.c < "m") * 0.7 + rng.randn(n) > 0, "yes", "no")
    df["m"] = rng.choice(["u", "v", "w"], n)
    df["r"] = (np.nan_to_num(X[:, 1]) + rng.randn(n)).astype(np.float32).astype(np.float64)
    return df, h2o3_amd.H2OFrame(df)


CASES = [(H2OGradientBoostingEstimator, dict(ntrees=15, max_depth=6, seed=1), "y"),
         (H2OGradientBoostingEstimator, dict(ntrees=8, max_depth=4, seed=1), "m"),
         (H2OGradientBoostingEstimator, dict(ntrees=8, max_depth=5, seed=1), "r"),
         (H2ORandomForestEstimator, dict(ntrees=10, max_depth=12, seed=1), "y"),
         (H2OXGBoostEstimator, dict(ntrees=10, max_depth=5, seed=1), "y"),
         (H2OXGBoostEstimator, dict(ntrees=6, max_depth=4, seed=1), "m"),
         (H2OXGBoostEstimator, dict(ntrees=10, max_depth=5, seed=1, booster="dart"), "y")]


@pytest.mark.parametrize("cls,kw,y", CASES)
def test_native_walk_equals_numpy_walk(data, cls, kw, y):
    df, fr = data
    lib = os.path.join(os.path.dirname(h2o_mojo.__file__), "..", "ops", "lib", "libmojo_forest.so")
    if not os.path.exists(lib):
        pytest.skip("libmojo_forest.so not built")
    xs = [f"x{i}" for i in range(5)] + ["c"]
    m = cls(**kw)
    m.train(x=xs, y=y, training_frame=fr)
    p = m.download_mojo(tempfile.mkdtemp(), format="h2o")
    test = df[xs].copy()
    test.loc[::9, "c"] = "unseen_level"
    out = {}
    try:
        for on in (True, False):
            _set_native(on)
            out[on] = MojoModel.load(p).predict(test)
    finally:
        _set_native(True)
    a, b = out[True], out[False]
    assert list(a.columns) == list(b.columns)
    for c in a.columns:
        if a[c].dtype == object:
            assert (a[c].astype(str) == b[c].astype(str)).all()
        else:
            np.testing.assert_array_equal(a[c].values, b[c].values)
