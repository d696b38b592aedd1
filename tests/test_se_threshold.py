"""Stacked ensemble labels come from the metalearner's threshold
(StackedEnsembleModel.java:251-258: predictions are metalearner.score of the
level-one frame), and the reference-layout MOJO labels identically."""
import tempfile

import numpy as np
import pandas as pd

import h2o3_amd
from h2o3_amd.estimators import H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator
from h2o3_amd.models.ensemble import H2OStackedEnsembleEstimator
from h2o3_amd.mojo.genmodel import MojoModel


def test_se_labels_use_metalearner_threshold_and_match_mojo():
    h2o3_amd.init(verbose=False)
    rng = np.random.RandomState(0)
    n = 3000
    X = rng.randn(n, 5).astype(np.float32).astype(np.float64)   # f32-exact: frame and MOJO see the same values
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(5)])
    df["y"] = np.where(X[:, 0] + X[:, 1] * X[:, 2] + rng.randn(n) > 0.8, "yes", "no")
    fr = h2o3_amd.H2OFrame(df)
    kw = dict(nfolds=3, fold_assignment="Modulo", keep_cross_validation_predictions=True, seed=1)
    g = H2OGradientBoostingEstimator(ntrees=10, max_depth=4, **kw)
    g.train(y="y", training_frame=fr)
    l = H2OGeneralizedLinearEstimator(family="binomial", **kw)
    l.train(y="y", training_frame=fr)
    se = H2OStackedEnsembleEstimator(base_models=[g, l])
    se.train(y="y", training_frame=fr)
    thr = se._meta._label_threshold()
    assert se._label_threshold() == thr
    pm = se.predict(fr).as_data_frame()
    np.testing.assert_array_equal(pm["predict"].values == "yes", pm["yes"].values >= thr)
    p = se.download_mojo(tempfile.mkdtemp(), format="h2o")
    pj = MojoModel.load(p).predict(df[[f"x{i}" for i in range(5)]])
    np.testing.assert_allclose(pj.iloc[:, -1].values, pm["yes"].values, rtol=1e-5, atol=1e-6)
    near = np.abs(pm["yes"].values - thr) < 1e-5
    agree = pj.iloc[:, 0].astype(str).values == pm["predict"].astype(str).values
    assert agree[~near].all()
