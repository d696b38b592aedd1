"""GLM training parity with numbers the reference hard-codes, on data that
ships in the reference tree (h2o-core/src/main/resources/extdata/prostate.csv).

hex/glm/GLMTest.java:1705-1740 (testProstate): binomial, lambda = 0,
standardize = false, ID ignored, RACE categorical (the test's
prostate_cat_replaced.csv relabels RACE 0/1/2 as R1/R2/R3, so RACE.R2 /
RACE.R3 are our RACE.1 / RACE.2); the reference model converges in 5
iterations, and capped at 4 its coefficients match R's to 1e-4, null
deviance 512.3, residual deviance 378.3, residual DOF 371, AIC 396.3.
GLMBasicTestBinomial.java:295-299 trains on prostate_cat_train.csv, which
does not ship: parity unpinned.  GBM / DRF: hex/tree/gbm/GBMTest.java and
hex/tree/drf/DRFTest.java hard-code no training numbers on the shipped files
(their prostate cases assert MOJO / POJO agreement and staged predictions
only; the numeric expectations use smalldata files that do not ship):
parity unpinned -- the tree engine is pinned against the reference's MOJO
fixtures instead (tests/test_mojo_reference.py).
"""
import os

import pytest

import h2o3_amd as h2o
from h2o3_amd.estimators import H2OGeneralizedLinearEstimator

PROSTATE = "/root/reference/h2o-core/src/main/resources/extdata/prostate.csv"
pytestmark = pytest.mark.skipif(not os.path.exists(PROSTATE), reason="reference tree not present")

# GLMTest.java:1712-1713
_NAMES = ["Intercept", "AGE", "RACE.1", "RACE.2", "DPROS", "DCAPS", "PSA", "VOL", "GLEASON"]
_VALS = [-8.14867, -0.01368, 0.32337, -0.38028, 0.55964, 0.49548, 0.02794, -0.01104, 0.97704]


@pytest.fixture(scope="module")
def prostate():
    h2o.init(verbose=False)
    fr = h2o.import_file(PROSTATE)
    fr["RACE"] = fr["RACE"].asfactor()
    fr["CAPSULE"] = fr["CAPSULE"].asfactor()
    return fr


@pytest.mark.parametrize("max_iterations", [None, 4])
def test_glm_prostate_binomial_matches_reference(prostate, max_iterations):
    kw = {} if max_iterations is None else {"max_iterations": max_iterations}
    m = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0, standardize=False, **kw)
    m.train(x=[c for c in prostate.names if c not in ("ID", "CAPSULE")], y="CAPSULE", training_frame=prostate)
    coef = m.coef()
    for n, v in zip(_NAMES, _VALS):
        assert coef[n] == pytest.approx(v, abs=1e-4), (n, coef[n], v)
    assert m.null_deviance() == pytest.approx(512.3, abs=0.1)
    assert m.residual_deviance() == pytest.approx(378.3, abs=0.1)
    assert m.residual_degrees_of_freedom() == 371
    assert m.aic() == pytest.approx(396.3, abs=0.1)
    # GLMTest.java:1721, :1726: bestSubmodel().iteration == 5 (converged) / == 4 (capped)
    assert m._output["model_summary"]["number_of_iterations"] == (5 if max_iterations is None else 4)


def test_scaled_cond_device_estimator_matches_lapack():
    """GLMDriver._scaled_cond_dev (Hager's estimate on a torch Cholesky, the
    device path of the wide IRLS system) equals LAPACK dpocon's estimate
    (_scaled_cond), including a zero-variance column left out of both."""
    import numpy as np
    import torch
    from h2o3_amd.models.glm.glm import GLMDriver
    g = np.random.default_rng(3)
    for n, P in ((2000, 50), (5000, 300)):
        X = g.standard_normal((n, P)) * np.exp(g.uniform(-2, 2, P))
        X[:, 1] = X[:, 0] + 0.05 * g.standard_normal(n)
        X[:, 7] = 0.0
        A = X.T @ X
        want = GLMDriver._scaled_cond(A)
        got = GLMDriver._scaled_cond_dev(torch.from_numpy(A))
        assert got == pytest.approx(want, rel=1e-8)
    assert GLMDriver._scaled_cond_dev(torch.from_numpy(-np.eye(4))) == 1.0
    bad = np.ones((3, 3))
    assert GLMDriver._scaled_cond_dev(torch.from_numpy(bad)) == float("inf")


def test_kappa_from_shared_factor_matches_lapack():
    """The device step's tier check reuses the solve's Cholesky factor
    (factor of D A D = D L): same estimate as LAPACK on the scaled matrix;
    a failed factor falls back to the filtered estimate."""
    import numpy as np
    import torch
    from h2o3_amd.models.glm.glm import GLMDriver
    g = np.random.default_rng(5)
    X = g.standard_normal((3000, 200)) * np.exp(g.uniform(-3, 3, 200))
    X[:, 5] = X[:, 4] + 0.01 * g.standard_normal(3000)
    A = X.T @ X
    At = torch.from_numpy(A)
    L, info = torch.linalg.cholesky_ex(At)
    assert GLMDriver._kappa_from_factor(At, L, info) == pytest.approx(GLMDriver._scaled_cond(A), rel=1e-8)
    A[:, 9] = A[9, :] = 0.0
    At = torch.from_numpy(A)
    L, info = torch.linalg.cholesky_ex(At)
    assert int(info) != 0
    assert GLMDriver._kappa_from_factor(At, L, info) == pytest.approx(GLMDriver._scaled_cond(A), rel=1e-8)


@pytest.mark.parametrize("intercept,l2", [(True, 0.0), (True, 0.3), (False, 0.3)])
def test_device_ridge_step_matches_host_solver(intercept, l2):
    """GLMDriver._step_solve_dev (the device Newton step of wide ridge-only
    systems; run here on CPU tensors) equals the host _solve_quadratic on
    the same system, penalty off the intercept, and reports the same
    max |gradient|."""
    from types import SimpleNamespace
    import numpy as np
    import torch
    from h2o3_amd.models.glm.glm import GLMDriver, _solve_quadratic
    g = np.random.default_rng(11)
    P = 40
    k = P + 1 if intercept else P
    A = g.standard_normal((500, k))
    Gn = A.T @ A / 500
    bn = g.standard_normal(k)
    beta = g.standard_normal(P + 1) * 0.1
    drv = SimpleNamespace(beta=beta, intercept=intercept, P=P)
    Gt, bt = torch.from_numpy(Gn), torch.from_numpy(bn)
    At = Gt.clone()
    pen = torch.full((k,), l2, dtype=torch.float64)
    if intercept:
        pen[-1] = 0.0
    At.diagonal().add_(pen)
    L, info = torch.linalg.cholesky_ex(At)
    gmax, new = GLMDriver._step_solve_dev(drv, Gt, bt, l2, L, info)
    want = _solve_quadratic(Gn, bn, 0.0, l2, intercept)
    np.testing.assert_allclose(new, want, rtol=1e-10, atol=1e-12)
    bcur = beta if intercept else beta[:-1]
    gq = Gn @ bcur - bn
    gq[:P] += l2 * bcur[:P]
    assert gmax == pytest.approx(float(np.abs(gq).max()), rel=1e-12)
