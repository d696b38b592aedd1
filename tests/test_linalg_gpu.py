"""Numerics of the GLM / Gram HIP kernels (ops/csrc/gram.hip) vs fp64 torch."""
import pytest
import torch

from h2o3_amd.models.glm.glm import _Fam
from h2o3_amd.ops import linalg_ops

pytestmark = pytest.mark.gpu


def _data(n, P, Pp, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.zeros(n, Pp)
    X[:, :P] = torch.randn(n, P, generator=g)
    beta = torch.zeros(Pp)
    beta[:P] = 0.1 * torch.randn(P, generator=g)
    return X, beta, g


def _close(a, b, rtol=2e-4):
    scale = b.abs().max().item() + 1e-12
    return (a.cpu() - b).abs().max().item() / scale < rtol


@pytest.mark.parametrize("family,link", [("binomial", "logit"), ("poisson", "log"), ("gaussian", "identity"),
                                         ("gamma", "log"), ("tweedie", "log")])
@pytest.mark.parametrize("P,Pp", [(30, 32), (60, 64), (100, 128), (200, 256)])
def test_glm_irls_fused(family, link, P, Pp):
    n = 50_003
    X, beta, g = _data(n, P, Pp)
    eta = X @ beta + 0.2
    if family == "binomial":
        y = (torch.rand(n, generator=g) < torch.sigmoid(eta)).float()
    elif family == "gaussian":
        y = eta + torch.randn(n, generator=g)
    else:
        y = torch.distributions.Poisson(torch.exp(eta)).sample() + (0.5 if family in ("gamma",) else 0.0)
    w = torch.rand(n, generator=g) + 0.5
    off = 0.1 * torch.randn(n, generator=g)
    fam = _Fam(family, link, tvp=1.5 if family == "tweedie" else 0.0)
    codes = linalg_ops.glm_fused_codes(family, link)
    Gk, dk = linalg_ops.glm_irls(X.cuda(), aug=P, beta=beta.cuda(), b0=0.2, y=y.cuda(), wprior=w.cuda(),
                                 offset=off.cuda(), codes=codes, tvp=fam.tvp, theta=fam.theta)
    Gr, dr = linalg_ops.glm_irls_reference(X, aug=P, beta=beta, b0=0.2, y=y, wprior=w, offset=off, fam=fam)
    assert _close(Gk[: P + 2, : P + 2], Gr[: P + 2, : P + 2])
    assert abs(dk.item() - dr.item()) / abs(dr.item()) < 1e-3


def test_glm_irls_external_and_gram():
    n, P, Pp = 77_777, 90, 96
    X, _, g = _data(n, P, Pp, seed=3)
    W = torch.rand(n, generator=g)
    z = torch.randn(n, generator=g)
    Gk, _ = linalg_ops.glm_irls(X.cuda(), aug=P, W=W.cuda(), z=z.cuda())
    Gr, _ = linalg_ops.glm_irls_reference(X, aug=P, W=W, z=z)
    assert _close(Gk[: P + 2, : P + 2], Gr[: P + 2, : P + 2])
    G2 = linalg_ops.weighted_gram(X.cuda(), W.cuda())
    G2r = X.double().T @ (X.double() * W.double().view(-1, 1))
    assert _close(G2, G2r)
    G3 = linalg_ops.weighted_gram(X[:1000].cuda())
    assert _close(G3, X[:1000].double().T @ X[:1000].double())


@pytest.mark.parametrize("signed", [False, True])
@pytest.mark.parametrize("P,Pp", [(61, 64), (100, 128), (200, 224), (400, 512)])
def test_glm_irls_external_widths(P, Pp, signed):
    n = 20_011
    X, _, g = _data(n, P, Pp, seed=5)
    W = torch.randn(n, generator=g) if signed else torch.rand(n, generator=g)
    z = torch.randn(n, generator=g)
    Gk, _ = linalg_ops.glm_irls(X.cuda(), aug=P, W=W.cuda(), z=z.cuda())
    Gr, _ = linalg_ops.glm_irls_reference(X, aug=P, W=W, z=z)
    assert _close(Gk[: P + 2, : P + 2], Gr[: P + 2, : P + 2])


def test_weighted_gram_aug_matches_fp64():
    """Wide-design augmented Gram (library GEMM path) vs fp64 torch."""
    import torch
    if not torch.cuda.is_available():
        import pytest
        pytest.skip("no GPU")
    from h2o3_amd.ops import linalg_ops
    g = torch.Generator(device="cuda").manual_seed(0)
    N, P = 300000, 600
    X = torch.randn(N, P + 8, generator=g, device="cuda")
    W = torch.rand(N, generator=g, device="cuda", dtype=torch.float64)
    z = torch.randn(N, generator=g, device="cuda", dtype=torch.float64)
    G, xw, xz, sw, swz = linalg_ops.weighted_gram_aug(X, W, z, P, step=100000)
    Xd = X[:, :P].double()
    torch.testing.assert_close(G, Xd.T @ (Xd * W.view(-1, 1)), rtol=2e-4, atol=2e-2)
    torch.testing.assert_close(xw, Xd.T @ W, rtol=2e-4, atol=2e-2)
    torch.testing.assert_close(xz, Xd.T @ (W * z), rtol=2e-4, atol=2e-2)
    torch.testing.assert_close(sw, W.sum(), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(swz, (W * z).sum(), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("bf3", ["1", "0"])
def test_glm_irls_bf3_elementwise(monkeypatch, bf3):
    """P = 100 (padded 128) runs the warp-specialised kernel; H2O3_GLM_BF3
    selects bf16x3 (hi*hi + hi*lo + lo*hi on 16x16x32 bf16 MFMA) or f32
    16x16x4 MFMA.  Both must match fp64 entry by entry, not just at the max."""
    monkeypatch.setenv("H2O3_GLM_BF3", bf3)
    n, P, Pp = 300_007, 100, 128
    X, beta, g = _data(n, P, Pp, seed=11)
    X[:, 7] = 3.0 + 0.01 * X[:, 7]          # near-constant column: large mean, small spread
    y = (torch.rand(n, generator=g) < torch.sigmoid(X @ beta)).float()
    fam = _Fam("binomial", "logit")
    codes = linalg_ops.glm_fused_codes("binomial", "logit")
    Gk, dk = linalg_ops.glm_irls(X.cuda(), aug=P, beta=beta.cuda(), b0=-0.1, y=y.cuda(), codes=codes)
    Gr, dr = linalg_ops.glm_irls_reference(X, aug=P, beta=beta, b0=-0.1, y=y, fam=fam)
    A, B = Gk[: P + 2, : P + 2].cpu(), Gr[: P + 2, : P + 2]
    diag = B.diagonal().abs().sqrt()
    rel = (A - B).abs() / (diag.view(-1, 1) * diag.view(1, -1))   # error relative to sqrt(G_ii G_jj)
    assert rel.max().item() < 2e-5
    assert abs(dk.item() - dr.item()) / abs(dr.item()) < 1e-4


def test_glm_fit_bf3_matches_f32(monkeypatch):
    """End-to-end IRLSM fit: bf16x3 and f32 MFMA Gram give the same model."""
    import numpy as np
    from h2o3_amd.core.frame import H2OFrame
    from h2o3_amd.models.glm.glm import H2OGeneralizedLinearEstimator
    g = np.random.default_rng(2)
    n, P = 200_000, 100
    X = g.standard_normal((n, P)).astype(np.float32)
    b = 0.2 * g.standard_normal(P)
    y = (g.random(n) < 1 / (1 + np.exp(-(X @ b)))).astype(int)
    cols = {f"x{j}": X[:, j] for j in range(P)}
    cols["y"] = y
    fr = H2OFrame(cols)
    fr["y"] = fr["y"].asfactor()
    coefs = []
    for v in ("1", "0"):
        monkeypatch.setenv("H2O3_GLM_BF3", v)
        m = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0.0)
        m.train(y="y", training_frame=fr)
        coefs.append(np.array([m.coef()[k] for k in sorted(m.coef())]))
    np.testing.assert_allclose(coefs[0], coefs[1], rtol=0, atol=2e-5)


@pytest.mark.parametrize("fused", [True, False])
def test_glm_irls_narrow_rows(fused):
    """X stored as [N, 100] (ldx = 100) with logical width 128 gives the same
    augmented Gram as the zero-padded [N, 128] matrix."""
    n, P, Pp = 123_457, 100, 128
    X, beta, g = _data(n, P, Pp, seed=13)
    Xn = X[:, :P].contiguous()
    if fused:
        y = (torch.rand(n, generator=g) < torch.sigmoid(X @ beta)).float()
        codes = linalg_ops.glm_fused_codes("binomial", "logit")
        kw = dict(aug=P, beta=beta.cuda(), b0=0.3, y=y.cuda(), codes=codes)
    else:
        kw = dict(aug=P, W=torch.randn(n, generator=g).cuda(), z=torch.randn(n, generator=g).cuda())
    Gp, dp = linalg_ops.glm_irls(X.cuda(), **kw)
    Gn, dn = linalg_ops.glm_irls(Xn.cuda(), width=Pp, **kw)
    torch.testing.assert_close(Gn, Gp, rtol=1e-9, atol=1e-9)
    if fused:
        torch.testing.assert_close(dn, dp, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("family,link", [("binomial", "logit"), ("poisson", "log"), ("gaussian", "identity")])
def test_glm_wide_irls_matches_fp64(family, link, fused):
    """Wide pass vs the fp64 reference, P = 601 (odd width: scalar tail
    loads), n = 40009 (a ragged last 64-row chunk).  fused=False: eta +
    family + bf16 hi/lo split + one bf16 library GEMM; fused=True: eta pass +
    the hand-written MFMA Gram kernel over the f32 rows (no z column)."""
    n, P, Pp = 40_009, 601, 640
    X, beta, g = _data(n, P, Pp, seed=17)
    beta *= 0.3
    eta = X @ beta - 0.2
    if family == "binomial":
        y = (torch.rand(n, generator=g) < torch.sigmoid(eta)).float()
    elif family == "gaussian":
        y = eta + torch.randn(n, generator=g)
    else:
        y = torch.distributions.Poisson(torch.exp(eta.clamp(max=3))).sample()
    w = torch.rand(n, generator=g) + 0.5
    off = 0.1 * torch.randn(n, generator=g)
    fam = _Fam(family, link)
    codes = linalg_ops.glm_fused_codes(family, link)
    Xn = X[:, :P].contiguous()
    Gk, dk, gk = linalg_ops.glm_wide_irls(Xn.cuda(), P, beta[:P].cuda(), -0.2, y.cuda(), w.cuda(), off.cuda(),
                                          codes, step=16_384, fused=fused)
    Gr, dr = linalg_ops.glm_irls_reference(X, aug=P, beta=beta, b0=-0.2, y=y, wprior=w, offset=off, fam=fam)
    m = P + 1 if fused else P + 2
    A, B = Gk[:m, :m].cpu(), Gr[:m, :m]
    diag = B.diagonal().abs().sqrt().clamp_min(1e-12)
    rel = (A - B).abs() / (diag.view(-1, 1) * diag.view(1, -1))
    assert rel.max().item() < 5e-5
    assert abs(dk.item() - dr.item()) / abs(dr.item()) < 1e-4
    # exact-gradient channel: X'r and sum r against fp64
    gr = _grad_reference(X[:, :P], beta[:P], -0.2, y, w, off, fam)
    _assert_grad_close(torch.cat([gk[:P], gk[P:P + 1]]).cpu(), gr, X[:, :P], y, w)


def _grad_reference(X, beta, b0, y, w, off, fam):
    """fp64 X'r (+ sum r last), r = w (y - mu) dmu/deta / var."""
    Xd = X.double()
    eta = Xd @ beta.double() + b0 + (0.0 if off is None else off.double())
    mu = fam.linkinv(eta)
    wd = torch.ones_like(eta) if w is None else w.double()
    if fam.family == "gaussian" and fam.link == "identity":
        r = wd * (y.double() - eta)
    else:
        r = wd * (y.double() - mu) * fam.dmu_deta(eta, mu) / fam.variance(mu)
    return torch.cat([Xd.T @ r, r.sum().view(1)])


def _assert_grad_close(gk, gr, X, y, w):
    # error bound: f32 rounding of the per-row terms, relative to sum |x r|
    # (the gradient itself may be near zero by cancellation)
    scale = (X.double().abs().sum(0).max() * (y.double().abs().max() + 1) *
             (1.0 if w is None else float(w.max()))).item()
    err = (gk.double() - gr).abs().max().item()
    assert err / scale < 1e-6, (err, scale)


@pytest.mark.parametrize("family,link", [("binomial", "logit"), ("poisson", "log"), ("gaussian", "identity"),
                                         ("gamma", "log"), ("tweedie", "log")])
@pytest.mark.parametrize("narrow,bf3,P,Pp", [(False, True, 100, 128), (True, True, 100, 128),
                                             (True, False, 100, 128), (False, False, 50, 64),
                                             (False, False, 30, 32)])
def test_glm_irls_grad_channel(family, link, narrow, bf3, P, Pp):
    """Exact-gradient channel of the fused ws kernel (bf16x3 or f32 Hessian):
    g = X'r and sum r with exact f64 products / f64 sums vs fp64 torch."""
    n = 200_003
    X, beta, g = _data(n, P, Pp, seed=21)
    eta = X @ beta + 0.2
    if family == "binomial":
        y = (torch.rand(n, generator=g) < torch.sigmoid(eta)).float()
    elif family == "gaussian":
        y = eta + torch.randn(n, generator=g)
    else:
        y = torch.distributions.Poisson(torch.exp(eta)).sample() + (0.5 if family == "gamma" else 0.0)
    w = torch.rand(n, generator=g) + 0.5
    off = 0.1 * torch.randn(n, generator=g)
    fam = _Fam(family, link, tvp=1.5 if family == "tweedie" else 0.0)
    codes = linalg_ops.glm_fused_codes(family, link)
    Xk = X[:, :P].contiguous() if narrow else X
    Gk, dk, gk = linalg_ops.glm_irls(Xk.cuda(), aug=P, beta=beta.cuda(), b0=0.2, y=y.cuda(), wprior=w.cuda(),
                                     offset=off.cuda(), codes=codes, tvp=fam.tvp, theta=fam.theta, width=Pp,
                                     grad=True, bf3=bf3)
    assert gk.shape == (Pp + 1,)
    assert gk[P:Pp].abs().max().item() == 0.0          # padding / augmented columns carry no gradient
    gr = _grad_reference(X[:, :P], beta[:P], 0.2, y, w, off, fam)
    _assert_grad_close(torch.cat([gk[:P], gk[Pp:]]).cpu(), gr, X[:, :P], y, w)
    # the Hessian and deviance of the same pass are unchanged by the channel
    G0, d0 = linalg_ops.glm_irls(Xk.cuda(), aug=P, beta=beta.cuda(), b0=0.2, y=y.cuda(), wprior=w.cuda(),
                                 offset=off.cuda(), codes=codes, tvp=fam.tvp, theta=fam.theta, width=Pp, bf3=bf3)
    assert torch.equal(G0, Gk) and torch.equal(d0, dk)


def _fp64_irls(X, y, beta0, iters=30):
    """Reference fp64 IRLS (binomial, intercept last) on a host design."""
    Xa = torch.cat([X.double(), torch.ones(X.shape[0], 1, dtype=torch.float64, device=X.device)], 1)
    b = torch.as_tensor(beta0, dtype=torch.float64, device=X.device).clone()
    for _ in range(iters):
        eta = Xa @ b
        mu = torch.sigmoid(eta)
        W = (mu * (1 - mu)).clamp_min(1e-10)
        G = Xa.T @ (Xa * W.view(-1, 1))
        nb = b + torch.linalg.solve(G, Xa.T @ (y.double() - mu))
        if (nb - b).abs().max() < 1e-13:
            b = nb
            break
        b = nb
    return b, G


def _glm_fit_modes(Xh, y, modes, monkeypatch, iters=30, est_kw=None):
    import numpy as np
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.core.frame import H2OFrame
    from h2o3_amd.models.glm.glm import GLMDriver, H2OGeneralizedLinearEstimator
    P = Xh.shape[1]
    cols = {f"x{j}": Xh[:, j] for j in range(P)}
    cols["y"] = y
    fr = H2OFrame(cols)
    fr["y"] = fr["y"].asfactor()
    res, drvs = {}, {}
    for name, env in modes.items():
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        est = H2OGeneralizedLinearEstimator(**(est_kw or dict(family="binomial", solver="IRLSM", lambda_=0.0)))
        spec = TrainSpec(fr, [f"x{j}" for j in range(P)], "y")
        est._spec = spec
        drv = GLMDriver(est, spec)
        assert drv.X.is_cuda
        for _ in range(iters):
            drv.step()
        res[name], drvs[name] = drv.beta.copy(), drv
    return res, drvs


_DEFAULT = {"H2O3_GLM_BF3": "1", "H2O3_GLM_EXACT_GRAD": "1", "H2O3_GLM_TIERS": "1"}
_LEGACY_F32 = {"H2O3_GLM_BF3": "0", "H2O3_GLM_EXACT_GRAD": "0", "H2O3_GLM_TIERS": "0"}
_LEGACY_BF3 = {"H2O3_GLM_BF3": "1", "H2O3_GLM_EXACT_GRAD": "0", "H2O3_GLM_TIERS": "0"}


@pytest.mark.parametrize("noise,tier", [(1e-3, "f64"), (2e-2, "f32"), (0.1, "bf3"), (None, "bf16")])
def test_glm_conditioning_tiers_match_fp64(monkeypatch, noise, tier):
    """Newton on the exact gradient channel with the Hessian precision tier
    picked from the scaled condition number: a well-conditioned design runs
    on the one-MFMA bf16 Hessian (kappa < 32), two columns at correlation
    ~0.995 (kappa ~ 400) on bf16x3, at 1 - 2e-4 (kappa ~ 1e4) move to the
    f32 Hessian, correlation 1 - 5e-7 (kappa >= 1e6) to fp64.  Every tier
    lands on the fp64 IRLS solution; at kappa >= 1e6 the legacy paths (Gram
    right-hand side, no tiers) are off by orders of magnitude more."""
    import numpy as np
    g = np.random.default_rng(5)
    n, P = 400_000, 100
    Xh = g.standard_normal((n, P)).astype(np.float32)
    if noise is not None:
        Xh[:, 1] = Xh[:, 0] + noise * g.standard_normal(n).astype(np.float32)
    b = np.zeros(P)
    b[:10] = g.standard_normal(10)
    b[0], b[1] = 1.0, -0.5
    y = (g.random(n) < 1 / (1 + np.exp(-(Xh.astype(np.float64) @ b)))).astype(int)
    modes = {"default": _DEFAULT}
    if tier == "f64":
        modes.update({"f32": _LEGACY_F32, "bf3_rhs": _LEGACY_BF3})
    res, drvs = _glm_fit_modes(Xh, y, modes, monkeypatch)
    drv = drvs["default"]
    assert drv._hprec == tier, (drv._hprec, drv.hessian_kappa)
    Xs = drv.X[:, :P].float()
    ref, G = _fp64_irls(Xs, drv.y, drv._init_beta)
    ref = ref.cpu().numpy()
    ev = torch.linalg.eigvalsh((G[:P, :P] / n).cpu())
    kappa = (ev.max() / ev.min()).item()
    if tier == "f64":
        assert kappa >= 1e6
    scale = np.abs(ref).max()
    err = {k: np.abs(v - ref).max() / scale for k, v in res.items()}
    assert err["default"] < 1e-6, (err, kappa)
    if tier == "f64":
        assert err["f32"] > 100 * err["default"] and err["bf3_rhs"] > 100 * err["default"], err


def test_glm_gaussian_reduced_tier_refines_to_fp64(monkeypatch):
    """Gaussian / identity on the one-MFMA bf16 Hessian tier: the one-step
    convergence shortcut only holds for an exact Hessian, so the driver keeps
    stepping on the exact-gradient channel until the coefficients are those of
    the fp64 least-squares solution (the bf16 step alone is ~kappa * 2^-8 off)."""
    import numpy as np
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.core.frame import H2OFrame
    from h2o3_amd.models.glm.glm import GLMDriver, H2OGeneralizedLinearEstimator
    for k, v in _DEFAULT.items():
        monkeypatch.setenv(k, v)
    g = np.random.default_rng(11)
    n, P = 300_000, 100
    Xh = g.standard_normal((n, P)).astype(np.float32)
    b = g.standard_normal(P)
    y = Xh.astype(np.float64) @ b + 0.3 * g.standard_normal(n)
    cols = {f"x{j}": Xh[:, j] for j in range(P)}
    cols["y"] = y
    fr = H2OFrame(cols)
    est = H2OGeneralizedLinearEstimator(family="gaussian", solver="IRLSM", lambda_=0.0)
    spec = TrainSpec(fr, [f"x{j}" for j in range(P)], "y")
    est._spec = spec
    drv = GLMDriver(est, spec)
    assert drv.X.is_cuda
    for _ in range(30):
        drv.step()
        if drv.converged:
            break
    assert drv.converged
    assert drv._hprec == "bf16", drv._hprec
    assert drv.iter > 1
    Xa = torch.cat([drv.X[:, :P].double(), torch.ones(n, 1, dtype=torch.float64, device=drv.X.device)], 1)
    yd = drv.y.double().view(-1, 1)
    ref = torch.linalg.lstsq(Xa.cpu(), yd.cpu()).solution.view(-1).numpy()
    err = np.abs(drv.beta - ref).max() / np.abs(ref).max()
    assert err < 1e-6, err


@pytest.mark.parametrize("noise,tier,P", [(None, "bf16", 600), (0.1, "bf3", 600), (2e-2, "f64", 600),
                                          (None, "bf16", 200), (0.1, "bf3", 200)])
def test_glm_wide_tiers_match_fp64(monkeypatch, noise, tier, P):
    """Wide design (P = 600: the fused wide pass -- eta kernel + hand-written
    Gram): a well-conditioned design runs on the one-MFMA bf16 Hessian
    (kappa < 32), a correlated pair (kappa ~ 400) on bf16x3, a
    strongly correlated one (kappa ~ 1e4) on fp64 (the wide path has no f32
    tier).  Every tier lands on the fp64 IRLS solution."""
    import numpy as np
    g = np.random.default_rng(8)
    n = 120_000
    if P < 512:
        # a mid-width design forced onto the wide path
        monkeypatch.setenv("H2O3_GLM_NARROW_MAX", "128")
    Xh = g.standard_normal((n, P)).astype(np.float32)
    if noise is not None:
        Xh[:, 1] = Xh[:, 0] + noise * g.standard_normal(n).astype(np.float32)
    b = np.zeros(P)
    b[:12] = 0.4 * g.standard_normal(12)
    y = (g.random(n) < 1 / (1 + np.exp(-(Xh.astype(np.float64) @ b)))).astype(int)
    res, drvs = _glm_fit_modes(Xh, y, {"default": _DEFAULT}, monkeypatch, iters=12)
    drv = drvs["default"]
    assert drv._hprec == tier, (drv._hprec, drv.hessian_kappa)
    Xs = drv.X[:, :P].float()
    ref, _ = _fp64_irls(Xs, drv.y, drv._init_beta)
    ref = ref.cpu().numpy()
    err = np.abs(res["default"] - ref).max() / np.abs(ref).max()
    assert err < 1e-6, (err, drv.hessian_kappa)


def test_gram_aug_bf3_matches_fp64():
    n, P = 30_011, 700
    g = torch.Generator().manual_seed(4)
    X = torch.randn(n, P, generator=g)
    W = torch.rand(n, generator=g)
    z = torch.randn(n, generator=g)
    G = linalg_ops.gram_aug_bf3(X.cuda(), W.cuda(), z.cuda(), P, step=8192).cpu()
    A = torch.cat([X.double(), torch.ones(n, 1, dtype=torch.float64), z.double().view(-1, 1)], 1)
    R = A.T @ (A * W.double().view(-1, 1))
    diag = R.diagonal().sqrt()
    rel = (G[: P + 2, : P + 2] - R).abs() / (diag.view(-1, 1) * diag.view(1, -1))
    assert rel.max().item() < 5e-5


@pytest.mark.gpu
def test_group_sum_matches_index_add():
    """One-hot GEMM grouped sums (core/groupsum.py) equal the f64 index_add_
    reference for few bins, and the large-bin fallback is index_add_ itself."""
    import torch
    from h2o3_amd.core.groupsum import group_sum
    g = torch.Generator(device="cuda").manual_seed(1)
    for nb in (2, 7, 300, 5000):
        idx = torch.randint(0, nb, (1_000_003,), generator=g, device="cuda")
        v = torch.randn((1_000_003, 3), generator=g, device="cuda", dtype=torch.float64)
        ref = torch.zeros((nb, 3), dtype=torch.float64, device="cuda").index_add_(0, idx, v)
        torch.testing.assert_close(group_sum(idx, v, nb), ref, rtol=1e-10, atol=1e-9)
        torch.testing.assert_close(group_sum(idx, v[:, 1], nb), ref[:, 1], rtol=1e-10, atol=1e-9)


@pytest.mark.gpu
def test_wide_split_gemm_overlap_matches_sequential(monkeypatch):
    """Double-buffered split / GEMM pipeline (side stream for the split
    kernels) gives exactly the sequential pass's Gram and deviance."""
    n, P = 50_021, 300
    g = torch.Generator().manual_seed(9)
    X = torch.randn(n, P, generator=g).cuda()
    beta = (0.05 * torch.randn(P, generator=g)).cuda()
    y = (torch.rand(n, generator=g) < 0.4).float().cuda()
    codes = linalg_ops.glm_fused_codes("binomial", "logit")
    W = torch.rand(n, generator=g).cuda()
    monkeypatch.setattr(linalg_ops, "_WIDE_GROUP", 2)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("H2O3_WIDE_OVERLAP", mode)
        G, d, gx = linalg_ops.glm_wide_irls(X, P, beta, 0.1, y, None, None, codes, step=4096)
        Ga = linalg_ops.gram_aug_bf3(X, W, y, P, step=4096)
        torch.cuda.synchronize()
        out[mode] = (G.cpu(), d.cpu(), Ga.cpu(), gx.cpu())
    for a, b in zip(out["0"], out["1"]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("tile,bf3", [(256, True), (128, True), (256, False)])
@pytest.mark.parametrize("n,P", [(100, 1000), (200_003, 1000), (70_001, 127), (5_000, 255), (9_000, 300)])
def test_glm_wide_fused_gram_matches_fp64(n, P, tile, bf3, monkeypatch):
    """glm_wide_gram_kernel alone: [X | 1]' W [X | 1] from the f32 rows vs
    fp64, at widths that fill 8 column tiles (P = 1000, the BASELINE wide
    config's width), exactly one tile with and without the intercept spilling
    into a second (127 / 128), with fewer chunks than slices (n = 100) and a
    ragged last chunk; both tile sizes (256: the default, diagonal tiles
    skip their lower-left quarter); the one-MFMA bf16 tier (64-row chunks)
    to bf16 rounding (~2^-9 per product)."""
    monkeypatch.setenv("H2O3_WIDE_TILE", str(tile))
    g = torch.Generator().manual_seed(n + P)
    X = torch.randn(n, P, generator=g)
    X[:, :3] *= 40.0                                # columns of very different scale
    beta = 0.02 * torch.randn(P, generator=g)
    y = (torch.rand(n, generator=g) < 0.4).float()
    codes = linalg_ops.glm_fused_codes("binomial", "logit")
    G, _, _ = linalg_ops.glm_wide_irls(X.cuda(), P, beta.cuda(), 0.1, y.cuda(), None, None, codes, step=1 << 16,
                                       fused=True, bf3=bf3)
    eta = X.double() @ beta.double() + 0.1
    mu = torch.sigmoid(eta)
    W = mu * (1 - mu)
    Xa = torch.cat([X.double(), torch.ones(n, 1, dtype=torch.float64)], 1)
    ref = Xa.T @ (Xa * W.view(-1, 1))
    A = G[:P + 1, :P + 1].cpu()
    d = ref.diagonal().sqrt()
    rel = (A - ref).abs() / (d.view(-1, 1) * d.view(1, -1))
    assert rel.max().item() < (3e-5 if bf3 else 8e-3), rel.max().item()
    assert torch.equal(A, A.T)
    assert float(G[P + 1].abs().sum()) == 0.0


@pytest.mark.parametrize("noise", [None, 0.1])
def test_glm_wide_device_solve_matches_host(monkeypatch, noise):
    """P = 600 (wide): the IRLS system conditioned (Hager 1-norm estimate on
    a device Cholesky) and solved on the device gives the same tier, kappa
    and coefficients as the host LAPACK path (H2O3_GLM_DEV_SOLVE=0)."""
    import numpy as np
    g = np.random.default_rng(9)
    n, P = 60_000, 600
    Xh = g.standard_normal((n, P)).astype(np.float32)
    if noise is not None:
        Xh[:, 1] = Xh[:, 0] + noise * g.standard_normal(n).astype(np.float32)
    b = np.zeros(P)
    b[:10] = 0.4 * g.standard_normal(10)
    y = (g.random(n) < 1 / (1 + np.exp(-(Xh.astype(np.float64) @ b)))).astype(int)
    res, drvs = _glm_fit_modes(Xh, y, {"host": dict(_DEFAULT, H2O3_GLM_DEV_SOLVE="0"),
                                       "dev": dict(_DEFAULT, H2O3_GLM_DEV_SOLVE="1")}, monkeypatch, iters=8)
    assert drvs["dev"]._dev_system_ok()
    assert drvs["dev"]._hprec == drvs["host"]._hprec
    assert drvs["dev"].hessian_kappa == pytest.approx(drvs["host"].hessian_kappa, rel=1e-6)
    err = np.abs(res["dev"] - res["host"]).max() / np.abs(res["host"]).max()
    assert err < 1e-9, err


def test_glm_wide_l1_device_tier_check_matches_host(monkeypatch):
    """P = 600, elastic net (alpha 0.5, lambda > 0: the host coordinate-descent
    solve): the condition estimate runs on the device statistics before they
    cross to the host; same tier, kappa and coefficients as the all-host
    path (H2O3_GLM_DEV_SOLVE=0)."""
    import numpy as np
    g = np.random.default_rng(12)
    n, P = 60_000, 600
    Xh = g.standard_normal((n, P)).astype(np.float32)
    b = np.zeros(P)
    b[:10] = 0.5 * g.standard_normal(10)
    y = (g.random(n) < 1 / (1 + np.exp(-(Xh.astype(np.float64) @ b)))).astype(int)
    kw = dict(family="binomial", solver="IRLSM", alpha=0.5, lambda_=1e-3)
    res, drvs = _glm_fit_modes(Xh, y, {"host": dict(_DEFAULT, H2O3_GLM_DEV_SOLVE="0"),
                                       "dev": dict(_DEFAULT, H2O3_GLM_DEV_SOLVE="1")}, monkeypatch, iters=8,
                               est_kw=kw)
    d = drvs["dev"]
    assert d._dev_tier_ok() and not d._dev_system_ok()
    assert d._hprec == drvs["host"]._hprec
    assert d.hessian_kappa == pytest.approx(drvs["host"].hessian_kappa, rel=1e-6)
    err = np.abs(res["dev"] - res["host"]).max() / np.abs(res["host"]).max()
    assert err < 1e-9, err
    assert np.count_nonzero(res["dev"][:P]) < P                  # the l1 penalty is active


@pytest.mark.parametrize("family", ["binomial", "poisson", "gaussian"])
def test_glm_wide_lambda_max_and_deviance_kernel_match_torch(family, monkeypatch):
    """P = 600: lambda_max (X'r at the intercept-only model) and the
    deviance at a coefficient vector from the wide eta kernel agree with the
    torch f64 paths (f32 products inside the kernel)."""
    import numpy as np
    from h2o3_amd.models.base import TrainSpec
    from h2o3_amd.core.frame import H2OFrame
    from h2o3_amd.models.glm.glm import GLMDriver, H2OGeneralizedLinearEstimator
    g = np.random.default_rng(21)
    n, P = 40_000, 600
    Xh = g.standard_normal((n, P)).astype(np.float32)
    eta = Xh[:, :5].astype(np.float64) @ (0.3 * g.standard_normal(5))
    if family == "binomial":
        y = (g.random(n) < 1 / (1 + np.exp(-eta))).astype(int)
    elif family == "poisson":
        y = g.poisson(np.exp(0.5 * eta)).astype(float)
    else:
        y = eta + g.standard_normal(n)
    cols = {f"x{j}": Xh[:, j] for j in range(P)}
    cols["y"] = y
    fr = H2OFrame(cols)
    if family == "binomial":
        fr["y"] = fr["y"].asfactor()
    est = H2OGeneralizedLinearEstimator(family=family, solver="IRLSM", alpha=0.5, lambda_search=True)
    spec = TrainSpec(fr, [f"x{j}" for j in range(P)], "y")
    est._spec = spec
    drv = GLMDriver(est, spec)
    assert drv._wide_eta_codes() is not None
    beta = np.concatenate([0.01 * g.standard_normal(P), [0.1]])
    lm_k, dv_k = drv._lambda_max(), drv.deviance(beta)
    monkeypatch.setattr(GLMDriver, "_wide_eta_codes", lambda self: None)
    lm_t, dv_t = drv._lambda_max(), drv.deviance(beta)
    assert lm_k == pytest.approx(lm_t, rel=1e-5)
    assert dv_k == pytest.approx(dv_t, rel=1e-5)


@pytest.mark.parametrize("method", ["Randomized", "Power", "GramSVD"])
def test_pca_methods_on_gram_kernel_match_fp64(method):
    """PCA Power / Randomized iterate on the covariance from ONE pass of the
    hand-written Gram kernel (no per-iteration pass over X, no library GEMM),
    and the projections run on the skinny MFMA kernel (cluster_ops.xv): the
    eigenvalues / eigenvectors match an fp64 eigendecomposition and the
    projections an fp64 product."""
    import numpy as np
    import h2o3_amd
    from h2o3_amd.core.frame import H2OFrame
    from h2o3_amd.models.clustering import H2OPrincipalComponentAnalysisEstimator
    from h2o3_amd.ops import _native, cluster_ops
    h2o3_amd.init(verbose=False)
    g = np.random.default_rng(3)
    n, P, k = 300_000, 100, 10
    # well-separated top-k spectrum (variance ratio 0.72 between neighbours and
    # between the k-th and the bulk) so Power's per-vector iterations converge
    # within max_iterations, as they would for the reference's PowerSVD
    scales = np.concatenate([3.0 * 0.85 ** np.arange(k + 1), np.linspace(0.5, 0.2, P - k - 1)])
    Xh = (g.standard_normal((n, P)) * scales).astype(np.float32)
    fr = H2OFrame({f"x{j}": Xh[:, j] for j in range(P)})
    m = H2OPrincipalComponentAnalysisEstimator(k=k, pca_method=method, transform="NONE", max_iterations=300, seed=1)
    m.train(training_frame=fr)
    Xd = torch.as_tensor(Xh, dtype=torch.float64)
    mu = Xd.mean(0)
    cov = (Xd - mu).T @ (Xd - mu) / (n - 1)
    ev, V = torch.linalg.eigh(cov)
    order = torch.argsort(ev, descending=True)[:k]
    ev, V = ev[order], V[:, order]
    sd = np.asarray(m._output["std_deviation"])
    np.testing.assert_allclose(sd, np.sqrt(ev.numpy()), rtol=1e-6)
    E = np.asarray(m._output["eigenvectors"])
    # eigenvectors up to sign
    cosv = np.abs((E * V.numpy()).sum(0))
    assert cosv.min() > 1 - 1e-6, cosv
    Z = m.predict(fr).as_data_frame().values
    Zref = ((Xd - mu) @ torch.as_tensor(E)).numpy()
    np.testing.assert_allclose(Z, Zref, rtol=1e-4, atol=1e-4 * np.abs(Zref).max())
    assert "libkmeans.so" in " ".join(_native.loaded_libs()) and "libgram.so" in " ".join(_native.loaded_libs())


def test_xv_kernel_matches_fp64():
    from h2o3_amd.ops import cluster_ops
    g = torch.Generator(device="cuda").manual_seed(4)
    for N, W, k in ((100_003, 100, 10), (70_000, 36, 40), (65_536, 256, 3), (80_000, 8, 17)):
        X = torch.randn((N, W), generator=g, device="cuda")
        V = torch.randn((W, k), generator=g, device="cuda", dtype=torch.float64)
        out = cluster_ops.xv(X, V)
        assert out.dtype == torch.float32 and out.shape == (N, k)
        ref = X.double() @ V
        torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-4 * float(ref.abs().max()))


@pytest.mark.parametrize("N,P,ldx", [(100_003, 5, 8), (65_536, 63, 64), (50_000, 64, 96), (40_000, 130, 130),
                                     (10, 3, 3)])
def test_gram_f64_aug_matches_fp64(N, P, ldx):
    """gram_f64_kernel (f64 MFMA) against torch fp64 on [X | 1]: exact f64
    products, so only summation order differs."""
    from h2o3_amd.ops import linalg_ops
    g = torch.Generator(device="cuda").manual_seed(P)
    Xs = torch.randn((N, ldx), generator=g, device="cuda")
    Xs[:, :P:3] = (Xs[:, :P:3] > 0.3).float()          # 0/1 rule-like columns
    W = torch.rand(N, generator=g, device="cuda", dtype=torch.float64)
    W[::11] = 0.0
    G = linalg_ops.gram_f64_aug(Xs, P, W)
    Xa = torch.cat([Xs[:, :P].double(), torch.ones((N, 1), dtype=torch.float64, device="cuda")], 1)
    ref = (Xa * W.view(-1, 1)).T @ Xa
    torch.testing.assert_close(G, ref, rtol=1e-12, atol=1e-9)
    # a row slice (the GLM passes chunks of a larger matrix)
    G2 = linalg_ops.gram_f64_aug(Xs[7:N // 2], P, W[7:N // 2])
    ref2 = (Xa[7:N // 2] * W[7:N // 2].view(-1, 1)).T @ Xa[7:N // 2]
    torch.testing.assert_close(G2, ref2, rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("N,P,ldx", [(100_003, 5, 8), (70_000, 300, 320), (3, 2, 2)])
def test_xv_xtr_f64_match_fp64(N, P, ldx):
    from h2o3_amd.ops import linalg_ops
    g = torch.Generator(device="cuda").manual_seed(N % 97)
    X = torch.randn((N, ldx), generator=g, device="cuda")
    b = torch.randn(P, generator=g, device="cuda", dtype=torch.float64)
    r = torch.randn(N, generator=g, device="cuda", dtype=torch.float64)
    Xd = X[:, :P].double()
    torch.testing.assert_close(linalg_ops.xv_f64(X, P, b, 0.25), Xd @ b + 0.25, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(linalg_ops.xtr_f64(X, P, r), Xd.T @ r, rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("n,p,q", [(100_003, 10, 3), (50_000, 7, 0), (30_000, 300, 2), (1000, 4, 4)])
def test_tmm_matches_matmul(n, p, q):
    from h2o3_amd.ops import linalg_ops
    g = torch.Generator(device="cuda").manual_seed(n % 13)
    A = torch.randn((n, p), generator=g, device="cuda", dtype=torch.float64)
    B = torch.randn((n, q), generator=g, device="cuda", dtype=torch.float64) if q else \
        torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    torch.testing.assert_close(linalg_ops.tmm(A, B), A.T @ B, rtol=1e-10, atol=1e-9)
