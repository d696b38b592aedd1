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
