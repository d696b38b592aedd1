"""ops/csrc/metrics.hip logit sketch against the torch fp64 reference
(index_add over the same bins, masked sums), and binomial_metrics through
the kernel against the torch path."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(y, p, w, nb):
    from h2o3_amd.models import metrics as mm
    ok = ~torch.isnan(y) & ~torch.isnan(p)
    y, p = y[ok].double(), p[ok].double()
    w = torch.ones_like(y) if w is None else w[ok].double()
    b = mm._logit_bins(p, nb)
    H = torch.zeros(2 * nb, dtype=torch.float64, device=p.device)
    H.index_add_(0, b + nb * (1 - y).long(), w)
    pc = p.clamp(1e-15, 1 - 1e-15)
    s = torch.stack([w.sum(), -(w * (y * pc.log() + (1 - y) * (1 - pc).log())).sum(), (w * (y - p) ** 2).sum(),
                     (w * y).sum(), torch.tensor(float(y.numel()), dtype=torch.float64, device=p.device)])
    return torch.cat([H, s])


@pytest.mark.parametrize("kind", ["random", "constant", "few", "weighted_nan"])
def test_logit_hist_matches_torch(kind):
    from h2o3_amd.ops import metrics_ops
    assert metrics_ops.available(torch.zeros(1, device="cuda")), "libmetrics.so must load on a GPU box"
    g = torch.Generator(device="cuda").manual_seed(3)
    n, nb = 300_001, 1 << 18
    y = (torch.rand(n, generator=g, device="cuda") < 0.3).double()
    if kind == "constant":
        p = torch.full((n,), 0.31, dtype=torch.float64, device="cuda")
    elif kind == "few":
        p = torch.sigmoid(torch.randint(-3, 4, (n,), generator=g, device="cuda").double())
    else:
        p = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
    w = None
    if kind == "weighted_nan":
        w = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
        p[::97] = float("nan")
        y[5::101] = float("nan")
    got = metrics_ops.logit_hist(y, p, w, nb)
    ref = _ref(y, p, w, nb)
    # atomic summation order differs: compare per bin with a relative tolerance
    torch.testing.assert_close(got, ref, rtol=1e-10, atol=1e-9)


def test_binomial_metrics_kernel_vs_torch(monkeypatch):
    from h2o3_amd.models import metrics as mm
    from h2o3_amd.ops import metrics_ops
    g = torch.Generator(device="cuda").manual_seed(5)
    n = 200_000
    x = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    y = (torch.rand(n, generator=g, device="cuda", dtype=torch.float64) < torch.sigmoid(2 * x)).double()
    p = torch.sigmoid(1.7 * x).float()
    a = mm.binomial_metrics(y, p)
    monkeypatch.setattr(metrics_ops, "available", lambda t: False)
    b = mm.binomial_metrics(y, p)
    for k in ("AUC", "pr_auc", "logloss", "MSE", "max_f1_threshold"):
        assert abs(a._m[k] - b._m[k]) < 1e-9, (k, a._m[k], b._m[k])


@pytest.mark.parametrize("n,nbins,C,kind", [(500_001, 1, 1, "const"), (500_001, 3, 4, "few"), (300_000, 2000, 4, "many"),
                                            (200_000, 50_000, 1, "many"), (100_000, 7, 300, "few"),
                                            (1000, 5, 2, "oob")])
def test_group_sum_matches_index_add(n, nbins, C, kind):
    from h2o3_amd.core.groupsum import index_add
    from h2o3_amd.ops import metrics_ops
    g = torch.Generator(device="cuda").manual_seed(11)
    if kind == "const":
        idx = torch.zeros(n, dtype=torch.int64, device="cuda")
    else:
        idx = torch.randint(0, nbins, (n,), generator=g, device="cuda")
    v = torch.randn((n, C), generator=g, device="cuda", dtype=torch.float64)
    ref = torch.zeros((nbins, C), dtype=torch.float64, device="cuda")
    if kind == "oob":
        # rows outside [0, nbins) are skipped by the kernel
        bad = torch.arange(n, device="cuda") % 7 == 0
        idx2 = torch.where(bad, torch.full_like(idx, nbins + 3), idx)
        idx2[1::14] = -1
        keep = (idx2 >= 0) & (idx2 < nbins)
        ref.index_add_(0, idx2[keep], v[keep])
        got = metrics_ops.group_sum(idx2, v, nbins)
    else:
        # the reference sum on the host (torch's device f64 index_add_ is
        # the contended path this kernel replaces)
        ref = torch.zeros((nbins, C), dtype=torch.float64).index_add_(0, idx.cpu(), v.cpu()).cuda()
        got = metrics_ops.group_sum(idx, v, nbins)
        out = torch.ones((nbins, C), dtype=torch.float64, device="cuda")
        index_add(out, idx, v if C > 1 else v.view(-1))
        torch.testing.assert_close(out, ref + 1, rtol=1e-9, atol=1e-8)
    torch.testing.assert_close(got, ref, rtol=1e-9, atol=1e-8)


@pytest.mark.parametrize("n,nbins,C", [(400_000, 1, 1), (400_000, 5, 3), (200_000, 30_000, 2)])
@pytest.mark.parametrize("op", ["min", "max"])
def test_group_extreme_matches_host(n, nbins, C, op):
    from h2o3_amd.core.groupsum import group_extreme
    g = torch.Generator(device="cuda").manual_seed(13)
    idx = torch.randint(0, nbins, (n,), generator=g, device="cuda")
    v = torch.randn((n, C), generator=g, device="cuda", dtype=torch.float64)
    fill = float("inf") if op == "min" else float("-inf")
    ref = torch.full((nbins, C), fill, dtype=torch.float64).scatter_reduce_(
        0, idx.cpu().view(-1, 1).expand(-1, C), v.cpu(), reduce="amin" if op == "min" else "amax")
    got = group_extreme(idx, v, nbins, op)
    assert torch.equal(got.cpu(), ref)
