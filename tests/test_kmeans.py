"""K-Means: reference semantics (hex/kmeans/KMeans.java) on CPU and the fused
HIP Lloyd kernel (ops/csrc/kmeans.hip) against a float64 torch reference on
the GPU."""
import math
import os

import numpy as np
import pandas as pd
import pytest
import torch

import h2o3_amd
from h2o3_amd.estimators import H2OKMeansEstimator
from h2o3_amd.ops import cluster_ops


def _blobs(n=300, seed=0):
    rng = np.random.RandomState(seed)
    cs = np.array([[0, 0], [8, 8], [-8, 8], [8, -8]])
    X = np.concatenate([c + rng.randn(n, 2) for c in cs])
    return X, cs


def _ref_distance(center, point, is_cat):
    """GenModel.KMeans_distance: squared euclidean on numerics, 0/1 mismatch
    on categoricals."""
    d = 0.0
    for c, x, cat in zip(center, point, is_cat):
        d += (1.0 if c != x else 0.0) if cat else (x - c) ** 2
    return d


def test_categorical_mismatch_distance_matches_reference():
    rng = np.random.RandomState(3)
    n = 400
    df = pd.DataFrame({"a": rng.randn(n), "b": rng.randn(n) * 3,
                       "c": rng.choice(["u", "v", "w"], n), "d": rng.choice(["p", "q"], n)})
    fr = h2o3_amd.H2OFrame(df)
    m = H2OKMeansEstimator(k=3, standardize=False, seed=7, max_iterations=20)
    m.train(training_frame=fr)
    cen = m.centers()
    # reference distances from the raw centers (cats as labels), row-wise closest
    pts = df[["c", "d", "a", "b"]].values.tolist()   # DataInfo order: categoricals first
    names = m._dinfo.x
    order = [names.index(c) for c in ["c", "d", "a", "b"]]
    cen_o = [[row[i] for i in order] for row in cen]
    is_cat = [True, True, False, False]
    ref = np.array([int(np.argmin([_ref_distance(c, p, is_cat) for c in cen_o])) for p in pts])
    got = m.predict(fr).as_data_frame()["predict"].values
    assert (ref == got).mean() > 0.995
    # categorical centers are the per-cluster modes
    for j in range(3):
        sel = df[got == j]
        if len(sel):
            assert cen_o[j][0] == sel["c"].mode().iloc[0] or (sel["c"] == cen_o[j][0]).sum() == sel["c"].value_counts().max()


def test_within_ss_and_totss_reference_definitions():
    X, _ = _blobs()
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=["a", "b"]))
    m = H2OKMeansEstimator(k=4, standardize=True, seed=1)
    m.train(training_frame=fr)
    Z = (X - X.mean(0)) / X.std(0, ddof=1)
    C = np.array(m.centers_std())
    a = ((Z[:, None, :] - C[None]) ** 2).sum(2).argmin(1)
    within = np.array([((Z[a == j] - C[j]) ** 2).sum() for j in range(4)])
    np.testing.assert_allclose(m.withinss(), within, rtol=1e-4)
    np.testing.assert_allclose(m.totss(), (Z ** 2).sum(), rtol=1e-5)
    np.testing.assert_allclose(m.betweenss(), m.totss() - m.tot_withinss(), rtol=1e-9)
    assert sum(m.size()) == len(X)


def test_estimate_k_finds_the_blobs():
    # cutoff = min(0.02 + 10/rows + 2.5/ncols^2, 0.8): 8 columns -> ~0.07
    rng = np.random.RandomState(2)
    cs = rng.randn(4, 8) * 10
    X = np.concatenate([c + rng.randn(300, 8) for c in cs])
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=[f"x{i}" for i in range(8)]))
    m = H2OKMeansEstimator(k=10, estimate_k=True, standardize=False, max_iterations=50)
    m.train(training_frame=fr)
    assert len(m.centers()) == 4
    got = np.array(sorted(map(tuple, np.round(np.array(m.centers()), 0))))
    assert np.abs(got - np.array(sorted(map(tuple, np.round(cs, 0))))).max() <= 1.0


@pytest.mark.parametrize("init", ["Random", "PlusPlus", "Furthest"])
def test_init_modes(init):
    X, cs = _blobs(seed=4)
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=["a", "b"]))
    m = H2OKMeansEstimator(k=4, init=init, standardize=False, seed=11, max_iterations=50)
    m.train(training_frame=fr)
    assert m.tot_withinss() < 0.05 * m.totss()
    assert m.num_iterations() >= 1
    hist = m.scoring_history()
    assert hist[-1]["number_of_reassigned_observations"] < max(1, len(X) * 1e-4) or len(hist) == 50


def test_user_points_and_convergence_rule():
    X, cs = _blobs(seed=5)
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=["a", "b"]))
    up = h2o3_amd.H2OFrame(pd.DataFrame(cs + 0.5, columns=["a", "b"]))
    m = H2OKMeansEstimator(k=4, user_points=up, standardize=False, max_iterations=100)
    m.train(training_frame=fr)
    np.testing.assert_allclose(np.array(m.centers()), np.array([X[i * 300:(i + 1) * 300].mean(0) for i in range(4)]),
                               atol=1e-6)
    # first pass: every row is "reassigned" (assignment starts at -1)
    assert m.scoring_history()[0]["number_of_reassigned_observations"] == len(X)


def test_empty_cluster_reseeded_at_worst_row():
    X, _ = _blobs(seed=6)
    X = np.concatenate([X, [[60.0, 60.0]]])
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=["a", "b"]))
    # two identical user points: one cluster goes empty on the first pass
    up = h2o3_amd.H2OFrame(pd.DataFrame([[0.0, 0.0], [0.0, 0.0], [8, 8], [-8, 8], [8, -8]], columns=["a", "b"]))
    m = H2OKMeansEstimator(k=5, user_points=up, standardize=False, max_iterations=30)
    m.train(training_frame=fr)
    assert min(m.size()) >= 1
    assert any(np.allclose(c, [60.0, 60.0]) for c in m.centers())


def test_cluster_size_constraints():
    rng = np.random.RandomState(8)
    X = np.concatenate([rng.randn(90, 2), rng.randn(10, 2) + 6])
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=["a", "b"]))
    m = H2OKMeansEstimator(k=2, cluster_size_constraints=[40, 40], standardize=False, seed=3, max_iterations=10)
    m.train(training_frame=fr)
    a = m._constrained_assign
    assert np.bincount(a, minlength=2).min() >= 40


def test_lloyd_pass_torch_matches_numpy():
    rng = np.random.RandomState(9)
    X = torch.tensor(rng.randn(5000, 12), dtype=torch.float32)
    C = X[:7].clone().double()
    w = torch.tensor(rng.rand(5000), dtype=torch.float32)
    a = torch.full((5000,), -1, dtype=torch.int32)
    st = cluster_ops.lloyd_pass(X, C, w, a)
    Xn, Cn, wn = X.double().numpy(), C.numpy(), w.double().numpy()
    d = ((Xn[:, None] - Cn[None]) ** 2).sum(2)
    ref = d.argmin(1)
    assert (a.numpy() == ref).mean() > 0.999
    sums = np.zeros((7, 12))
    np.add.at(sums, ref, Xn * wn[:, None])
    np.testing.assert_allclose(st.sums.numpy(), sums, rtol=1e-4, atol=1e-3)
    assert st.changed == 5000


def test_kmeans_two_rank_equals_one(tmp_path):
    """Row-sharded Lloyd (gloo, 2 ranks): same centers as one rank with the
    same user points (one all-reduce per iteration)."""
    import subprocess
    import sys
    import os
    X, cs = _blobs(seed=12)
    np.save(tmp_path / "X.npy", X)
    script = tmp_path / "w.py"
    script.write_text(f"""
import sys, json, numpy as np, pandas as pd
sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
import h2o3_amd
from h2o3_amd.estimators import H2OKMeansEstimator
from h2o3_amd.parallel import cloud
h2o3_amd.init(verbose=False)
X = np.load({repr(str(tmp_path / 'X.npy'))})
fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=['a', 'b']))
up = h2o3_amd.H2OFrame(pd.DataFrame({cs.tolist()!r}, columns=['a', 'b']) + 0.3)
m = H2OKMeansEstimator(k=4, user_points=up, standardize=True, max_iterations=20)
m.train(training_frame=fr)
if cloud.rank() == 0:
    print('RES', json.dumps({{'c': m.centers(), 'w': m.tot_withinss()}}))
""")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0", CUDA_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr", "127.0.0.1", "--master-port", "29631", str(script)],
                         capture_output=True, text=True, env=env, timeout=300)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("RES")]
    assert line, out.stderr[-3000:]
    import json
    r2 = json.loads(line[0][4:])
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=["a", "b"]))
    up = h2o3_amd.H2OFrame(pd.DataFrame(cs, columns=["a", "b"]) + 0.3)
    m = H2OKMeansEstimator(k=4, user_points=up, standardize=True, max_iterations=20)
    m.train(training_frame=fr)
    np.testing.assert_allclose(np.array(r2["c"]), np.array(m.centers()), rtol=1e-6, atol=1e-8)
    assert math.isclose(r2["w"], m.tot_withinss(), rel_tol=1e-6)


# ---------------------------------------------------------------- GPU kernel
@pytest.mark.gpu
@pytest.mark.parametrize("fx", [False, True])
@pytest.mark.parametrize("N,P,k", [(100_003, 12, 5), (70_001, 100, 40), (33_333, 256, 16), (20_000, 36, 130),
                                   (65, 4, 1)])
def test_lloyd_kernel_matches_f64_reference(N, P, k, fx):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from h2o3_amd.ops import _native
    g = torch.Generator(device="cuda").manual_seed(N + P + k)
    X = torch.randn((N, P), generator=g, device="cuda")
    C = X[torch.randperm(N, generator=g, device="cuda")[:k]].double() + 0.01
    w = torch.rand(N, generator=g, device="cuda")
    w[::7] = 0
    a = torch.full((N,), -1, dtype=torch.int32, device="cuda")
    dmin = torch.empty(N, dtype=torch.float32, device="cuda")
    assert cluster_ops.native_ok(X, k)
    xa = cluster_ops.abs_bound(X, w) if fx else None
    st = cluster_ops.lloyd_pass(X, C, w, a, dmin=dmin, xabs_max=xa)
    assert "libkmeans.so" in " ".join(_native.loaded_libs())
    torch.cuda.synchronize()
    Xd = X.double()
    D = (Xd * Xd).sum(1, keepdim=True) - 2 * Xd @ C.T + (C * C).sum(1).view(1, -1)
    ref = D.argmin(1)
    if k > 1:
        gap = D.topk(2, dim=1, largest=False).values
        clear = (gap[:, 1] - gap[:, 0]) > 1e-3 * (1 + gap[:, 0].abs())
    else:
        clear = torch.ones(N, dtype=torch.bool, device="cuda")
    got = a.long()
    assert bool((got[clear] == ref[clear]).all())
    assert float(st.changed) == N
    # statistics from the kernel's own assignment, in f64
    oh = torch.zeros((N, k), dtype=torch.float64, device="cuda")
    oh[torch.arange(N, device="cuda"), got] = w.double()
    sums = oh.T @ Xd
    torch.testing.assert_close(st.sums, sums, rtol=2e-5, atol=2e-3)
    torch.testing.assert_close(st.weights, oh.sum(0), rtol=1e-5, atol=1e-3)
    dsel = D.gather(1, got.view(-1, 1)).view(-1).clamp_min(0)
    torch.testing.assert_close(dmin.double(), dsel, rtol=1e-4, atol=1e-3 * P)
    torch.testing.assert_close(st.withinss, (oh * dsel.view(-1, 1)).sum(0), rtol=1e-4, atol=1e-2 * P)
    # second pass from the same centers: nothing changes
    st2 = cluster_ops.lloyd_pass(X, C, w, a, xabs_max=xa)
    assert float(st2.changed) == 0
    # assignment-only mode agrees
    a2 = torch.empty(N, dtype=torch.int32, device="cuda")
    cluster_ops.lloyd_pass(X, C, accumulate=False, assign=a2)
    assert bool((a2 == a).all())


@pytest.mark.gpu
@pytest.mark.parametrize("N,P,k", [(200_003, 100, 128), (100_001, 100, 64), (50_000, 36, 200), (9_999, 8, 17)])
def test_split_path_wave_assign_kernel(monkeypatch, N, P, k):
    """Large-k split path with the wave-persistent assignment kernel
    (kmeans_assign_kernel: X rows in registers, centers in LDS): the same
    per-accumulator MFMA order as the Lloyd kernel, so the assignment equals
    the Lloyd kernel's bit for bit and the f64 reference wherever the two
    closest centers are not within rounding; the sums pass statistics match f64."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = torch.Generator(device="cuda").manual_seed(N + k)
    X = torch.randn((N, P), generator=g, device="cuda")
    C = X[torch.randperm(N, generator=g, device="cuda")[:k]].double() + 0.01
    xa = cluster_ops.abs_bound(X)
    monkeypatch.setenv("H2O3_KM_SPLIT", "1")
    a = torch.full((N,), -1, dtype=torch.int32, device="cuda")
    st = cluster_ops.lloyd_pass(X, C, None, a, xabs_max=xa)
    monkeypatch.setenv("H2O3_KM_ASSIGN", "lloyd")
    a_ref = torch.full((N,), -1, dtype=torch.int32, device="cuda")
    cluster_ops.lloyd_pass(X, C, None, a_ref, xabs_max=xa)
    torch.cuda.synchronize()
    assert bool((a == a_ref).all())
    Xd = X.double()
    D = (Xd * Xd).sum(1, keepdim=True) - 2 * Xd @ C.T + (C * C).sum(1).view(1, -1)
    gap = D.topk(2, dim=1, largest=False).values
    clear = (gap[:, 1] - gap[:, 0]) > 1e-3 * (1 + gap[:, 0].abs())
    assert bool((a.long()[clear] == D.argmin(1)[clear]).all())
    oh = torch.zeros((N, k), dtype=torch.float64, device="cuda")
    oh[torch.arange(N, device="cuda"), a.long()] = 1.0
    torch.testing.assert_close(st.sums, oh.T @ Xd, rtol=2e-5, atol=2e-3)
    torch.testing.assert_close(st.weights, oh.sum(0), rtol=0, atol=0)
    assert float(st.changed) == N


@pytest.mark.gpu
def test_kmeans_estimator_gpu_uses_kernel():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    X, cs = _blobs(n=5000, seed=13)
    rng = np.random.RandomState(0)
    df = pd.DataFrame(X, columns=["a", "b"])
    df["c"] = rng.choice(["x", "y", "z"], len(df))
    fr = h2o3_amd.H2OFrame(df)
    m = H2OKMeansEstimator(k=4, seed=3, standardize=False)
    m.train(x=["a", "b"], training_frame=fr)
    assert m.tot_withinss() < 0.05 * m.totss()
    m2 = H2OKMeansEstimator(k=6, seed=3, estimate_k=False)
    m2.train(training_frame=fr)
    assert len(m2.centers()) == 6 and sum(m2.size()) == len(df)


@pytest.mark.gpu
@pytest.mark.parametrize("fx", [False, True])
def test_lloyd_kernel_large_n_f64_accumulation(fx):
    """20M rows (~80K rows per workgroup): the per-workgroup partials are f64
    and no f32 running sum spans more than a few thousand rows, so the
    cluster sums, weights and within-SS match an f64 reduction of the same
    per-row quantities far below f32 resolution of the totals."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    N, P, k = 20_000_000, 8, 4
    g = torch.Generator(device="cuda").manual_seed(5)
    X = torch.randn((N, P), generator=g, device="cuda") + 3.0
    C = X[:k].double()
    w = torch.rand(N, generator=g, device="cuda")
    a = torch.full((N,), -1, dtype=torch.int32, device="cuda")
    dmin = torch.empty(N, dtype=torch.float32, device="cuda")
    xa = cluster_ops.abs_bound(X, w) if fx else None
    st = cluster_ops.lloyd_pass(X, C, w, a, dmin=dmin, xabs_max=xa)
    torch.cuda.synchronize()
    idx = a.long()
    wd = w.double()
    oh = torch.nn.functional.one_hot(idx, k).double() * wd.view(-1, 1)   # f64 GEMMs, no contended atomics
    sums = oh.T @ X.double()
    wts = oh.sum(0)
    wss = oh.T @ dmin.double()
    torch.testing.assert_close(st.sums, sums, rtol=1e-7, atol=0)
    torch.testing.assert_close(st.weights, wts, rtol=1e-7, atol=0)
    torch.testing.assert_close(st.withinss, wss, rtol=1e-6, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("N,P,k", [(200_003, 100, 64), (50_001, 36, 130), (9_999, 8, 3), (400_001, 16, 128)])
def test_lloyd_split_path_matches_fused(N, P, k, monkeypatch):
    """Large-k split path (assignment pass + kmeans_sums_kernel) vs the fused
    kernel: same assignment / distances, same f64 statistics (both 64-bit
    fixed-point sums), same changed count."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = torch.Generator(device="cuda").manual_seed(N + k)
    X = torch.randn((N, P), generator=g, device="cuda")
    C = X[torch.randperm(N, generator=g, device="cuda")[:k]].double() + 0.01
    w = torch.rand(N, generator=g, device="cuda")
    w[::5] = 0
    xa = cluster_ops.abs_bound(X, w)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("H2O3_KM_SPLIT", mode)
        a = torch.full((N,), -1, dtype=torch.int32, device="cuda")
        a[::3] = 0
        dmin = torch.empty(N, dtype=torch.float32, device="cuda")
        st = cluster_ops.lloyd_pass(X, C, w, a, dmin=dmin, xabs_max=xa)
        torch.cuda.synchronize()
        out[mode] = (a.clone(), dmin.clone(), st.vec.clone())
    assert bool((out["0"][0] == out["1"][0]).all())
    # distances: same f32 terms, the wave kernel's interleaved MFMA chains may
    # sum them in another order (last-ulp differences at small k)
    torch.testing.assert_close(out["0"][1], out["1"][1], rtol=2e-6, atol=2e-6)
    assert float(out["1"][2][-1]) == float(out["0"][2][-1]) > 0
    # f64 statistics of the common assignment: the split path's fixed-point sums
    # are exact up to the f32 product w*x; the fused kernel at this k may hold
    # f32 private sums (folded every 16 tiles), so it gets the looser bound
    idx = out["1"][0].long()
    oh = torch.nn.functional.one_hot(idx, k).double() * w.double().view(-1, 1)
    ref = torch.cat([(oh.T @ X.double()).reshape(-1), oh.sum(0), oh.T @ out["1"][1].double()])
    m = k * P + 2 * k
    torch.testing.assert_close(out["1"][2][:k * P], ref[:k * P], rtol=1e-6, atol=1e-4)
    torch.testing.assert_close(out["1"][2][k * P:m], ref[k * P:], rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(out["0"][2][:k * P], ref[:k * P], rtol=2e-5, atol=2e-3)


IRIS = "/root/reference/h2o-core/src/main/resources/extdata/iris.csv"


@pytest.mark.skipif(not os.path.exists(IRIS), reason="reference extdata not present")
def test_kmeans_nfolds_cv_metrics_iris():
    """KMeans N-fold CV (hex/kmeans/KMeansTest.java:576-606 testNfolds): fold
    models train on the whole frame with the holdout at weight 0 (full-frame
    standardization), the CV metrics pool the holdout rows.  The reference's
    CV totss 695.9999869341457 is pinned to its own tolerance (1e-4); its
    tot_withinss / betweenss depend on the Java RNG's initial centers (its
    main model lands on a worse optimum, 240.8 vs 158.8 here), so only the
    identity betweenss = totss - tot_withinss and tot_withinss >= the main
    model's training optimum's order are checked -- parity unpinned there."""
    h2o3_amd.init(verbose=False)
    fr = h2o3_amd.import_file(IRIS)
    m = H2OKMeansEstimator(k=3, seed=0xdecaf, nfolds=3)
    m.train(training_frame=fr)
    assert m.totss(xval=True) == pytest.approx(695.9999869341457, abs=1e-4)
    assert m.totss() == pytest.approx(695.9999869341457, abs=1e-4)
    cv = m.model_performance(xval=True)
    assert cv.betweenss() == pytest.approx(cv.totss() - cv.tot_withinss(), abs=1e-9)
    assert 100 < cv.tot_withinss() < 400
    assert len(m.cross_validation_models()) == 3
    assert m._output["cross_validation_metrics_summary"]["tot_withinss"]["values"].__len__() == 3
    # holdout within-SS of the folds add up to the CV tot_withinss
    s = sum(cm._validation_metrics.tot_withinss() for cm in m.cross_validation_models())
    assert cv.tot_withinss() == pytest.approx(s, rel=1e-12)
