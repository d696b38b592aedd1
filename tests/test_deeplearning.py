import numpy as np
import pandas as pd

import h2o3_amd
from h2o3_amd.estimators import H2ODeepLearningEstimator


def test_dl_binomial_and_regression():
    rng = np.random.RandomState(0)
    X = rng.randn(3000, 5)
    logit = 2 * X[:, 0] - X[:, 1] ** 2 + X[:, 2]
    y = (rng.rand(3000) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame(X, columns=list("abcde"))
    df["y"] = np.where(y == 1, "t", "f")
    df["r"] = X[:, 0] * 3 + np.sin(X[:, 1])
    fr = h2o3_amd.H2OFrame(df)
    m = H2ODeepLearningEstimator(hidden=[32, 32], epochs=20, seed=1)
    m.train(x=list("abcde"), y="y", training_frame=fr)
    assert m.auc() > 0.85
    assert m.varimp() is not None
    m2 = H2ODeepLearningEstimator(hidden=[32], epochs=30, seed=1, activation="Tanh")
    m2.train(x=list("abcde"), y="r", training_frame=fr)
    assert m2.r2() > 0.9


def test_autoencoder_anomaly():
    rng = np.random.RandomState(1)
    X = rng.randn(2000, 4)
    X[:, 3] = X[:, 0] + X[:, 1]
    fr = h2o3_amd.H2OFrame(pd.DataFrame(X, columns=list("abcd")))
    m = H2ODeepLearningEstimator(autoencoder=True, hidden=[3], epochs=20, seed=2)
    m.train(training_frame=fr)
    a = m.anomaly(fr)
    assert a.nrows == 2000
    assert m.deepfeatures(fr, 0).ncols == 3


# ---------------------------------------------------------------- reference semantics
import math

import pytest
import torch

from h2o3_amd.ops import dl_ops


def _frame_cls(n=2000, seed=3):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, 6)
    logit = 2 * X[:, 0] - X[:, 1] + X[:, 2] * X[:, 3]
    y = (rng.rand(n) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(6)])
    df["y"] = np.where(y == 1, "yes", "no")
    df["r"] = X[:, 0] * 2 + np.sin(X[:, 1]) + 0.05 * rng.randn(n)
    df["cnt"] = rng.poisson(np.exp(0.5 * X[:, 0]))
    return h2o3_amd.H2OFrame(df), [f"x{i}" for i in range(6)]


def test_manual_backprop_matches_autograd():
    """The step's hand-written backward (GEMMs + dl_ops.bwd) equals autograd
    of the same forward (no dropout)."""
    torch.manual_seed(0)
    m = H2ODeepLearningEstimator(hidden=[7, 5], activation="Tanh", seed=4)
    layers = m._build(4, 3, True)
    m._layers = layers
    m._parms["input_dropout_ratio"] = 0.0
    X = torch.randn(16, 4)
    y = torch.randint(0, 3, (16,))
    acts, zs = m._forward(X.clone(), True, 1)
    _, dZ, _ = dl_ops.softmax(zs[-1], layers[-1].b, y, None, 1.0 / 16)
    grads = {}
    for li in range(len(layers) - 1, -1, -1):
        L = layers[li]
        if li == len(layers) - 1:
            db = dZ.sum(0)
        grads[li] = (dZ.t() @ acts[li], db)
        if li > 0:
            dZ, db = dl_ops.bwd(dZ @ L.W, acts[li], zs[li - 1], layers[li - 1].act)
    Ws = [L.W.clone().requires_grad_(True) for L in layers]
    bs = [L.b.clone().requires_grad_(True) for L in layers]
    h = X
    for i in range(len(layers) - 1):
        h = torch.tanh(h @ Ws[i].t() + bs[i])
    loss = torch.nn.functional.cross_entropy(h @ Ws[-1].t() + bs[-1], y)
    loss.backward()
    for li in range(len(layers)):
        torch.testing.assert_close(grads[li][0], Ws[li].grad, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(grads[li][1], bs[li].grad, rtol=1e-4, atol=1e-6)


def test_adadelta_row_update_matches_reference_formulas():
    """Neurons.bprop + computeAdaDeltaRateForWeight / ForBias, per row."""
    rng = np.random.RandomState(5)
    U, I = 3, 5
    W = torch.tensor(rng.randn(U, I), dtype=torch.float32)
    b = torch.tensor(rng.randn(U), dtype=torch.float32)
    dW = torch.tensor(rng.randn(U, I), dtype=torch.float32)
    db = torch.tensor(rng.randn(U), dtype=torch.float32)
    rho, eps, l1, l2 = 0.95, 1e-6, 1e-3, 1e-2
    Wn, bn = W.double().numpy().copy(), b.double().numpy().copy()
    E = np.zeros((U, I, 2))
    Eb = np.zeros((U, 2))
    for _ in range(3):   # three steps exercise the accumulators
        st = {} if _ == 0 else st
        for r in range(U):
            g2s = 0.0
            for c in range(I):
                g = dW[r, c].item() + np.sign(Wn[r, c]) * l1 + Wn[r, c] * l2
                E[r, c, 1] = rho * E[r, c, 1] + (1 - rho) * g * g
                rate = math.sqrt((E[r, c, 0] + eps) / (E[r, c, 1] + eps))
                E[r, c, 0] = rho * E[r, c, 0] + (1 - rho) * rate * rate * g * g
                Wn[r, c] -= rate * g
                g2s += g * g
            avg = g2s / I
            pg = db[r].item() + np.sign(bn[r]) * l1 + bn[r] * l2
            Eb[r, 1] = rho * Eb[r, 1] + (1 - rho) * avg
            rate = math.sqrt((Eb[r, 0] + eps) / (Eb[r, 1] + eps))
            Eb[r, 0] = rho * Eb[r, 0] + (1 - rho) * rate * rate * avg
            bn[r] -= rate * pg
        dl_ops.update(W, dW, b, db, st, dl_ops.UpdateParams(ada=True, rho=rho, eps=eps, l1=l1, l2=l2))
    np.testing.assert_allclose(W.numpy(), Wn, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(b.numpy(), bn, rtol=1e-5, atol=1e-6)


def test_momentum_nesterov_and_max_w2():
    W = torch.ones((2, 4))
    b = torch.zeros(2)
    dW = torch.full((2, 4), 0.5)
    db = torch.full((2,), 0.1)
    st = {}
    up = dl_ops.UpdateParams(ada=False, rate=0.1, momentum=0.5, nesterov=True, has_momenta=True, max_w2=2.0)
    dl_ops.update(W, dW, b, db, st, up)
    # nesterov: m = 0.5*0 - g = -0.5 ; w = 1 + 0.1*(-0.5) = 0.95 -> row |w|^2 = 3.61 > 2 -> rescale
    s = math.sqrt(2.0 / (4 * 0.95 ** 2))
    np.testing.assert_allclose(W.numpy(), np.full((2, 4), 0.95 * s), rtol=1e-6)
    np.testing.assert_allclose(b.numpy(), np.full(2, -0.01), rtol=1e-6)


def test_dropout_mask_rate_and_test_scaling():
    mask = dl_ops.keep_mask(12345, 2000, 300, 0.3, "cpu")
    assert abs(float(mask.float().mean()) - 0.7) < 0.005
    # same seed -> same bits (forward and backward recompute them)
    assert bool((mask == dl_ops.keep_mask(12345, 2000, 300, 0.3, "cpu")).all())
    Z = torch.randn(4, 3)
    A = dl_ops.fwd(Z.clone(), torch.zeros(3), "rectifier", 0.5, train=False, test_scale=0.5)
    torch.testing.assert_close(A, torch.relu(Z) * 0.5)


@pytest.mark.parametrize("act", ["TanhWithDropout", "RectifierWithDropout", "Maxout", "ExpRectifier"])
def test_activations_train(act):
    fr, x = _frame_cls()
    m = H2ODeepLearningEstimator(hidden=[24, 24], epochs=15, seed=1, activation=act)
    m.train(x=x, y="y", training_frame=fr)
    assert m.auc() > 0.8, (act, m.auc())
    p = m.predict(fr)
    assert p.ncols == 3


def test_regression_losses_and_distributions():
    fr, x = _frame_cls()
    for kw in ({"loss": "Huber"}, {"loss": "Absolute"}, {"loss": "Quantile", "quantile_alpha": 0.5}):
        m = H2ODeepLearningEstimator(hidden=[16], epochs=20, seed=2, **kw)
        m.train(x=x, y="r", training_frame=fr)
        assert m.r2() > 0.8, (kw, m.r2())
    mp = H2ODeepLearningEstimator(hidden=[16], epochs=20, seed=2, distribution="poisson")
    mp.train(x=x, y="cnt", training_frame=fr)
    pred = mp.predict(fr).as_data_frame().iloc[:, 0].values
    assert (pred > 0).all()
    cnt = fr.as_data_frame()["cnt"].values
    assert np.corrcoef(pred, cnt)[0, 1] > 0.3


def test_early_stopping_and_best_model():
    fr, x = _frame_cls(n=3000)
    tr, va = fr.split_frame(ratios=[0.7], seed=1)
    # score every iteration: no minimum interval, no duty-cycle cap
    m = H2ODeepLearningEstimator(hidden=[32, 32], epochs=200, seed=3, stopping_rounds=2, stopping_tolerance=0.05,
                                 train_samples_per_iteration=500, score_interval=0, score_duty_cycle=1.0)
    m.train(x=x, y="y", training_frame=tr, validation_frame=va)
    hist = m.scoring_history()
    assert len(hist) < 200 * 2100 / 500          # stopped early
    assert "validation_logloss" in hist[-1]
    best = min(h["validation_logloss"] for h in hist)
    assert m.logloss(valid=True) <= best * 1.02  # overwrite_with_best_model


def test_checkpoint_and_pretrained_autoencoder():
    fr, x = _frame_cls()
    ae = H2ODeepLearningEstimator(autoencoder=True, hidden=[12], epochs=5, seed=1, activation="Tanh")
    ae.train(x=x, training_frame=fr)
    m = H2ODeepLearningEstimator(hidden=[12], epochs=5, seed=1, activation="Tanh", pretrained_autoencoder=ae)
    m.train(x=x, y="y", training_frame=fr)
    assert m.auc() > 0.8
    m2 = H2ODeepLearningEstimator(hidden=[12], epochs=5, seed=1, activation="Tanh", checkpoint=m)
    m2.train(x=x, y="y", training_frame=fr)
    assert m2._processed > m._processed
    assert m2.auc() > 0.8


def test_sparse_autoencoder_and_rate_schedule():
    fr, x = _frame_cls()
    ae = H2ODeepLearningEstimator(autoencoder=True, hidden=[8], epochs=3, seed=1, activation="Tanh",
                                  sparsity_beta=0.1, average_activation=-0.5)
    ae.train(x=x, training_frame=fr)
    assert ae.anomaly(fr).nrows == fr.nrows
    m = H2ODeepLearningEstimator(hidden=[16], epochs=10, seed=1, adaptive_rate=False, rate=0.01,
                                 momentum_start=0.5, momentum_stable=0.9, momentum_ramp=1000, rate_decay=0.9,
                                 l1=1e-5, l2=1e-5, max_w2=10.0)
    m.train(x=x, y="y", training_frame=fr)
    assert m.auc() > 0.8
    for L in m._layers:
        assert float((L.W ** 2).sum(1).max()) <= 10.0 * (1 + 1e-5)


# ---------------------------------------------------------------- GPU kernels
@pytest.mark.gpu
@pytest.mark.parametrize("act", ["tanh", "rectifier", "exprectifier", "maxout"])
def test_dl_kernels_match_torch(act):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from h2o3_amd.ops import _native
    g = torch.Generator(device="cuda").manual_seed(7)
    B, U, I = 777, 300, 129
    k = 2 if act == "maxout" else 1
    Z = torch.randn((B, U * k), generator=g, device="cuda")
    b = torch.randn(U * k, generator=g, device="cuda")
    Zn, Zt = Z.clone(), Z.clone()
    An = dl_ops.fwd(Zn, b, act, 0.3, seed=99, train=True)
    At = dl_ops.fwd(Zt, b, act, 0.3, seed=99, train=True, use_native=False)
    assert "libdl.so" in " ".join(_native.loaded_libs())
    torch.testing.assert_close(An, At, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(Zn, Zt)
    dA = torch.randn((B, U), generator=g, device="cuda")
    dZn, dbn = dl_ops.bwd(dA, An, Zn, act, 0.3, seed=99)
    dZt, dbt = dl_ops.bwd(dA, At, Zt, act, 0.3, seed=99, use_native=False)
    torch.testing.assert_close(dZn, dZt, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dbn, dbt, rtol=1e-4, atol=1e-3)
    # per-row update, ADADELTA and Nesterov momentum with max_w2
    for up in (dl_ops.UpdateParams(ada=True, l1=1e-4, l2=1e-3, max_w2=5.0),
               dl_ops.UpdateParams(ada=False, rate=0.01, momentum=0.9, has_momenta=True, nesterov=True, max_w2=5.0)):
        W = torch.randn((U, I), generator=g, device="cuda") * 0.3
        bb = torch.randn(U, generator=g, device="cuda")
        dW = torch.randn((U, I), generator=g, device="cuda")
        db = torch.randn(U, generator=g, device="cuda")
        Wt, bt, sn, stt = W.clone(), bb.clone(), {}, {}
        for _ in range(3):
            dl_ops.update(W, dW, bb, db, sn, up)
            dl_ops.update(Wt, dW, bt, db, stt, up, use_native=False)
        torch.testing.assert_close(W, Wt, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(bb, bt, rtol=1e-4, atol=1e-5)
    # softmax + CE gradient
    Zs = torch.randn((B, 5), generator=g, device="cuda")
    y = torch.randint(0, 5, (B,), generator=g, device="cuda")
    y[::11] = -1
    bs = torch.randn(5, generator=g, device="cuda")
    Pn, gn, ln = dl_ops.softmax(Zs.clone(), bs, y, None, 1.0 / B)
    Pt, gt, lt = dl_ops.softmax(Zs.clone(), bs, y, None, 1.0 / B, use_native=False)
    torch.testing.assert_close(Pn, Pt, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(gn, gt, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(ln, lt, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_dl_estimator_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fr, x = _frame_cls(n=20000)
    m = H2ODeepLearningEstimator(hidden=[64, 64], epochs=5, seed=1, activation="RectifierWithDropout",
                                 input_dropout_ratio=0.1)
    m.train(x=x, y="y", training_frame=fr)
    assert m.auc() > 0.85


@pytest.mark.gpu
def test_dl_step_graph_matches_eager():
    """The hipGraph-captured step (gather + forward + backward + updates +
    seed advance) equals the same steps launched eagerly."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn((5000, 12), generator=g, device="cuda")
    Y = (X[:, 0] > 0).long()
    hp = dict(K=2, ae=False, bs=256, ada=True, rate0=0.005, anneal=1e-6, decay=1.0, mom_start=0.0, mom_ramp=1e6,
              mom_stable=0.0, has_mom=False, l1=1e-5, l2=1e-5, max_w2=10.0, sparsity=0.0)
    mk = lambda: H2ODeepLearningEstimator(hidden=[32, 16], activation="RectifierWithDropout", seed=3,
                                          input_dropout_ratio=0.1)
    a, b = mk(), mk()
    for m in (a, b):
        m._layers = m._build(12, 2, True)
        m._processed = 0.0
    idxs = [torch.randint(0, 5000, (256,), generator=g, device="cuda") for _ in range(3)]
    gs = a._step_graph(X, Y, None, hp, None)
    for idx in idxs:
        gs["idx"].copy_(idx)
        gs["g"].replay()
    seed = torch.tensor([b._seed() * 1000003 & ((1 << 62) - 1)], dtype=torch.int64, device="cuda")
    # the capture's warm-up steps are rolled back: both models see only idxs
    for idx in idxs:
        dl_ops.seed_advance(seed)
        b._train_step(X.index_select(0, idx), Y.index_select(0, idx), None, 0, hp, None, seed_dev=seed)
    torch.cuda.synchronize()
    for La, Lb in zip(a._layers, b._layers):
        torch.testing.assert_close(La.W, Lb.W, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(La.b, Lb.b, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(La.state["ada"], Lb.state["ada"], rtol=1e-5, atol=1e-7)
    assert a._processed == 0.0


def _cat_frame(n=3000, seed=4):
    rng = np.random.RandomState(seed)
    lv = np.array([f"L{i}" for i in range(40)])
    c = rng.choice(lv, n)
    eff = dict(zip(lv, rng.randn(40)))
    x1 = rng.randn(n)
    y = (np.array([eff[v] for v in c]) + x1 + 0.3 * rng.randn(n)) > 0
    df = pd.DataFrame({"c": c, "x1": x1, "y": np.where(y, "a", "b")})
    return df, h2o3_amd.H2OFrame(df)


def test_max_categorical_features_hash_trick():
    """max_categorical_features (Neurons.Input.setInput): 40 one-hot levels
    hashed into 8 input slots; the input layer shrinks and scoring hashes
    the same way."""
    import pytest
    df, fr = _cat_frame()
    m = H2ODeepLearningEstimator(hidden=[16], epochs=10, seed=1, max_categorical_features=8)
    m.train(x=["c", "x1"], y="y", training_frame=fr)
    assert m._layers[0].fin == 8 + 1
    full = H2ODeepLearningEstimator(hidden=[16], epochs=10, seed=1)
    full.train(x=["c", "x1"], y="y", training_frame=fr)
    assert full._layers[0].fin == 40 + 1
    assert 0.6 < m.auc() < full.auc() + 0.02         # collisions cost accuracy, never help much
    p1 = m.predict(fr).as_data_frame().iloc[:, -1].values
    p2 = m.predict(h2o3_amd.H2OFrame(df.iloc[::-1].reset_index(drop=True))).as_data_frame().iloc[:, -1].values
    np.testing.assert_allclose(p1[::-1], p2, atol=1e-6)
    with pytest.raises(ValueError, match="max_categorical_features"):
        H2ODeepLearningEstimator(max_categorical_features=0).train(x=["c", "x1"], y="y", training_frame=fr)


def test_export_weights_shuffle_reproducible_and_checks():
    import pytest
    _, fr = _cat_frame(1500, seed=5)
    m = H2ODeepLearningEstimator(hidden=[8], epochs=2, seed=2, export_weights_and_biases=True)
    m.train(x=["c", "x1"], y="y", training_frame=fr)
    W0 = m.weights(0).as_data_frame().values
    np.testing.assert_allclose(W0, m._layers[0].W.cpu().numpy(), atol=1e-6)
    assert m.biases(1).nrows == 2
    q = H2ODeepLearningEstimator(hidden=[8], epochs=2, seed=2)
    q.train(x=["c", "x1"], y="y", training_frame=fr)
    with pytest.raises(ValueError, match="export_weights_and_biases"):
        q.weights(0)
    # iterations smaller than the data: row order is kept unless shuffle_training_data
    kw = dict(hidden=[8], epochs=3, seed=2, train_samples_per_iteration=300)
    a = H2ODeepLearningEstimator(shuffle_training_data=False, **kw)
    a.train(x=["c", "x1"], y="y", training_frame=fr)
    b = H2ODeepLearningEstimator(shuffle_training_data=True, **kw)
    b.train(x=["c", "x1"], y="y", training_frame=fr)
    assert not np.allclose(a._layers[0].W.cpu().numpy(), b._layers[0].W.cpu().numpy())
    r1 = H2ODeepLearningEstimator(reproducible=True, **kw)
    r1.train(x=["c", "x1"], y="y", training_frame=fr)
    r2 = H2ODeepLearningEstimator(reproducible=True, **kw)
    r2.train(x=["c", "x1"], y="y", training_frame=fr)
    np.testing.assert_array_equal(r1._layers[0].W.cpu().numpy(), r2._layers[0].W.cpu().numpy())
    with pytest.raises(ValueError, match="duty"):
        H2ODeepLearningEstimator(score_duty_cycle=2).train(x=["c", "x1"], y="y", training_frame=fr)
    with pytest.raises(ValueError, match="moving rate"):
        H2ODeepLearningEstimator(elastic_averaging=True, elastic_averaging_moving_rate=2).train(
            x=["c", "x1"], y="y", training_frame=fr)


def test_score_validation_samples():
    df, fr = _cat_frame(3000, seed=6)
    tr, va = fr.split_frame(ratios=[0.5], seed=1)
    m = H2ODeepLearningEstimator(hidden=[8], epochs=2, seed=2, score_validation_samples=200,
                                 score_validation_sampling="Stratified")
    m.train(x=["c", "x1"], y="y", training_frame=tr, validation_frame=va)
    full = H2ODeepLearningEstimator(hidden=[8], epochs=2, seed=2)
    full.train(x=["c", "x1"], y="y", training_frame=tr, validation_frame=va)
    h1, h2 = m.scoring_history()[-1], full.scoring_history()[-1]
    # same training, the history's validation numbers come from a 200-row sample
    assert h1["training_logloss"] == h2["training_logloss"]
    assert h1["validation_logloss"] != h2["validation_logloss"]


def _fused_vs_unfused(mk, P, K, B, Y, w, hp, steps=3, graph=False):
    """Train two copies of the same network for `steps` mini-batches, one
    through the fused HIP step and one through the unfused path (library
    GEMMs + element-wise kernels); returns the two layer lists."""
    import os
    g = torch.Generator(device="cuda").manual_seed(11)
    X = torch.randn((4000, P), generator=g, device="cuda")
    a, b = mk(), mk()
    from h2o3_amd.models.distributions import get_distribution
    for m in (a, b):
        m._layers = m._build(P, K, K > 1)
        m._processed = 0.0
        m._dist = get_distribution("AUTO" if K > 1 else "gaussian", K)
    idxs = [torch.randint(0, 4000, (B,), generator=g, device="cuda") for _ in range(steps)]
    old = os.environ.get("H2O3_DL_FUSED")
    try:
        for m, flag in ((a, "1"), (b, "0")):
            os.environ["H2O3_DL_FUSED"] = flag
            assert (m._fused_kind(hp, None) is not None) == (flag == "1")
            for t, idx in enumerate(idxs):
                m._train_step(X.index_select(0, idx), Y.index_select(0, idx),
                              None if w is None else w.index_select(0, idx), 1000 + t, hp)
    finally:
        if old is None:
            os.environ.pop("H2O3_DL_FUSED", None)
        else:
            os.environ["H2O3_DL_FUSED"] = old
    torch.cuda.synchronize()
    return a._layers, b._layers


def _assert_layers_close(La, Lb):
    for x, y in zip(La, Lb):
        for ta, tb in ((x.W, y.W), (x.b, y.b), (x.state["ada"], y.state["ada"])):
            # f32 sums in another order; an ADADELTA step is ~sign(g) sqrt(eps / (1 - rho))
            # at the first steps, so a gradient within rounding of 0 may flip one weight
            bad = ((ta - tb).abs() > 2e-5 + 2e-4 * tb.abs()).sum().item()
            assert bad <= 2, (bad, (ta - tb).abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["bench", "tanh_multiclass_ragged", "regression_elu", "momentum"])
def test_dl_fused_step_matches_unfused(case):
    """The fused HIP MLP step (dl.hip dl_mlp_*: f32 MFMA forward/backward per
    16-row tile, dW tiles, per-row updates) gives the weights, biases and
    ADADELTA state of the unfused step (hipBLASLt GEMMs + element-wise
    kernels) on the same batches and dropout seeds."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from h2o3_amd.ops import _native
    g = torch.Generator(device="cuda").manual_seed(5)
    base = dict(ae=False, ada=True, rate0=0.005, anneal=1e-6, decay=1.0, mom_start=0.0, mom_ramp=1e6,
                mom_stable=0.0, has_mom=False, l1=0.0, l2=0.0, max_w2=3.4e38, sparsity=0.0)
    if case == "bench":
        P, K, B = 100, 2, 1024
        Y = torch.randint(0, 2, (4000,), generator=g, device="cuda")
        mk = lambda: H2ODeepLearningEstimator(hidden=[200, 200], activation="RectifierWithDropout", seed=42,
                                              input_dropout_ratio=0.1)
        w = None
    elif case == "tanh_multiclass_ragged":
        P, K, B = 13, 5, 333
        Y = torch.randint(0, 5, (4000,), generator=g, device="cuda")
        mk = lambda: H2ODeepLearningEstimator(hidden=[37, 19], activation="TanhWithDropout", seed=3,
                                              hidden_dropout_ratios=[0.2, 0.3])
        w = torch.rand(4000, generator=g, device="cuda") + 0.5
        base.update(l1=1e-4, l2=1e-3, max_w2=2.0)
    elif case == "regression_elu":
        P, K, B = 24, 1, 100
        Y = torch.randn((4000, 1), generator=g, device="cuda")
        mk = lambda: H2ODeepLearningEstimator(hidden=[50], activation="ExpRectifier", seed=8)
        w = None
    else:
        P, K, B = 32, 3, 256
        Y = torch.randint(0, 3, (4000,), generator=g, device="cuda")
        mk = lambda: H2ODeepLearningEstimator(hidden=[64, 32], activation="Rectifier", seed=9,
                                              adaptive_rate=False, momentum_start=0.5, momentum_stable=0.9,
                                              nesterov_accelerated_gradient=True)
        w = None
        base.update(ada=False, rate0=0.01, has_mom=True, mom_start=0.5, mom_stable=0.9, mom_ramp=1000.0,
                    decay=0.9, max_w2=5.0)
    hp = dict(base, K=K, bs=B)
    La, Lb = _fused_vs_unfused(mk, P, K, B, Y, w, hp)
    assert "libdl.so" in " ".join(_native.loaded_libs())
    _assert_layers_close(La, Lb)
    if not hp["ada"]:
        for x, y in zip(La, Lb):
            torch.testing.assert_close(x.state["mom"], y.state["mom"], rtol=2e-4, atol=2e-5)


@pytest.mark.gpu
def test_dl_gemm_kernel_matches_fp64():
    """dl.hip dl_gemm_kernel (f32 MFMA tiles, any strides) against an fp64
    product, for the three per-step products and ragged shapes."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from h2o3_amd.ops import dl_ops
    g = torch.Generator(device="cuda").manual_seed(3)
    for M, K, N in ((1024, 1024, 1024), (333, 37, 19), (1, 5, 7), (1000, 100, 200), (64, 2000, 3), (1024, 1000, 2),
                    (1024, 0, 5)):
        A = torch.randn((M, K), generator=g, device="cuda")
        W = torch.randn((N, K), generator=g, device="cuda")
        C = dl_ops.gemm(A, W.t())                       # Z = A W^T
        torch.testing.assert_close(C.double(), A.double() @ W.double().t(), rtol=1e-4, atol=1e-4 * K ** 0.5)
        dZ = torch.randn((M, N), generator=g, device="cuda")
        dA = dl_ops.gemm(dZ, W)                          # dA = dZ W
        torch.testing.assert_close(dA.double(), dZ.double() @ W.double(), rtol=1e-4, atol=1e-4 * N ** 0.5)
        dW = dl_ops.gemm(dZ.t(), A)                      # dW = dZ^T A
        torch.testing.assert_close(dW.double(), dZ.double().t() @ A.double(), rtol=1e-4, atol=1e-4 * M ** 0.5)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["wide1024", "maxout", "autoencoder"])
def test_dl_wide_layers_on_mfma_gemm(monkeypatch, case):
    """Networks beyond the LDS-resident fused step (hidden=[1024, 1024],
    maxout, autoencoders) train through dl_gemm_kernel: the same weights /
    ADADELTA state as the same steps with torch (library) matmuls."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import copy
    from h2o3_amd.ops import dl_ops
    g = torch.Generator(device="cuda").manual_seed(21)
    P, B = 100, 512
    X = torch.randn((3000, P), generator=g, device="cuda")
    if case == "wide1024":
        mk = lambda: H2ODeepLearningEstimator(hidden=[1024, 1024], activation="RectifierWithDropout", seed=1)
        K, ae = 2, False
    elif case == "maxout":
        mk = lambda: H2ODeepLearningEstimator(hidden=[200, 100], activation="Maxout", seed=2)
        K, ae = 3, False
    else:
        mk = lambda: H2ODeepLearningEstimator(hidden=[300, 20, 300], activation="Tanh", seed=3, autoencoder=True)
        K, ae = P, True
    Y = torch.randint(0, max(K, 2), (3000,), generator=g, device="cuda") if not ae else None
    hp = dict(K=K if not ae else P, ae=ae, bs=B, ada=True, rate0=0.005, anneal=1e-6, decay=1.0, mom_start=0.0,
              mom_ramp=1e6, mom_stable=0.0, has_mom=False, l1=0.0, l2=0.0, max_w2=3.4e38, sparsity=0.0)
    from h2o3_amd.models.distributions import get_distribution
    nets = []
    for mode in ("mfma", "torch"):
        monkeypatch.setenv("H2O3_DL_GEMM", mode)
        m = mk()
        m._layers = m._build(P, hp["K"], (K > 1) and not ae)
        m._processed = 0.0
        m._dist = get_distribution("AUTO" if (K > 1 and not ae) else "gaussian", K)
        assert m._fused_kind(hp, None) is None
        gg = torch.Generator(device="cuda").manual_seed(5)
        for t in range(3):
            idx = torch.randint(0, 3000, (B,), generator=gg, device="cuda")
            m._train_step(X.index_select(0, idx), X.index_select(0, idx) if ae else Y.index_select(0, idx), None,
                          500 + t, hp)
        nets.append(m._layers)
    for x, y in zip(nets[0], nets[1]):
        for ta, tb in ((x.W, y.W), (x.b, y.b), (x.state["ada"], y.state["ada"])):
            # f32 sums in another order; the first ADADELTA steps move a weight by
            # ~sign(g) sqrt(eps / (1 - rho)), so gradients within rounding of 0 may
            # flip: allow a few per million
            bad = ((ta - tb).abs() > 2e-5 + 2e-4 * tb.abs()).sum().item()
            assert bad <= max(2, int(2e-5 * ta.numel())), (bad, ta.numel(), (ta - tb).abs().max().item())


@pytest.mark.gpu
def test_dl_multi_step_graph_matches_single_steps(monkeypatch):
    """S steps captured in one graph (H2O3_DL_GRAPH_STEPS) train the model
    that S single-step replays train: same batches, same dropout seeds."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fr, x = _frame_cls(n=60000)
    out = []
    for S in ("1", "8"):
        monkeypatch.setenv("H2O3_DL_GRAPH_STEPS", S)
        m = H2ODeepLearningEstimator(hidden=[50], epochs=3, seed=1, activation="RectifierWithDropout",
                                     hidden_dropout_ratios=[0.1], input_dropout_ratio=0.05)
        m.train(x=x, y="y", training_frame=fr)
        out.append(([L.W.detach().clone() for L in m._layers], m.logloss()))
    for Wa, Wb in zip(out[0][0], out[1][0]):
        torch.testing.assert_close(Wa, Wb, rtol=1e-5, atol=1e-6)
    assert abs(out[0][1] - out[1][1]) < 1e-6
