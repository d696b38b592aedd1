"""Deep Learning (multi-layer perceptron, autoencoder).

Reference: hex/deeplearning/DeepLearning.java, DeepLearningModel.java,
DeepLearningModelInfo.java, Neurons.java (Tanh / Rectifier / Maxout /
ExpRectifier, each +WithDropout; Softmax / Linear outputs), Dropout.java,
DeepLearningTask.java.  Semantics kept from the reference:
  * layer-wise UniformAdaptive / Uniform / Normal init, user initial weights
    and biases, pretrained_autoencoder;
  * ADADELTA per weight (rho, epsilon) with the bias rate driven by the
    row's mean squared weight gradient (Neurons.update_bias), or plain SGD:
    rate / (1 + rate_annealing * samples) * rate_decay^layer, momentum ramp
    momentum_start -> momentum_stable over momentum_ramp samples, Nesterov;
  * L1 / L2 on weights and biases, max_w2 per-neuron row rescale;
  * unit dropout without rescaling while training, activations scaled by
    (1 - ratio) at test time; input dropout;
  * Softmax + CrossEntropy / Quadratic, Linear output with the
    distribution's gradient (gaussian, poisson, gamma, tweedie, laplace,
    quantile, huber), standardized regression response;
  * autoencoder (reconstruction gradient, sparsity_beta / average_activation),
    anomaly(), deepfeatures(), Gedeon variable importance;
  * scoring every iteration (train_samples_per_iteration), early stopping
    (stopping_rounds / metric / tolerance, classification_stop,
    regression_stop), overwrite_with_best_model, max_runtime_secs,
    checkpoint restart.

MI355X design: the standardized design matrix is one HBM tensor; a training
step is mini-batch data parallel: the dense products go to the library GEMM
(hipBLASLt), every element-wise / per-neuron part is a hand-written HIP
kernel (ops/csrc/dl.hip: fused bias + activation + hashed dropout forward,
fused backward with bias-gradient column sums, one per-neuron-row update
kernel doing gradient + L1/L2 + ADADELTA / momentum + max_w2 + bias update,
softmax + output gradient).  The reference's per-row Hogwild updates are a
CPU-cache idiom; here a mini-batch gradient (mini_batch_size, at least 32
rows) is applied per step.  With several GPUs each rank trains its own
copy for an iteration with no collective in the (graph-captured) step and
the models are averaged by one bucketed RCCL all-reduce per iteration -- the
reference's model averaging (DeepLearningTask.reduce), with its elastic
averaging, replicate_training_data, single_node_mode and the
target_ratio_comm_to_comp auto-tuning of the iteration size.
"""
from __future__ import annotations

import copy
import math
import os
import time

import numpy as np
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_REAL, Vec
from ..ops import dl_ops
from ..parallel import cloud
from ..parallel import collectives as coll
from ..utils import graphs
from . import metrics as mm
from .base import H2OEstimator, ScoreKeeper, _LESS_IS_BETTER
from .datainfo import DataInfo

DL_DEFAULTS = dict(activation="Rectifier", hidden=[200, 200], epochs=10.0, train_samples_per_iteration=-2,
                   target_ratio_comm_to_comp=0.05, seed=-1, adaptive_rate=True, rho=0.99, epsilon=1e-8, rate=0.005,
                   rate_annealing=1e-6, rate_decay=1.0, momentum_start=0.0, momentum_ramp=1e6, momentum_stable=0.0,
                   nesterov_accelerated_gradient=True, input_dropout_ratio=0.0, hidden_dropout_ratios=None,
                   l1=0.0, l2=0.0, max_w2=3.4028235e38, initial_weight_distribution="UniformAdaptive",
                   initial_weight_scale=1.0, initial_weights=None, initial_biases=None, loss="Automatic",
                   distribution="auto", quantile_alpha=0.5, tweedie_power=1.5, huber_alpha=0.9,
                   score_interval=5.0, score_training_samples=10000, score_validation_samples=0,
                   score_duty_cycle=0.1, classification_stop=0.0, regression_stop=1e-6, stopping_rounds=5,
                   stopping_metric="auto", stopping_tolerance=0.0, max_runtime_secs=0.0,
                   score_validation_sampling="Uniform", diagnostics=True, fast_mode=True, force_load_balance=True,
                   variable_importances=True, replicate_training_data=True, single_node_mode=False,
                   shuffle_training_data=False, missing_values_handling="MeanImputation", quiet_mode=False,
                   autoencoder=False, sparse=False, col_major=False, average_activation=0.0, sparsity_beta=0.0,
                   max_categorical_features=2147483647, reproducible=False, export_weights_and_biases=False,
                   mini_batch_size=1, categorical_encoding="auto", elastic_averaging=False,
                   elastic_averaging_moving_rate=0.9, elastic_averaging_regularization=0.001,
                   pretrained_autoencoder=None, standardize=True, balance_classes=False,
                   class_sampling_factors=None, max_after_balance_size=5.0, max_confusion_matrix_size=20,
                   use_all_factor_levels=True, checkpoint=None, overwrite_with_best_model=True)

_MIN_GPU_BATCH = 32


def _murmur3_int(v, seed):
    """32-bit murmur3 of one big-endian int (the hash trick of
    Neurons.Input.setInput)."""
    c1, c2, m32 = 0xCC9E2D51, 0x1B873593, 0xFFFFFFFF
    k = int.from_bytes(int(v & m32).to_bytes(4, "big"), "little")
    h = seed & m32
    k = (k * c1) & m32
    k = ((k << 15) | (k >> 17)) & m32
    k = (k * c2) & m32
    h ^= k
    h = ((h << 13) | (h >> 19)) & m32
    h = (h * 5 + 0xE6546B64) & m32
    h ^= 4
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & m32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & m32
    h ^= h >> 16
    return h


def _act_name(activation):
    a = (activation or "Rectifier").lower()
    drop = a.endswith("withdropout")
    base = a.replace("withdropout", "")
    return {"tanh": "tanh", "rectifier": "rectifier", "maxout": "maxout", "exprectifier": "exprectifier"}[base], drop


class _Layer:
    """One dense layer: W [out*k, in] (k = 2 for maxout), b [out*k]."""

    def __init__(self, fin, fout, act, drop, k=1):
        self.fin, self.fout, self.act, self.drop, self.k = fin, fout, act, drop, k
        self.W = None
        self.b = None
        self.state = {}

    def state_dict(self):
        return {"W": self.W.detach().cpu().clone(), "b": self.b.detach().cpu().clone()}


class H2ODeepLearningEstimator(H2OEstimator):
    algo = "deeplearning"
    _defaults = DL_DEFAULTS

    def __init__(self, **kw):
        super().__init__(**kw)
        if self._parms.get("autoencoder"):
            self.supervised_learning = False

    def _seed(self):
        s = self._parms.get("seed", -1)
        return 12345 if s is None or s == -1 else int(s) & 0x7FFFFFFF

    # ------------------------------------------------------------------ network
    def _build(self, P, out_dim, classification):
        p = self._parms
        hidden = list(p.get("hidden") or [200, 200])
        act, with_drop = _act_name(p.get("activation"))
        hdr = p.get("hidden_dropout_ratios")
        if hdr is None:
            hdr = [0.5] * len(hidden) if with_drop else [0.0] * len(hidden)
        if len(hdr) != len(hidden):
            raise ValueError("hidden_dropout_ratios must have one entry per hidden layer")
        if not with_drop and any(h > 0 for h in hdr):
            raise ValueError("hidden_dropout_ratios requires a *WithDropout activation")
        layers, fin = [], P
        for h, d in zip(hidden, hdr):
            layers.append(_Layer(fin, h, act, float(d), 2 if act == "maxout" else 1))
            fin = h
        out_act = "softmax" if classification else "linear"
        layers.append(_Layer(fin, out_dim, out_act, 0.0))
        g = torch.Generator().manual_seed(self._seed())
        dist = (p.get("initial_weight_distribution") or "UniformAdaptive").lower()
        scale = float(p.get("initial_weight_scale", 1.0))
        iw, ib = p.get("initial_weights"), p.get("initial_biases")
        dev = cloud.device()
        for li, L in enumerate(layers):
            rows = L.fout * L.k
            if dist == "uniform":
                W = (torch.rand((rows, L.fin), generator=g) * 2 - 1) * scale
            elif dist == "normal":
                W = torch.randn((rows, L.fin), generator=g) * scale
            else:   # UniformAdaptive (Neurons.randomize: +-sqrt(6 / (fan_in + fan_out)))
                r = math.sqrt(6.0 / (L.fin + L.fout))
                W = (torch.rand((rows, L.fin), generator=g) * 2 - 1) * r
            b = torch.zeros(rows)
            if iw is not None and li < len(iw) and iw[li] is not None:
                W = self._frame_matrix(iw[li]).view(rows, L.fin)
            if ib is not None and li < len(ib) and ib[li] is not None:
                b = self._frame_matrix(ib[li]).view(rows)
            L.W = W.to(dev, torch.float32).contiguous()
            L.b = b.to(dev, torch.float32).contiguous()
        pre = p.get("pretrained_autoencoder")
        if pre is not None:
            from ..core import dkv
            ae = dkv.get(pre) if isinstance(pre, str) else pre
            for L, A in zip(layers[:-1], ae._layers[:len(layers) - 1]):
                if A.W.shape != L.W.shape:
                    raise ValueError("pretrained_autoencoder hidden layers do not match this network")
                L.W.copy_(A.W)
                L.b.copy_(A.b)
        return layers

    @staticmethod
    def _frame_matrix(fr):
        from ..core import dkv
        fr = dkv.get(fr) if isinstance(fr, str) else fr
        cols = [fr.vec(c).as_float(torch.float32) for c in fr.names]
        return torch.stack(cols, 1).cpu()

    def _forward(self, X, train, seed=0, seed_dev=None):
        """Returns (activations list [A_0 = input, ...], pre-activations list).
        Dropout masks hash (seed + per-layer offset [+ *seed_dev])."""
        p = self._parms
        A = X
        ratio_in = float(p.get("input_dropout_ratio") or 0.0)
        if train and ratio_in > 0:
            # input dropout: the forward kernel with a linear activation and no bias
            A = dl_ops.fwd(X.clone(), None, "linear", ratio_in, seed=seed + 0x5bd1e995, train=True,
                           seed_dev=seed_dev)
        acts, zs = [A], []
        for li, L in enumerate(self._layers[:-1]):
            Z = dl_ops.gemm(A, L.W.t())
            Ah = dl_ops.fwd(Z, L.b, L.act, L.drop, seed=seed + 7919 * (li + 1), train=train,
                            test_scale=1.0 - L.drop, seed_dev=seed_dev)
            zs.append(Z)
            acts.append(Ah)
            A = Ah
        Lo = self._layers[-1]
        Zo = dl_ops.gemm(A, Lo.W.t())
        zs.append(Zo)
        return acts, zs

    # ------------------------------------------------------------------ inputs
    def _validate_dl(self, spec, di):
        """DeepLearningParameters.validate (DeepLearningModel.java:1760-1940)."""
        p = self._parms
        if not 0 <= float(p.get("score_duty_cycle", 0.1)) <= 1:
            raise ValueError("ERRR on field: _score_duty_cycle: Score duty cycle must be >= 0 and <=1.")
        if int(p.get("score_validation_samples") or 0) < 0:
            raise ValueError("ERRR on field: _score_validation_samples: Number of training samples for scoring must "
                             "be >= 0 (0 for all).")
        if int(p.get("max_categorical_features", 2147483647)) < 1:
            raise ValueError("ERRR on field: _max_categorical_features: max_categorical_features must be at least 1.")
        if p.get("elastic_averaging"):
            if not 0 <= float(p.get("elastic_averaging_moving_rate", 0.9)) <= 1:
                raise ValueError("ERRR on field: _elastic_averaging_moving_rate: Elastic averaging moving rate must "
                                 "be between 0 and 1.")
            if float(p.get("elastic_averaging_regularization", 1e-3)) < 0:
                raise ValueError("ERRR on field: _elastic_averaging_regularization: Elastic averaging "
                                 "regularization strength must be >= 0.")
            if p.get("sparse"):
                raise ValueError("ERRR on field: _elastic_averaging: Cannot use elastic averaging with sparse input.")
        if str(p.get("score_validation_sampling") or "Uniform").lower() not in ("uniform", "stratified"):
            raise ValueError("score_validation_sampling must be Uniform or Stratified")
        if p.get("reproducible") and p.get("seed", -1) in (None, -1):
            import warnings
            warnings.warn("reproducible=True without a seed: the run is deterministic for the default seed only")

    def _hash_slots(self, di):
        """max_categorical_features (Neurons.Input.setInput, hash trick): the
        one-hot categorical columns are folded into that many slots by a
        seeded murmur3 hash of the expanded column index; numeric columns
        stay.  Returns the slot of every categorical column, or None."""
        p = self._parms
        mc = int(p.get("max_categorical_features", 2147483647))
        ncat = di.n_cat_expanded
        if mc >= ncat:
            return None
        if p.get("autoencoder"):
            raise ValueError("max_categorical_features below the categorical width is not supported for "
                             "autoencoders (the reconstruction would be of hashed slots)")
        seed = int(p.get("seed", -1) if p.get("seed", -1) is not None else -1)
        slots = np.array([_murmur3_int(j, seed) % mc for j in range(ncat)], dtype=np.int64)
        return torch.as_tensor(slots, device=cloud.device())

    def _design(self, frame):
        """(X, ok): the expanded input matrix, categorical columns hashed into
        max_categorical_features slots when that is below their count."""
        X, ok = self._dinfo.expand(frame, pad=False)
        slots = getattr(self, "_cat_slots", None)
        if slots is None:
            return X, ok
        ncat = self._dinfo.n_cat_expanded
        mc = int(self._parms.get("max_categorical_features"))
        H = torch.zeros((X.shape[0], mc), dtype=X.dtype, device=X.device)
        H.index_add_(1, slots, X[:, :ncat])
        return torch.cat([H, X[:, ncat:]], 1).contiguous(), ok

    def _valid_sample(self, spec):
        """score_validation_samples / score_validation_sampling
        (DeepLearning.java:428): the validation frame scored during training
        is a seeded uniform or class-stratified sample of that many rows."""
        p = self._parms
        ns = int(p.get("score_validation_samples") or 0)
        vf = spec.valid
        if vf is None or ns <= 0 or ns >= vf.nrows:
            return vf
        g = torch.Generator(device=cloud.device())
        g.manual_seed((self._seed() + 1) * 1000003 + cloud.rank())
        frac = ns / vf.nrows
        if str(p.get("score_validation_sampling") or "Uniform").lower() == "stratified" and spec.is_classification:
            y = spec.y_tensor(vf).long()
            u = torch.rand(y.numel(), generator=g, device=y.device)
            keep = torch.zeros_like(u, dtype=torch.bool)
            for k in range(spec.nclasses):
                m = y == k
                keep |= m & (u < frac)
            keep |= (y < 0) & (u < frac)
        else:
            keep = torch.rand(vf.nlocal, generator=g, device=cloud.device()) < frac
        return vf[keep]

    # ------------------------------------------------------------------ fit
    def _fit(self, spec):
        p = self._parms
        torch.manual_seed(self._seed())
        di = DataInfo(spec.frame, spec.x, standardize=bool(p.get("standardize", True)),
                      use_all_factor_levels=bool(p.get("use_all_factor_levels", True)),
                      missing_values_handling=p.get("missing_values_handling"), pad_to=0)
        self._dinfo = di
        self._validate_dl(spec, di)
        self._cat_slots = self._hash_slots(di)
        X, ok = self._design(spec.frame)
        ae = bool(p.get("autoencoder"))
        self._ae = ae
        K = spec.nclasses if (spec.is_classification and not ae) else 1
        self._K = K
        Y = None
        from .distributions import get_distribution
        dname = (p.get("distribution") or "auto")
        if not ae:
            y = spec.y_tensor()
            if spec.is_classification:
                ok = ok & (y >= 0)
                Y = y.long()
            else:
                yf = y.to(torch.float32)
                ok = ok & ~torch.isnan(yf)
                n_ok = coll.allreduce_scalar(float(ok.sum()))
                self._ymu = coll.allreduce_scalar(float(yf[ok].sum())) / max(n_ok, 1)
                var = coll.allreduce_scalar(float(((yf[ok] - self._ymu) ** 2).sum())) / max(n_ok - 1, 1)
                self._ysd = math.sqrt(var) if var > 0 else 1.0
                if dname.lower() not in ("auto", "gaussian", "laplace", "quantile", "huber"):
                    self._ymu, self._ysd = 0.0, 1.0   # log-link families train on the raw response
                Y = ((yf - self._ymu) / self._ysd).view(-1, 1)
        self._dist = get_distribution(dname if not spec.is_classification else "AUTO", max(K, 1),
                                      tweedie_power=float(p.get("tweedie_power", 1.5)),
                                      quantile_alpha=float(p.get("quantile_alpha", 0.5)),
                                      huber_alpha=float(p.get("huber_alpha", 0.9)))
        if not bool(ok.all()):
            X = X[ok]
            Y = Y[ok] if Y is not None else None
        w = spec.w_tensor()
        w = None if w is None else w[ok].to(torch.float32)
        P = X.shape[1]
        out_dim = P if ae else K
        ckpt = p.get("checkpoint")
        if ckpt is not None:
            from ..core import dkv
            prev = dkv.get(ckpt) if isinstance(ckpt, str) else ckpt
            self._layers = copy.deepcopy(prev._layers)
            self._processed = getattr(prev, "_processed", 0.0)
        else:
            self._layers = self._build(P, out_dim, K > 1)
            self._processed = 0.0
        self._train_loop(spec, X, Y, w, ae, K)
        self._output["model_summary"] = {
            "layers": [P] + [L.fout for L in self._layers],
            "activation": p.get("activation"), "epochs": self._epochs_done,
            "units": [L.fout for L in self._layers],
            "dropout": [float(p.get("input_dropout_ratio") or 0.0)] + [L.drop for L in self._layers[:-1]]}
        if p.get("variable_importances", True) and not ae:
            self._output["variable_importances"] = self._gedeon(di)

    def _loss_name(self, K, ae):
        loss = (self._parms.get("loss") or "Automatic").lower()
        if loss == "automatic":
            return "crossentropy" if K > 1 else "quadratic"
        return loss

    def _output_grad(self, Zo, yb, wb, inv_n, K, ae, xb):
        """dE/dnet of the output layer (already / n) and the per-row loss."""
        Lo = self._layers[-1]
        if K > 1:
            loss = self._loss_name(K, ae)
            _, dZ, lo = dl_ops.softmax(Zo, Lo.b, yb, wb, inv_n, "quadratic" if loss == "quadratic" else "crossentropy")
            return dZ, lo
        Zo += Lo.b.view(1, -1)
        t = xb if ae else yb
        loss = self._loss_name(K, ae)
        d = Zo - t
        if loss == "absolute":
            g, lo = torch.sign(d), d.abs()
        elif loss == "huber":
            delta = float(self._parms.get("huber_alpha", 0.9))
            g = torch.clamp(d, -delta, delta)
            lo = torch.where(d.abs() <= delta, 0.5 * d * d, delta * (d.abs() - 0.5 * delta))
        elif loss == "quantile":
            a = float(self._parms.get("quantile_alpha", 0.5))
            g = torch.where(d > 0, torch.full_like(d, 1 - a), torch.full_like(d, -a))
            lo = torch.where(d > 0, (1 - a) * d, -a * d)
        elif not ae and self._dist.family not in ("gaussian",):
            # Linear.setOutputLayerGradient: g = -2 * negHalfGradient(t, y)
            g = -2.0 * self._dist.neg_half_gradient(t, Zo)
            lo = d * d
        else:
            g, lo = 2.0 * d, d * d
        lo = lo.sum(1)
        if wb is not None:
            g = g * wb.view(-1, 1)
            lo = lo * wb
        return g * inv_n, lo

    def _train_loop(self, spec, X, Y, w, ae, K):
        """Iterations of train_samples_per_iteration samples.  One GPU runs
        mini-batch steps (hipGraph-captured).  Several GPUs run the
        reference's model averaging (DeepLearningTask.reduce/postGlobal):
        every rank trains its own copy for the iteration with no collective
        in the step, then ONE all-reduce averages weights, biases and the
        ADADELTA / momentum state; with elastic_averaging the consensus is
        the moving time-average of the per-iteration averages
        (DeepLearningModelInfo.timeAverage) and local models keep training,
        pulled toward it by elastic_averaging_regularization.  With
        train_samples_per_iteration=-2 the iteration size is re-tuned each
        iteration so that averaging costs target_ratio_comm_to_comp of the
        compute time (DeepLearningModel.java:310)."""
        p = self._parms
        W_ = cloud.world()
        single = W_ > 1 and bool(p.get("single_node_mode"))
        replicate = W_ > 1 and (bool(p.get("replicate_training_data", True)) or single)
        if replicate:
            # replicate_training_data: every rank holds the whole training set
            X = coll.all_gather_var(X)
            Y = None if Y is None else coll.all_gather_var(Y)
            w = None if w is None else coll.all_gather_var(w)
        n = X.shape[0]
        ntot = n if replicate else coll.allreduce_scalar(float(n))
        contrib = 1 if single else W_          # ranks whose samples count
        epochs = float(p.get("epochs", 10))
        mbs = int(p.get("mini_batch_size") or 1)
        # mini_batch_size=1 (the reference's per-row updates): a GPU batch that
        # still gives >= ~256 updates per epoch (ADADELTA's step size does not
        # grow with the batch, so progress per epoch follows the update count)
        bs = max(mbs, _MIN_GPU_BATCH) if mbs > 1 else int(min(1024, max(_MIN_GPU_BATCH, ntot // (256 * contrib))))
        n_min = n if replicate or W_ == 1 else int(coll.allreduce_scalar(float(n), op="min"))
        bs = max(1, min(bs, n_min))      # the same batch on every rank keeps the step counts aligned
        total_samples = epochs * ntot
        tspi = int(p.get("train_samples_per_iteration", -2))
        if tspi == 0:
            per_iter = float(ntot)
        elif tspi == -1:
            per_iter = float(ntot * contrib if replicate else ntot)
        elif tspi == -2:
            per_iter = float(ntot) if contrib == 1 else float(min(ntot * contrib, max(16 * bs * contrib, 1)))
        else:
            per_iter = max(float(tspi), float(bs * contrib))
        auto_tune = tspi == -2 and contrib > 1
        target_ratio = float(p.get("target_ratio_comm_to_comp", 0.05))
        ada = bool(p.get("adaptive_rate", True))
        rate0, anneal, decay = float(p["rate"]), float(p["rate_annealing"]), float(p["rate_decay"])
        mom_start, mom_ramp, mom_stable = float(p["momentum_start"]), float(p["momentum_ramp"]), \
            float(p["momentum_stable"])
        has_mom = (not ada) and (mom_start > 0 or mom_stable > 0)
        l1, l2 = float(p.get("l1", 0)), float(p.get("l2", 0))
        max_w2 = float(p.get("max_w2") or 3.4028235e38)
        sparsity = float(p.get("sparsity_beta") or 0.0) if ae else 0.0
        avg_act = [torch.zeros(L.fout, device=X.device) for L in self._layers[:-1]] if sparsity > 0 else None
        gen = torch.Generator(device=X.device).manual_seed(self._seed() * 31 + cloud.rank())
        # shuffle_training_data: a fresh permutation per pass; otherwise the
        # rows are walked in order -- unless one pass is one iteration over a
        # single-chunk shard, where DeepLearning.java:448 turns shuffling on
        shuffle = bool(p.get("shuffle_training_data")) or per_iter >= ntot or auto_tune
        elastic = contrib > 1 and bool(p.get("elastic_averaging"))
        self._ea = None
        self._ea_started = False
        t0 = time.time()
        max_rt = float(p.get("max_runtime_secs") or 0)
        self._scoring_history = []
        stop_rounds = int(p.get("stopping_rounds") or 0)
        smetric = (p.get("stopping_metric") or "auto").lower()
        if smetric == "auto":
            smetric = "logloss" if K > 1 else ("mse" if ae else "deviance")
        history, best = [], None
        hp = dict(K=K, ae=ae, bs=bs, ada=ada, rate0=rate0, anneal=anneal, decay=decay, mom_start=mom_start,
                  mom_ramp=mom_ramp, mom_stable=mom_stable, has_mom=has_mom, l1=l1, l2=l2, max_w2=max_w2,
                  sparsity=sparsity, ea_reg=float(p.get("elastic_averaging_regularization", 1e-3)) if elastic else 0.0)
        if elastic:
            self._ea = [(L.W.clone(), L.b.clone()) for L in self._layers]
        step_seed = self._seed() * 1000003 + 7 * cloud.rank()
        perm, pos = None, n
        samples_done = 0.0
        next_iter = per_iter
        it = 0
        nstep = 0
        valid_sample = self._valid_sample(spec)
        score_iv = float(p.get("score_interval", 5.0))
        duty = float(p.get("score_duty_cycle", 0.1))
        last_start = last_end = None
        iter_t0 = time.time()
        det = bool(p.get("reproducible"))
        prev_det = torch.are_deterministic_algorithms_enabled()
        if det:
            torch.use_deterministic_algorithms(True, warn_only=True)
        graph = self._step_graph(X, Y, w, hp, avg_act) if self._graph_ok(X, hp, avg_act) else None
        try:
            while samples_done < total_samples:
                if pos + bs > n:
                    perm = torch.randperm(n, generator=gen, device=X.device) if shuffle else \
                        torch.arange(n, device=X.device)
                    pos = 0
                S = graph.get("S", 1) if graph is not None else 1
                nstep0 = nstep
                if S > 1 and W_ == 1 and pos + S * bs <= n and \
                        samples_done + (S - 1) * bs * contrib < min(next_iter, total_samples):
                    # S steps in one replay (one GPU: no collective is paced by
                    # the step count); no iteration boundary inside the group
                    # -- its last step may end one, handled below as usual
                    graph["idxm"].copy_(perm[pos:pos + S * bs].view(S, bs))
                    graph["gm"].replay()
                    pos += S * bs
                    self._processed += S * bs * contrib
                    samples_done += S * bs * contrib
                    nstep += S
                    final = samples_done >= total_samples
                    idx = None
                else:
                    idx = perm[pos:pos + bs]
                    pos += bs
                if idx is not None:
                    if graph is not None:
                        # ONE graph launch per step: the batch gather, forward, backward,
                        # updates and the dropout-seed advance were captured once
                        graph["idx"].copy_(idx)
                        graph["g"].replay()
                    else:
                        xb = X.index_select(0, idx)
                        yb = None if Y is None else Y.index_select(0, idx)
                        wb = None if w is None else w.index_select(0, idx)
                        step_seed = (step_seed * 6364136223846793005 + 1442695040888963407) & ((1 << 63) - 1)
                        self._train_step(xb, yb, wb, step_seed, hp, avg_act)
                    self._processed += bs * contrib
                    samples_done += bs * contrib
                    nstep += 1
                    final = samples_done >= total_samples
                if samples_done >= next_iter or final:
                    it += 1
                    t_comp = time.time() - iter_t0
                    t_comm = 0.0
                    if contrib > 1 or single:
                        tc = time.time()
                        self._average_models(single, elastic)
                        t_comm = time.time() - tc
                    if auto_tune and t_comp > 0:
                        # DeepLearningModel.java:310: keep comm / comp near the target
                        corr = (t_comm / t_comp) / max(target_ratio, 1e-9)
                        if corr > 0 and (corr < 0.8 or corr > 1.2):
                            per_iter = min(float(ntot * contrib), max(float(bs * contrib), per_iter / corr))
                        per_iter = float(cloud.agree([per_iter])[0]) if cloud.is_distributed() else per_iter
                    next_iter = samples_done + per_iter
                    self._epochs_done = samples_done / max(ntot, 1)
                    now = time.time()
                    due = final or bool(p.get("score_each_iteration")) or last_start is None or (
                        (now - last_start) > score_iv and
                        (last_end - last_start) / max(now - last_start, 1e-9) < duty)
                    if cloud.is_distributed():
                        due = bool(cloud.agree([due])[0])
                    if due:
                        last_start = time.time()
                        swapped = None
                        if elastic and self._ea_started:
                            # the consensus model is "the" model: score (and keep) it
                            swapped = [(L.W.clone(), L.b.clone()) for L in self._layers]
                            for L, (We, be) in zip(self._layers, self._ea):
                                L.W.copy_(We)
                                L.b.copy_(be)
                        entry = self._score_history_entry(spec, X, Y, w, ae, K, t0, valid_sample)
                        last_end = time.time()
                        self._scoring_history.append(entry)
                        val = entry.get(("validation_" if valid_sample is not None else "training_") + smetric)
                        history.append(val)
                        if val is not None and p.get("overwrite_with_best_model", True):
                            better = best is None or (val < best[0] if smetric in _LESS_IS_BETTER else val > best[0])
                            if better:
                                best = (val, [(L.W.clone(), L.b.clone()) for L in self._layers])
                        if swapped is not None:
                            for L, (Wl, bl) in zip(self._layers, swapped):
                                L.W.copy_(Wl)
                                L.b.copy_(bl)
                        if self._stop_on_error(entry, K, ae):
                            break
                        if stop_rounds > 0 and ScoreKeeper.stop_early(history, stop_rounds,
                                                                      float(p.get("stopping_tolerance", 0.0)),
                                                                      smetric in _LESS_IS_BETTER, metric=smetric):
                            break
                    iter_t0 = time.time()
                # job progress / cancel and the max_runtime_secs clock, agreed across
                # ranks every 64 mini-batches (not per step: a 0.14 ms step)
                if nstep // 64 != nstep0 // 64 or final:
                    _, timed_out = self._tick(samples_done, total_samples, None, False, t0, max_rt)
                    if timed_out:
                        if contrib > 1 or single:
                            self._average_models(single, elastic)
                        break
        finally:
            if det:
                torch.use_deterministic_algorithms(prev_det, warn_only=True)
        self._epochs_done = samples_done / max(ntot, 1)
        if elastic and self._ea is not None:
            # the consensus (elastic average) is the model
            for L, (We, be) in zip(self._layers, self._ea):
                L.W.copy_(We)
                L.b.copy_(be)
        if best is not None and p.get("overwrite_with_best_model", True):
            for L, (Wb, bb) in zip(self._layers, best[1]):
                L.W.copy_(Wb)
                L.b.copy_(bb)
        if p.get("export_weights_and_biases"):
            self._export_weights()

    def _average_models(self, single, elastic):
        """Model averaging at an iteration boundary: one bucketed all-reduce of
        every layer's weights, biases and optimizer state (divided by the
        number of ranks), or rank 0's model broadcast (single_node_mode)."""
        W_ = cloud.world()
        ts = []
        for L in self._layers:
            ts += [L.W, L.b] + [v for _, v in sorted(L.state.items()) if v is not None]
        if single:
            for t in ts:
                coll.broadcast_(t, 0)
            return
        if elastic:
            local = [(L.W.clone(), L.b.clone()) for L in self._layers]
        coll.allreduce_many_(ts)
        for t in ts:
            t.div_(W_)
        if elastic:
            # DeepLearningModelInfo.timeAverage: consensus <- (1 - pa) consensus
            # + pa * node average; the local models resume from their own weights
            pa = float(self._parms.get("elastic_averaging_moving_rate", 0.9))
            first = getattr(self, "_ea_started", False) is False
            for (We, be), L in zip(self._ea, self._layers):
                if first or pa == 1:
                    We.copy_(L.W)
                    be.copy_(L.b)
                else:
                    We.mul_(1 - pa).add_(L.W, alpha=pa)
                    be.mul_(1 - pa).add_(L.b, alpha=pa)
            self._ea_started = True
            for L, (Wl, bl) in zip(self._layers, local):
                L.W.copy_(Wl)
                L.b.copy_(bl)

    def _export_weights(self):
        """export_weights_and_biases (DeepLearning.java:354): one frame per
        weight matrix and bias vector in the DKV, keyed by the model id."""
        from ..core import dkv
        wk, bk = [], []
        for i, L in enumerate(self._layers):
            kw, kb = f"{self.model_id}.weights.{i}", f"{self.model_id}.biases.{i}"
            dkv.put(kw, H2OFrame.from_tensor(L.W.detach().float()))
            dkv.put(kb, H2OFrame.from_tensor(L.b.detach().float().view(-1, 1)))
            wk.append({"name": kw})
            bk.append({"name": kb})
        self._output["weights"] = wk
        self._output["biases"] = bk

    def _train_step(self, xb, yb, wb, step_seed, hp, avg_act=None, seed_dev=None):
        """One mini-batch step.  On the GPU, networks the fused kernels cover
        run dl_ops.mlp_step (three hand-written kernels, no library GEMM);
        otherwise forward, output gradient, backward through the HIP bwd
        kernel + GEMMs, per-row update kernels.  With seed_dev the dropout
        seed is read from device memory (graph replays)."""
        K, ae, bs = hp["K"], hp["ae"], xb.shape[0]
        kind = self._fused_kind(hp, avg_act) if xb.device.type == "cuda" else None
        if kind is not None:
            self._fused_step(xb, None, yb, wb, step_seed, hp, kind, seed_dev, False)
            return
        acts, zs = self._forward(xb, True, step_seed, seed_dev)
        dZ, _ = self._output_grad(zs[-1], yb, wb, 1.0 / bs, K, ae, xb)
        grads = []
        for li in range(len(self._layers) - 1, -1, -1):
            L = self._layers[li]
            if li == len(self._layers) - 1:
                db = dZ.sum(0)
            dW = dl_ops.gemm(dZ.t(), acts[li])
            grads.append((li, dW, db))
            if li > 0:
                dA = dl_ops.gemm(dZ, L.W)
                Lp = self._layers[li - 1]
                dZ, db = dl_ops.bwd(dA, acts[li], zs[li - 1], Lp.act, Lp.drop, seed=step_seed + 7919 * li,
                                    seed_dev=seed_dev)
        ea = getattr(self, "_ea", None)
        if ea is not None and hp.get("ea_reg", 0.0) > 0 and getattr(self, "_ea_started", False):
            # elastic averaging (Neurons.java:262): gradient += reg * (w - w_consensus)
            reg = hp["ea_reg"]
            grads = [(li, dW + reg * (self._layers[li].W - ea[li][0]),
                      db + reg * (self._layers[li].b - ea[li][1])) for (li, dW, db) in grads]
        if avg_act is not None:
            for li in range(len(self._layers) - 1):
                avg_act[li].mul_(0.999).add_(0.001 * acts[li + 1].mean(0))
        for (li, dW, db) in grads:
            L = self._layers[li]
            dl_ops.update(L.W, dW.contiguous(), L.b, db.contiguous(), L.state, self._update_params(hp, li),
                          avg_act=avg_act[li] if (avg_act is not None and li < len(avg_act)) else None)

    def _update_params(self, hp, li):
        """Per-layer update knobs at the current sample count: rate annealing
        and decay per layer, the momentum ramp (Neurons.java rate / momentum)."""
        p = self._parms
        m = hp["mom_start"]
        if hp["mom_ramp"] > 0:
            m = hp["mom_stable"] if self._processed >= hp["mom_ramp"] else \
                hp["mom_start"] + (hp["mom_stable"] - hp["mom_start"]) * self._processed / hp["mom_ramp"]
        r = hp["rate0"] / (1 + hp["anneal"] * self._processed) * hp["decay"] ** li
        return dl_ops.UpdateParams(ada=hp["ada"], rho=float(p["rho"]), eps=float(p["epsilon"]),
                                   rate=r * (1 - m) if not hp["ada"] else 0.0, momentum=m,
                                   nesterov=bool(p.get("nesterov_accelerated_gradient", True)),
                                   has_momenta=hp["has_mom"], l1=hp["l1"], l2=hp["l2"], max_w2=hp["max_w2"],
                                   sparsity_beta=hp["sparsity"],
                                   average_activation=float(p.get("average_activation") or 0.0))

    def _fused_kind(self, hp, avg_act):
        """Output kind of the fused HIP step (dl_ops.mlp_step: 0 softmax +
        CrossEntropy, 1 softmax + Quadratic, 2 linear + Quadratic Gaussian),
        or None for the networks it does not cover: maxout units,
        autoencoders, other regression losses / distributions, sparsity and
        elastic-averaging terms, layers beyond the LDS budget."""
        import os
        if os.environ.get("H2O3_DL_FUSED", "1") != "1" or avg_act is not None or hp.get("ea_reg", 0.0) > 0 \
                or hp["ae"]:
            return None
        if any(L.act not in dl_ops._FUSED_ACTS or L.k != 1 for L in self._layers[:-1]) or self._layers[-1].k != 1:
            return None
        K = hp["K"]
        loss = self._loss_name(K, False)
        if K > 1:
            kind = 1 if loss == "quadratic" else 0
        else:
            dist = getattr(self, "_dist", None)
            if loss != "quadratic" or (dist is not None and dist.family != "gaussian"):
                return None
            kind = 2
        widths = [self._layers[0].W.shape[1]] + [L.W.shape[0] for L in self._layers]
        return kind if dl_ops.mlp_fits(widths) else None

    def _fused_step(self, X, idx, Y, w, step_seed, hp, kind, seed_dev, advance):
        p = self._parms
        bs = int(idx.shape[0]) if idx is not None else int(X.shape[0])
        if not hasattr(self, "_mlp_bufs"):
            self._mlp_bufs = {}
        dl_ops.mlp_step(X, idx, Y, w, self._layers, [L.act for L in self._layers[:-1]],
                        [L.drop for L in self._layers[:-1]], float(p.get("input_dropout_ratio") or 0.0), kind,
                        1.0 / bs, [self._update_params(hp, li) for li in range(len(self._layers))],
                        seed=step_seed, seed_dev=seed_dev, advance=advance, bufs=self._mlp_bufs)

    def _graph_ok(self, X, hp, avg_act):
        """HIP-graph the step when nothing in it changes between steps on the
        host side: ADADELTA (no rate / momentum schedule), no sparsity
        running averages, no elastic-averaging pull (its consensus changes
        between iterations).  Model averaging keeps collectives out of the
        step, so several ranks graph their steps too."""
        import os
        return X.device.type == "cuda" and hp["ada"] and avg_act is None and not hp.get("ea_reg") and \
            os.environ.get("H2O3_DL_GRAPH", "1") == "1"

    def _step_graph(self, X, Y, w, hp, avg_act):
        """Capture gather + step + seed advance into one hipGraph (static
        batch buffers, weights / ADADELTA state updated in place)."""
        bs = hp["bs"]
        dev = X.device
        gs = {"idx": torch.zeros(bs, dtype=torch.int64, device=dev),
              "seed": torch.tensor([self._seed() * 1000003 & ((1 << 62) - 1)], dtype=torch.int64, device=dev)}

        kind = self._fused_kind(hp, avg_act)

        def body(idx=None):
            idx = gs["idx"] if idx is None else idx
            if kind is not None:
                # the whole step in three kernels: gather + forward + backward,
                # weight gradients, updates + seed advance
                self._fused_step(X, idx, Y, w, 0, hp, kind, gs["seed"], True)
                return
            xb = X.index_select(0, idx)
            yb = None if Y is None else Y.index_select(0, idx)
            wb = None if w is None else w.index_select(0, idx)
            dl_ops.seed_advance(gs["seed"])
            self._train_step(xb, yb, wb, 0, hp, avg_act, seed_dev=gs["seed"])
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        # The warm-up steps only allocate the optimizer state and let the GEMM
        # library pick its algorithms: weights, biases, optimizer state and the
        # dropout seed are snapshotted first and restored after capture, so the
        # model trains on exactly the batches the caller replays (and the
        # sample counters are untouched).
        saved = [(L.W.clone(), L.b.clone(), {k: v.clone() for k, v in L.state.items() if v is not None})
                 for L in self._layers]
        seed0 = gs["seed"].clone()
        with torch.cuda.stream(side):
            for i in range(2):
                gs["idx"].copy_(torch.arange(i * bs, (i + 1) * bs, device=dev) % X.shape[0])
                body()
        cur.wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with graphs.capture(g):
            body()
        # S consecutive steps in one graph (their batches in one [S, bs] index
        # buffer): a small net's step is ~10 us of GPU work and ~37 us of host
        # time per replay + index copy, so single-step replays are launch bound
        S = int(os.environ.get("H2O3_DL_GRAPH_STEPS", "8"))
        if S > 1:
            gs["idxm"] = torch.zeros((S, bs), dtype=torch.int64, device=dev)
            gm = torch.cuda.CUDAGraph()
            with graphs.capture(gm):
                for k in range(S):
                    body(gs["idxm"][k])
            gs["gm"], gs["S"] = gm, S
        for L, (Wb, bb, st) in zip(self._layers, saved):
            L.W.copy_(Wb)
            L.b.copy_(bb)
            for k, v in L.state.items():
                if v is not None:
                    v.copy_(st[k]) if k in st else v.zero_()   # state created by the warm-up starts at 0
        gs["seed"].copy_(seed0)
        gs["g"] = g
        return gs

    def _stop_on_error(self, entry, K, ae):
        """classification_stop / regression_stop on the training error."""
        p = self._parms
        if K > 1:
            cs = float(p.get("classification_stop", 0.0))
            err = entry.get("training_classification_error")
            return cs >= 0 and err is not None and err <= cs
        rs = float(p.get("regression_stop", 1e-6))
        mse = entry.get("training_mse")
        return rs >= 0 and mse is not None and mse <= rs

    def _score_history_entry(self, spec, X, Y, w, ae, K, t0, valid=None):
        from .tree.gbm import H2OGradientBoostingEstimator as _G
        p = self._parms
        entry = {"timestamp": time.time(), "duration_s": time.time() - t0, "epochs": self._epochs_done,
                 "samples": self._processed}
        ns = int(p.get("score_training_samples") or 0)
        Xs, Ys = X, Y
        if 0 < ns < X.shape[0]:
            sel = torch.randperm(X.shape[0], device=X.device)[:ns]
            Xs = X[sel]
            Ys = None if Y is None else Y[sel]
        with torch.no_grad():
            out = self._predict_matrix(Xs)
        if ae:
            entry["training_mse"] = float(((out - Xs) ** 2).mean())
            return entry
        if K > 1:
            yy = Ys
            raw = out
            if K == 2:
                m = mm.binomial_metrics(yy.to(torch.float64), raw[:, 1], None, spec.response_domain)
            else:
                m = mm.multinomial_metrics(yy, raw, None, spec.response_domain)
        else:
            pred = out[:, 0] * self._ysd + self._ymu
            m = mm.regression_metrics((Ys[:, 0] * self._ysd + self._ymu).to(torch.float64), pred, None, self._dist)
        _G._add_metrics(entry, "training", m)
        if valid is not None:
            vm = self._metrics_from_raw(spec, valid, self._predict_raw(valid))
            _G._add_metrics(entry, "validation", vm)
        return entry

    # ------------------------------------------------------------------ scoring
    def _predict_matrix(self, X):
        """Output-layer values for a design matrix: class probabilities,
        standardized regression values or the reconstruction."""
        acts, zs = self._forward(X, False)
        Zo = zs[-1]
        Lo = self._layers[-1]
        if self._K > 1:
            P, _, _ = dl_ops.softmax(Zo, Lo.b, None, want_grad=False)
            return P
        Zo += Lo.b.view(1, -1)
        return Zo

    def _predict_raw(self, frame):
        X, _ = self._design(frame)
        with torch.no_grad():
            out = self._predict_matrix(X)
        if self._ae or self._K > 1:
            return out
        f = out * self._ysd + self._ymu
        if self._dist.family not in ("gaussian", "laplace", "quantile", "huber"):
            f = self._dist.linkinv(f)
        return f

    def _gedeon(self, di):
        """Gedeon (1997) input importance from the weight matrices."""
        with torch.no_grad():
            imp = None
            for L in reversed(self._layers):
                W = L.W.abs()
                if L.k > 1:
                    W = W.view(L.fout, L.k, L.fin).sum(1)
                W = W / W.sum(1, keepdim=True).clamp_min(1e-30)
                imp = W if imp is None else imp @ W
            v = imp.sum(0)
        vi = {}
        for n_, val in zip(di.coef_names, v.tolist()):
            base = n_.split(".")[0] if n_ not in di.num_cols else n_
            vi[base] = vi.get(base, 0.0) + val
        return vi

    def predict(self, test_data, **kw):
        if self._ae:
            out = self._predict_raw(test_data)
            names = [f"reconstr_{n}" for n in self._dinfo.coef_names]
            return H2OFrame.from_vecs([Vec(out[:, j].contiguous(), T_REAL) for j in range(out.shape[1])], names)
        return super().predict(test_data, **kw)

    def anomaly(self, test_data, per_feature=False):
        X, _ = self._design(test_data)
        with torch.no_grad():
            out = self._predict_matrix(X)
        err = (out - X) ** 2
        if per_feature:
            return H2OFrame.from_vecs([Vec(err[:, j].contiguous(), T_REAL) for j in range(err.shape[1])],
                                      [f"reconstr_{n}.SE" for n in self._dinfo.coef_names])
        return H2OFrame.from_vecs([Vec(err.mean(1).contiguous(), T_REAL)], ["Reconstruction.MSE"])

    def deepfeatures(self, test_data, layer):
        X, _ = self._design(test_data)
        with torch.no_grad():
            acts, _ = self._forward(X, False)
        h = acts[layer + 1]
        return H2OFrame.from_vecs([Vec(h[:, j].contiguous(), T_REAL) for j in range(h.shape[1])],
                                  [f"DF.L{layer + 1}.C{j + 1}" for j in range(h.shape[1])])

    def weights(self, matrix_id=0):
        """Weight matrix frame (needs export_weights_and_biases=True, as the
        reference's model.weights())."""
        from ..core import dkv
        ws = self._output.get("weights")
        if not ws:
            raise ValueError("weights are only available with export_weights_and_biases=True")
        return dkv.get(ws[matrix_id]["name"])

    def biases(self, vector_id=0):
        from ..core import dkv
        bs_ = self._output.get("biases")
        if not bs_:
            raise ValueError("biases are only available with export_weights_and_biases=True")
        return dkv.get(bs_[vector_id]["name"])

    def _score_unsupervised(self, spec):
        if self._ae:
            X, _ = self._design(spec.frame)
            with torch.no_grad():
                out = self._predict_matrix(X)
            mse = float(((out - X) ** 2).mean())
            self._training_metrics = mm.ModelMetricsAutoEncoder(MSE=mse, RMSE=math.sqrt(mse), nobs=spec.frame.nrows)

    def scoring_history(self):
        return self._scoring_history
