"""Deep Learning (multi-layer perceptron, autoencoder).

Reference: hex/deeplearning/DeepLearning.java, DeepLearningModel.java,
Neurons.java (Tanh / Rectifier / Maxout / ExpRectifier (+WithDropout)),
Dropout.java, DeepLearningTask.java (Hogwild SGD per node, model averaging
across nodes), ADADELTA adaptive rate (rho, epsilon), momentum schedule,
L1/L2, input/hidden dropout, autoencoder with reconstruction error, Gedeon
variable importance, deep features.

MI355X design: the standardized / one-hot design matrix is one HBM tensor;
training runs mini-batches (the reference's per-row Hogwild updates are a
CPU-cache idiom) of bf16-capable GEMMs through torch on the GPU, the
optimizer is ADADELTA with the reference's defaults; with several GPUs each
rank trains on its row shard and gradients are averaged with a bucketed
RCCL all-reduce every step (synchronous data parallel instead of the
reference's periodic model averaging).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch
import torch.nn as nn

from ..core.frame import H2OFrame
from ..core.vec import T_REAL, Vec
from ..parallel import cloud
from ..parallel import collectives as coll
from . import metrics as mm
from .base import H2OEstimator
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


class _Maxout(nn.Module):
    def __init__(self, fin, fout, k=2):
        super().__init__()
        self.lin = nn.Linear(fin, fout * k)
        self.k = k
        self.fout = fout

    def forward(self, x):
        return self.lin(x).view(x.shape[0], self.fout, self.k).max(2).values


def _act(name):
    n = name.lower().replace("withdropout", "")
    if n == "tanh":
        return nn.Tanh()
    if n == "rectifier":
        return nn.ReLU()
    if n == "exprectifier":
        return nn.ELU()
    return None


class H2ODeepLearningEstimator(H2OEstimator):
    algo = "deeplearning"
    _defaults = DL_DEFAULTS

    def __init__(self, **kw):
        super().__init__(**kw)
        if self._parms.get("autoencoder"):
            self.supervised_learning = False

    def _build_net(self, P, out_dim):
        p = self._parms
        hidden = list(p.get("hidden") or [200, 200])
        act = p.get("activation", "Rectifier")
        drop = "withdropout" in act.lower()
        hdr = p.get("hidden_dropout_ratios") or ([0.5] * len(hidden) if drop else [0.0] * len(hidden))
        layers = []
        if float(p.get("input_dropout_ratio", 0) or 0) > 0:
            layers.append(nn.Dropout(float(p["input_dropout_ratio"])))
        fin = P
        self._hidden_idx = []
        for h, d in zip(hidden, hdr):
            if act.lower().startswith("maxout"):
                layers.append(_Maxout(fin, h))
            else:
                layers.append(nn.Linear(fin, h))
                layers.append(_act(act))
            self._hidden_idx.append(len(layers) - 1)
            if d and d > 0:
                layers.append(nn.Dropout(d))
            fin = h
        layers.append(nn.Linear(fin, out_dim))
        net = nn.Sequential(*layers)
        # UniformAdaptive init (reference Neurons: U(-sqrt(6/(fan_in+fan_out)), +))
        g = torch.Generator().manual_seed(self._seed())
        scale = float(p.get("initial_weight_scale", 1.0))
        dist = (p.get("initial_weight_distribution") or "UniformAdaptive").lower()
        for m in net.modules():
            if isinstance(m, nn.Linear):
                fi, fo = m.in_features, m.out_features
                with torch.no_grad():
                    if dist == "uniform":
                        m.weight.uniform_(-scale, scale, generator=g)
                    elif dist == "normal":
                        m.weight.normal_(0, scale, generator=g)
                    else:
                        r = math.sqrt(6.0 / (fi + fo))
                        m.weight.uniform_(-r, r, generator=g)
                    m.bias.zero_()
        return net.to(cloud.device())

    def _seed(self):
        s = self._parms.get("seed", -1)
        return 12345 if s is None or s == -1 else int(s) & 0x7FFFFFFF

    def _fit(self, spec):
        p = self._parms
        torch.manual_seed(self._seed())
        di = DataInfo(spec.frame, spec.x, standardize=bool(p.get("standardize", True)),
                      use_all_factor_levels=bool(p.get("use_all_factor_levels", True)),
                      missing_values_handling=p.get("missing_values_handling"), pad_to=0)
        self._dinfo = di
        X, ok = di.expand(spec.frame, pad=False)
        ae = bool(p.get("autoencoder"))
        K = spec.nclasses if spec.is_classification else 1
        if not ae:
            y = spec.y_tensor()
            if spec.is_classification:
                ok = ok & (y >= 0)
                Y = y.long()
            else:
                yf = y.to(torch.float32)
                ok = ok & ~torch.isnan(yf)
                # standardize regression targets (reference normalizes the response)
                self._ymu = coll.allreduce_scalar(float(yf[ok].sum())) / max(coll.allreduce_scalar(float(ok.sum())), 1)
                var = coll.allreduce_scalar(float(((yf[ok] - self._ymu) ** 2).sum())) / max(coll.allreduce_scalar(float(ok.sum())) - 1, 1)
                self._ysd = math.sqrt(var) if var > 0 else 1.0
                Y = ((yf - self._ymu) / self._ysd).view(-1, 1)
        X = X[ok]
        if not ae:
            Y = Y[ok]
        w = spec.w_tensor()
        w = None if w is None else w[ok]
        P = X.shape[1]
        out_dim = P if ae else (K if K > 1 else 1)
        if p.get("checkpoint") is not None:
            from ..core import dkv
            prev = dkv.get(p["checkpoint"]) if isinstance(p["checkpoint"], str) else p["checkpoint"]
            net = prev._net
        else:
            net = self._build_net(P, out_dim)
        self._net = net
        if bool(p.get("adaptive_rate", True)):
            opt = torch.optim.Adadelta(net.parameters(), lr=1.0, rho=float(p["rho"]), eps=float(p["epsilon"]))
        else:
            opt = torch.optim.SGD(net.parameters(), lr=float(p["rate"]), momentum=float(p.get("momentum_stable", 0)),
                                  nesterov=bool(p.get("nesterov_accelerated_gradient")) and float(p.get("momentum_stable", 0)) > 0)
        l1, l2 = float(p.get("l1", 0)), float(p.get("l2", 0))
        n = X.shape[0]
        ntot = coll.allreduce_scalar(float(n))
        epochs = float(p.get("epochs", 10))
        bs = max(int(p.get("mini_batch_size", 1)), 32)   # GPU minibatch (reference default 1 = Hogwild per row)
        bs = min(bs if p.get("mini_batch_size", 1) > 1 else 256, max(n, 1))
        steps = int(math.ceil(epochs * ntot / (bs * cloud.world())))
        loss_name = (p.get("loss") or "Automatic").lower()
        gen = torch.Generator(device=X.device).manual_seed(self._seed() + cloud.rank())
        t0 = time.time()
        max_rt = float(p.get("max_runtime_secs") or 0)
        self._scoring_history = []
        net.train()
        params = [q for q in net.parameters()]
        lr0 = float(p.get("rate", 0.005))
        for step in range(max(1, steps)):
            idx = torch.randint(0, max(n, 1), (bs,), generator=gen, device=X.device)
            xb = X[idx]
            out = net(xb)
            if ae:
                loss = ((out - xb) ** 2).mean()
            elif K > 1:
                loss = nn.functional.cross_entropy(out, Y[idx], reduction="none")
                loss = (loss * w[idx]).mean() if w is not None else loss.mean()
            else:
                d = out - Y[idx]
                if loss_name == "absolute":
                    l_ = d.abs()
                elif loss_name == "huber":
                    l_ = torch.nn.functional.huber_loss(out, Y[idx], reduction="none")
                else:
                    l_ = d * d
                loss = (l_.view(-1) * w[idx]).mean() if w is not None else l_.mean()
            if l1 > 0 or l2 > 0:
                for m in net.modules():
                    if isinstance(m, nn.Linear):
                        if l1 > 0:
                            loss = loss + l1 * m.weight.abs().sum()
                        if l2 > 0:
                            loss = loss + 0.5 * l2 * (m.weight ** 2).sum()
            opt.zero_grad(set_to_none=False)
            loss.backward()
            if cloud.is_distributed():
                grads = [q.grad for q in params if q.grad is not None]
                coll.allreduce_many_(grads)
                for g_ in grads:
                    g_.div_(cloud.world())
            if not p.get("adaptive_rate", True):
                for gr in opt.param_groups:
                    gr["lr"] = lr0 / (1 + float(p.get("rate_annealing", 1e-6)) * step * bs)
            opt.step()
            if max_rt > 0 and time.time() - t0 > max_rt:
                break
            if step % max(1, steps // 10) == 0:
                self._scoring_history.append({"iterations": step, "epochs": step * bs * cloud.world() / max(ntot, 1),
                                              "training_loss": float(loss.detach())})
        net.eval()
        self._K = K
        self._ae = ae
        if p.get("variable_importances", True) and not ae:
            self._output["variable_importances"] = self._gedeon(di)
        self._output["model_summary"] = {"layers": [P] + list(p.get("hidden") or []) + [out_dim],
                                         "activation": p.get("activation"), "epochs": epochs}

    def _gedeon(self, di):
        """Gedeon (1997) input importance from the weight matrices."""
        lins = [m for m in self._net.modules() if isinstance(m, nn.Linear)]
        with torch.no_grad():
            imp = None
            for m in reversed(lins):
                W = m.weight.abs()
                W = W / W.sum(1, keepdim=True).clamp_min(1e-30)
                imp = W if imp is None else imp @ W
            v = imp.sum(0)
        names = di.coef_names
        vi = {}
        for n_, val in zip(names, v.tolist()):
            base = n_.split(".")[0] if n_ not in di.num_cols else n_
            vi[base] = vi.get(base, 0.0) + val
        return vi

    def _forward(self, frame):
        X, _ = self._dinfo.expand(frame, pad=False)
        with torch.no_grad():
            return self._net(X), X

    def _predict_raw(self, frame):
        out, X = self._forward(frame)
        if self._ae:
            return out
        if self._K > 1:
            return torch.softmax(out, 1)
        return (out * self._ysd + self._ymu)

    def predict(self, test_data, **kw):
        if self._ae:
            out = self._predict_raw(test_data)
            names = [f"reconstr_{n}" for n in self._dinfo.coef_names]
            return H2OFrame.from_vecs([Vec(out[:, j].contiguous(), T_REAL) for j in range(out.shape[1])], names)
        return super().predict(test_data, **kw)

    def anomaly(self, test_data, per_feature=False):
        out, X = self._forward(test_data)
        err = (out - X) ** 2
        if per_feature:
            return H2OFrame.from_vecs([Vec(err[:, j].contiguous(), T_REAL) for j in range(err.shape[1])],
                                      [f"reconstr_{n}.SE" for n in self._dinfo.coef_names])
        return H2OFrame.from_vecs([Vec(err.mean(1).contiguous(), T_REAL)], ["Reconstruction.MSE"])

    def deepfeatures(self, test_data, layer):
        X, _ = self._dinfo.expand(test_data, pad=False)
        idx = self._hidden_idx[layer]
        with torch.no_grad():
            h = self._net[: idx + 1](X)
        return H2OFrame.from_vecs([Vec(h[:, j].contiguous(), T_REAL) for j in range(h.shape[1])],
                                  [f"DF.L{layer + 1}.C{j + 1}" for j in range(h.shape[1])])

    def weights(self, matrix_id=0):
        lins = [m for m in self._net.modules() if isinstance(m, nn.Linear)]
        return H2OFrame.from_tensor(lins[matrix_id].weight.detach())

    def biases(self, vector_id=0):
        lins = [m for m in self._net.modules() if isinstance(m, nn.Linear)]
        return H2OFrame.from_tensor(lins[vector_id].bias.detach().view(-1, 1))

    def _score_unsupervised(self, spec):
        if self._ae:
            out, X = self._forward(spec.frame)
            mse = float(((out - X) ** 2).mean())
            self._training_metrics = mm.ModelMetricsAutoEncoder(MSE=mse, RMSE=math.sqrt(mse), nobs=spec.frame.nrows)
