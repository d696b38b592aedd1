"""Distribution families and link functions.

Reference: h2o-core/src/main/java/hex/Distribution.java,
hex/DistributionFactory.java, hex/LinkFunction*.java (and the GBM leaf
estimates `gammaNum/gammaDenom` used by GBM.GammaPass, gbm/GBM.java:1286).

All functions operate on device tensors (vectorized over rows).  `f` is the
link-scale prediction, `y` the response.
"""
from __future__ import annotations

import math

import torch

FAMILIES = ("AUTO", "bernoulli", "quasibinomial", "multinomial", "gaussian", "poisson", "gamma", "tweedie",
            "laplace", "quantile", "huber", "modified_huber", "fractionalbinomial", "negativebinomial",
            "ordinal", "custom")


def _exp(f):
    return torch.exp(torch.clamp(f, max=88.0 if f.dtype == torch.float32 else 700.0))


class Distribution:
    family = "gaussian"
    link = "identity"

    def __init__(self, tweedie_power=1.5, quantile_alpha=0.5, huber_alpha=0.9, theta=1e-10):
        self.tweedie_power = tweedie_power
        self.quantile_alpha = quantile_alpha
        self.huber_alpha = huber_alpha
        self.huber_delta = None
        self.theta = theta

    # link
    def link_fn(self, mu):
        if self.link == "identity":
            return mu
        if self.link == "logit":
            mu = torch.clamp(mu, 1e-15, 1 - 1e-15) if isinstance(mu, torch.Tensor) else min(max(mu, 1e-15), 1 - 1e-15)
            return torch.log(mu / (1 - mu)) if isinstance(mu, torch.Tensor) else math.log(mu / (1 - mu))
        if self.link == "log":
            return torch.log(mu) if isinstance(mu, torch.Tensor) else math.log(max(mu, 1e-300))
        raise ValueError(self.link)

    def linkinv(self, f):
        if self.link == "identity":
            return f
        if self.link == "logit":
            return torch.sigmoid(f)
        if self.link == "log":
            return _exp(f)
        raise ValueError(self.link)

    # boosting
    def neg_half_gradient(self, y, f):
        return y - f

    def gamma_num(self, w, y, z, f):
        return w * z

    def gamma_denom(self, w, y, z, f):
        return w

    def gamma(self, num, den):
        return num / den if den != 0 else 0.0

    def init_f(self, y, w, offset=None):
        mu = float((w * y).sum() / w.sum())
        return self.link_fn(mu) if self.link != "identity" else mu

    # deviance (per row, weighted later)
    def deviance(self, w, y, f_mu):
        return w * (y - f_mu) ** 2

    # second-order stats (XGBoost-style)
    def grad_hess(self, y, f):
        return f - y, torch.ones_like(f)

    @property
    def is_classification(self):
        return False


class Gaussian(Distribution):
    family = "gaussian"


class Bernoulli(Distribution):
    family = "bernoulli"
    link = "logit"

    def neg_half_gradient(self, y, f):
        return y - torch.sigmoid(f)

    def gamma_denom(self, w, y, z, f):
        p = y - z
        return w * p * (1 - p)

    def deviance(self, w, y, mu):
        mu = torch.clamp(mu, 1e-15, 1 - 1e-15)
        return -2 * w * (y * torch.log(mu) + (1 - y) * torch.log(1 - mu))

    def grad_hess(self, y, f):
        p = torch.sigmoid(f)
        return p - y, torch.clamp(p * (1 - p), min=1e-16)

    @property
    def is_classification(self):
        return True


class QuasiBinomial(Bernoulli):
    family = "quasibinomial"


class FractionalBinomial(Bernoulli):
    family = "fractionalbinomial"


class ModifiedHuber(Bernoulli):
    family = "modified_huber"

    def neg_half_gradient(self, y, f):
        yf = (2 * y - 1) * f
        return torch.where(yf < -1, 2 * (2 * y - 1), torch.where(yf > 1, torch.zeros_like(f), -f * (2 * y - 1) ** 2 + (2 * y - 1)))

    def linkinv(self, f):
        return torch.clamp((f + 1) / 2, 0, 1)


class Multinomial(Distribution):
    family = "multinomial"
    link = "log"

    @property
    def is_classification(self):
        return True


class Poisson(Distribution):
    family = "poisson"
    link = "log"

    def neg_half_gradient(self, y, f):
        return y - _exp(f)

    def gamma_num(self, w, y, z, f):
        return w * y

    def gamma_denom(self, w, y, z, f):
        return w * _exp(f)

    def gamma(self, num, den):
        if num <= 0 or den <= 0:
            return -19.0 if num <= 0 else 0.0
        return math.log(num / den)

    def deviance(self, w, y, mu):
        t = torch.where(y > 0, y * torch.log(y / mu.clamp_min(1e-300)), torch.zeros_like(y))
        return 2 * w * (t - (y - mu))

    def grad_hess(self, y, f):
        mu = _exp(f)
        return mu - y, mu


class Gamma(Distribution):
    family = "gamma"
    link = "log"

    def neg_half_gradient(self, y, f):
        return y * _exp(-f) - 1

    def gamma_num(self, w, y, z, f):
        return w * y * _exp(-f)

    def gamma_denom(self, w, y, z, f):
        return w

    def gamma(self, num, den):
        if num <= 0 or den <= 0:
            return 0.0
        return math.log(num / den)

    def deviance(self, w, y, mu):
        return 2 * w * (-torch.log(y / mu) + (y - mu) / mu)

    def grad_hess(self, y, f):
        e = y * _exp(-f)
        return 1 - e, e


class Tweedie(Distribution):
    family = "tweedie"
    link = "log"

    def neg_half_gradient(self, y, f):
        p = self.tweedie_power
        return y * _exp(f * (1 - p)) - _exp(f * (2 - p))

    def gamma_num(self, w, y, z, f):
        return w * y * _exp(f * (1 - self.tweedie_power))

    def gamma_denom(self, w, y, z, f):
        return w * _exp(f * (2 - self.tweedie_power))

    def gamma(self, num, den):
        if num <= 0 or den <= 0:
            return -19.0 if num <= 0 else 0.0
        return math.log(num / den)

    def deviance(self, w, y, mu):
        p = self.tweedie_power
        t1 = torch.where(y > 0, torch.pow(y, 2 - p) / ((1 - p) * (2 - p)), torch.zeros_like(y))
        return 2 * w * (t1 - y * torch.pow(mu, 1 - p) / (1 - p) + torch.pow(mu, 2 - p) / (2 - p))

    def grad_hess(self, y, f):
        p = self.tweedie_power
        a, b = _exp(f * (1 - p)), _exp(f * (2 - p))
        return -y * a + b, -y * (1 - p) * a + (2 - p) * b


class Laplace(Distribution):
    family = "laplace"

    def neg_half_gradient(self, y, f):
        return torch.sign(y - f)

    def deviance(self, w, y, mu):
        return w * (y - mu).abs()


class Quantile(Distribution):
    family = "quantile"

    def neg_half_gradient(self, y, f):
        a = self.quantile_alpha
        return torch.where(y > f, torch.full_like(f, a), torch.full_like(f, a - 1))

    def deviance(self, w, y, mu):
        a = self.quantile_alpha
        d = y - mu
        return w * torch.where(d > 0, a * d, (a - 1) * d)


class Huber(Distribution):
    family = "huber"

    def neg_half_gradient(self, y, f):
        d = y - f
        delta = self.huber_delta if self.huber_delta is not None else float("inf")
        return torch.where(d.abs() <= delta, d, delta * torch.sign(d))

    def deviance(self, w, y, mu):
        d = (y - mu).abs()
        delta = self.huber_delta if self.huber_delta is not None else float("inf")
        return w * torch.where(d <= delta, d * d, 2 * delta * d - delta * delta)


class NegativeBinomial(Poisson):
    family = "negativebinomial"


_REG = {"gaussian": Gaussian, "bernoulli": Bernoulli, "quasibinomial": QuasiBinomial,
        "fractionalbinomial": FractionalBinomial, "multinomial": Multinomial, "poisson": Poisson,
        "gamma": Gamma, "tweedie": Tweedie, "laplace": Laplace, "quantile": Quantile, "huber": Huber,
        "modified_huber": ModifiedHuber, "negativebinomial": NegativeBinomial}


def get_distribution(name, nclasses=1, **kw):
    n = (name or "AUTO")
    if n in ("AUTO", "auto"):
        n = "gaussian" if nclasses == 1 else ("bernoulli" if nclasses == 2 else "multinomial")
    if n == "custom":
        from ..core.udf import CustomDistribution
        if kw.get("custom_distribution_func") is None:
            raise ValueError("distribution='custom' needs custom_distribution_func (h2o.upload_custom_distribution)")
        return CustomDistribution(kw.pop("custom_distribution_func"), **kw)
    kw.pop("custom_distribution_func", None)
    if n not in _REG:
        raise ValueError(f"unsupported distribution {name}")
    return _REG[n](**kw)
