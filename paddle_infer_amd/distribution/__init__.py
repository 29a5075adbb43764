"""``paddle.distribution`` (reference `python/paddle/distribution/`): probability distributions,
bijective transforms, KL registry.

Each Paddle distribution wraps the matching ``torch.distributions`` object (sampling runs on the
device RNG of the parameters' device; ``rsample`` is reparameterised where the family allows it)
and exposes Paddle's surface: ``batch_shape``, ``event_shape``, ``mean``, ``variance``,
``sample(shape)``, ``rsample(shape)``, ``entropy()``, ``log_prob``, ``prob``, ``probs``,
``kl_divergence(other)``; ``kl_divergence(p, q)`` / ``register_kl`` dispatch on the class pair.
"""
from __future__ import annotations

import torch
import torch.distributions as D

from . import transform  # noqa: F401
from .transform import *  # noqa: F401,F403

__all__ = ["Beta", "Categorical", "Dirichlet", "Distribution", "ExponentialFamily", "Multinomial",
           "Normal", "Uniform", "kl_divergence", "register_kl", "Independent",
           "TransformedDistribution", "Laplace", "LogNormal", "Gumbel", "Geometric", "Cauchy",
           "Bernoulli", "Poisson", "Exponential", "Gamma", "Binomial"]
__all__.extend(transform.__all__)


def _t(x, dtype=torch.float32):
    if isinstance(x, torch.Tensor):
        return x if x.is_floating_point() else x.to(dtype)
    return torch.as_tensor(x, dtype=dtype)


class Distribution:
    """Base class. Subclasses set ``self._d`` (a torch distribution)."""
    _d: D.Distribution

    def __init__(self, batch_shape=(), event_shape=()):
        self._batch_shape = tuple(batch_shape)
        self._event_shape = tuple(event_shape)

    @property
    def batch_shape(self):
        return tuple(self._d.batch_shape) if hasattr(self, "_d") else self._batch_shape

    @property
    def event_shape(self):
        return tuple(self._d.event_shape) if hasattr(self, "_d") else self._event_shape

    @property
    def mean(self):
        return self._d.mean

    @property
    def variance(self):
        return self._d.variance

    def sample(self, shape=()):
        with torch.no_grad():
            return self._d.sample(torch.Size(shape))

    def rsample(self, shape=()):
        return self._d.rsample(torch.Size(shape))

    def entropy(self):
        return self._d.entropy()

    def log_prob(self, value):
        return self._d.log_prob(_t(value))

    def prob(self, value):
        return torch.exp(self.log_prob(value))

    probs = prob

    def kl_divergence(self, other):
        return kl_divergence(self, other)


class ExponentialFamily(Distribution):
    """Marker base of the exponential-family members (entropy via the torch Bregman form)."""


class Normal(ExponentialFamily):
    def __init__(self, loc, scale, name=None):
        self.loc, self.scale = _t(loc), _t(scale)
        self._d = D.Normal(self.loc, self.scale)
        super().__init__(self._d.batch_shape)


class Uniform(Distribution):
    def __init__(self, low, high, name=None):
        self.low, self.high = _t(low), _t(high)
        self._d = D.Uniform(self.low, self.high)
        super().__init__(self._d.batch_shape)

    def log_prob(self, value):  # Paddle: -inf outside the support instead of raising
        v = _t(value)
        inside = (v >= self.low) & (v < self.high)
        lp = -torch.log(self.high - self.low)
        return torch.where(inside, lp.expand_as(inside) if lp.dim() else lp, torch.full_like(v, float("-inf")))


class Categorical(Distribution):
    """Paddle's Categorical takes (unnormalised, non-negative) ``logits`` as weights."""

    def __init__(self, logits, name=None):
        self.logits = _t(logits)
        self._d = D.Categorical(probs=self.logits / self.logits.sum(-1, keepdim=True))
        super().__init__(self._d.batch_shape)

    def probs(self, value):
        return self._d.probs.gather(-1, _t(value, torch.long).long().unsqueeze(-1)).squeeze(-1) \
            if self._d.probs.dim() > 1 else self._d.probs[_t(value, torch.long).long()]


class Beta(ExponentialFamily):
    def __init__(self, alpha, beta):
        self.alpha, self.beta = _t(alpha), _t(beta)
        self._d = D.Beta(self.alpha, self.beta)
        super().__init__(self._d.batch_shape)


class Dirichlet(ExponentialFamily):
    def __init__(self, concentration):
        self.concentration = _t(concentration)
        self._d = D.Dirichlet(self.concentration)
        super().__init__(self._d.batch_shape, self._d.event_shape)


class Multinomial(Distribution):
    def __init__(self, total_count, probs):
        self.total_count, self.probs_ = int(total_count), _t(probs)
        self._d = D.Multinomial(self.total_count, probs=self.probs_)
        super().__init__(self._d.batch_shape, self._d.event_shape)


class Independent(Distribution):
    def __init__(self, base, reinterpreted_batch_rank):
        self.base = base
        self._d = D.Independent(base._d, reinterpreted_batch_rank)
        super().__init__(self._d.batch_shape, self._d.event_shape)


class TransformedDistribution(Distribution):
    def __init__(self, base, transforms):
        self.base, self.transforms = base, list(transforms)
        self._d = D.TransformedDistribution(base._d, [t._t for t in self.transforms])
        super().__init__(self._d.batch_shape, self._d.event_shape)


def _simple(name, cls, *params):
    def __init__(self, *args, **kw):
        kw.pop("name", None)
        vals = [_t(a) if not isinstance(a, int) or name in ("Binomial",) else a for a in args]
        for p, v in zip(params, vals):
            setattr(self, p, v)
        self._d = cls(*vals, **kw)
        Distribution.__init__(self, self._d.batch_shape, self._d.event_shape)
    return type(name, (ExponentialFamily,), {"__init__": __init__})


Laplace = _simple("Laplace", D.Laplace, "loc", "scale")
LogNormal = _simple("LogNormal", D.LogNormal, "loc", "scale")
Gumbel = _simple("Gumbel", D.Gumbel, "loc", "scale")
Cauchy = _simple("Cauchy", D.Cauchy, "loc", "scale")
Geometric = _simple("Geometric", D.Geometric, "probs")
Bernoulli = _simple("Bernoulli", D.Bernoulli, "probs")
Poisson = _simple("Poisson", D.Poisson, "rate")
Exponential = _simple("Exponential", D.Exponential, "rate")
Gamma = _simple("Gamma", D.Gamma, "concentration", "rate")
Binomial = _simple("Binomial", D.Binomial, "total_count", "probs")

_KL = {}


def register_kl(cls_p, cls_q):
    """Decorator registering ``fn(p, q)`` as KL(p‖q) for the class pair (reference `kl.py`)."""
    def deco(fn):
        _KL[(cls_p, cls_q)] = fn
        return fn
    return deco


def kl_divergence(p, q):
    for (a, b), fn in _KL.items():
        if isinstance(p, a) and isinstance(q, b):
            return fn(p, q)
    return D.kl_divergence(p._d, q._d)
