"""Bijective transforms (reference `python/paddle/distribution/transform.py`) over
``torch.distributions.transforms``: ``forward``, ``inverse``, ``forward_log_det_jacobian``,
``inverse_log_det_jacobian``, ``forward_shape``, ``inverse_shape``."""
from __future__ import annotations

import torch
import torch.distributions.transforms as T

__all__ = ["Transform", "AbsTransform", "AffineTransform", "ChainTransform", "ExpTransform",
           "IndependentTransform", "PowerTransform", "ReshapeTransform", "SigmoidTransform",
           "SoftmaxTransform", "StackTransform", "StickBreakingTransform", "TanhTransform"]


class Transform:
    _t: T.Transform

    def __call__(self, x):
        return self.forward(x)

    def forward(self, x):
        return self._t(x)

    def inverse(self, y):
        return self._t.inv(y)

    def forward_log_det_jacobian(self, x):
        return self._t.log_abs_det_jacobian(x, self._t(x))

    def inverse_log_det_jacobian(self, y):
        return -self._t.log_abs_det_jacobian(self._t.inv(y), y)

    def forward_shape(self, shape):
        return tuple(self._t.forward_shape(torch.Size(shape)))

    def inverse_shape(self, shape):
        return tuple(self._t.inverse_shape(torch.Size(shape)))


class _AbsT(T.Transform):
    domain = T.constraints.real
    codomain = T.constraints.positive

    def _call(self, x):
        return x.abs()

    def _inverse(self, y):
        return y


class AbsTransform(Transform):
    """y = |x| (not injective: the inverse returns the non-negative branch)."""

    def __init__(self):
        self._t = _AbsT()

    def inverse(self, y):
        return (-y, y)


class AffineTransform(Transform):
    def __init__(self, loc, scale):
        self.loc, self.scale = torch.as_tensor(loc), torch.as_tensor(scale)
        self._t = T.AffineTransform(self.loc, self.scale)


class ChainTransform(Transform):
    def __init__(self, transforms):
        self.transforms = list(transforms)
        self._t = T.ComposeTransform([t._t for t in self.transforms])


class ExpTransform(Transform):
    def __init__(self):
        self._t = T.ExpTransform()


class IndependentTransform(Transform):
    def __init__(self, base, reinterpreted_batch_rank):
        self.base = base
        self._t = T.IndependentTransform(base._t, reinterpreted_batch_rank)


class PowerTransform(Transform):
    def __init__(self, power):
        self.power = torch.as_tensor(power)
        self._t = T.PowerTransform(self.power)


class ReshapeTransform(Transform):
    def __init__(self, in_event_shape, out_event_shape):
        self._t = T.ReshapeTransform(torch.Size(in_event_shape), torch.Size(out_event_shape))


class SigmoidTransform(Transform):
    def __init__(self):
        self._t = T.SigmoidTransform()


class SoftmaxTransform(Transform):
    def __init__(self):
        self._t = T.SoftmaxTransform()


class StackTransform(Transform):
    def __init__(self, transforms, axis=0):
        self.transforms = list(transforms)
        self._t = T.StackTransform([t._t for t in self.transforms], axis)


class StickBreakingTransform(Transform):
    def __init__(self):
        self._t = T.StickBreakingTransform()


class TanhTransform(Transform):
    def __init__(self):
        self._t = T.TanhTransform()
