"""Gradient clipping (reference `python/paddle/nn/clip.py`).

``ClipGradByGlobalNorm`` computes Σg² with the HIP ``sumsq`` kernel per gradient (one device scalar,
no host sync) and scales in place; flat-buffer training uses the engine's fused path instead.
"""
from __future__ import annotations

import torch

from ..ops.optim import sumsq


class ClipGradBase:
    def __call__(self, params_grads):
        return self._clip(params_grads)


class ClipGradByValue(ClipGradBase):
    def __init__(self, max, min=None):  # noqa: A002
        self.max, self.min = max, (-max if min is None else min)

    def _clip(self, params_grads):
        out = []
        for p, g in params_grads:
            if g is not None and getattr(p, "need_clip", True):
                g = g.clamp(self.min, self.max)
            out.append((p, g))
        return out


class ClipGradByNorm(ClipGradBase):
    def __init__(self, clip_norm):
        self.clip_norm = clip_norm

    def _clip(self, params_grads):
        out = []
        for p, g in params_grads:
            if g is not None and getattr(p, "need_clip", True):
                n = g.float().norm()
                g = g * torch.clamp(self.clip_norm / (n + 1e-6), max=1.0).to(g.dtype)
            out.append((p, g))
        return out


class ClipGradByGlobalNorm(ClipGradBase):
    def __init__(self, clip_norm, group_name="default_group", auto_skip_clip=False):
        self.clip_norm = clip_norm

    def global_norm(self, grads):
        if not grads:
            return torch.zeros(())
        acc = torch.zeros((), device=grads[0].device, dtype=torch.float32)
        for g in grads:
            sumsq(g.reshape(-1), out=acc, accumulate=True)
        return acc.sqrt()

    def _clip(self, params_grads):
        gs = [g for p, g in params_grads if g is not None and getattr(p, "need_clip", True)]
        if not gs:
            return params_grads
        coef = torch.clamp(self.clip_norm / (self.global_norm(gs) + 1e-6), max=1.0)
        out = []
        for p, g in params_grads:
            if g is not None and getattr(p, "need_clip", True):
                g.mul_(coef.to(g.dtype))
            out.append((p, g))
        return out


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False):
    params = [parameters] if isinstance(parameters, torch.Tensor) else list(parameters)
    return torch.nn.utils.clip_grad_norm_(params, max_norm, norm_type, error_if_nonfinite)


def clip_grad_value_(parameters, clip_value):
    params = [parameters] if isinstance(parameters, torch.Tensor) else list(parameters)
    return torch.nn.utils.clip_grad_value_(params, clip_value)
