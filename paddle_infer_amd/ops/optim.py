"""Flat-buffer optimizer kernels (``csrc/kernels/optim.hip``) with PyTorch reference paths.

Parity: reference `paddle/phi/kernels/gpu/adamw_kernel.cu` / `momentum_kernel.cu` and
``ClipGradByGlobalNorm`` (`python/paddle/nn/clip.py`).
"""
from __future__ import annotations

import math

import torch

from . import _lib


def adamw_flat(p, m, v, grad, lr, beta1, beta2, eps, wd, step, model=None, grad_scale=None,
               static_grad_scale: float = 1.0, lr_tensor=None):
    """In-place AdamW (Paddle semantics: decoupled decay ``p *= 1 - lr*wd`` then Adam with
    ``eps * sqrt(1 - beta2^t)``) over flat f32 ``p/m/v``; ``grad`` bf16/f32; ``model`` optional
    bf16 copy written in the same pass; ``grad_scale`` optional device scalar."""
    bc1 = 1.0 - beta1 ** step
    bc2s = math.sqrt(1.0 - beta2 ** step)
    if p.is_cuda:
        _lib.call("piamd_adamw_flat", p.data_ptr(), m.data_ptr(), v.data_ptr(), grad.data_ptr(),
                  1 if grad.dtype == torch.bfloat16 else 0, _lib.ptr(model), p.numel(), float(lr),
                  _lib.ptr(lr_tensor), float(beta1), float(beta2), float(eps), float(wd),
                  float(bc1), float(bc2s), _lib.ptr(grad_scale), float(static_grad_scale),
                  _lib.stream())
        return
    g = grad.float() * static_grad_scale
    if grad_scale is not None:
        g = g * grad_scale.float()
    lr_ = float(lr_tensor) if lr_tensor is not None else lr
    p.mul_(1.0 - lr_ * wd)
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    step_size = lr_ * bc2s / bc1
    p.addcdiv_(m, v.sqrt().add_(eps * bc2s), value=-step_size)
    if model is not None:
        model.copy_(p)


def momentum_flat(p, vel, grad, lr, mu, wd=0.0, nesterov=False, model=None, grad_scale=None):
    if p.is_cuda:
        _lib.call("piamd_momentum_flat", p.data_ptr(), vel.data_ptr(), grad.data_ptr(),
                  1 if grad.dtype == torch.bfloat16 else 0, _lib.ptr(model), p.numel(), float(lr),
                  None, float(mu), float(wd), int(nesterov), _lib.ptr(grad_scale), _lib.stream())
        return
    g = grad.float()
    if grad_scale is not None:
        g = g * grad_scale.float()
    g = g + wd * p
    vel.mul_(mu).add_(g)
    p.sub_(lr * (g + mu * vel if nesterov else vel))
    if model is not None:
        model.copy_(p)


def sumsq(x, out=None, accumulate=False):
    """Σ x² of a flat tensor into a f32 device scalar (no host sync)."""
    if out is None:
        out = torch.zeros((), device=x.device, dtype=torch.float32)
    if x.is_cuda:
        part = torch.empty(2048, device=x.device, dtype=torch.float32)
        _lib.call("piamd_sumsq", x.data_ptr(), 1 if x.dtype == torch.bfloat16 else 0, x.numel(),
                  part.data_ptr(), out.data_ptr(), int(accumulate), _lib.stream())
        return out
    s = x.float().pow(2).sum()
    if accumulate:
        out.add_(s)
    else:
        out.copy_(s)
    return out
