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


_MT_CHUNK = 2048


def multi_tensor_update(op, entries, lr, cache=None, mu=0.0, nesterov=False, beta1=0.9,
                        beta2=0.999, eps=1e-8, step=1, grad_scale=None):
    """Merged optimizer update of many tensors in ONE kernel launch (reference
    ``merged_momentum`` / ``merged_adam``; ``optim.hip`` multi_tensor_kernel).

    ``op``: 0 SGD, 1 Momentum, 2 Adam (L2 decay), 3 AdamW (decoupled decay). ``entries``: list of
    ``(p, grad, s1, s2, wd, lr_mult)`` with f32 contiguous ``p`` / states and bf16 or f32 ``grad``.
    ``cache`` (a dict owned by the optimizer) keeps the device table while no pointer changes."""
    dev = entries[0][0].device
    if dev.type != "cuda":
        for p, g, s1, s2, wd, lm in entries:
            gf = g.float()
            lr_ = lr * lm
            if op == 0:
                p.sub_(lr_ * (gf + wd * p))
            elif op == 1:
                gf = gf + wd * p
                s1.mul_(mu).add_(gf)
                p.sub_(lr_ * (gf + mu * s1 if nesterov else s1))
            else:
                if op == 2:
                    gf = gf + wd * p
                else:
                    p.mul_(1.0 - lr_ * wd)
                s1.mul_(beta1).add_(gf, alpha=1 - beta1)
                s2.mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
                bc2 = math.sqrt(1 - beta2 ** step)
                p.addcdiv_(s1, s2.sqrt().add_(eps * bc2), value=-lr_ * bc2 / (1 - beta1 ** step))
        return
    key = tuple((e[0].data_ptr(), e[1].data_ptr(), _lib.ptr(e[2]) or 0, _lib.ptr(e[3]) or 0,
                 e[1].dtype == torch.bfloat16, e[4], e[5]) for e in entries)
    ent = cache.get("table") if cache is not None else None
    if ent is None or ent[0] != key:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("merged optimizer: parameter / gradient buffers changed inside hipGraph "
                               "capture (keep gradients allocated across steps: clear_grad(set_to_zero=True) "
                               "and run one eager step before capturing)")
        meta, fmeta, offs, c = [], [], [0], 0
        for (pp, gp, s1p, s2p, bf, wd, lm), e in zip(key, entries):
            n = e[0].numel()
            meta += [pp, gp, s1p, s2p, n, int(bf)]
            fmeta += [float(wd), float(lm)]
            c += -(-n // _MT_CHUNK)
            offs.append(c)
        t_meta = torch.tensor(meta, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
        t_f = torch.tensor(fmeta, dtype=torch.float32).pin_memory().to(dev, non_blocking=True)
        t_o = torch.tensor(offs, dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
        ent = (key, t_meta, t_f, t_o, c)
        if cache is not None:
            cache["table"] = ent
    _, t_meta, t_f, t_o, total = ent
    bc1 = 1.0 - beta1 ** step
    bc2s = math.sqrt(1.0 - beta2 ** step)
    _lib.call("piamd_multi_tensor_update", int(op), t_meta.data_ptr(), t_f.data_ptr(), t_o.data_ptr(),
              len(entries), int(total), float(lr), float(mu), int(nesterov), float(beta1),
              float(beta2), float(eps), float(bc1), float(bc2s), _lib.ptr(grad_scale), _lib.stream())
