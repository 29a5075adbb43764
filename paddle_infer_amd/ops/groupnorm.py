"""GroupNorm / InstanceNorm on the own HIP kernels (``csrc/kernels/groupnorm.hip``): f32 / bf16 /
fp16 NCHW-contiguous activations, f32 statistics, forward and backward (dx, dγ, dβ).

Parity: reference `phi/kernels/gpu/group_norm_kernel.cu` / `group_norm_grad_kernel.cu`,
`instance_norm_kernel.cu` / `instance_norm_grad_kernel.cu` (InstanceNorm = GroupNorm with one
channel per group; with running statistics and ``use_input_stats=False`` it is the per-channel
affine y = (x − μ_c)·rsqrt(σ²_c + ε)·γ_c + β_c, run through the same apply kernel).
"""
from __future__ import annotations

import torch

from . import _lib

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def supported(x, num_groups: int) -> bool:
    return (x.is_cuda and x.dtype in _DT and x.dim() >= 2 and x.shape[1] % num_groups == 0
            and x.numel() > 0 and _lib.available())


def _ws(N, C, G, dev):
    return torch.empty(max(3 * N * C, 2 * N * C + 2 * N * G), dtype=torch.float32, device=dev)


def _f32(t, dev=None):
    if t is None:
        return None
    t = t.detach().float()
    return (t.to(dev) if dev is not None else t).contiguous()


class _GroupNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, G, eps):
        xc = x.contiguous()
        N, C = xc.shape[0], xc.shape[1]
        HW = xc.numel() // (N * C)
        dev = xc.device
        y = torch.empty_like(xc)
        mean = torch.empty(N * G, dtype=torch.float32, device=dev)
        rstd = torch.empty(N * G, dtype=torch.float32, device=dev)
        g, b = _f32(weight, dev), _f32(bias, dev)
        _lib.call("piamd_group_norm_fwd", _DT[xc.dtype], xc.data_ptr(), y.data_ptr(), _lib.ptr(g), _lib.ptr(b),
                  mean.data_ptr(), rstd.data_ptr(), _ws(N, C, G, dev).data_ptr(), N, C, HW, G, float(eps),
                  _lib.stream())
        ctx.save_for_backward(xc, g, mean, rstd)
        ctx.meta = (N, C, HW, G, weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, g, mean, rstd = ctx.saved_tensors
        N, C, HW, G, weight, bias = ctx.meta
        dyc = dy.contiguous()
        dev = xc.device
        dx = torch.empty_like(xc) if ctx.needs_input_grad[0] else None
        want_w = weight is not None and ctx.needs_input_grad[1]
        want_b = bias is not None and ctx.needs_input_grad[2]
        dg = torch.empty(C, dtype=torch.float32, device=dev) if want_w else None
        db = torch.empty(C, dtype=torch.float32, device=dev) if want_b else None
        _lib.call("piamd_group_norm_bwd", _DT[xc.dtype], dyc.data_ptr(), xc.data_ptr(), _lib.ptr(g),
                  mean.data_ptr(), rstd.data_ptr(), _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db),
                  _ws(N, C, G, dev).data_ptr(), N, C, HW, G, _lib.stream())
        return (dx, dg.to(weight.dtype) if want_w else None, db.to(bias.dtype) if want_b else None,
                None, None)


def group_norm(x, num_groups, weight=None, bias=None, eps=1e-5):
    """GroupNorm over NC[*] (channels second, contiguous or not)."""
    return _GroupNorm.apply(x, weight, bias, int(num_groups), float(eps))


def instance_norm_eval(x, running_mean, running_var, weight=None, bias=None, eps=1e-5):
    """InstanceNorm with the running statistics (``use_input_stats=False``, no autograd): the
    per-channel affine y = x·s_c + t_c (s = γ·rsqrt(σ² + ε), t = β − μ·s) on the apply kernel."""
    xc = x.contiguous()
    N, C = xc.shape[0], xc.shape[1]
    HW = xc.numel() // (N * C)
    dev = x.device
    s = torch.rsqrt(_f32(running_var, dev) + eps)
    if weight is not None:
        s = s * _f32(weight, dev)
    t = -_f32(running_mean, dev) * s
    if bias is not None:
        t = t + _f32(bias, dev)
    y = torch.empty_like(xc)
    zero = torch.zeros(N * C, dtype=torch.float32, device=dev)  # per-(n, c) "statistics": 0 / 1
    one = torch.ones(N * C, dtype=torch.float32, device=dev)
    _lib.call("piamd_group_norm_apply", _DT[xc.dtype], xc.data_ptr(), y.data_ptr(), s.contiguous().data_ptr(),
              t.contiguous().data_ptr(), zero.data_ptr(), one.data_ptr(), N, C, HW, C, _lib.stream())
    return y
