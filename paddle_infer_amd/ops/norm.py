"""LayerNorm ops backed by ``csrc/kernels/layernorm.hip``.

Parity: ``paddle.nn.functional.layer_norm`` (reference `python/paddle/nn/functional/norm.py`) and
``paddle.incubate.nn.functional.fused_bias_dropout_residual_layer_norm``
(reference `python/paddle/incubate/nn/functional/fused_transformer.py:275`).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from ..framework import random as _random


def _hip_ok(*ts) -> bool:
    return all(t is None or t.is_cuda for t in ts)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        shp = x.shape
        N = shp[-1]
        x2 = x.contiguous().view(-1, N)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        _lib.call("piamd_layernorm_fwd", _lib.dtype_code(x2), x2.data_ptr(), None, None,
                  _lib.ptr(weight), _lib.ptr(bias), y.data_ptr(), None, mean.data_ptr(),
                  rstd.data_ptr(), rows, N, float(eps), 0.0, 0, 0, _lib.stream())
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.has_bias = bias is not None
        ctx.shp = shp
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, mean, rstd = ctx.saved_tensors
        rows, N = x2.shape
        dy2 = dy.contiguous().view(rows, N)
        dx = torch.empty_like(x2)
        G = _lib.lib().piamd_layernorm_bwd_grid(rows)
        need_w = weight is not None and ctx.needs_input_grad[1]
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        part = torch.empty((2, N), device=x2.device, dtype=torch.float32)
        dw = torch.empty_like(weight) if need_w else None
        db = torch.empty(N, device=x2.device, dtype=weight.dtype if weight is not None else x2.dtype) if need_b else None
        _lib.call("piamd_layernorm_bwd", _lib.dtype_code(x2), dy2.data_ptr(), x2.data_ptr(),
                  _lib.ptr(weight), mean.data_ptr(), rstd.data_ptr(), None, dx.data_ptr(), None,
                  _lib.ptr(dw), _lib.ptr(db), None, part[0].data_ptr(), part[1].data_ptr(), None,
                  rows, N, 0.0, 0, 0, _lib.stream())
        return dx.view(ctx.shp), dw, db, None


def layer_norm(x, weight=None, bias=None, eps: float = 1e-5):
    """LayerNorm over the last dim."""
    N = x.shape[-1]
    if _hip_ok(x, weight, bias) and x.dtype in (torch.bfloat16, torch.float32) and N % 8 == 0 \
            and N <= 4096 and (weight is None or weight.dtype == x.dtype):
        return _LayerNormFn.apply(x, weight, bias, eps)
    if x.is_cuda and _lib.available() is False:
        raise RuntimeError("paddle_infer_amd kernels missing on a GPU run")
    return F.layer_norm(x, (N,), weight, bias, eps)


class _FusedAddLNFn(torch.autograd.Function):
    """(y, h) = (LN(h), h) with h = residual + dropout(x + x_bias)."""

    @staticmethod
    def forward(ctx, x, residual, weight, bias, x_bias, eps, p, seed, offset):
        shp = x.shape
        N = shp[-1]
        x2 = x.contiguous().view(-1, N)
        r2 = residual.contiguous().view(-1, N)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        h = torch.empty_like(x2)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        _lib.call("piamd_layernorm_fwd", _lib.dtype_code(x2), x2.data_ptr(), _lib.ptr(x_bias),
                  r2.data_ptr(), _lib.ptr(weight), _lib.ptr(bias), y.data_ptr(), h.data_ptr(),
                  mean.data_ptr(), rstd.data_ptr(), rows, N, float(eps), float(p), seed, offset,
                  _lib.stream())
        ctx.save_for_backward(h, weight, mean, rstd)
        ctx.meta = (shp, bias is not None, x_bias is not None, p, seed, offset)
        return y.view(shp), h.view(shp)

    @staticmethod
    def backward(ctx, dy, dh):
        h, weight, mean, rstd = ctx.saved_tensors
        shp, has_b, has_xb, p, seed, offset = ctx.meta
        rows, N = h.shape
        dy2 = dy.contiguous().view(rows, N) if dy is not None else torch.zeros_like(h)
        dh2 = dh.contiguous().view(rows, N) if dh is not None else None
        dres = torch.empty_like(h)
        separate_dx = p > 0.0 or has_xb
        dx = torch.empty_like(h) if (p > 0.0) else None
        G = _lib.lib().piamd_layernorm_bwd_grid(rows)
        need_w = weight is not None and ctx.needs_input_grad[2]
        need_b = has_b and ctx.needs_input_grad[3]
        need_xb = has_xb and ctx.needs_input_grad[4]
        part = torch.empty((3, N), device=h.device, dtype=torch.float32)
        dw = torch.empty_like(weight) if need_w else None
        db = torch.empty(N, device=h.device, dtype=weight.dtype if weight is not None else h.dtype) if need_b else None
        dxb = torch.empty(N, device=h.device, dtype=h.dtype) if need_xb else None
        # dbias (of x_bias) = column sums of dx; when no dropout dx == dres, computed on dres.
        dx_ptr = dx.data_ptr() if dx is not None else (dres.data_ptr() if need_xb else None)
        if dx is None and need_xb:
            # kernel writes dres then dx (same values) into the same buffer: column sums of dx.
            pass
        _lib.call("piamd_layernorm_bwd", _lib.dtype_code(h), dy2.data_ptr(), h.data_ptr(),
                  _lib.ptr(weight), mean.data_ptr(), rstd.data_ptr(), _lib.ptr(dh2),
                  dres.data_ptr(), dx_ptr, _lib.ptr(dw), _lib.ptr(db), _lib.ptr(dxb),
                  part[0].data_ptr(), part[1].data_ptr(), part[2].data_ptr(), rows, N, float(p),
                  seed, offset, _lib.stream())
        dxo = (dx if dx is not None else dres).view(shp)
        del separate_dx
        return dxo, dres.view(shp), dw, db, dxb, None, None, None, None


def fused_add_layer_norm(x, residual, weight=None, bias=None, eps: float = 1e-5, x_bias=None,
                         dropout_p: float = 0.0, training: bool = True):
    """Returns ``(LN(h), h)`` with ``h = residual + dropout(x + x_bias)``."""
    p = float(dropout_p) if training else 0.0
    N = x.shape[-1]
    if _hip_ok(x, residual, weight, bias, x_bias) and x.dtype in (torch.bfloat16, torch.float32) \
            and N % 8 == 0 and N <= 4096:
        seed, offset = _random.next_seed_offset(x.numel()) if p > 0 else (0, 0)
        return _FusedAddLNFn.apply(x, residual, weight, bias, x_bias, eps, p, seed, offset)
    t = x if x_bias is None else x + x_bias
    if p > 0:
        t = F.dropout(t, p, training=True)
    h = residual + t
    return F.layer_norm(h, (N,), weight, bias, eps), h


def rms_norm(x, weight=None, eps: float = 1e-6):
    """RMSNorm (LLaMA-style) — composed from torch ops on every device (bandwidth-bound)."""
    var = x.float().pow(2).mean(-1, keepdim=True)
    y = (x.float() * torch.rsqrt(var + eps)).to(x.dtype)
    return y * weight if weight is not None else y
