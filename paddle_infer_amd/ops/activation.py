"""Fused bias + activation (+ dropout) ops backed by ``csrc/kernels/elementwise.hip``.

Parity: reference `paddle/fluid/operators/fused/fused_dropout_act_bias.h` (FusedFeedForward's
``act(x + bias)``), ``paddle.nn.functional.gelu`` (`nn/functional/activation.py`),
``paddle.nn.functional.dropout`` and the fused masked softmax ops.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from ..framework import random as _random

_H16 = (torch.bfloat16, torch.float16)
_KDT = {torch.bfloat16: 0, torch.float16: 1, torch.float32: 2}  # element types of the HIP kernels


def _f16(t) -> int:
    """dtype code of elementwise.hip's entry points: 0 bf16, 1 fp16, 2 f32."""
    return _KDT[t.dtype]


ACTS = {"none": 0, "identity": 0, "gelu_tanh": 1, "gelu": 2, "relu": 3, "silu": 4, "swish": 4}


def _ref_act(x, act):
    if act == 0:
        return x
    if act == 1:
        return F.gelu(x, approximate="tanh")
    if act == 2:
        return F.gelu(x)
    if act == 3:
        return F.relu(x)
    return F.silu(x)


class _BiasActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act):
        N = x.shape[-1]
        x2 = x.contiguous()
        y = torch.empty_like(x2)
        # the pre-activation is NOT materialised: backward re-adds the bias to the saved GEMM
        # output in registers (saves one [tokens x 4h] write per layer)
        _lib.call("piamd_bias_act_fwd", _f16(x2), act, x2.data_ptr(), _lib.ptr(bias), y.data_ptr(),
                  None, x2.numel(), N, _lib.stream())
        ctx.save_for_backward(x2)
        ctx.act = act
        ctx.has_bias = bias is not None
        ctx.bias_param = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        (h,) = ctx.saved_tensors
        N = h.shape[-1]
        rows = h.numel() // N
        dy = dy.contiguous()
        dx = torch.empty_like(h)
        need_b = ctx.has_bias and ctx.needs_input_grad[1]
        db, part, acc = None, None, 0
        if need_b:
            mg = _lib.main_grad(ctx.bias_param)
            if mg is not None:  # add straight into the engine's flat gradient view
                db, acc = mg.view(-1), 1
            else:
                db = torch.empty(N, device=h.device, dtype=h.dtype)
            part = torch.empty((N,), device=h.device, dtype=torch.float32)
        # h is the GEMM output without bias: the kernel adds the bias before act'()
        _lib.call("piamd_bias_act_bwd", _f16(h), ctx.act, dy.data_ptr(), h.data_ptr(),
                  _lib.ptr(ctx.bias_param), dx.data_ptr(), _lib.ptr(db), _lib.ptr(part), rows, N,
                  acc, _lib.stream())
        if acc:
            _lib.fire(ctx.bias_param)
            db = None
        return dx, db, None


def bias_act(x, bias=None, act: str = "gelu"):
    """``act(x + bias)``; bias broadcast over the last dim."""
    a = ACTS[act]
    N = x.shape[-1]
    if x.is_cuda:
        if x.dtype in _KDT and N % 8 == 0:
            b = bias if bias is None or bias.dtype == x.dtype else bias.to(x.dtype)
            return _BiasActFn.apply(x, b, a)
        _lib.fallback("bias_act", f"dtype {x.dtype} / N {N} (kernel: bf16/fp16/f32, N % 8 == 0)")
    return _ref_act(x if bias is None else x + bias, a)


def gelu(x, approximate: bool = False):
    return bias_act(x, None, "gelu_tanh" if approximate else "gelu")


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, offset):
        x2 = x.contiguous()
        y = torch.empty_like(x2)
        _lib.call("piamd_dropout", _f16(x2), x2.data_ptr(), y.data_ptr(), x2.numel(), float(p), seed, offset,
                  _lib.stream())
        ctx.meta = (p, seed, offset)
        return y

    @staticmethod
    def backward(ctx, dy):
        p, seed, offset = ctx.meta
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        _lib.call("piamd_dropout", _f16(dy), dy.data_ptr(), dx.data_ptr(), dy.numel(), float(p), seed, offset,
                  _lib.stream())
        return dx, None, None, None


def dropout(x, p: float = 0.5, training: bool = True):
    if not training or p == 0.0:
        return x
    if x.is_cuda:
        if x.dtype in _KDT and x.numel() % 8 == 0:
            seed, offset = _random.next_seed_offset(x.numel())
            return _DropoutFn.apply(x, p, seed, offset)
        _lib.fallback("dropout", f"dtype {x.dtype} / numel % 8 (kernel: bf16/fp16/f32)")
    return F.dropout(x, p, training=True)


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask, causal_q, scale):
        N = x.shape[-1]
        x2 = x.contiguous()
        rows = x2.numel() // N
        y = torch.empty_like(x2)
        mrows = 0
        if mask is not None:
            mask = mask.contiguous()
            mrows = mask.numel() // N
        _lib.call("piamd_softmax_fwd", _f16(x2), x2.data_ptr(), _lib.ptr(mask), mrows, causal_q, y.data_ptr(),
                  rows, N, float(scale), _lib.stream())
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        N = y.shape[-1]
        dy = dy.contiguous()
        dx = torch.empty_like(y)
        _lib.call("piamd_softmax_bwd", _f16(y), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), y.numel() // N, N,
                  float(ctx.scale), _lib.stream())
        return dx, None, None, None


def fused_softmax_mask(x, mask=None, scale: float = 1.0, causal: bool = False):
    """softmax(scale*x + mask) over the last dim; ``causal`` masks the upper triangle (the
    reference's ``fused_softmax_mask_upper_triangle``). mask broadcasts over leading rows."""
    N = x.shape[-1]
    if x.is_cuda:
        if x.dtype in _KDT and N % 8 == 0 and N <= 4096 and \
                (mask is None or x.numel() % mask.numel() == 0):
            cq = x.shape[-2] if causal else 0
            m = mask if mask is None or mask.dtype == x.dtype else mask.to(x.dtype)
            return _SoftmaxFn.apply(x, m, cq, scale)
        _lib.fallback("fused_softmax_mask", f"dtype {x.dtype} / N {N} / mask shape")
    s = x.float() * scale
    if mask is not None:
        s = s + mask.float()
    if causal:
        Sq = x.shape[-2]
        i = torch.arange(Sq, device=x.device)[:, None]
        j = torch.arange(N, device=x.device)[None, :]
        s = s.masked_fill(j > i + (N - Sq), float("-inf"))
    return torch.softmax(s, -1).to(x.dtype)
