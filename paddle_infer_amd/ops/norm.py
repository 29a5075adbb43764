"""LayerNorm / RMSNorm ops backed by ``csrc/kernels/layernorm.hip`` (f32 / bf16 / fp16, N <= 16384).

Parity: ``paddle.nn.functional.layer_norm`` (reference `python/paddle/nn/functional/norm.py`) and
``paddle.incubate.nn.functional.fused_bias_dropout_residual_layer_norm``
(reference `python/paddle/incubate/nn/functional/fused_transformer.py:275`).

Parameter gradients: when a parameter carries a ``main_grad`` view (flat gradient buffer of the
training engine), the kernel's column-sum epilogue ADDS into it directly and the op returns no
gradient for that parameter — no temporary, no autograd AccumulateGrad launch.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from ..framework import random as _random


_DTYPES = (torch.bfloat16, torch.float16, torch.float32)
MAX_N = 16384
RMS = 1  # kernel flag bit


def _hip_ok(*ts) -> bool:
    return all(t is None or t.is_cuda for t in ts)


def _hip_path(op, x, *params) -> bool:
    """True: run the HIP kernel. CPU tensors take the reference path silently; a GPU tensor the
    kernel cannot take is recorded + warned once (``_lib.fallback``)."""
    if not (x.is_cuda and _hip_ok(*params)):
        return False
    N = x.shape[-1]
    if x.dtype not in _DTYPES:
        _lib.fallback(op, f"dtype {x.dtype}")
        return False
    if N % 8 != 0 or N > MAX_N:
        _lib.fallback(op, f"row length {N} (kernel: multiple of 8, <= {MAX_N})")
        return False
    return True


def _cast(p, dtype):
    """Params in the activation dtype (AMP O1 keeps LN weights f32 under bf16/fp16 activations):
    a differentiable cast of an N-vector, so gradients flow back in the parameter's dtype.
    Without autograd (inference, AMP predictors keeping LN params f32) the cast is cached on the
    parameter until it changes, so a run launches no per-layer cast kernels."""
    if p is None or p.dtype == dtype:
        return p
    if torch.is_grad_enabled() and p.requires_grad:
        return p.to(dtype)
    c = getattr(p, "_piamd_cast", None)
    key = (dtype, p._version, p.data_ptr())
    if c is not None and c[0] == key:
        return c[1]
    out = p.detach().to(dtype)
    try:
        p._piamd_cast = (key, out)
    except (AttributeError, RuntimeError):
        pass
    return out


def _grad_target(p, needed, N, dtype, device):
    """(tensor the kernel writes, accumulate?, return-to-autograd?)."""
    if p is None or not needed:
        return None, False, False
    mg = _lib.main_grad(p)
    if mg is not None:
        return mg.view(-1), True, False
    return torch.empty(N, device=device, dtype=dtype), False, True


def _ln_bwd(dtype, dy2, h, weight, mean, rstd, dh2, dres, dx_ptr, targets, rows, N, p, seed, off,
            flags=0):
    ws = torch.empty(_lib.lib().piamd_layernorm_bwd_ws(rows, N), device=h.device, dtype=torch.float32)
    mask = 0
    outs = []
    for i, (t, acc, _) in enumerate(targets):
        outs.append(_lib.ptr(t))
        if acc:
            mask |= 1 << i
    _lib.call("piamd_layernorm_bwd", dtype, dy2.data_ptr(), h.data_ptr(), _lib.ptr(weight),
              mean.data_ptr(), rstd.data_ptr(), _lib.ptr(dh2), _lib.ptr(dres), dx_ptr, outs[0],
              outs[1], outs[2], ws.data_ptr(), rows, N, float(p), seed, off, mask, flags,
              _lib.stream())


def _finish(params, targets):
    out = []
    for prm, (t, acc, ret) in zip(params, targets):
        if acc:
            _lib.fire(prm)
        out.append(t.view(prm.shape) if ret else None)
    return out


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, flags=0):
        shp = x.shape
        N = shp[-1]
        x2 = x.contiguous().view(-1, N)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        _lib.call("piamd_layernorm_fwd", _lib.dtype_code(x2, fp16=True), x2.data_ptr(), None, None,
                  _lib.ptr(weight), _lib.ptr(bias), y.data_ptr(), None, mean.data_ptr(),
                  rstd.data_ptr(), rows, N, float(eps), 0.0, 0, 0, flags, _lib.stream())
        ctx.save_for_backward(x2, weight, bias, mean, rstd)
        ctx.shp = shp
        ctx.flags = flags
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, bias, mean, rstd = ctx.saved_tensors
        rows, N = x2.shape
        dy2 = dy.contiguous().view(rows, N)
        dx = torch.empty_like(x2)
        pdt = weight.dtype if weight is not None else x2.dtype
        targets = [_grad_target(weight, ctx.needs_input_grad[1], N, pdt, x2.device),
                   _grad_target(bias, ctx.needs_input_grad[2], N, pdt, x2.device),
                   (None, False, False)]
        _ln_bwd(_lib.dtype_code(x2, fp16=True), dy2, x2, weight, mean, rstd, None, dx, None,
                targets, rows, N, 0.0, 0, 0, ctx.flags)
        dw, db = _finish([weight, bias], targets[:2])
        return dx.view(ctx.shp), dw, db, None, None


def layer_norm(x, weight=None, bias=None, eps: float = 1e-5):
    """LayerNorm over the last dim."""
    N = x.shape[-1]
    if _hip_path("layer_norm", x, weight, bias):
        return _LayerNormFn.apply(x, _cast(weight, x.dtype), _cast(bias, x.dtype), eps)
    return F.layer_norm(x, (N,), weight, bias, eps)


class _FusedAddLNFn(torch.autograd.Function):
    """(y, h) = (LN(h), h) with h = residual + dropout(x + x_bias)."""

    @staticmethod
    def forward(ctx, x, residual, weight, bias, x_bias, eps, p, seed, offset, flags=0):
        ctx.set_materialize_grads(False)
        shp = x.shape
        N = shp[-1]
        x2 = x.contiguous().view(-1, N)
        r2 = residual.contiguous().view(-1, N) if residual is not None else None
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        h = torch.empty_like(x2)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        _lib.call("piamd_layernorm_fwd", _lib.dtype_code(x2, fp16=True), x2.data_ptr(),
                  _lib.ptr(x_bias), _lib.ptr(r2), _lib.ptr(weight), _lib.ptr(bias), y.data_ptr(),
                  h.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows, N, float(eps), float(p),
                  seed, offset, flags, _lib.stream())
        ctx.save_for_backward(h, weight, bias, x_bias, mean, rstd)
        ctx.meta = (shp, p, seed, offset, residual is not None, flags)
        return y.view(shp), h.view(shp)

    @staticmethod
    def backward(ctx, dy, dh):
        h, weight, bias, x_bias, mean, rstd = ctx.saved_tensors
        shp, p, seed, offset, has_res, flags = ctx.meta
        rows, N = h.shape
        if dy is None and dh is None:
            return (None,) * 10
        dy2 = dy.contiguous().view(rows, N) if dy is not None else torch.zeros_like(h)
        dh2 = dh.contiguous().view(rows, N) if dh is not None else None
        dres = torch.empty_like(h)
        dx = torch.empty_like(h) if p > 0.0 else None
        pdt = weight.dtype if weight is not None else h.dtype
        targets = [_grad_target(weight, ctx.needs_input_grad[2], N, pdt, h.device),
                   _grad_target(bias, ctx.needs_input_grad[3], N, pdt, h.device),
                   _grad_target(x_bias, ctx.needs_input_grad[4], N, h.dtype, h.device)]
        # dbias(x_bias) = column sums of dx; without dropout dx == dres (same buffer)
        dx_ptr = dx.data_ptr() if dx is not None else (dres.data_ptr() if targets[2][0] is not None else None)
        _ln_bwd(_lib.dtype_code(h, fp16=True), dy2, h, weight, mean, rstd, dh2, dres, dx_ptr,
                targets, rows, N, p, seed, offset, flags)
        dw, db, dxb = _finish([weight, bias, x_bias], targets)
        dxo = (dx if dx is not None else dres).view(shp)
        return (dxo, (dres.view(shp) if has_res else None), dw, db, dxb, None, None, None, None,
                None)


def fused_add_layer_norm(x, residual, weight=None, bias=None, eps: float = 1e-5, x_bias=None,
                         dropout_p: float = 0.0, training: bool = True, need_residual: bool = True):
    """Returns ``(LN(h), h)`` with ``h = residual + dropout(x + x_bias)`` (residual may be None).
    ``need_residual=False`` (post-LN blocks, whose residual stream is the LN output): without
    autograd the kernel writes only LN(h) — no h, mean or rstd stores — and ``h`` is None."""
    p = float(dropout_p) if training else 0.0
    N = x.shape[-1]
    if _hip_path("fused_add_layer_norm", x, residual, weight, bias, x_bias) \
            and (residual is None or residual.dtype == x.dtype):
        seed, offset = _random.next_seed_offset(x.numel()) if p > 0 else (0, 0)
        dt = x.dtype
        if not need_residual and not (torch.is_grad_enabled() and any(
                t is not None and t.requires_grad for t in (x, residual, weight, bias, x_bias))):
            x2 = x.contiguous().view(-1, N)
            r2 = residual.contiguous().view(-1, N) if residual is not None else None
            y = torch.empty_like(x2)
            _lib.call("piamd_layernorm_fwd", _lib.dtype_code(x2, fp16=True), x2.data_ptr(),
                      _lib.ptr(_cast(x_bias, dt)), _lib.ptr(r2), _lib.ptr(_cast(weight, dt)),
                      _lib.ptr(_cast(bias, dt)), y.data_ptr(), None, None, None, x2.shape[0], N, float(eps),
                      float(p), seed, offset, 0, _lib.stream())
            return y.view(x.shape), None
        return _FusedAddLNFn.apply(x, residual, _cast(weight, dt), _cast(bias, dt), _cast(x_bias, dt),
                                   eps, p, seed, offset)
    t = x if x_bias is None else x + x_bias
    if p > 0:
        t = F.dropout(t, p, training=True)
    h = t if residual is None else residual + t
    return F.layer_norm(h, (N,), weight, bias, eps), h


def _rms_ref(h, weight, eps):
    hf = h.float() if h.element_size() < 4 else h  # 16-bit math in fp32; fp32/fp64 as is
    var = hf.pow(2).mean(-1, keepdim=True)
    y = (hf * torch.rsqrt(var + eps)).to(h.dtype)
    return y * weight if weight is not None else y


def rms_norm(x, weight=None, eps: float = 1e-6):
    """RMSNorm (LLaMA-style): ``x * rsqrt(mean(x^2) + eps) * weight`` — the LayerNorm kernels with
    the mean term dropped (one HBM read + one write per element, fused dweight column sums)."""
    if _hip_path("rms_norm", x, weight):
        return _LayerNormFn.apply(x, _cast(weight, x.dtype), None, eps, RMS)
    return _rms_ref(x, weight, eps)


def fused_add_rms_norm(x, residual, weight=None, eps: float = 1e-6, x_bias=None,
                       dropout_p: float = 0.0, training: bool = True):
    """Returns ``(RMSNorm(h), h)`` with ``h = residual + dropout(x + x_bias)``: the pre-norm
    residual stream of a LLaMA-style block in one pass (one kernel forward, one backward)."""
    p = float(dropout_p) if training else 0.0
    if _hip_path("fused_add_rms_norm", x, residual, weight, x_bias) \
            and (residual is None or residual.dtype == x.dtype):
        seed, offset = _random.next_seed_offset(x.numel()) if p > 0 else (0, 0)
        dt = x.dtype
        return _FusedAddLNFn.apply(x, residual, _cast(weight, dt), None, _cast(x_bias, dt), eps, p,
                                   seed, offset, RMS)
    t = x if x_bias is None else x + x_bias
    if p > 0:
        t = F.dropout(t, p, training=True)
    h = t if residual is None else residual + t
    return _rms_ref(h, weight, eps), h
