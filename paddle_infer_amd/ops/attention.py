"""Flash attention ops backed by ``csrc/kernels/flash_attn.hip``.

Parity: ``paddle.nn.functional.flash_attention`` / ``scaled_dot_product_attention``
(reference `python/paddle/nn/functional/flash_attention.py:142,440`), and the fork's
``memory_efficient_attention`` (`paddle/phi/kernels/fusion/cutlass/memory_efficient_attention.cu`).

Layout is Paddle's: ``[batch, seq, heads, head_dim]``. ``flash_attention_packed`` takes the fused
QKV projection output ``[B, S, Hq + 2*Hk, D]`` and returns the fused gradient, so neither forward
nor backward copies Q/K/V.
"""
from __future__ import annotations

import math

import torch

from . import _lib


def _strides(t):
    s = t.stride()
    return s[0], s[1], s[2]


def _fwd(q, k, v, causal, scale):
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    o = torch.empty((B, Sq, Hq, D), device=q.device, dtype=q.dtype)
    lse = torch.empty((B, Hq, Sq), device=q.device, dtype=torch.float32)
    _lib.call("piamd_flash_attn_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
              lse.data_ptr(), B, Sq, Sk, Hq, Hk, D, *_strides(q), *_strides(k), *_strides(v),
              *_strides(o), float(scale), int(causal), _lib.stream())
    return o, lse


def _bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale):
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    do = do.contiguous()
    assert o.stride() == do.stride()
    delta = torch.empty((B, Hq, Sq), device=q.device, dtype=torch.float32)
    dq_acc = torch.empty((B, Sq, Hq, D), device=q.device, dtype=torch.float32)
    _lib.call("piamd_flash_attn_bwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
              do.data_ptr(), lse.data_ptr(), delta.data_ptr(), dq_acc.data_ptr(), dq.data_ptr(),
              dk.data_ptr(), dv.data_ptr(), None, B, Sq, Sk, Hq, Hk, D, *_strides(q),
              *_strides(k), *_strides(v), *_strides(o), float(scale), int(causal), _lib.stream())


class _FlashAttnPackedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, hq, hk, causal, scale):
        q = qkv[:, :, :hq]
        k = qkv[:, :, hq:hq + hk]
        v = qkv[:, :, hq + hk:]
        o, lse = _fwd(q, k, v, causal, scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.meta = (hq, hk, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        hq, hk, causal, scale = ctx.meta
        dqkv = torch.empty_like(qkv)
        sl = lambda t: (t[:, :, :hq], t[:, :, hq:hq + hk], t[:, :, hq + hk:])
        q, k, v = sl(qkv)
        dq, dk, dv = sl(dqkv)
        _bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale)
        return dqkv, None, None, None, None


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        o, lse = _fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.meta = (causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        causal, scale = ctx.meta
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale)
        return dq, dk, dv, None, None


def attention_reference(q, k, v, causal=False, scale=None, attn_mask=None):
    """fp32 math attention on [B, S, H, D] (the numerics reference; also the CPU path)."""
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2)
    vf = v.float().transpose(1, 2)
    if Hk != Hq:
        rep = Hq // Hk
        kf = kf.repeat_interleave(rep, dim=1)
        vf = vf.repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if attn_mask is not None:
        s = s + attn_mask.float()
    if causal:
        i = torch.arange(Sq, device=q.device)[:, None]
        j = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill(j > i + (Sk - Sq), float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vf).transpose(1, 2)
    return o.to(q.dtype)


def _kernel_ok(q, k, v) -> bool:
    return (q.is_cuda and q.dtype == torch.bfloat16 and k.dtype == q.dtype and v.dtype == q.dtype
            and q.shape[-1] in (64, 128) and q.shape[2] % k.shape[2] == 0)


def flash_attention(q, k, v, causal: bool = False, scale: float | None = None):
    """q [B, Sq, Hq, D], k/v [B, Sk, Hk, D] → o [B, Sq, Hq, D]."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if _kernel_ok(q, k, v):
        return _FlashAttnFn.apply(q, k, v, causal, scale)
    if q.is_cuda and q.dtype == torch.bfloat16:
        raise RuntimeError(f"flash_attention: unsupported shape {tuple(q.shape)} on GPU")
    return attention_reference(q, k, v, causal, scale)


def flash_attention_packed(qkv, num_heads: int, num_kv_heads: int | None = None,
                           causal: bool = True, scale: float | None = None):
    """qkv [B, S, Hq + 2*Hk, D] (fused projection output) → o [B, S, Hq, D]."""
    hk = num_kv_heads or num_heads
    D = qkv.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and D in (64, 128):
        return _FlashAttnPackedFn.apply(qkv, num_heads, hk, causal, scale)
    q = qkv[:, :, :num_heads]
    k = qkv[:, :, num_heads:num_heads + hk]
    v = qkv[:, :, num_heads + hk:]
    return attention_reference(q, k, v, causal, scale)


# ------------------------------------------------------------------ variable length (packed)
def _varlen_fwd(q, k, v, cu_q, cu_k, max_q, max_k, causal, scale):
    T, Hq, D = q.shape
    Hk = k.shape[1]
    o = torch.empty((T, Hq, D), device=q.device, dtype=q.dtype)
    lse = torch.empty((Hq, T), device=q.device, dtype=torch.float32)
    _lib.call("piamd_flash_attn_varlen_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
              lse.data_ptr(), cu_q.numel() - 1, int(max_q), int(max_k), Hq, Hk, D,
              0, q.stride(0), q.stride(1), 0, k.stride(0), k.stride(1), 0, v.stride(0), v.stride(1),
              0, o.stride(0), o.stride(1), float(scale), int(causal), cu_q.data_ptr(),
              cu_k.data_ptr(), T, _lib.stream())
    return o, lse


class _FlashAttnVarlenFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, cu_q, cu_k, max_q, max_k, causal, scale):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        o, lse = _varlen_fwd(q, k, v, cu_q, cu_k, max_q, max_k, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse, cu_q, cu_k)
        ctx.meta = (max_q, max_k, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, cu_q, cu_k = ctx.saved_tensors
        max_q, max_k, causal, scale = ctx.meta
        do = do.contiguous()
        T, Hq, D = q.shape
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty((Hq, T), device=q.device, dtype=torch.float32)
        _lib.call("piamd_flash_attn_varlen_bwd", q.data_ptr(), k.data_ptr(), v.data_ptr(),
                  o.data_ptr(), do.data_ptr(), lse.data_ptr(), delta.data_ptr(), dq.data_ptr(),
                  dk.data_ptr(), dv.data_ptr(), cu_q.numel() - 1, int(max_q), int(max_k), Hq,
                  k.shape[1], D, 0, q.stride(0), q.stride(1), 0, k.stride(0), k.stride(1), 0,
                  v.stride(0), v.stride(1), 0, o.stride(0), o.stride(1), float(scale), int(causal),
                  cu_q.data_ptr(), cu_k.data_ptr(), T, _lib.stream())
        return dq, dk, dv, None, None, None, None, None, None


def attention_varlen_reference(q, k, v, cu_q, cu_k, causal=False, scale=None):
    cq, ck = cu_q.tolist(), cu_k.tolist()
    outs = []
    for i in range(len(cq) - 1):
        outs.append(attention_reference(q[cq[i]:cq[i + 1]][None], k[ck[i]:ck[i + 1]][None],
                                        v[ck[i]:ck[i + 1]][None], causal, scale)[0])
    return torch.cat(outs, 0) if outs else q[:0].clone()


def flash_attention_varlen(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                           causal: bool = False, scale: float | None = None):
    """Packed variable-length attention in ONE launch per pass: q [Tq, Hq, D], k/v [Tk, Hk, D],
    ``cu_seqlens_*`` int32 [B+1] cumulative offsets (device), ``max_seqlen_*`` host ints sizing the
    grid (blocks past a sequence's end exit). Causal masking is bottom-right aligned per sequence.
    Reference: `flash_attn_unpadded` / `variable_length_memory_efficient_attention.cu`."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if (q.is_cuda and q.dtype == torch.bfloat16 and k.dtype == q.dtype and v.dtype == q.dtype
            and q.shape[-1] in (64, 128) and q.shape[1] % k.shape[1] == 0):
        cu_q = cu_seqlens_q.to(device=q.device, dtype=torch.int32).contiguous()
        cu_k = cu_seqlens_k.to(device=q.device, dtype=torch.int32).contiguous()
        return _FlashAttnVarlenFn.apply(q, k, v, cu_q, cu_k, int(max_seqlen_q), int(max_seqlen_k),
                                        causal, scale)
    if q.is_cuda and q.dtype == torch.bfloat16:
        raise RuntimeError(f"flash_attention_varlen: unsupported shape {tuple(q.shape)} on GPU")
    return attention_varlen_reference(q, k, v, cu_seqlens_q, cu_seqlens_k, causal, scale)
