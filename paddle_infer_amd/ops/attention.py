"""Flash attention ops backed by ``csrc/kernels/flash_attn.hip``.

Parity: ``paddle.nn.functional.flash_attention`` / ``scaled_dot_product_attention``
(reference `python/paddle/nn/functional/flash_attention.py:142,440`), and the fork's
``memory_efficient_attention`` (`paddle/phi/kernels/fusion/cutlass/memory_efficient_attention.cu`).

Layout is Paddle's: ``[batch, seq, heads, head_dim]``. ``flash_attention_packed`` takes the fused
QKV projection output ``[B, S, Hq + 2*Hk, D]`` and returns the fused gradient, so neither forward
nor backward copies Q/K/V.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch
import torch.nn.functional as F

from . import _lib
from ..framework import random as _random


NATIVE_D = (64, 96, 128)  # forward + backward kernels
WIDE_D = 256  # forward kernel; the backward runs on the own batched GEMMs (_bwd_wide_own)


def _padded_d(D: int, wide: bool = False) -> int | None:
    """Kernel head dim for a model head dim: native, or the next native size (zero-padded
    channels change neither Q·Kᵀ nor the real output columns). None if unsupported. ``wide``:
    head dims up to 256 run on the wide forward kernel."""
    if D % 8:
        return None
    for n in NATIVE_D + ((WIDE_D,) if wide else ()):
        if D <= n:
            return n
    return None


def _strides(t):
    s = t.stride()
    return s[0], s[1], s[2]


def _prep_mask(mask, B, H, Sq, Sk, dtype):
    """Additive mask for the kernel: input dtype, [1|B, 1|H, Sq, Skp] with Skp % 4 == 0, element
    strides % 4 == 0 (8-B reads of 4 keys). bool masks: True = attend (0), False = -inf."""
    if mask is None:
        return None
    m = mask.detach()
    if m.dtype == torch.bool:
        m = torch.zeros(m.shape, device=m.device, dtype=dtype).masked_fill(~m, float("-inf"))
    while m.dim() < 4:
        m = m.unsqueeze(0)
    mb, mh = m.shape[0], m.shape[1]
    if mb not in (1, B) or mh not in (1, H) or m.shape[-2] not in (1, Sq) or m.shape[-1] != Sk:
        raise ValueError(f"attention mask {tuple(mask.shape)} does not broadcast to "
                         f"[{B}, {H}, {Sq}, {Sk}]")
    m = m.to(dtype)
    Skp = (Sk + 3) // 4 * 4
    ok = (m.shape[-2] == Sq and m.stride(-1) == 1 and Sk == Skp and m.data_ptr() % 8 == 0
          and all((st % 4 == 0) or n == 1 for st, n in zip(m.stride()[:3], m.shape[:3])))
    if not ok:
        buf = torch.zeros((mb, mh, Sq, Skp), device=m.device, dtype=dtype)
        buf[..., :Sk] = m
        m = buf
    return m


def _args(q, k, v, o, lse, causal, scale, mask, p, seed, off, B, Sq, Sk, Hq, Hk, D,
          cu_q=None, cu_k=None, ltot=0):
    a = _lib.FaArgs()
    a.q, a.k, a.v, a.o, a.lse = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), _lib.ptr(lse)
    a.cu_q, a.cu_k = _lib.ptr(cu_q), _lib.ptr(cu_k)
    a.B, a.Sq, a.Sk, a.Hq, a.Hk, a.D, a.ltot, a.causal = B, Sq, Sk, Hq, Hk, D, ltot, int(causal)
    if cu_q is None:
        (a.sqb, a.sqs, a.sqh), (a.skb, a.sks, a.skh) = _strides(q), _strides(k)
        (a.svb, a.svs, a.svh), (a.sob, a.sos, a.soh) = _strides(v), _strides(o)
    else:  # packed [T, H, D]
        a.sqs, a.sqh, a.sks, a.skh = q.stride(0), q.stride(1), k.stride(0), k.stride(1)
        a.svs, a.svh, a.sos, a.soh = v.stride(0), v.stride(1), o.stride(0), o.stride(1)
    if mask is not None:
        a.mask = mask.data_ptr()
        a.smb = mask.stride(0) if mask.shape[0] > 1 else 0
        a.smh = mask.stride(1) if mask.shape[1] > 1 else 0
        a.smq = mask.stride(2) if mask.shape[2] > 1 else 0
    a.scale, a.p_drop, a.seed, a.offset = float(scale), float(p), int(seed), int(off)
    return a


def _f16(t) -> int:
    return int(t.dtype == torch.float16)


def _fwd(q, k, v, causal, scale, mask=None, p=0.0, seed=0, off=0):
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    o = torch.empty((B, Sq, Hq, D), device=q.device, dtype=q.dtype)
    lse = torch.empty((B, Hq, Sq), device=q.device, dtype=torch.float32)
    a = _args(q, k, v, o, lse, causal, scale, mask, p, seed, off, B, Sq, Sk, Hq, Hk, D)
    _fa_asm_load()
    _lib.call("piamd_fa_fwd", ctypes.byref(a), _f16(q), _lib.stream())
    return o, lse


_FA_ASM_READY = [False]


def _fa_asm_load():
    """Load the assembly flash-attention backward code object (`_lib/piamd_fa.hsaco`, from
    `csrc/asm/fa_gen.py`) once; `piamd_fa_bwd` then runs its dK/dV kernel where it applies."""
    if _FA_ASM_READY[0]:
        return
    import os
    from .. import _build
    path = os.environ.get("PIAMD_FA_HSACO") or _build.FA_HSACO  # ablation builds (measurement)
    if not os.path.exists(path):
        raise RuntimeError(f"assembly flash-attention code object missing ({path}); run "
                           "`python -m paddle_infer_amd._build`")
    _lib.call("piamd_fa_asm_load", path.encode())
    _FA_ASM_READY[0] = True


def _bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale, mask=None, p=0.0, seed=0, off=0):
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    if do.stride() != o.stride():
        do = do.contiguous() if o.is_contiguous() else torch.empty_like(o).copy_(do)
    assert o.stride() == do.stride()
    assert dq.stride() == q.stride() and dk.stride() == k.stride() and dv.stride() == v.stride()
    # per-row backward constants: [0] = −δ (rowsum dO·O), [1] = −lse/scale (flash_attn.h pre-pass)
    delta = torch.empty((2, B, Hq, Sq), device=q.device, dtype=torch.float32)
    a = _args(q, k, v, o, lse, causal, scale, mask, p, seed, off, B, Sq, Sk, Hq, Hk, D)
    a.dout, a.delta, a.dq, a.dk, a.dv = do.data_ptr(), delta.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
    a.ds = None
    _fa_asm_load()
    _lib.call("piamd_fa_bwd", ctypes.byref(a), _f16(q), _lib.stream())


class _FlashAttnPackedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, hq, hk, causal, scale, p, seed, off):
        q = qkv[:, :, :hq]
        k = qkv[:, :, hq:hq + hk]
        v = qkv[:, :, hq + hk:]
        o, lse = _fwd(q, k, v, causal, scale, None, p, seed, off)
        ctx.save_for_backward(qkv, o, lse)
        ctx.meta = (hq, hk, causal, scale, p, seed, off)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        hq, hk, causal, scale, p, seed, off = ctx.meta
        dqkv = torch.empty_like(qkv)
        sl = lambda t: (t[:, :, :hq], t[:, :, hq:hq + hk], t[:, :, hq + hk:])
        q, k, v = sl(qkv)
        dq, dk, dv = sl(dqkv)
        _bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale, None, p, seed, off)
        return dqkv, None, None, None, None, None, None, None


def _ceil_to(x, m, lo=0):
    return max(lo, -(-x // m) * m)


def _bwd_wide_own(q, k, v, o, lse, do, causal, scale, mask, chunk_bytes=1 << 30):
    """Backward of the wide-head (D > 128) forward on the framework's own kernels: per
    (batch · head) and query chunk, five batched assembly GEMMs (csrc/asm/gemm_gen.py) —
    S = Q·Kᵀ and dP = dO·Vᵀ into f32, dV += Pᵀ·dO and dK += dSᵀ·Q accumulated in f32, dQ = dS·K —
    with P = exp(S − lse) and dS = P∘(dP − δ) in f32 between them (P and dS rounded to the
    operands' dtype for the GEMMs, as the fused kernels do). Rows / keys / head dim are
    zero-padded to the GEMM's 64-multiples; padded keys are masked, padded queries carry lse = +inf
    (P = 0). Memory O(chunk · Sk)."""
    from .gemm import asm_gemm as _asm
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    rep = Hq // Hk
    dt, dev = q.dtype, q.device

    def asm_gemm(a, b, trans_a=False, trans_b=False, out=None, out_f32=False, accumulate=False):
        if a.is_cuda:
            return _asm(a, b, trans_a, trans_b, out=out, out_f32=out_f32, accumulate=accumulate)
        # CPU: the same contract in PyTorch (the numerics reference of the CPU tier)
        r = torch.matmul(a.transpose(-1, -2) if trans_a else a, b.transpose(-1, -2) if trans_b else b)
        if out is not None:
            if accumulate:
                out += r.to(out.dtype)
            else:
                out.copy_(r)
            return out
        return r.to(torch.float32 if out_f32 else a.dtype)

    Dp, Sqp, Skp = _ceil_to(D, 64, 128), _ceil_to(Sq, 64, 128), _ceil_to(Sk, 64, 128)
    BH = B * Hq

    def heads(t, S, Sp, H):
        x = t.transpose(1, 2)
        if H != Hq:
            x = x.repeat_interleave(rep, dim=1)
        out = torch.zeros((B, Hq, Sp, Dp), dtype=dt, device=dev)
        out[:, :, :S, :D] = x
        return out.view(BH, Sp, Dp)

    qh, doh = heads(q, Sq, Sqp, Hq), heads(do, Sq, Sqp, Hq)
    kh, vh = heads(k, Sk, Skp, Hk), heads(v, Sk, Skp, Hk)
    st = torch.float32 if dt in (torch.bfloat16, torch.float16) else dt  # statistics dtype
    delta = torch.zeros((BH, Sqp), dtype=st, device=dev)
    delta[:, :Sq] = (do.to(st) * o.to(st)).sum(-1).transpose(1, 2).reshape(BH, Sq)
    lse_p = torch.full((BH, Sqp), float("inf"), dtype=st, device=dev)
    lse_p[:, :Sq] = lse.to(st).reshape(BH, Sq)
    mk = None
    if mask is not None:
        mk = torch.zeros((B, mask.shape[1], mask.shape[2] if mask.shape[2] == 1 else Sqp, Skp),
                         dtype=st, device=dev)
        mk[..., :mask.shape[2], :Sk] = mask[..., :Sk].to(st)
    dq = torch.empty((BH, Sqp, Dp), dtype=dt, device=dev)
    acc_t = torch.float32 if dt in (torch.bfloat16, torch.float16) else dt
    dk = torch.zeros((BH, Skp, Dp), dtype=acc_t, device=dev)
    dv = torch.zeros((BH, Skp, Dp), dtype=acc_t, device=dev)
    kj = torch.arange(Skp, device=dev)
    ch = max(128, min(Sqp, (chunk_bytes // max(1, BH * Skp * 4 * 3)) // 64 * 64))
    q0 = 0
    while q0 < Sqp:
        q1 = Sqp if Sqp - q0 < ch + 128 else q0 + ch  # no tail chunk shorter than 128 rows
        qs, dos = qh[:, q0:q1], doh[:, q0:q1]
        s = asm_gemm(qs, kh, trans_b=True, out_f32=True).mul_(scale)
        s = s.view(B, Hq, q1 - q0, Skp)
        if mk is not None:
            s += mk if mk.shape[2] == 1 else mk[:, :, q0:q1]
        bad = kj >= Sk
        if causal:
            qi = torch.arange(q0, q1, device=dev)[:, None]
            bad = bad | (kj[None, :] > qi + (Sk - Sq))
        s = s.masked_fill(bad, float("-inf")).view(BH, q1 - q0, Skp)
        p = torch.exp(s - lse_p[:, q0:q1, None])
        pb = p.to(dt)
        asm_gemm(pb, dos, trans_a=True, out=dv, accumulate=True)
        dp = asm_gemm(dos, vh, trans_b=True, out_f32=True)
        dsb = (p * (dp - delta[:, q0:q1, None])).mul_(scale).to(dt)
        dq[:, q0:q1] = asm_gemm(dsb, kh)
        asm_gemm(dsb, qs, trans_a=True, out=dk, accumulate=True)
        q0 = q1
    dq = dq.view(B, Hq, Sqp, Dp)[:, :, :Sq, :D].transpose(1, 2)
    dk = dk.view(B, Hq, Skp, Dp)[:, :, :Sk, :D]
    dv = dv.view(B, Hq, Skp, Dp)[:, :, :Sk, :D]
    if rep > 1:
        dk = dk.reshape(B, Hk, rep, Sk, D).sum(2)
        dv = dv.reshape(B, Hk, rep, Sk, D).sum(2)
    return dq.contiguous(), dk.transpose(1, 2).to(dt).contiguous(), dv.transpose(1, 2).to(dt).contiguous()


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, mask, p, seed, off):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        o, lse = _fwd(q, k, v, causal, scale, mask, p, seed, off)
        ctx.save_for_backward(q, k, v, o, lse, mask)
        ctx.meta = (causal, scale, p, seed, off)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, mask = ctx.saved_tensors
        causal, scale, p, seed, off = ctx.meta
        if q.shape[-1] > NATIVE_D[-1]:  # wide heads: the backward on the own batched GEMMs
            dq, dk, dv = _bwd_wide_own(q, k, v, o, lse, do.contiguous(), causal, scale, mask)
            return dq, dk, dv, None, None, None, None, None, None
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale, mask, p, seed, off)
        return dq, dk, dv, None, None, None, None, None, None


def attention_reference(q, k, v, causal=False, scale=None, attn_mask=None, dropout_p=0.0,
                        training=True):
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
        if attn_mask.dtype == torch.bool:
            s = s.masked_fill(~attn_mask, float("-inf"))
        else:
            s = s + attn_mask.float()
    if causal:
        i = torch.arange(Sq, device=q.device)[:, None]
        j = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill(j > i + (Sk - Sq), float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)  # fully masked rows -> 0 (kernel convention)
    if dropout_p > 0 and training:
        p = F.dropout(p, dropout_p)
    o = torch.matmul(p, vf).transpose(1, 2)
    return o.to(q.dtype)


def _kernel_ok(op, q, k, v, wide=False) -> bool:
    """True: the MFMA kernel takes it. GPU inputs it cannot take are recorded (warn once)."""
    if not (q.is_cuda and k.is_cuda and v.is_cuda):
        return False
    if q.dtype not in (torch.bfloat16, torch.float16) or k.dtype != q.dtype or v.dtype != q.dtype:
        _lib.fallback(op, f"dtype {q.dtype} (kernel: bf16/fp16)")
        return False
    if _padded_d(q.shape[-1], wide) is None:
        _lib.fallback(op, f"head dim {q.shape[-1]} (kernel: multiple of 8, <= {WIDE_D if wide else 128})")
        return False
    if q.shape[-2] % k.shape[-2]:
        _lib.fallback(op, "q heads not a multiple of kv heads")
        return False
    return True


def _drop_state(p, training, B, H, Sq, Sk):
    p = float(p) if training else 0.0
    if p <= 0.0:
        return 0.0, 0, 0
    seed, off = _random.next_seed_offset(B * H * Sq * Sk)
    return p, seed, off


def flash_attention(q, k, v, causal: bool = False, scale: float | None = None, attn_mask=None,
                    dropout_p: float = 0.0, training: bool = True):
    """q [B, Sq, Hq, D], k/v [B, Sk, Hk, D] → o [B, Sq, Hq, D]. ``attn_mask``: additive (or bool,
    True = attend) mask broadcastable to [B, Hq, Sq, Sk]; ``dropout_p``: attention-probability
    dropout, regenerated in backward from the counter RNG (nothing stored)."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    # wide heads (129..256): native forward; without dropout (the chunked backward cannot replay
    # the kernel's dropout mask)
    wide = D > NATIVE_D[-1] and (dropout_p == 0.0 or not training)
    if _kernel_ok("flash_attention", q, k, v, wide):
        B, Sq, Hq, _ = q.shape
        Sk = k.shape[1]
        mask = _prep_mask(attn_mask, B, Hq, Sq, Sk, q.dtype)
        p, seed, off = _drop_state(dropout_p, training, B, Hq, Sq, Sk)
        Dp = _padded_d(D, wide)
        if Dp != D:  # zero channels: Q·Kᵀ unchanged, extra output columns are zero (sliced off)
            pad = (0, Dp - D)
            o = _FlashAttnFn.apply(F.pad(q, pad), F.pad(k, pad), F.pad(v, pad), causal, scale, mask,
                                   p, seed, off)
            return o[..., :D]
        return _FlashAttnFn.apply(q, k, v, causal, scale, mask, p, seed, off)
    return attention_reference(q, k, v, causal, scale, attn_mask, dropout_p, training)


def flash_attention_packed(qkv, num_heads: int, num_kv_heads: int | None = None,
                           causal: bool = True, scale: float | None = None,
                           dropout_p: float = 0.0, training: bool = True):
    """qkv [B, S, Hq + 2*Hk, D] (fused projection output) → o [B, S, Hq, D]."""
    hk = num_kv_heads or num_heads
    D = qkv.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    q = qkv[:, :, :num_heads]
    k = qkv[:, :, num_heads:num_heads + hk]
    v = qkv[:, :, num_heads + hk:]
    if _kernel_ok("flash_attention_packed", q, k, v):
        if D not in NATIVE_D:
            return flash_attention(q, k, v, causal, scale, None, dropout_p, training)
        B, S = qkv.shape[0], qkv.shape[1]
        p, seed, off = _drop_state(dropout_p, training, B, num_heads, S, S)
        return _FlashAttnPackedFn.apply(qkv, num_heads, hk, causal, scale, p, seed, off)
    return attention_reference(q, k, v, causal, scale, None, dropout_p, training)


# ------------------------------------------------------------------ variable length (packed)
def _varlen_args(q, k, v, o, lse, cu_q, cu_k, max_q, max_k, causal, scale, p, seed, off):
    T, Hq, D = q.shape
    return _args(q, k, v, o, lse, causal, scale, None, p, seed, off, cu_q.numel() - 1, int(max_q),
                 int(max_k), Hq, k.shape[1], D, cu_q, cu_k, T)


class _FlashAttnVarlenFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, cu_q, cu_k, max_q, max_k, causal, scale, p, seed, off):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        T, Hq, D = q.shape
        o = torch.empty((T, Hq, D), device=q.device, dtype=q.dtype)
        lse = torch.empty((Hq, T), device=q.device, dtype=torch.float32)
        a = _varlen_args(q, k, v, o, lse, cu_q, cu_k, max_q, max_k, causal, scale, p, seed, off)
        _lib.call("piamd_fa_fwd", ctypes.byref(a), _f16(q), _lib.stream())
        ctx.save_for_backward(q, k, v, o, lse, cu_q, cu_k)
        ctx.meta = (max_q, max_k, causal, scale, p, seed, off)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, cu_q, cu_k = ctx.saved_tensors
        max_q, max_k, causal, scale, p, seed, off = ctx.meta
        do = do.contiguous()
        T, Hq, D = q.shape
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty((2, Hq, T), device=q.device, dtype=torch.float32)  # −δ, −lse/scale
        a = _varlen_args(q, k, v, o, lse, cu_q, cu_k, max_q, max_k, causal, scale, p, seed, off)
        a.dout, a.delta, a.dq, a.dk, a.dv = (do.data_ptr(), delta.data_ptr(), dq.data_ptr(),
                                             dk.data_ptr(), dv.data_ptr())
        _lib.call("piamd_fa_bwd", ctypes.byref(a), _f16(q), _lib.stream())
        return dq, dk, dv, None, None, None, None, None, None, None, None, None


def attention_varlen_reference(q, k, v, cu_q, cu_k, causal=False, scale=None):
    cq, ck = cu_q.tolist(), cu_k.tolist()
    outs = []
    for i in range(len(cq) - 1):
        outs.append(attention_reference(q[cq[i]:cq[i + 1]][None], k[ck[i]:ck[i + 1]][None],
                                        v[ck[i]:ck[i + 1]][None], causal, scale)[0])
    return torch.cat(outs, 0) if outs else q[:0].clone()


def flash_attention_varlen(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                           causal: bool = False, scale: float | None = None,
                           dropout_p: float = 0.0, training: bool = True):
    """Packed variable-length attention in ONE launch per pass: q [Tq, Hq, D], k/v [Tk, Hk, D],
    ``cu_seqlens_*`` int32 [B+1] cumulative offsets (device), ``max_seqlen_*`` host ints sizing the
    grid (blocks past a sequence's end exit). Causal masking is bottom-right aligned per sequence.
    Reference: `flash_attn_unpadded` / `variable_length_memory_efficient_attention.cu`."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if _kernel_ok("flash_attention_varlen", q, k, v):
        cu_q = cu_seqlens_q.to(device=q.device, dtype=torch.int32).contiguous()
        cu_k = cu_seqlens_k.to(device=q.device, dtype=torch.int32).contiguous()
        p, seed, off = _drop_state(dropout_p, training, cu_q.numel() - 1, q.shape[1],
                                   int(max_seqlen_q), int(max_seqlen_k))
        Dp = _padded_d(D)
        if Dp != D:
            pad = (0, Dp - D)
            q, k, v = F.pad(q, pad), F.pad(k, pad), F.pad(v, pad)
        o = _FlashAttnVarlenFn.apply(q, k, v, cu_q, cu_k, int(max_seqlen_q), int(max_seqlen_k),
                                     causal, scale, p, seed, off)
        return o[..., :D] if Dp != D else o
    return attention_varlen_reference(q, k, v, cu_seqlens_q, cu_seqlens_k, causal, scale)
