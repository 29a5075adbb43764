"""``paddle.incubate.nn.functional`` — fused transformer ops on the MI355X kernel library.

Parity: reference `python/paddle/incubate/nn/functional/fused_transformer.py`
(fused_feedforward:31, fused_bias_dropout_residual_layer_norm:275, fused_multi_head_attention:465,
fused_multi_transformer:833) and `fused_matmul_bias.py` (fused_matmul_bias, fused_linear), plus
the fork's weight-only / MoE fused multi-transformer variants
(`fluid/operators/fused/fused_multi_transformer_{weight_only,moe}_op.cu`).

How they map onto the hardware (instead of the reference's one-CUDA-op-per-layer):
* GEMMs: the framework's own kernels (``ops.gemm``: assembly GEMM / skinny MFMA kernel with bias +
  activation epilogues) — or the in-tree weight-only int8/int4 MFMA kernel;
* LN + residual + bias (+dropout) → one pass of ``layernorm.hip`` (fused_add_layer_norm);
* bias + activation → ``elementwise.hip``; QKV bias + RoPE + KV-cache write → ``infer.hip``;
* context attention → ``flash_attn.hip``; decode attention → split-K ``infer.hip``;
* the per-layer launch chain is replayed as a hipGraph by ``inference.generation``.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from ... import ops
from ...ops import inference as _inf


# ----------------------------------------------------------------------------- helpers
def _to_additive_mask(mask, dtype):
    if mask is None:
        return None
    if mask.dtype == torch.bool:
        return torch.zeros(mask.shape, dtype=dtype, device=mask.device).masked_fill(~mask, float("-inf"))
    if not mask.is_floating_point():
        return torch.zeros(mask.shape, dtype=dtype, device=mask.device).masked_fill(mask == 0, float("-inf"))
    return mask.to(dtype)


def _dropout(x, p, training, mode):
    if p == 0.0:
        return x
    if not training:
        return x * (1.0 - p) if mode == "downscale_in_infer" else x
    if mode == "downscale_in_infer":
        return ops.dropout(x, p, True) * (1.0 - p)
    return ops.dropout(x, p, True)


def _ln(x, w, b, eps):
    return ops.layer_norm(x, w, b, eps)


def _mm(x, w, bias=None, transpose=False):
    """x @ w (+ bias), w stored [in, out] (Paddle) unless ``transpose`` (own GEMMs for bf16 / fp16:
    2-D weights through the linear path, bias in the GEMM epilogue)."""
    if w.dim() == 2 and not transpose:
        from ...ops.linear import linear
        return linear(x, w, bias)
    from ...ops.gemm import matmul
    y = matmul(x, w, False, transpose)
    return y + bias if bias is not None else y


def attention_core(qkv, num_heads, num_kv_heads=None, attn_mask=None, causal=False,
                   attn_dropout=0.0, training=False, mode="upscale_in_train", scale=None):
    """qkv: [B, S, Hq+2Hk, D] → [B, S, Hq*D]. Flash kernel (with in-kernel mask add and attention
    dropout) whenever dropout is upscale_in_train; the downscale_in_infer dropout convention takes
    GEMM + fused masked softmax (``elementwise.hip``)."""
    B, S, _, D = qkv.shape
    hq, hk = num_heads, num_kv_heads or num_heads
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    drop = attn_dropout if training else 0.0
    if attn_mask is None and (drop == 0.0 or mode == "upscale_in_train"):
        o = ops.flash_attention_packed(qkv, hq, hk, causal=causal, scale=scale, dropout_p=drop,
                                       training=training)
        return o.reshape(B, S, hq * D)
    if drop == 0.0 or mode == "upscale_in_train":
        q = qkv[:, :, :hq]
        k = qkv[:, :, hq:hq + hk]
        v = qkv[:, :, hq + hk:]
        m = _to_additive_mask(attn_mask, qkv.dtype)
        o = ops.flash_attention(q, k, v, causal, scale, attn_mask=m, dropout_p=drop,
                                training=training)
        return o.reshape(B, S, hq * D)
    q = qkv[:, :, :hq].transpose(1, 2)
    k = qkv[:, :, hq:hq + hk].transpose(1, 2)
    v = qkv[:, :, hq + hk:].transpose(1, 2)
    if hk != hq:
        k = k.repeat_interleave(hq // hk, 1)
        v = v.repeat_interleave(hq // hk, 1)
    from ...ops.gemm import matmul
    s = matmul(q, k, False, True)
    m = _to_additive_mask(attn_mask, s.dtype)
    if m is not None:
        m = m.expand(B, hq, S, s.shape[-1]) if m.dim() == 4 else m
    p = ops.fused_softmax_mask(s, m.contiguous() if m is not None else None, scale, causal)
    p = _dropout(p, attn_dropout, training, mode)
    o = matmul(p, v)
    return o.transpose(1, 2).reshape(B, S, hq * D)


# ----------------------------------------------------------------------------- small fused ops
def fused_matmul_bias(x, y, bias=None, transpose_x=False, transpose_y=False, name=None):
    """Reference `fused_matmul_bias.py:21` (cublasLt bias epilogue, `fused_gemm_epilogue_op.cu`).
    bf16 / fp16: the framework's own GEMM with the bias in its epilogue — through the linear path
    (own forward AND backward kernels) for a 2-D [in, out] weight, ``ops.gemm.gemm_nt`` for a
    [out, in] one; other layouts / dtypes: ``ops.gemm.matmul`` + bias."""
    from ...ops import gemm as G
    if bias is not None and not transpose_x and x.dim() >= 2 and y.dim() == 2 and G.own_dtype(x, y):
        if not transpose_y:
            from ...ops.linear import linear
            return linear(x, y, bias)
        if not (torch.is_grad_enabled() and (x.requires_grad or y.requires_grad or bias.requires_grad)):
            lead = x.shape[:-1]
            out = G.gemm_nt(x.reshape(-1, x.shape[-1]), y.contiguous(), bias=bias)
            return out.reshape(*lead, y.shape[0])
    out = G.matmul(x, y, transpose_x, transpose_y)
    return out + bias if bias is not None else out


def fused_linear(x, weight, bias=None, transpose_weight=False, name=None):
    return fused_matmul_bias(x, weight, bias, False, transpose_weight)


def fused_linear_activation(x, y, bias, trans_x=False, trans_y=False, activation=None):
    """Reference `fused_matmul_bias.py` fused_linear_activation (GELU / ReLU epilogue): one own GEMM
    with bias + activation in its epilogue at inference (GELU: the tanh form, as cublasLt's)."""
    from ...ops import gemm as G
    act = activation or "none"
    if (not trans_x and x.dim() >= 2 and y.dim() == 2 and bias is not None and G.own_dtype(x, y)
            and not (torch.is_grad_enabled() and (x.requires_grad or y.requires_grad))):
        from ...ops.linear import linear_bias_act
        return linear_bias_act(x, y.contiguous(), bias, act, weight_out_in=trans_y)
    out = fused_matmul_bias(x, y, None, trans_x, trans_y)
    return ops.bias_act(out, bias, act)


def fused_bias_dropout_residual_layer_norm(x, residual, bias=None, ln_scale=None, ln_bias=None,
                                           dropout_rate=0.5, ln_epsilon=1e-5, training=True,
                                           mode="upscale_in_train", name=None):
    """y = layer_norm(residual + dropout(bias + x)) — one ``layernorm.hip`` pass."""
    if mode == "downscale_in_infer" and dropout_rate > 0:
        h = residual + _dropout(x + (bias if bias is not None else 0), dropout_rate, training, mode)
        return _ln(h, ln_scale, ln_bias, ln_epsilon)
    y, _ = ops.fused_add_layer_norm(x, residual, ln_scale, ln_bias, ln_epsilon, bias,
                                    dropout_rate if training else 0.0, training)
    return y


def fused_feedforward(x, linear1_weight, linear2_weight, linear1_bias=None, linear2_bias=None,
                      ln1_scale=None, ln1_bias=None, ln2_scale=None, ln2_bias=None,
                      dropout1_rate=0.5, dropout2_rate=0.5, seed=None, activation="relu",
                      ln1_epsilon=1e-5, ln2_epsilon=1e-5, pre_layer_norm=False, training=True,
                      mode="upscale_in_train", ring_id=-1, add_residual=True, name=None, group=None):
    residual = x
    out = _ln(x, ln1_scale, ln1_bias, ln1_epsilon) if pre_layer_norm else x
    from ...ops.linear import fused_mlp, fused_mlp_supported
    if ((dropout1_rate == 0.0 or not training) and linear1_bias is not None
            and fused_mlp_supported(out, linear1_weight, linear1_bias, linear2_weight, activation)):
        # relu / gelu_tanh: both GEMMs on the assembly kernel, bias + activation in the FFN1
        # epilogue and the activation backward in the FFN2 data-gradient epilogue (exact-erf GELU
        # keeps the separate bias-act kernel: the epilogue GELU is the tanh form)
        o = fused_mlp(out, linear1_weight, linear1_bias, linear2_weight, activation)
    else:
        h = ops.bias_act(_mm(out, linear1_weight), linear1_bias, activation)
        h = _dropout(h, dropout1_rate, training, mode)
        o = _mm(h, linear2_weight)
    if group is not None:
        torch.distributed.all_reduce(o, group=group)
    if pre_layer_norm:
        o = o + linear2_bias if linear2_bias is not None else o
        o = _dropout(o, dropout2_rate, training, mode)
        return residual + o if add_residual else o
    return fused_bias_dropout_residual_layer_norm(
        o, residual if add_residual else torch.zeros_like(o), linear2_bias, ln2_scale, ln2_bias,
        dropout2_rate, ln2_epsilon, training, mode)


def fused_multi_head_attention(x, qkv_weight, linear_weight, pre_layer_norm=False,
                               pre_ln_scale=None, pre_ln_bias=None, ln_scale=None, ln_bias=None,
                               pre_ln_epsilon=1e-5, qkv_bias=None, linear_bias=None, cache_kv=None,
                               attn_mask=None, dropout_rate=0.5, attn_dropout_rate=0.5,
                               dropout_seed=None, attn_dropout_seed=None, ln_epsilon=1e-5,
                               training=True, mode="upscale_in_train", ring_id=-1,
                               add_residual=True, name=None, group=None, causal=False,
                               transpose_qkv_wb=False, num_heads=None):
    """qkv_weight [3, H, D, E] (or [E, 3E] with ``transpose_qkv_wb``), linear_weight [E, E].
    With ``cache_kv`` ([2, B, H, S_cache, D]) returns (out, new_cache_kv) like the reference."""
    B, S, E = x.shape
    residual = x
    out = _ln(x, pre_ln_scale, pre_ln_bias, pre_ln_epsilon) if pre_layer_norm else x
    if transpose_qkv_wb:
        H = num_heads
        D = E // H
        qkv = _mm(out, qkv_weight)
    else:
        _, H, D, _ = qkv_weight.shape
        from ...ops.gemm import matmul
        qkv = matmul(out, qkv_weight.reshape(3 * H * D, E), False, True)
    if qkv_bias is not None:
        qkv = qkv + qkv_bias.reshape(-1)
    qkv = qkv.reshape(B, S, 3 * H, D)
    new_cache = None
    if cache_kv is not None:
        k = torch.cat([cache_kv[0], qkv[:, :, H:2 * H].transpose(1, 2)], 2)
        v = torch.cat([cache_kv[1], qkv[:, :, 2 * H:].transpose(1, 2)], 2)
        new_cache = torch.stack([k, v])
        q = qkv[:, :, :H].transpose(1, 2)
        from ...ops.gemm import matmul
        s = matmul(q, k, False, True)
        m = _to_additive_mask(attn_mask, s.dtype)
        p = ops.fused_softmax_mask(s, m.expand_as(s).contiguous() if m is not None else None,
                                   1.0 / math.sqrt(D))
        p = _dropout(p, attn_dropout_rate, training, mode)
        a = matmul(p, v).transpose(1, 2).reshape(B, S, H * D)
    else:
        a = attention_core(qkv, H, H, attn_mask, causal, attn_dropout_rate, training, mode)
    o = _mm(a, linear_weight)
    if group is not None:
        torch.distributed.all_reduce(o, group=group)
    if pre_layer_norm:
        o = o + linear_bias if linear_bias is not None else o
        o = _dropout(o, dropout_rate, training, mode)
        res = residual + o if add_residual else o
    else:
        res = fused_bias_dropout_residual_layer_norm(
            o, residual if add_residual else torch.zeros_like(o), linear_bias, ln_scale, ln_bias,
            dropout_rate, ln_epsilon, training, mode)
    return (res, new_cache) if cache_kv is not None else res


# ----------------------------------------------------------------------------- multi-transformer
class _Linear:
    """A projection: bf16 weight ([in, out] Paddle layout, or [out, in] when ``trans``) or a
    weight-only packed weight + scale. ``packed``: an optional MFMA-tile packed bf16 copy used for
    small-M (decode) calls, where the GEMM is a weight stream (see ops.inference.pack_bf16)."""
    __slots__ = ("w", "scale", "bits", "trans", "packed", "act_scale", "lnf")
    PACKED_MAX_M = 64
    # serving batches with short K: the skinny MFMA GEMM on the K-contiguous weight beats the packed
    # weight stream from 8 rows (M=32 QKV 14.7 -> 11.5 us, out-proj 8.8 -> 6.5; K = 8192 stays on
    # the packed GEMV: profiles/decode_linear_r5.txt)
    # the skinny GEMM takes every serving-batch projection incl. FFN2 (K = 8192, tuned split-K config):
    # batch 8 1.368 -> 1.312 ms/step vs the packed GEMV at K = 8192, batch 32 equal (profiles/decode_r6.txt)
    DENSE_MIN_M, DENSE_MAX_K = 8, int(os.environ.get("PIAMD_DENSE_MAX_K", "8192"))

    def _packed_for(self, M, K):
        return (self.packed is not None and M <= self.PACKED_MAX_M
                and not (M >= self.DENSE_MIN_M and K <= self.DENSE_MAX_K))

    def _dense_epilogue(self, x, bias, act, resid):
        """act(x·W + bias) + resid as ONE own GEMM (bias / activation / residual in the epilogue)."""
        from ...ops.gemm import gemm_nt
        from ...ops.linear import transposed
        x2 = x.reshape(-1, x.shape[-1])
        wk = self.w if self.trans else transposed(self.w)
        r2 = resid.reshape(x2.shape[0], -1) if resid is not None else None
        y = gemm_nt(x2.contiguous(), wk, bias=bias, act=act, resid=r2)
        return y.reshape(*x.shape[:-1], y.shape[-1])

    def __init__(self, w, scale=None, bits=0, trans=False, packed=None, act_scale=None):
        self.w, self.scale, self.bits, self.trans, self.packed = w, scale, bits, trans, packed
        self.act_scale = act_scale  # bits == -8: int8 activations (None → dynamic per token)
        self.lnf = {}  # LayerNorm folds of the K-contiguous weight, keyed by (γ, β, bias)

    def _kn(self):
        """(K, N) of the projection."""
        return (self.w.shape[1], self.w.shape[0]) if self.trans else tuple(self.w.shape)

    def ln_fold_ok(self, M, act="none"):
        """A pre-LN call with M rows runs as ONE skinny GEMM on the LayerNorm-folded weight
        (``ops.gemm.ln_fold``: row statistics gathered from the raw rows inside the GEMM, no
        LayerNorm launch) — serving batches (M ≥ DENSE_MIN_M) on the dense path, bf16 / fp16."""
        from ...ops.gemm import use_small
        K, N = self._kn()
        return (not self.bits and self.packed is not None and self.w.dtype in (torch.bfloat16, torch.float16)
                and M >= self.DENSE_MIN_M and not self._packed_for(M, K) and K % 64 == 0
                and N % 4 == 0 and use_small(M, N, K) and act in ("none", "gelu", "gelu_tanh", "relu"))

    def fused_rows(self, M, ln, act="none"):
        """True when a call with M rows takes its pre-LN (``ln``) or residual add in the kernel
        that computes it: the weight-stream GEMV at few rows, the LN-folded / residual-epilogue
        skinny GEMM at serving batches."""
        if self.fused_gemv(M):
            return True
        if self.bits or self.packed is None or M < self.DENSE_MIN_M:
            return False
        return self.ln_fold_ok(M, act) if ln else True

    def _dense_ln(self, x, ln, bias, act, resid):
        from ...ops.gemm import ln_fold, small_gemm
        from ...ops.linear import transposed
        from ...ops.linear import _PARAM_EPOCH
        g, b, eps = ln
        # an in-place reload (set_state_dict / copy_) of any folded operand bumps its version;
        # the flat optimizers that write outside autograd bump the parameter epoch
        key = (g.data_ptr(), b.data_ptr(), bias.data_ptr() if bias is not None else 0)
        ver = (_PARAM_EPOCH[0], self.w.data_ptr(), self.w._version, g._version, b._version,
               bias._version if bias is not None else 0)
        f = self.lnf.get(key)
        if f is not None and f[3] != ver:
            f = None
            del self.lnf[key]
        if f is None and torch.cuda.is_current_stream_capturing():
            # a fold built inside a capture would only be computed at replay: explicit LN instead
            return self._dense_epilogue(ops.layer_norm(x, g, b, eps), bias, act, resid)
        if f is None:
            wk = self.w if self.trans else transposed(self.w)
            f = self.lnf[key] = tuple(ln_fold(wk, g, b, bias)) + (ver,)
        x2 = x.reshape(-1, x.shape[-1])
        if x2.stride(-1) != 1 or x2.stride(0) != x2.shape[1]:
            x2 = x2.contiguous()
        r2 = resid.reshape(x2.shape[0], -1) if resid is not None else None
        y = small_gemm(x2, f[0], act=act, resid=r2, ln=(f[1], f[2], eps))
        return y.reshape(*x.shape[:-1], y.shape[-1])

    def prepack(self):
        if not self.bits and self.packed is None:
            w = self.w.t() if self.trans else self.w
            if w.shape[1] % 32 == 0 and w.shape[0] % 16 == 0:
                self.packed = _inf.pack_bf16(w.detach())
        return self

    def fused_gemv(self, M):
        """True when a call with M rows runs the weight-stream GEMV, which takes the pre-LN in its
        prologue and the residual add in its epilogue (no separate launches)."""
        if M > FUSED_LN_MAX_M:  # the per-workgroup LN prologue grows with M; the saved launch does not
            return False
        return self.bits in (4, 8) or self.packed is not None

    def __call__(self, x, bias=None, act="none", ln=None, resid=None):
        if ln is not None or resid is not None:
            M = x.numel() // x.shape[-1]
            if self.bits in (4, 8):
                return _inf.weight_only_linear(x, self.w, bias, self.scale,
                                               "int4" if self.bits == 4 else "int8", act, ln=ln,
                                               resid=resid)
            if x.is_cuda and self._packed_for(M, x.shape[-1]):
                return _inf.packed_linear(x, self.packed, bias, act, ln=ln, resid=resid)
            if (ln is not None and x.is_cuda and x.dtype == torch.bfloat16 and LN_FOLD
                    and self.ln_fold_ok(M, act)):
                return self._dense_ln(x, ln, bias, act, resid)
            if ln is not None:
                x = ops.layer_norm(x, ln[0], ln[1], ln[2])
            if (x.is_cuda and self.packed is not None and x.dtype == self.w.dtype
                    and act in ("none", "gelu", "gelu_tanh", "relu")):
                return self._dense_epilogue(x, bias, act, resid)
            y = self(x, bias, act)
            return y + resid.reshape(y.shape) if resid is not None else y
        if self.bits == -8:  # int8 x int8 MFMA GEMM, dequantising epilogue (FusedMultiTransformerINT8)
            return _inf.int8_linear(x, self.w, self.scale, bias, self.act_scale, act)
        if self.bits:
            return _inf.weight_only_linear(x, self.w, bias, self.scale,
                                           "int4" if self.bits == 4 else "int8", act)
        if x.is_cuda and self._packed_for(x.numel() // x.shape[-1], x.shape[-1]):
            return _inf.packed_linear(x, self.packed, bias, act)
        from ...ops.linear import linear as _dense, linear_bias_act
        if act != "none" and bias is not None:  # one epilogue GEMM when eligible (inference)
            return linear_bias_act(x, self.w, bias, act, weight_out_in=self.trans)
        if self.trans:  # [out, in] weight: already K-contiguous
            from ...ops.linear import mm_nt
            x2 = x.reshape(-1, x.shape[-1])
            y = mm_nt(x2, self.w, bias if act == "none" else None).reshape(*x.shape[:-1], -1)
        else:  # [in, out] weight: cached K-contiguous copy, bias in the GEMM epilogue
            y = _dense(x, self.w, bias if act == "none" else None)
        return ops.bias_act(y, bias, act) if act != "none" else y


# decode rows up to which each layer's pre-LN / residual adds ride in the GEMV prologue / epilogue.
# Measured (GPT-1.3B decode, profiles/decode_fused_ln_sweep_r1.txt): fusing wins at batch 1-2
# (+4-12 % tok/s) and loses from batch 4 (the LN prologue forces KS=1 and grows with M).
FUSED_LN_MAX_M = int(os.environ.get("PIAMD_FUSED_LN_MAX_M", "2"))
# serving batches (M ≥ 8 rows, E ≤ 2048): each pre-LN folded into the skinny GEMM that consumes it
# (ops.gemm.ln_fold) and each residual add in the producing GEMM's epilogue — no LayerNorm launches
LN_FOLD = os.environ.get("PIAMD_LN_FOLD", "1") != "0"


def _lin(w, scale=None, bits=0, trans=False, act_scale=None):
    return _Linear(w, scale, bits, trans, act_scale=act_scale)


def _rope_table(x, cos, sin, chunks, decode):
    """Rotary embedding from an EXTERNAL cos / sin table (reference ``RotaryPosEmb`` input,
    `fused_multi_transformer_op.h:1600` RotrayKernel / mmha `apply_rotary_emb`): the head dim is
    cut into ``chunks`` pieces of width L, each rotated half-against-half (neox style). x
    [B, S, H, D]; cos / sin [B, S, D]. Context rows take the table entry of the first-half index for
    both halves (RotrayKernel); the decode step takes each element's own entry (mmha)."""
    B, S, H, D = x.shape
    L = D // chunks
    h = L // 2
    xf = x.float().reshape(B, S, H, chunks, 2, h)
    c = cos.float().reshape(B, S, 1, chunks, 2, h)
    sn = sin.float().reshape(B, S, 1, chunks, 2, h)
    left, right = xf[..., 0, :], xf[..., 1, :]
    if decode:
        ol = left * c[..., 0, :] - right * sn[..., 0, :]
        orr = right * c[..., 1, :] + left * sn[..., 1, :]
    else:
        ol = left * c[..., 0, :] - right * sn[..., 0, :]
        orr = right * c[..., 0, :] + left * sn[..., 0, :]
    return torch.stack([ol, orr], -2).reshape(B, S, H, D).to(x.dtype)


def _attend_ext(qkv, bias, kc, vc, B, S, hq, hk, D, attn_mask, causal, rope, pre_kv, decode,
                lens=None, max_len=None):
    """Attention with an external RoPE table and / or prefix K/V (reference ``PreCaches``
    [2, B, Hk, P, D]): bias + table rotation on the QKV rows, the prefix written to cache slots
    [0, P) ahead of the new tokens, queries attending to [prefix | new] keys (bottom-right causal
    band, or SrcMask [B, 1|H, S, P+S])."""
    x = qkv.view(B, S, hq + 2 * hk, D)
    if bias is not None:
        x = x + bias.view(hq + 2 * hk, D).to(x.dtype)
    q, k, v = x[:, :, :hq], x[:, :, hq:hq + hk], x[:, :, hq + hk:]
    if rope is not None:
        cos, sin, chunks = rope
        q = _rope_table(q, cos, sin, chunks, decode)
        k = _rope_table(k, cos, sin, chunks, decode)
    if decode:  # rotated row → the split-K decode kernel (cache write of the new k / v in-kernel)
        row = torch.cat([q, k, v], 2).reshape(B, (hq + 2 * hk) * D).contiguous()
        return _inf.decode_attention(row, kc, vc, lens, hq, hk, attn_mask, max_len=max_len,
                                     prep_bias=None, prep=True, rot_dim=0)
    P = 0
    if pre_kv is not None:
        P = pre_kv.shape[3]
        pk = pre_kv[0].transpose(1, 2).to(k.dtype)  # [B, P, Hk, D]
        pv = pre_kv[1].transpose(1, 2).to(v.dtype)
        kf, vf = torch.cat([pk, k], 1), torch.cat([pv, v], 1)
    else:
        kf, vf = k, v
    if kc is not None:  # reference write_cache_kv: slots [0, P + S)
        kc[:, :, :P + S].copy_(kf.transpose(1, 2))
        vc[:, :, :P + S].copy_(vf.transpose(1, 2))
    m = _to_additive_mask(attn_mask, x.dtype) if attn_mask is not None else None
    o = ops.flash_attention(q.contiguous(), kf.contiguous(), vf.contiguous(),
                            causal and m is None, 1.0 / math.sqrt(D), attn_mask=m)
    return o.reshape(B * S, hq * D)


def multi_transformer_forward(x, layers, num_heads, num_kv_heads=None, pre_layer_norm=True,
                              epsilon=1e-5, caches=None, pos=None, lens=None, attn_mask=None,
                              decode=False, activation="gelu", rotary_dim=0, neox_rotary=True,
                              rope_base=10000.0, causal=None, group=None, max_len=None,
                              moe_fn=None, final_ln=None, rope_table=None, pre_caches=None):
    """Core of every fused multi-transformer variant.

    x: [B, S, E]; ``layers``: list of dicts with keys ln_scale, ln_bias, qkv (_Linear producing
    [(Hq+2Hk)*D]), qkv_bias, out (_Linear), out_bias, ffn_ln_scale, ffn_ln_bias, ffn1, ffn1_bias,
    ffn2, ffn2_bias (or ``moe`` — a callable replacing the FFN). ``caches``: per layer
    (k_cache, v_cache) [B, Hk, maxS, D]. Context (decode=False): writes positions
    pos[b] + [0, S). Decode (S == 1): writes position pos[b] and attends to keys [0, lens[b]).
    ``pos``/``lens`` are device int32 [B] (graph-replayable). ``rope_table``: (cos, sin, chunks) —
    RoPE from an external table instead of the in-kernel angles; ``pre_caches``: per layer prefix
    K/V [2, B, Hk, P, D] attended ahead of the context tokens (both: reference
    ``fused_multi_transformer`` RotaryPosEmb / PreCaches inputs).
    """
    B, S, E = x.shape
    hq = num_heads
    hk = num_kv_heads or num_heads
    D = E // hq if layers[0].get("head_dim") is None else layers[0]["head_dim"]
    T = B * S
    act = {"gelu": "gelu", "relu": "relu", "silu": "silu", "swiglu": "silu",
           "geglu": "gelu"}.get(activation, activation)
    gated = activation in ("swiglu", "geglu")
    causal = (attn_mask is None) if causal is None else causal
    if decode and attn_mask is not None:
        attn_mask = _to_additive_mask(attn_mask, x.dtype).reshape(B, -1).contiguous()
    xf = x.reshape(T, E)
    ext = rope_table is not None or pre_caches is not None
    if (decode and pre_layer_norm and group is None and not gated and moe_fn is None and not ext
            and x.dtype == torch.bfloat16
            and all(L.get("moe") is None
                    and all(L.get(k) is not None and L[k].dtype == torch.bfloat16
                            for k in ("ln_scale", "ln_bias", "ffn_ln_scale", "ffn_ln_bias"))
                    and all(isinstance(L[k], _Linear)
                            and (L[k].fused_gemv(T)
                                 or (LN_FOLD and L[k].fused_rows(T, k in ("qkv", "ffn1"),
                                                                 act if k == "ffn1" else "none")))
                            for k in ("qkv", "out", "ffn1", "ffn2")) for L in layers)):
        # decode: each pre-LN runs inside the projection that consumes it (GEMV prologue at few
        # rows, LayerNorm-folded skinny GEMM at serving batches) and each residual add in the
        # epilogue of the projection that produces it — per layer QKV → attention → out → FFN1 →
        # FFN2, with no LayerNorm launches (2 fewer kernels per layer on a launch-bound step)
        residual = xf
        for li, L in enumerate(layers):
            qkv = L["qkv"](residual, ln=(L["ln_scale"], L["ln_bias"], epsilon))
            kc, vc = caches[li] if caches is not None else (None, None)
            a = _inf.decode_attention(qkv, kc, vc, lens, hq, hk, attn_mask, max_len=max_len,
                                      prep_bias=L.get("qkv_bias"), prep=True, rot_dim=rotary_dim,
                                      neox=neox_rotary, base=rope_base)
            residual = L["out"](a, L.get("out_bias"), resid=residual)
            h = L["ffn1"](residual, L.get("ffn1_bias"), act,
                          ln=(L["ffn_ln_scale"], L["ffn_ln_bias"], epsilon))
            residual = L["ffn2"](h, L.get("ffn2_bias"), resid=residual)
        if final_ln is not None:
            out = ops.layer_norm(residual, final_ln[0], final_ln[1],
                                 final_ln[2] if len(final_ln) > 2 else epsilon)
        else:
            out = residual
        return out.reshape(B, S, E)
    residual = xf
    pending = None  # (ffn2_out, ffn2_bias) to fold into the next LN pass
    n = len(layers)
    for li, L in enumerate(layers):
        if pre_layer_norm:
            if pending is None:
                xn = _ln(residual, L["ln_scale"], L["ln_bias"], epsilon)
            else:
                xn, residual = ops.fused_add_layer_norm(pending[0], residual, L["ln_scale"],
                                                        L["ln_bias"], epsilon, pending[1])
        else:
            if pending is not None:
                residual, _ = ops.fused_add_layer_norm(pending[0], residual, pending[2],
                                                       pending[3], epsilon, pending[1])
            xn = residual
        pending = None
        qkv = L["qkv"](xn)  # [T, (Hq+2Hk)*D]
        kc, vc = caches[li] if caches is not None else (None, None)
        if ext:
            a = _attend_ext(qkv, L.get("qkv_bias"), kc, vc, B, S, hq, hk, D, attn_mask, causal,
                            rope_table, pre_caches[li] if pre_caches is not None else None, decode,
                            lens, max_len)
        elif decode:  # bias + RoPE + cache write fused into the split-K attention kernel
            a = _inf.decode_attention(qkv, kc, vc, lens, hq, hk, attn_mask, max_len=max_len,
                                      prep_bias=L.get("qkv_bias"), prep=True, rot_dim=rotary_dim,
                                      neox=neox_rotary, base=rope_base)
        else:
            ops.qkv_prep(qkv, L.get("qkv_bias"), kc, vc, pos, B, S, hq, hk, D, rotary_dim,
                         neox_rotary, rope_base)
            a = attention_core(qkv.view(B, S, hq + 2 * hk, D), hq, hk, attn_mask, causal)
            a = a.reshape(T, hq * D)
        o = L["out"](a)
        if group is not None:
            torch.distributed.all_reduce(o, group=group)
        if pre_layer_norm:
            yn, residual = ops.fused_add_layer_norm(o, residual, L["ffn_ln_scale"],
                                                    L["ffn_ln_bias"], epsilon, L.get("out_bias"))
        else:
            residual, _ = ops.fused_add_layer_norm(o, residual, L["ln_scale"], L["ln_bias"],
                                                   epsilon, L.get("out_bias"))
            yn = residual
        if moe_fn is not None and L.get("moe") is not None:
            f2 = L["moe"](yn)
            b2 = None
        else:
            if gated:
                h = L["ffn1"](yn, L.get("ffn1_bias"))
                g, u = h.chunk(2, -1)
                h = ops.bias_act(g.contiguous(), None, act) * u
            else:
                h = L["ffn1"](yn, L.get("ffn1_bias"), act)
            f2 = L["ffn2"](h)
            b2 = L.get("ffn2_bias")
        if group is not None:
            torch.distributed.all_reduce(f2, group=group)
        if pre_layer_norm:
            pending = (f2, b2)
        else:
            pending = (f2, b2, L["ffn_ln_scale"], L["ffn_ln_bias"])
    if pre_layer_norm and final_ln is not None:  # final add + LN in one pass (GPT head)
        out, _ = ops.fused_add_layer_norm(pending[0], residual, final_ln[0], final_ln[1],
                                          final_ln[2] if len(final_ln) > 2 else epsilon, pending[1])
    elif pre_layer_norm:
        out = residual + pending[0]
        if pending[1] is not None:
            out = out + pending[1]
    else:
        out, _ = ops.fused_add_layer_norm(pending[0], residual, pending[2], pending[3], epsilon,
                                          pending[1])
    return out.reshape(B, S, E)


def _qkv_linear(w, trans_qkvw, scale=None, bits=0):
    if bits:
        return _lin(w, scale, bits)
    if trans_qkvw:  # [3, H, D, E] (or [(Hq+2Hk), D, E])
        return _lin(w.reshape(-1, w.shape[-1]), trans=True)
    return _lin(w.reshape(w.shape[0], -1))  # [E, 3, H, D]


def _positions(B, time_step, seq_lens, S, device, decode):
    """Reference semantics: context writes cache positions [0, S); decode writes position
    ``time_step`` (or per-batch ``seq_lens``) and attends to keys [0, pos]."""
    if decode:
        if seq_lens is not None:
            p = seq_lens.reshape(-1).to(device=device, dtype=torch.int32)
        else:
            t = int(time_step.reshape(-1)[0]) if torch.is_tensor(time_step) else int(time_step)
            p = torch.full((B,), t, dtype=torch.int32, device=device)
        return p, p + 1
    return torch.zeros(B, dtype=torch.int32, device=device), None


def ext_inputs(rotary_embs, rotary_table_dims, pre_caches, B, D, device, decode):
    """(rope_table, pre_caches) for multi_transformer_forward from the op's RotaryPosEmb
    [2, B, 1, S, D] and PreCaches inputs (a prefix only matters to the context stage: afterwards it
    lives in the cache)."""
    rope = None
    if rotary_embs is not None:
        t = rotary_embs.to(device)
        rope = (t[0].reshape(B, -1, D), t[1].reshape(B, -1, D), int(rotary_table_dims or 1))
    return rope, (None if decode else pre_caches)


def _caches_from(cache_kvs):
    if cache_kvs is None:
        return None
    return [(c[0], c[1]) for c in cache_kvs]


def fused_multi_transformer(x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights,
                            linear_biases, ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_biases,
                            ffn2_weights, ffn2_biases, pre_layer_norm=True, epsilon=1e-05,
                            cache_kvs=None, beam_offset=None, seq_lens=None, time_step=None,
                            attn_mask=None, dropout_rate=0.0, activation="gelu", training=False,
                            mode="upscale_in_train", trans_qkvw=True, ring_id=-1, name=None,
                            num_kv_heads=None, rotary_emb_dims=0, use_neox_rotary_style=True,
                            rope_base=10000.0, group=None, causal=False, pre_caches=None,
                            rotary_embs=None, rotary_table_dims=1):
    """Reference `incubate/nn/functional/fused_transformer.py:833`. cache_kvs: per layer
    [2, B, Hk, max_seq_len, D], updated in place; returns (out, cache_kvs) when given. Context
    attention is full (the reference op's semantics without SrcMask) unless ``causal`` (an
    extension: the bottom-right causal band without materialising a mask).
    ``rotary_emb_dims`` here (dygraph extension) = rotated head dims with in-kernel angles;
    ``rotary_embs`` = the op's RotaryPosEmb table [2, B, 1, S, D] (``rotary_table_dims`` = its
    reference ``rotary_emb_dims``: the head-dim chunk count); ``pre_caches`` = PreCaches, per
    layer [2, B, Hk, P, D] prefix K/V (context stage)."""
    B, S, E = x.shape
    w0 = qkv_weights[0]
    if trans_qkvw:
        nh_total, D = w0.shape[-3] * (w0.shape[0] if w0.dim() == 4 else 1), w0.shape[-2]
    else:
        nh_total, D = w0.numel() // E // w0.shape[-1], w0.shape[-1]
    hk = num_kv_heads
    hq = nh_total // 3 if hk is None else nh_total - 2 * hk
    hk = hk or hq
    decode = time_step is not None
    if beam_offset is not None and cache_kvs is not None:
        src = beam_offset.reshape(-1)[:B].long().to(x.device)
        for c in cache_kvs:
            c.copy_(c.index_select(1, src))
    pos, lens = _positions(B, time_step, seq_lens, S, x.device, decode)
    rope, pre_caches = ext_inputs(rotary_embs, rotary_table_dims, pre_caches, B, D, x.device, decode)
    if rope is not None:
        rotary_emb_dims = 0
    layers = []
    for i in range(len(qkv_weights)):
        layers.append(dict(
            head_dim=D, ln_scale=ln_scales[i], ln_bias=ln_biases[i] if ln_biases else None,
            qkv=_qkv_linear(qkv_weights[i], trans_qkvw),
            qkv_bias=qkv_biases[i].reshape(-1) if qkv_biases and qkv_biases[i] is not None else None,
            out=_lin(linear_weights[i]), out_bias=linear_biases[i] if linear_biases else None,
            ffn_ln_scale=ffn_ln_scales[i], ffn_ln_bias=ffn_ln_biases[i] if ffn_ln_biases else None,
            ffn1=_lin(ffn1_weights[i]), ffn1_bias=ffn1_biases[i] if ffn1_biases else None,
            ffn2=_lin(ffn2_weights[i]), ffn2_bias=ffn2_biases[i] if ffn2_biases else None))
    with torch.no_grad():
        out = multi_transformer_forward(
            x, layers, hq, hk, pre_layer_norm, epsilon, _caches_from(cache_kvs), pos, lens,
            attn_mask, decode, activation, rotary_emb_dims, use_neox_rotary_style, rope_base,
            causal=causal and attn_mask is None, group=group, rope_table=rope,
            pre_caches=pre_caches)
    return (out, cache_kvs) if cache_kvs is not None else out


def fused_multi_transformer_weight_only(x, ln_scales, ln_biases, qkv_weights, qkv_scales,
                                        qkv_biases, linear_weights, linear_scales, linear_biases,
                                        ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_scales,
                                        ffn1_biases, ffn2_weights, ffn2_scales, ffn2_biases,
                                        pre_layer_norm=True, epsilon=1e-5, cache_kvs=None,
                                        beam_offset=None, seq_lens=None, time_step=None,
                                        attn_mask=None, activation="gelu", weight_dtype="int8",
                                        num_heads=None, num_kv_heads=None, rotary_emb_dims=0,
                                        use_neox_rotary_style=True, rope_base=10000.0, group=None,
                                        causal=False, pre_caches=None, rotary_embs=None,
                                        rotary_table_dims=1):
    """Reference `fused_multi_transformer_weight_only_op.cu`: every projection is a
    weight-only int8/int4 GEMM (packed [N, K] / [N/2, K] weights, per-channel f32 scales).
    RotaryPosEmb / PreCaches as :func:`fused_multi_transformer`."""
    B, S, E = x.shape
    bits = 4 if weight_dtype == "int4" else 8
    hk = num_kv_heads or num_heads
    D = E // num_heads
    decode = time_step is not None
    pos, lens = _positions(B, time_step, seq_lens, S, x.device, decode)
    rope, pre_caches = ext_inputs(rotary_embs, rotary_table_dims, pre_caches, B, D, x.device, decode)
    if rope is not None:
        rotary_emb_dims = 0
    layers = []
    for i in range(len(qkv_weights)):
        layers.append(dict(
            head_dim=D, ln_scale=ln_scales[i], ln_bias=ln_biases[i],
            qkv=_lin(qkv_weights[i], qkv_scales[i], bits),
            qkv_bias=qkv_biases[i].reshape(-1) if qkv_biases[i] is not None else None,
            out=_lin(linear_weights[i], linear_scales[i], bits), out_bias=linear_biases[i],
            ffn_ln_scale=ffn_ln_scales[i], ffn_ln_bias=ffn_ln_biases[i],
            ffn1=_lin(ffn1_weights[i], ffn1_scales[i], bits), ffn1_bias=ffn1_biases[i],
            ffn2=_lin(ffn2_weights[i], ffn2_scales[i], bits), ffn2_bias=ffn2_biases[i]))
    with torch.no_grad():
        out = multi_transformer_forward(
            x, layers, num_heads, hk, pre_layer_norm, epsilon, _caches_from(cache_kvs), pos, lens,
            attn_mask, decode, activation, rotary_emb_dims, use_neox_rotary_style, rope_base,
            causal=causal and attn_mask is None, group=group, rope_table=rope,
            pre_caches=pre_caches)
    return (out, cache_kvs) if cache_kvs is not None else out


# ----------------------------------------------------------------------------- misc fused ops
def fused_rotary_position_embedding(q, k=None, v=None, sin=None, cos=None, position_ids=None,
                                    use_neox_rotary_style=True, rotary_base=10000.0):
    """q/k/v: [B, S, H, D]; rotates q and k (v passes through)."""
    outs = []
    for t in (q, k, v):
        if t is None:
            outs.append(None)
            continue
        if t is v:
            outs.append(v)
            continue
        B, S, H, D = t.shape
        pos = position_ids[0].cpu() if position_ids is not None else torch.arange(S)
        if sin is not None and cos is not None:
            c = cos.reshape(S, -1)[:, :D].float().to(t.device)
            s_ = sin.reshape(S, -1)[:, :D].float().to(t.device)
            if use_neox_rotary_style:
                x1, x2 = t.float()[..., :D // 2], t.float()[..., D // 2:]
                rot = torch.cat([-x2, x1], -1)
            else:
                x1, x2 = t.float()[..., 0::2], t.float()[..., 1::2]
                rot = torch.stack([-x2, x1], -1).flatten(-2)
            outs.append((t.float() * c[None, :, None] + rot * s_[None, :, None]).to(t.dtype))
        else:
            r = _inf._rope_ref(t.float().transpose(1, 2).cpu(), pos, D, use_neox_rotary_style,
                               rotary_base)
            outs.append(r.transpose(1, 2).to(t.device, t.dtype))
    return tuple(outs)


def masked_multihead_attention(x, cache_kv=None, src_mask=None, sequence_lengths=None,
                               rotary_tensor=None, beam_cache_offset=None, seq_len=1,
                               rotary_emb_dims=0, use_neox_rotary_style=False, num_heads=None,
                               num_kv_heads=None, rope_base=10000.0):
    """Reference mmha: x [B, (Hq+2Hk)*D] (one new token, QKV bias already added), cache_kv
    [2, B, Hk, maxS, D]; sequence_lengths [B] = cached length (the new token goes there).
    Returns (out [B, Hq*D], cache_kv)."""
    B = x.shape[0]
    _, _, hk, maxS, D = cache_kv.shape
    hq = num_heads or (x.shape[1] // D - 2 * hk)
    if sequence_lengths is None:
        raise ValueError("masked_multihead_attention needs sequence_lengths")
    pos = sequence_lengths.reshape(-1).to(x.device, torch.int32)
    qkv = x.clone()
    ops.qkv_prep(qkv, None, cache_kv[0], cache_kv[1], pos, B, 1, hq, hk, D, rotary_emb_dims,
                 use_neox_rotary_style, rope_base)
    out = _inf.decode_attention(qkv, cache_kv[0], cache_kv[1], pos + 1, hq, hk, src_mask)
    return out, cache_kv


def variable_length_memory_efficient_attention(query, key, value, seq_lens, kv_seq_lens,
                                               mask=None, scale=None, causal=False):
    """query [B, H, S, D], key/value [B, Hk, Sk, D]; per-batch valid lengths (reference
    `variable_length_memory_efficient_attention.cu`). Without a mask the valid prefixes are packed
    and run as ONE variable-length flash launch (``ops.flash_attention_varlen``); rows past a
    sequence's length are zero."""
    B, H, S, D = query.shape
    Sk = key.shape[2]
    lq = seq_lens.reshape(-1).to(torch.long)
    lk = kv_seq_lens.reshape(-1).to(torch.long)
    dev = query.device
    if mask is None:
        out = torch.zeros_like(query)
        ar_q = torch.arange(S, device=dev)
        ar_k = torch.arange(Sk, device=dev)
        vq = (ar_q[None, :] < lq.to(dev)[:, None]).reshape(-1)
        vk = (ar_k[None, :] < lk.to(dev)[:, None]).reshape(-1)
        iq = vq.nonzero().squeeze(1)
        ik = vk.nonzero().squeeze(1)
        q = query.transpose(1, 2).reshape(B * S, H, D).index_select(0, iq)
        k = key.transpose(1, 2).reshape(B * Sk, -1, D).index_select(0, ik)
        v = value.transpose(1, 2).reshape(B * Sk, -1, D).index_select(0, ik)
        cu_q = torch.zeros(B + 1, dtype=torch.int32, device=dev)
        cu_k = torch.zeros(B + 1, dtype=torch.int32, device=dev)
        cu_q[1:] = torch.cumsum(lq.to(dev), 0)
        cu_k[1:] = torch.cumsum(lk.to(dev), 0)
        o = ops.flash_attention_varlen(q, k, v, cu_q, cu_k, S, Sk, causal, scale)
        flat = out.transpose(1, 2).reshape(B * S, H, D).clone()
        flat.index_copy_(0, iq, o.to(flat.dtype))
        return flat.view(B, S, H, D).transpose(1, 2).contiguous()
    # Masked: ONE padded flash launch, no host sync. Key-length limits and the per-sequence
    # (bottom-right aligned) causal band are folded into the additive mask on the device; rows
    # past a sequence's length are zeroed.
    lqd, lkd = lq.to(dev), lk.to(dev)
    ar_q = torch.arange(S, device=dev)[None, :, None]
    ar_k = torch.arange(Sk, device=dev)[None, None, :]
    allow = ar_k < lkd[:, None, None]
    if causal:
        allow = allow & (ar_k <= ar_q + (lkd - lqd)[:, None, None])
    m = mask.to(query.dtype)
    if m.dim() == 3:
        m = m.unsqueeze(1)
    m = m.masked_fill(~allow[:, None], float("-inf"))
    o = ops.flash_attention(query.transpose(1, 2), key.transpose(1, 2), value.transpose(1, 2),
                            False, scale, attn_mask=m)
    o = o.transpose(1, 2)
    rows = (torch.arange(S, device=dev)[None, :] < lqd[:, None])[:, None, :, None]
    return torch.where(rows, o, torch.zeros((), device=dev, dtype=o.dtype)).contiguous()


def softmax_mask_fuse(x, mask, name=None):
    return ops.fused_softmax_mask(x, mask)


def softmax_mask_fuse_upper_triangle(x):
    return ops.fused_softmax_mask(x, None, 1.0, causal=True)
