"""Serving-path ops backed by ``csrc/kernels/infer.hip``.

* :func:`qkv_prep` — QKV bias + rotary embedding + KV-cache write, in place on the packed
  QKV GEMM output (reference `fused_multi_transformer_op.cu.h`: add bias / rotary_qk /
  write_cache_kv).
* :func:`decode_attention` — one new token per sequence attending to its KV cache (reference
  `masked_multihead_attention_kernel`), split-K over the cache with a combine pass.
* :func:`weight_quantize` / :func:`weight_dequantize` / :func:`weight_only_linear` — weight-only
  int8/int4 (reference `python/paddle/nn/quant/quantized_linear.py`). The quantized weight keeps
  Paddle's logical shape ([N, K] for int8, [N/2, K] for int4, from an input of [K, N]) but its
  bytes are in the MI355X MFMA-tile order documented in infer.hip, exactly as the reference's own
  weight_quantize emits a CUTLASS-interleaved order for sm80.

Every op has a PyTorch reference path (CPU tensors) used by the CPU tests and as the numerics
reference of the GPU tests.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from . import _lib
from .activation import ACTS, _ref_act


# ------------------------------------------------------------------------------- rotary / prep
def _rope_ref(x, pos, rot, neox, base):
    """x: [..., T, D] float; pos: [T] positions."""
    if rot <= 0:
        return x
    half = rot // 2
    inv = base ** (-(2.0 * torch.arange(half, dtype=torch.float64) / rot))
    ang = pos.double()[:, None] * inv[None, :]  # [T, half]
    cos, sin = ang.cos().float(), ang.sin().float()
    xr, xp = x[..., :rot], x[..., rot:]
    if neox:
        a, b = xr[..., :half], xr[..., half:]
        out = torch.cat([a * cos - b * sin, b * cos + a * sin], -1)
    else:
        a, b = xr[..., 0::2], xr[..., 1::2]
        out = torch.stack([a * cos - b * sin, b * cos + a * sin], -1).flatten(-2)
    return torch.cat([out, xp], -1)


def qkv_prep(qkv, bias, k_cache, v_cache, pos0, B, S, Hq, Hk, D, rot_dim=0, neox=True,
             base=10000.0, pos_from_lens=None):
    """In place on ``qkv`` ([B*S, (Hq+2Hk)*D] rows, any row stride): add bias, rotate q/k,
    write k/v into ``k_cache``/``v_cache`` ([B, Hk, maxS, D]) at positions pos0[b] + s
    (``pos_from_lens``: pos0 = lens - 1, the decode convention)."""
    if pos_from_lens is not None:
        pos0 = (pos_from_lens - 1).to(torch.int32)
    H = Hq + 2 * Hk
    if qkv.is_cuda:
        assert qkv.dtype == torch.bfloat16 and qkv.stride(-1) == 1 and qkv.shape[-1] >= H * D
        if k_cache is not None:
            assert k_cache.is_contiguous() and v_cache.is_contiguous() and k_cache.shape[1] == Hk
        if pos0 is not None:
            assert pos0.dtype == torch.int32 and pos0.is_cuda and pos0.numel() >= B
        maxS = k_cache.shape[2] if k_cache is not None else 0
        _lib.call("piamd_qkv_prep", qkv.data_ptr(), qkv.stride(0), _lib.ptr(bias),
                  _lib.ptr(k_cache), _lib.ptr(v_cache), _lib.ptr(pos0), B, S, Hq, Hk, D, maxS,
                  int(rot_dim), int(bool(neox)), float(base), _lib.stream())
        return qkv
    x = qkv[:, :H * D].float().view(B, S, H, D)
    if bias is not None:
        x = x + bias.float().view(H, D)
    p0 = pos0.long().cpu() if pos0 is not None else torch.zeros(B, dtype=torch.long)
    for b in range(B):
        pos = p0[b] + torch.arange(S)
        qk = x[b, :, :Hq + Hk].transpose(0, 1)  # [H', S, D]
        x[b, :, :Hq + Hk] = _rope_ref(qk, pos, rot_dim, neox, base).transpose(0, 1)
        if k_cache is not None:
            maxS = k_cache.shape[2]
            ok = pos < maxS
            kk = x[b, :, Hq:Hq + Hk].transpose(0, 1)[:, ok]
            vv = x[b, :, Hq + Hk:].transpose(0, 1)[:, ok]
            k_cache[b, :, pos[ok]] = kk.to(k_cache.dtype)
            v_cache[b, :, pos[ok]] = vv.to(v_cache.dtype)
    qkv[:, :H * D] = x.view(B * S, H * D).to(qkv.dtype)
    return qkv


# ------------------------------------------------------------------------------- decode attn
_PART_CACHE = {}


DECODE_CHUNK = int(os.environ.get("PIAMD_DECODE_CHUNK", "0"))  # A/B knob: fixed keys per split


def decode_chunking(max_len, chunk=None):
    if chunk is None and DECODE_CHUNK:
        chunk = DECODE_CHUNK
    if chunk is None:
        # short caches: 64-key splits (one K pass + one V pass per workgroup, 4x the workgroups of
        # a 256-key split at batch 1); long caches keep the per-split partial count bounded
        # (≤ 256 keys: ONE split — the single-pass kernel variant keeps all K/V rows in flight and
        # skips the partial/combine round trips)
        chunk = (max(16, max_len) if max_len <= 256 else
                 64 if max_len <= 1024 else (128 if max_len <= 4096 else 256))
    chunk = max(16, min(512, chunk))
    return chunk, max(1, -(-max_len // chunk))


def decode_attention(q, k_cache, v_cache, lens, Hq, Hk, mask=None, scale=None, out=None,
                     max_len=None, chunk=None, prep_bias=None, prep=False, rot_dim=0, neox=True,
                     base=10000.0):
    """q: [B, >=Hq*D] rows (head h at columns h*D); caches [B, Hk, maxS, D]; lens: [B] int32
    number of valid keys (including the new token, which sits at lens-1). Returns [B, Hq*D].

    ``prep=True``: ``q`` is the raw QKV GEMM row of the new token ([Hq | Hk | Hk] heads); the
    kernel adds ``prep_bias``, applies RoPE (``rot_dim`` 0 or D) and writes the new k/v into the
    caches itself — one launch per layer for the whole decode attention.
    ``max_len`` bounds lens (defaults to the cache capacity, which is what a captured graph
    needs); it sets the split count."""
    B, _, maxS, D = k_cache.shape
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if out is None:
        out = torch.empty((B, Hq * D), dtype=q.dtype, device=q.device)
    if q.is_cuda:
        assert q.dtype == torch.bfloat16 and q.stride(-1) == 1 and k_cache.is_contiguous() \
            and v_cache.is_contiguous() and lens.dtype == torch.int32 and lens.is_cuda
        assert Hq % Hk == 0 and (Hq // Hk) in (1, 2, 4, 8) and D in (64, 128)
        if prep and rot_dim not in (0, D):  # partial rotary: separate prologue kernel
            q = qkv_prep(q.clone(), prep_bias, k_cache, v_cache, None, B, 1, Hq, Hk, D, rot_dim, neox, base,
                     pos_from_lens=lens)
            prep, prep_bias, rot_dim = False, None, 0
        ck, ns = decode_chunking(max_len or maxS, chunk)
        part = cnt = None
        if ns > 1:
            key = (q.device, B, Hq, Hk, ns, D)  # cnt is [B·Hk]: models of equal Hq share no buffer
            ent = _PART_CACHE.get(key)
            if ent is None:
                ent = _PART_CACHE[key] = (
                    torch.empty(B * Hq * ns * (D + 2), dtype=torch.float32, device=q.device),
                    torch.zeros(B * Hk, dtype=torch.int32, device=q.device))
            part, cnt = ent
        ldm = 0
        if mask is not None:
            mask = mask.reshape(B, -1)
            assert mask.dtype == torch.bfloat16 and mask.stride(-1) == 1
            ldm = mask.stride(0)
        _lib.call("piamd_decode_attn", q.data_ptr(), q.stride(0), _lib.ptr(prep_bias), int(prep),
                  int(rot_dim), int(bool(neox)), float(base), k_cache.data_ptr(),
                  v_cache.data_ptr(), lens.data_ptr(), B, Hq, Hk, D, maxS, ck, ns, _lib.ptr(mask),
                  ldm, float(scale), _lib.ptr(part), _lib.ptr(cnt), out.data_ptr(), out.stride(0),
                  _lib.stream())
        return out
    if prep:
        q = q.clone()
        qkv_prep(q, prep_bias, k_cache, v_cache, None, B, 1, Hq, Hk, D, rot_dim, neox, base,
                 pos_from_lens=lens)
    G = Hq // Hk
    for b in range(B):
        n = int(lens[b])
        qb = q[b, :Hq * D].float().view(Hq, 1, D)
        kb = k_cache[b, :, :n].float().repeat_interleave(G, 0)
        vb = v_cache[b, :, :n].float().repeat_interleave(G, 0)
        s = (qb @ kb.transpose(-1, -2)) * scale
        if mask is not None:
            s = s + mask.reshape(B, -1)[b, :n].float()
        out[b] = (torch.softmax(s, -1) @ vb).reshape(-1).to(out.dtype)
    return out


# ------------------------------------------------------------------------------- weight-only
def _pack(q, bits):
    """int8 q [N, K] (values in the bit range) → packed uint8 bytes in MFMA-tile order."""
    N, K = q.shape
    if bits == 8:
        assert N % 32 == 0 and K % 32 == 0, "weight-only int8 needs N % 32 == 0 and K % 32 == 0"
        t = q.view(N // 32, 32, K // 32, 2, 16).permute(0, 2, 3, 1, 4)
        return t.contiguous().view(torch.uint8).reshape(N, K)
    assert N % 32 == 0 and K % 64 == 0, "weight-only int4 needs N % 32 == 0 and K % 64 == 0"
    u = (q.to(torch.int16) & 15).to(torch.uint8)
    t = u.view(N // 32, 32, K // 64, 2, 16, 2).permute(0, 2, 3, 1, 4, 5).contiguous()
    packed = t[..., 0] | (t[..., 1] << 4)
    return packed.reshape(N // 2, K)


def _unpack(wp, bits, N, K):
    """Inverse of :func:`_pack` → int8 [N, K]."""
    if bits == 8:
        t = wp.reshape(N // 32, K // 32, 2, 32, 16).permute(0, 3, 1, 2, 4)
        return t.contiguous().view(torch.int8).reshape(N, K)
    b = wp.reshape(N // 32, K // 64, 2, 32, 16)
    lo = (b & 15).to(torch.int16)
    hi = (b >> 4).to(torch.int16)
    t = torch.stack([lo, hi], -1)
    t = torch.where(t >= 8, t - 16, t).to(torch.int8)
    return t.permute(0, 3, 1, 2, 4, 5).contiguous().reshape(N, K)


def pack_bf16(w_kn):
    """bf16 serving weight [K, N] (Paddle [in, out]) → MFMA-tile packed [N, K] (see infer.hip)."""
    K, N = w_kn.shape
    assert N % 32 == 0 and K % 16 == 0, "packed bf16 GEMM needs N % 32 == 0 and K % 16 == 0"
    t = w_kn.t().contiguous().view(N // 32, 32, K // 16, 2, 8).permute(0, 2, 3, 1, 4)
    return t.contiguous().view(N, K)


def _ln_ref(x2, ln):
    g, b, eps = ln
    return torch.nn.functional.layer_norm(x2.float(), (x2.shape[-1],), g.float(), b.float(), eps)


def ln_fusable(M, K, KS=1):
    """Whether :func:`packed_linear` / :func:`weight_only_linear` can take ``ln=`` (the LayerNorm
    computed in the GEMV prologue): one K split, M ≤ 8 rows, K % 512 == 0, K ≤ 2048 (beyond that
    the per-workgroup prologue costs more than the LayerNorm launch it replaces:
    profiles/decode_gemv_rows_r5.txt)."""
    return KS == 1 and K % 512 == 0 and K <= 2048 and 1 <= M <= 8



def _wo_call(bits, x2, w, scale, bias, y, M, N, K, KS, act, ln, resid, ws, cnt):
    lg, lb, eps = ln if ln is not None else (None, None, 0.0)
    _lib.call("piamd_wo_gemm_ex", bits, x2.data_ptr(), x2.stride(0), w.data_ptr(), _lib.ptr(scale),
              _lib.ptr(bias), y.data_ptr(), y.stride(0), _lib.ptr(ws), _lib.ptr(cnt), M, N, K, KS,
              act, _lib.ptr(lg), _lib.ptr(lb), float(eps), _lib.ptr(resid),
              resid.stride(0) if resid is not None else 0, _lib.stream())


def packed_linear(x, wp, bias=None, act="none", ln=None, resid=None):
    """y = act(LN?(x) @ W + bias) (+ resid) with W pre-packed by :func:`pack_bf16` (small-M decode
    GEMMs: one fully-coalesced 1 KB weight load per wave per MFMA, split-K to fill 256 CUs).
    ``ln = (gamma, beta, eps)``: the pre-LayerNorm of the input runs in the GEMV prologue (no LN
    launch); ``resid`` [M, N]: residual added after the activation in the epilogue."""
    N, K = wp.shape
    lead = x.shape[:-1]
    x2 = x.reshape(-1, K)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    M = x2.shape[0]
    r2 = resid.reshape(M, N) if resid is not None else None
    if ln is not None and x.is_cuda and not ln_fusable(M, K):
        from .norm import layer_norm
        x2, ln = layer_norm(x2, ln[0], ln[1], ln[2]), None
    if not x.is_cuda:
        w = wp.view(N // 32, K // 16, 2, 32, 8).permute(0, 3, 1, 2, 4).reshape(N, K)
        xin = _ln_ref(x2, ln).to(x.dtype) if ln is not None else x2
        y = xin.float() @ w.float().t()
        if bias is not None:
            y = y + bias.float()
        y = _ref_act(y, ACTS[act])
        if r2 is not None:
            y = y + r2.float()
        return y.to(x.dtype).reshape(*lead, N)
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    tiles = (N // 32) * ((M + 31) // 32)
    KS = 1 if ln is not None else _split_k(tiles, K // 16)
    ws, cnt = _splitk_bufs(x.device, KS, M, N, tiles)
    _wo_call(16, x2, wp, None, bias, y, M, N, K, KS, ACTS[act], ln, r2, ws, cnt)
    return y.reshape(*lead, N)


def _split_k(tiles, kb):
    """Split-K factor of the weight-stream GEMV. Measured on MI355X with the weights streamed
    from HBM (tools/bench_gemv.py → profiles/gemv_decode_r1.txt): with the software-pipelined
    kernel the fastest split is the smallest one giving ≥ ~192 workgroups (QKV / FFN1: 1,
    out-proj / FFN2: 4), as long as each split keeps ≥ 16 k-blocks."""
    KS = 1
    while tiles * KS < 192 and kb // (KS * 2) >= 16:
        KS *= 2
    return KS


FIXUP_MAX_M = int(os.environ.get("PIAMD_WO_FIXUP_MAX_M", "8"))  # split-K reduction: in-kernel atomic fixup up to this M, slices + finalize above


def _splitk_bufs(device, KS, M, N, tiles):
    if KS == 1:
        return None, None
    if M <= FIXUP_MAX_M:
        return _ws_buf(device, M * N, tiles)
    return _ws_buf(device, KS * M * N, 0)[0], None


def _ws_buf(device, n, tiles):
    """Split-K partial workspace + per-tile arrival counters (kept zeroed by the kernel). Shared
    by every launch on the stream: GEMMs on one stream never overlap."""
    key = (device, n, tiles)
    ent = _WS.get(key)
    if ent is None:
        ent = _WS[key] = (torch.zeros(n, dtype=torch.float32, device=device),
                          torch.zeros(tiles, dtype=torch.int32, device=device))
    return ent


def weight_quantize(x, algo="weight_only_int8"):
    """x: [K, N] float → (quantized weight, scale[N] f32). Symmetric per-output-channel.
    ``weight_only_int8`` / ``weight_only_int4``: MFMA-tile packed bytes for the weight-only GEMM;
    ``llm.int8``: plain row-major int8 [N, K] for the int8×int8 GEMM (``int8_linear``)."""
    bits = 4 if algo == "weight_only_int4" else 8
    w = x.float().t().contiguous()  # [N, K]
    qmax = 7.0 if bits == 4 else 127.0
    scale = w.abs().amax(1).clamp_min(1e-10) / qmax
    q = torch.round(w / scale[:, None]).clamp(-qmax - (1 if bits == 4 else 0), qmax).to(torch.int8)
    if algo == "llm.int8":
        return q, scale
    return _pack(q, bits), scale


def weight_dequantize(x, scale, algo="weight_only_int8", out_dtype="bfloat16"):
    """Packed weight → dequantized [K, N] (Paddle's layout of the original weight)."""
    bits = 4 if algo == "weight_only_int4" else 8
    N = scale.shape[0]
    K = x.numel() * (2 if bits == 4 else 1) // N
    from ..framework.dtype import to_torch_dtype
    dt = to_torch_dtype(out_dtype)
    if x.is_cuda:
        out = torch.empty((N, K), dtype=torch.bfloat16, device=x.device)
        _lib.call("piamd_wo_dequant", bits, x.data_ptr(), scale.float().contiguous().data_ptr(),
                  out.data_ptr(), N, K, _lib.stream())
        return out.t().to(dt)
    return (_unpack(x, bits, N, K).float() * scale.float()[:, None]).t().to(dt)


_WS = {}

# rows above which the weight-only GEMM dequantises once and runs the bf16 MFMA GEMM instead of
# the weight-stream kernel (which re-streams the packed weight once per 32-row tile)
WO_GEMV_MAX_M = int(os.environ.get("PIAMD_WO_GEMV_MAX_M", "256"))


def weight_only_linear(x, weight, bias=None, weight_scale=None, weight_dtype="int8",
                       act_method="none", ln=None, resid=None):
    """y = act(LN?(x) @ dequant(weight)ᵀ + bias) (+ resid); x [..., K], weight packed [N, K] /
    [N/2, K]. ``ln`` / ``resid`` as :func:`packed_linear` (GEMV path only)."""
    bits = 4 if weight_dtype == "int4" else 8
    N = weight_scale.shape[0]
    K = x.shape[-1]
    act = ACTS[act_method]
    lead = x.shape[:-1]
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if ln is not None or resid is not None:
        # fused prologue / epilogue (decode GEMV); other paths apply them around the GEMM
        if ln is not None and x.is_cuda and not ln_fusable(M, K):
            from .norm import layer_norm
            x2, ln = layer_norm(x2, ln[0], ln[1], ln[2]), None
        if x.is_cuda and M <= 256:
            assert x.dtype == torch.bfloat16, "weight-only GEMV takes bf16 activations"
            if x2.stride(-1) != 1:
                x2 = x2.contiguous()
            if resid is not None:
                resid = resid.reshape(M, N).contiguous()
            scale = weight_scale if weight_scale.dtype == torch.float32 else weight_scale.float()
            y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
            tiles = (N // 32) * ((M + 31) // 32)
            KS = 1 if ln is not None else _split_k(tiles, K // (32 if bits == 8 else 64))
            ws, cnt = _splitk_bufs(x.device, KS, M, N, tiles)
            _wo_call(bits, x2, weight, scale, bias, y, M, N, K, KS, act, ln,
                     resid.reshape(M, N) if resid is not None else None, ws, cnt)
            return y.reshape(*lead, N)
        xin = _ln_ref(x2, ln).to(x.dtype) if ln is not None else x2
        y = weight_only_linear(xin, weight, bias, weight_scale, weight_dtype, act_method)
        if resid is not None:
            y = (y.float() + resid.reshape(M, N).float()).to(y.dtype)
        return y.reshape(*lead, N)
    if x.is_cuda:
        assert x.dtype == torch.bfloat16, "weight-only GEMM takes bf16 activations"
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        scale = weight_scale if weight_scale.dtype == torch.float32 else weight_scale.float()
        if M > WO_GEMV_MAX_M:  # compute-bound: dequantize once, the own bf16 MFMA GEMM
            from .gemm import gemm_nt
            w = torch.empty((N, K), dtype=torch.bfloat16, device=x.device)
            _lib.call("piamd_wo_dequant", bits, weight.data_ptr(), scale.data_ptr(), w.data_ptr(),
                      N, K, _lib.stream())
            fused = {0: "none", 1: "gelu_tanh", 2: "gelu", 3: "relu"}.get(act)
            y = gemm_nt(x2, w, bias=bias.to(torch.bfloat16) if bias is not None else None,
                        act=fused or "none")
            if fused is None:
                y = _ref_act(y, act)
            return y.reshape(*lead, N)
        y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
        tiles = (N // 32) * ((M + 31) // 32)
        KS = _split_k(tiles, K // (32 if bits == 8 else 64))
        ws, cnt = _splitk_bufs(x.device, KS, M, N, tiles)
        _lib.call("piamd_wo_gemm", bits, x2.data_ptr(), x2.stride(0), weight.data_ptr(),
                  scale.data_ptr(), _lib.ptr(bias), y.data_ptr(), y.stride(0), _lib.ptr(ws),
                  _lib.ptr(cnt), M, N, K, KS, act, _lib.stream())
        return y.reshape(*lead, N)
    w = _unpack(weight, bits, N, K).float() * weight_scale.float()[:, None]
    y = x2.float() @ w.t()
    if bias is not None:
        y = y + bias.float()
    return _ref_act(y, act).to(x.dtype).reshape(*lead, N)


def quantize_rows(x, scale=None):
    """bf16 [M, K] → (int8 [M, K], per-row scale [M] f32). ``scale`` (float > 0): static
    per-tensor scale (x ≈ q · scale); None: dynamic per-token absmax / 127."""
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if not x.is_cuda:
        xf = x2.float()
        s = (xf.abs().amax(1).clamp_min(1e-30) / 127.0) if scale is None else \
            torch.full((M,), float(scale))
        s = torch.where(xf.abs().amax(1) > 0, s, torch.ones_like(s)) if scale is None else s
        q = torch.round(xf / s[:, None]).clamp(-127, 127).to(torch.int8)
        return q, s
    if x2.stride(-1) != 1 or x2.dtype != torch.bfloat16:
        x2 = x2.to(torch.bfloat16).contiguous()
    q = torch.empty((M, K), dtype=torch.int8, device=x.device)
    if scale is None:
        s = torch.empty(M, dtype=torch.float32, device=x.device)
        _lib.call("piamd_quant_rows", x2.data_ptr(), x2.stride(0), q.data_ptr(), K, s.data_ptr(),
                  0.0, M, K, _lib.stream())
    else:
        s = torch.full((M,), float(scale), dtype=torch.float32, device=x.device)
        _lib.call("piamd_quant_rows", x2.data_ptr(), x2.stride(0), q.data_ptr(), K, None,
                  float(scale), M, K, _lib.stream())
    return q, s


def int8_gemm(xq, xs, wq, ws, bias=None, act="none"):
    """y = act((xq · wqᵀ) · xs[m] · ws[n] + bias) → bf16. xq [M, K] int8, wq [N, K] int8."""
    M, K = xq.shape
    N = wq.shape[0]
    if not xq.is_cuda:
        y = (xq.double() @ wq.double().t()) * xs.double()[:, None] * ws.double()[None, :]
        if bias is not None:
            y = y + bias.double()
        return _ref_act(y.float(), ACTS[act]).to(torch.bfloat16)
    assert K % 128 == 0 and N % 4 == 0, "int8 GEMM needs K % 128 == 0 and N % 4 == 0"
    y = torch.empty((M, N), dtype=torch.bfloat16, device=xq.device)
    wsf = ws.float().contiguous()
    _lib.call("piamd_gemm_i8", xq.data_ptr(), xq.stride(0), wq.data_ptr(), wq.stride(0),
              xs.data_ptr(), 0.0, wsf.data_ptr(), _lib.ptr(bias), y.data_ptr(), y.stride(0), M, N,
              K, ACTS[act], _lib.stream())
    return y


def int8_linear(x, weight, weight_scale, bias=None, act_scale=None, act="none"):
    """Activation-quantised int8 linear (reference `fused_multi_transformer_int8` GEMMs):
    x [..., K] bf16 is quantised per token (``act_scale=None``) or with the static per-tensor
    ``act_scale``; weight [N, K] int8 row-major (``weight_quantize(w, "llm.int8")``) with per-channel
    ``weight_scale`` [N]; int8 MFMA GEMM with int32 accumulation and a dequantising epilogue."""
    K = x.shape[-1]
    lead = x.shape[:-1]
    xq, xs = quantize_rows(x.reshape(-1, K), act_scale)
    y = int8_gemm(xq, xs, weight, weight_scale, bias, act)
    return y.reshape(*lead, weight.shape[0]).to(x.dtype if x.dtype != torch.float32 else torch.float32)


def llm_int8_linear(x, weight, bias=None, weight_scale=None, threshold=6.0):
    """LLM.int8 (reference `nn/quant/quantized_linear.py:llm_int8_linear`): input features with an
    outlier (|x| > threshold in any row) run in bf16 against the dequantised weight columns; the rest
    is quantised per token to int8 and multiplied by the int8 weight [N, K] on the int8 MFMA GEMM."""
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    outl = (x2.abs() > threshold).any(0)
    xi = x2.masked_fill(outl[None, :], 0)
    y = int8_linear(xi, weight, weight_scale, bias).float()
    if bool(outl.any()):
        wd = weight.float() * weight_scale.float()[:, None]  # [N, K]
        y = y + x2[:, outl].float() @ wd[:, outl].t()
    return y.to(x.dtype).reshape(*x.shape[:-1], weight.shape[0])
