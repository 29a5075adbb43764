"""The framework's own GEMMs: the hand-scheduled gfx950 assembly GEMM (``csrc/asm/gemm_gen.py``,
``asm_gemm``) for bf16 / fp16 products with at least a few hundred rows, and the skinny MFMA kernel
(``csrc/kernels/gemm_small.hip``, ``small_gemm``) for few-row products (inference, prefill of short
prompts). ``matmul`` is the dispatcher every framework matmul goes through.

Operand convention: ``trans_a`` means ``a`` is stored [K, M] and ``trans_b`` means ``b`` is stored
[N, K] (so weights kept [in, out] serve forward, data-gradient and weight-gradient products without
copies). Epilogues:

* ``epi="bias_act"``: ``pre = A·B + bias`` is written to ``aux`` and ``act(pre)`` to C (FFN1);
* ``epi="dact"``: ``C = (A·B) ⊙ act'(aux)`` (the FFN1 activation backward fused into the FFN2
  data-gradient GEMM);
* ``out`` f32 with ``accumulate=True``: C += A·B (weight gradient straight into main_grad).

CPU tensors run the PyTorch reference of the same contract (tests' numerics reference).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from .activation import ACTS, _ref_act

_EPI = {"none": 0, "bias_act": 1, "dact": 2}


def _act_grad_ref(h, act):
    h = h.float().detach().requires_grad_(True)
    with torch.enable_grad():
        y = _ref_act(h, act)
        (g,) = torch.autograd.grad(y.sum(), h)
    return g


NUM_CUS = 256

_AGEMM_READY = [False]


def _agemm_load():
    """Load the assembled code object (`_lib/piamd_agemm.hsaco`) into the HIP runtime once."""
    if _AGEMM_READY[0]:
        return
    import os
    from .. import _build
    path = os.environ.get("PIAMD_AGEMM_HSACO") or _build.AGEMM_HSACO  # ablation builds (tools/)
    if not os.path.exists(path):
        raise RuntimeError(f"assembly GEMM code object missing ({path}); run "
                           "`python -m paddle_infer_amd._build`")
    _lib.call("piamd_agemm_load", path.encode())
    _AGEMM_READY[0] = True


_HALF = (torch.bfloat16, torch.float16)


def asm_supported(a, b, trans_a=False, trans_b=False, ksplit=1):
    """Contract of the assembly GEMM (`csrc/asm/gemm_gen.py`): bf16 or fp16 operands of one dtype,
    K % (64·ksplit) with ≥ 2 K-blocks per split, N % 4, 8-element aligned leading dims < 2^22,
    M % 8 when A is stored [K, M], N % 8 when B is stored [K, N], 16-byte aligned operands."""
    if not (a.is_cuda and a.dtype in _HALF and b.dtype == a.dtype):
        return False
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    return (K % (64 * ksplit) == 0 and K // ksplit >= 128 and N % 4 == 0 and M > 0
            and (not trans_a or M % 8 == 0) and (trans_b or N % 8 == 0)
            and a.stride(-1) == 1 and b.stride(-1) == 1
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and a.stride(0) < (1 << 22) and b.stride(0) < (1 << 22))


def asm_gemm(a, b, trans_a=False, trans_b=False, out=None, out_f32=False, accumulate=False,
             ksplit=1, epi="none", act="none", bias=None, aux=None, colsum=None):
    """C (+)= op(A)·op(B) on the hand-scheduled assembly kernels (bf16 or fp16 operands; the
    16-bit output has the operands' dtype). 3-D ``a`` / ``b`` / ``out`` run one batched launch
    (a 2-D operand, or a batch stride of 0, broadcasts over the batch). Fused epilogues (2-D, A
    stored [M, K], B stored [N, K], 16-bit C): ``epi="bias_act"`` — pre = 16-bit(A·B + bias)
    written to ``aux`` (optional), C = act(pre), act ∈ none / gelu_tanh / gelu (exact erf) / relu;
    ``epi="dact"`` — C = (A·B) ⊙ act'(aux), act ∈ gelu_tanh / relu; with ``colsum`` (f32
    [ceil(M/128), N]) the epilogue also writes C's column sums per 128-row band (bias gradient of
    the activation's producer without another pass over C: reduce with :func:`colsum_parts`)."""
    _agemm_load()
    batched = a.dim() == 3 or b.dim() == 3
    nb = max(a.shape[0] if a.dim() == 3 else 1, b.shape[0] if b.dim() == 3 else 1)
    M = a.shape[-1] if trans_a else a.shape[-2]
    K = a.shape[-2] if trans_a else a.shape[-1]
    N = b.shape[-2] if trans_b else b.shape[-1]
    f16 = a.dtype == torch.float16
    half = torch.float16 if f16 else torch.bfloat16
    oshape = (nb, M, N) if batched else (M, N)
    if out is None:
        out = torch.empty(oshape, dtype=torch.float32 if out_f32 else half, device=a.device)
    assert tuple(out.shape) == oshape and out.stride(-1) == 1 and out.data_ptr() % 16 == 0
    assert out.dtype in (torch.float32, half)
    ws = None
    if ksplit > 1:
        assert not batched
        ws = torch.empty((ksplit, M, N), dtype=torch.float32, device=a.device)
    if aux is not None:
        assert aux.shape == (M, N) and aux.dtype == half and aux.stride(-1) == 1
    if bias is not None:
        assert bias.dtype == half and bias.is_contiguous()

    def bstride(t):
        return t.stride(0) if t.dim() == 3 and t.shape[0] > 1 else 0
    sa, sb = bstride(a), bstride(b)
    sc = out.stride(0) if batched else 0
    if batched:
        assert epi == "none" and (nb == 1 or sc > 0)
    if colsum is not None:
        assert epi == "dact" and colsum.dtype == torch.float32 and colsum.is_contiguous() \
            and tuple(colsum.shape) == ((M + 127) // 128, N)
        _lib.call("piamd_agemm2", a.data_ptr(), a.stride(-2), int(trans_a), b.data_ptr(), b.stride(-2),
                  int(trans_b), out.data_ptr(), out.stride(-2), int(out.dtype == torch.float32),
                  int(accumulate), M, N, K, _EPI[epi], ACTS[act], _lib.ptr(bias), _lib.ptr(aux),
                  aux.stride(0) if aux is not None else 0, ksplit, _lib.ptr(ws), int(f16), nb,
                  sa, sb, max(sc, 1), colsum.data_ptr(), _lib.stream())
        return out
    _lib.call("piamd_agemm", a.data_ptr(), a.stride(-2), int(trans_a), b.data_ptr(), b.stride(-2),
              int(trans_b), out.data_ptr(), out.stride(-2), int(out.dtype == torch.float32),
              int(accumulate), M, N, K, _EPI[epi], ACTS[act], _lib.ptr(bias), _lib.ptr(aux),
              aux.stride(0) if aux is not None else 0, ksplit, _lib.ptr(ws), int(f16), nb,
              sa, sb, max(sc, 1), _lib.stream())
    return out


def colsum_parts(part, out, accumulate=True):
    """out[N] (+)= Σ_rows part[rows, N] (f32 partial planes; ``out`` f32 / bf16 / fp16)."""
    G, N = part.shape
    _lib.call("piamd_colsum_parts", _lib.dtype_code(out, fp16=True), part.data_ptr(), G, N,
              out.data_ptr(), int(accumulate), _lib.stream())
    return out


def pick_ksplit(M, N, K):
    """Split-K degree for the assembly GEMM: fill the 256 CUs (one 256x256 tile per CU) when the
    tile grid is small and K is long (weight gradients: 2048 x 2048 tiles over 98k tokens; the
    tall-skinny 1x1-conv weight gradients: one or two tiles over a million pixel rows). Any
    divisor of the 64-block count up to 256 that leaves >= 8 blocks per split; the fewest waves per
    split wins, ties to the smaller split (less f32 plane traffic)."""
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    nk = K // 64
    if tiles >= 2 * NUM_CUS or nk < 16:
        return 1
    best, best_t = 1, None
    for ks in range(1, min(256, nk // 8) + 1):
        if nk % ks:
            continue
        waves = -(-tiles * ks // NUM_CUS)
        t = waves / ks
        if best_t is None or t < best_t - 1e-9:
            best, best_t = ks, t
    return best


F  # noqa


# ---------------------------------------------------------------------------------------------
# skinny kernel (csrc/kernels/gemm_small.hip) and the dispatcher every framework matmul uses
# ---------------------------------------------------------------------------------------------
_SG_SHAPES = {(1, 1), (1, 2), (1, 4), (2, 1), (2, 2), (2, 4), (4, 1), (4, 2), (4, 4), (8, 1), (8, 2)}
# (M, N, K) -> (mb, nb, wn, depth, ks): the fastest configs of the graph-timed sweep
# (tools/tune_small_gemm.py, fp16, weights streamed from HBM; profiles/small_gemm_tune_r4.jsonl)
_SG_TUNED: dict = {
    (16, 3072, 1024): (1, 1, 1, 1, 1), (16, 1024, 4096): (1, 1, 1, 1, 4),
    (32, 3072, 1024): (1, 2, 1, 1, 1), (32, 1024, 4096): (1, 1, 1, 1, 2),
    (64, 3072, 1024): (2, 2, 1, 1, 1), (64, 1024, 4096): (1, 1, 1, 1, 1),
    # M = 128 (BERT-Large batch 1): B-deep rings (depth = 1 | DB << 4; profiles/small_gemm_bdeep_r6.jsonl)
    (128, 3072, 1024): (2, 4, 1, 0x41, 1), (128, 1024, 1024): (1, 2, 1, 0x81, 1),
    (128, 4096, 1024): (2, 4, 1, 0x41, 1), (128, 1024, 4096): (2, 1, 1, 0x81, 1),
    (128, 6144, 2048): (4, 4, 1, 2, 1), (128, 2048, 2048): (2, 2, 1, 1, 1),
    (128, 8192, 2048): (4, 4, 1, 2, 1),
    # GPT-1.3B serving-batch decode (bf16, graph-timed sweep incl. the B-deep rings;
    # profiles/small_gemm_decode_r6.jsonl): QKV / FFN1 (LN-folded), out-proj, FFN2 (K = 8192, split-K)
    (8, 6144, 2048): (1, 2, 1, 2, 1), (8, 8192, 2048): (1, 1, 1, 2, 1),
    (8, 2048, 2048): (1, 1, 1, 0x81, 1), (8, 2048, 8192): (1, 2, 1, 2, 4),
    (16, 2048, 2048): (1, 1, 1, 0x81, 1), (16, 2048, 8192): (1, 2, 1, 2, 4),
    (32, 6144, 2048): (2, 2, 1, 0x21, 1), (32, 8192, 2048): (2, 2, 1, 0x21, 1),
    (32, 2048, 2048): (1, 1, 1, 0x81, 1), (32, 2048, 8192): (2, 2, 1, 1, 4),
    (256, 3072, 1024): (4, 4, 1, 1, 1), (256, 1024, 4096): (2, 2, 1, 2, 1),
    (256, 2048, 2048): (4, 2, 1, 1, 1), (512, 2048, 2048): (4, 4, 1, 1, 1),
}


def small_cfg(M, N, K):
    """(mb, nb, wn, depth, ks) of the skinny kernel: 16·mb rows × 16·nb·wn columns per workgroup
    (wn waves side by side along N, 4/wn splitting K), ``depth`` k64 steps of loads in flight per
    wave (``1 | DB << 4``: DB steps of the weight operand in flight, one of the activations), K split ks ways over workgroups when the tile grid alone cannot fill the 256 CUs."""
    hit = _SG_TUNED.get((M, N, K))
    if hit is not None:
        return hit
    # The sweep's winners all keep the 4 waves splitting K (wn = 1) and take the biggest tile
    # (most operand reuse) whose grid still gives every CU a workgroup (≥ 192); among equal areas
    # the squarest, then the wider. Split K only when even 16x16 tiles cannot fill the chip.
    nkb = K // 64
    best = None
    for mb, nb in _SG_SHAPES:
        if mb > 1 and 16 * mb > M:
            continue
        wgs = -(-M // (16 * mb)) * -(-N // (16 * nb))
        if wgs < 192:
            continue
        key = (mb * nb, -abs(mb - nb), nb)
        if best is None or key > best[0]:
            best = (key, mb, nb, wgs)
    if best is None:
        mb, nb = 1, 1
        wgs = -(-M // 16) * -(-N // 16)
        ks = 1
        while wgs * ks < 192 and ks * 2 <= nkb // 4:
            ks *= 2
        return mb, nb, 1, 1, ks
    _, mb, nb, wgs = best
    depth = 2 if (mb * nb >= 16 and K >= 2048 and wgs <= 256) else 1
    return mb, nb, 1, depth, 1


_SG_WS: dict = {}
# activation codes of the skinny kernel: the shared set plus tanh (code 5, skinny kernel only)
_SG_ACTS = dict(ACTS, tanh=5)


def _sg_fixup_bufs(device, M, N, tiles):
    """Zeroed f32 [M·N] partial tile + per-tile arrival counters for the fixup mode (left zeroed
    by the kernel's last arrival); one pair per (device, stream): launches on one stream never
    overlap."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    ws, cnt = _SG_WS.get(key, (None, None))
    if ws is None or ws.numel() < M * N or cnt.numel() < tiles:
        ws = torch.zeros(max(M * N, ws.numel() if ws is not None else 0), dtype=torch.float32, device=device)
        cnt = torch.zeros(max(tiles, cnt.numel() if cnt is not None else 0, 4096), dtype=torch.int32,
                          device=device)
        _SG_WS[key] = (ws, cnt)
    return ws, cnt


def small_gemm(a, b, out=None, out_f32=False, alpha=1.0, bias=None, act="none", resid=None, cfg=None,
               slices=False, ln=None, ln_stats=None, resid_ln=None):
    """C[M, N] = act(alpha·a[M, K]·b[N, K]ᵀ + bias) (+ resid) on the skinny MFMA kernel (both
    operands K-contiguous bf16 / fp16, K % 64 == 0, N % 4 == 0). Split-K runs in fixup mode (one
    launch; ``slices=True``: deterministic slices + a finish launch). ``ln = (c1, b2, eps)``: the
    LayerNorm fold (see :func:`ln_fold`) — ``b`` is the folded weight, C = act(LN(a)·Wᵀ + bias)
    from the raw rows of ``a`` (no K split; ``bias`` is inside b2); ``ln_stats`` (f32 [M, 2]):
    receives each raw row's (mean, rstd). ``resid_ln = (stats, gamma, beta)``: ``resid`` holds raw
    rows whose LayerNorm was deferred; (r − mean)·rstd·γ + β is added instead of r."""
    M, K = a.shape
    N = b.shape[0]
    half = a.dtype
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32 if out_f32 else half, device=a.device)
    mb, nb, wn, depth, ks = cfg or small_cfg(M, N, K)
    if ln is not None or resid_ln is not None:
        if ln is not None:
            ks = 1
        return _small_gemm_ln(a, b, out, M, N, K, (mb, nb, wn, depth, ks), act, resid, ln, ln_stats,
                              resid_ln, bias, alpha)
    ws = cnt = None
    if ks > 1:
        if slices:
            ws = torch.empty((ks, M, N), dtype=torch.float32, device=a.device)
        else:
            tiles = -(-M // (16 * mb)) * -(-N // (16 * nb * wn))
            ws, cnt = _sg_fixup_bufs(a.device, M, N, tiles)
    _lib.call("piamd_small_gemm", int(half == torch.float16), a.data_ptr(), a.stride(0),
              b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0),
              int(out.dtype == torch.float32), M, N, K, mb, nb, wn, depth, ks, float(alpha), _lib.ptr(bias),
              _SG_ACTS[act], _lib.ptr(resid), resid.stride(0) if resid is not None else 0,
              _lib.ptr(ws), _lib.ptr(cnt), _lib.stream())
    return out


def ln_fold(w_nk, gamma, beta, bias=None):
    """LayerNorm fold of a K-contiguous weight w [N, K] for :func:`small_gemm` ``ln=``:
    (w∘γ as bf16 [N, K], c1 = Σ_k (w∘γ)[n, k] of the ROUNDED fold (f32 [N]), b2 = bias + w·β (f32
    [N])), so that LN(a)·wᵀ + bias = rstd·(a·(w∘γ)ᵀ − mean·c1) + b2."""
    wf = (w_nk.float() * gamma.float().view(1, -1)).to(w_nk.dtype).contiguous()
    c1 = wf.float().sum(1).contiguous()
    b2 = w_nk.float() @ beta.float()
    if bias is not None:
        b2 = b2 + bias.float().view(-1)
    return wf, c1, b2.contiguous()


def _small_gemm_ln(a, b, out, M, N, K, cfg, act, resid, ln, ln_stats=None, resid_ln=None, bias=None,
                   alpha=1.0):
    assert a.dtype == b.dtype and a.dtype in _HALF, "LayerNorm fold: bf16 / fp16 operands of one dtype"
    mb, nb, wn, depth, ks = cfg
    c1 = b2 = None
    eps = 0.0
    if ln is not None:
        c1, b2, eps = ln
        assert c1.dtype == torch.float32 and b2.dtype == torch.float32 and c1.numel() == N == b2.numel()
        if not (depth >> 4 in (2, 4) and depth & 15 == 1 and wn == 1):  # LN fold: one ring depth, or B 2 / 4 deep
            depth &= 15
        ks, bias, alpha = 1, None, 1.0
    if ln_stats is not None:
        assert ln is not None and ln_stats.dtype == torch.float32 and ln_stats.numel() >= 2 * M
    rs = rg = rb = None
    if resid_ln is not None:
        rs, rg, rb = resid_ln
        assert resid is not None and rs.dtype == torch.float32 and rs.numel() >= 2 * M
        assert rg.dtype == a.dtype and rb.dtype == a.dtype and rg.numel() == N == rb.numel()
        rg, rb = rg.contiguous(), rb.contiguous()
    ws = cnt = None
    if ks > 1:
        tiles = -(-M // (16 * mb)) * -(-N // (16 * nb * wn))
        ws, cnt = _sg_fixup_bufs(a.device, M, N, tiles)
    _lib.call("piamd_small_gemm_ln", int(a.dtype == torch.float16), a.data_ptr(), a.stride(0),
              b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0), int(out.dtype == torch.float32),
              M, N, K, mb, nb, wn, depth, ks, float(alpha), _lib.ptr(bias), _SG_ACTS[act], _lib.ptr(resid),
              resid.stride(0) if resid is not None else 0, _lib.ptr(ws), _lib.ptr(cnt), _lib.ptr(c1),
              _lib.ptr(b2), float(eps), _lib.ptr(ln_stats), _lib.ptr(rs), _lib.ptr(rg), _lib.ptr(rb),
              _lib.stream())
    return out


def own_dtype(*ts):
    """The own GEMMs take bf16 / fp16 CUDA operands of one dtype."""
    t0 = ts[0]
    return t0.is_cuda and t0.dtype in _HALF and all(t.dtype == t0.dtype for t in ts)


# ---------------------------------------------------------------------------------------------
# fp32 GEMMs as split-bf16 products (Paddle's default dtype; reference `blas_impl.cu.h:32`
# CUBlas<float>): x·w ≈ x_hi·w_hi + x_lo·w_hi + x_hi·w_lo with t = hi + lo (both bf16), the three
# products run as ONE bf16 MFMA GEMM over a 3×-long reduction ([x_hi | x_lo | x_hi] ·
# [w_hi | w_hi | w_lo]) with an f32 result: ≈2^-16 relative per product, at 3× the bf16 work —
# still ≈3× the f32 MFMA rate (`MI355X_MICROARCH.md` § Matrix cores: f32-input MFMA = 1/16 bf16).
# The operand split is one HIP pass (`piamd_split3_f32`).
# ---------------------------------------------------------------------------------------------
FP32_SPLIT = True  # False: fp32 GEMMs on the library (exact fp32)
_LO = {"hlh": 0b010, "hhl": 0b100}


def own_f32(*ts):
    """fp32 CUDA operands the split-bf16 path takes."""
    return FP32_SPLIT and all(t.is_cuda and t.dtype == torch.float32 for t in ts)


def split3(t, order, axis=0, Rp=None, Cp=None):
    """f32 [R, C] → bf16 segments (order "hlh" / "hhl"): axis 0 → [R, 3·Cp] (segments along the
    row, C zero-padded to Cp), axis 1 → [3·Rp, C] (stacked rows, R zero-padded to Rp)."""
    R, C = t.shape
    if t.stride(-1) != 1 or (R > 1 and t.stride(0) < C):
        t = t.contiguous()
    if axis == 0:
        Cp = Cp or _ceil(C, 64)
        Rp = R
        out = torch.empty((R, 3 * Cp), dtype=torch.bfloat16, device=t.device)
    else:
        Rp = Rp or _ceil(R, 64)
        Cp = C
        assert C % 8 == 0, "row-stacked split needs C % 8 == 0"
        out = torch.empty((3 * Rp, C), dtype=torch.bfloat16, device=t.device)
    _lib.call("piamd_split3_f32", t.data_ptr(), t.stride(0) if R > 1 else C, out.data_ptr(), R, C, Rp, Cp,
              _LO[order], axis, _lib.stream())
    return out


def gemm_nt_f32(a, b=None, alpha=1.0, bias=None, act="none", resid=None, b3=None):
    """fp32 C[M, N] = act(alpha·a[M, K]·b[N, K]ᵀ + bias) (+ resid) on the split-bf16 path; ``b3``:
    a pre-split right operand ([N, 3·Kp], "hhl", e.g. a cached weight)."""
    M, K = a.shape
    Kp = _ceil(K, 64)
    a3 = split3(a, "hlh", 0, Cp=Kp)
    if b3 is None:
        b3 = split3(b, "hhl", 0, Cp=Kp)
    N = b3.shape[0] if b is None else b.shape[0]
    Np = _ceil(N, 4)
    if Np != N:
        b3 = torch.nn.functional.pad(b3, (0, 0, 0, Np - N))
    K3 = 3 * Kp
    if use_small(M, Np, K3):
        out = small_gemm(a3, b3, out_f32=True)
    else:
        ks = pick_ksplit(M, Np, K3)
        if not asm_supported(a3, b3, trans_b=True, ksplit=ks):
            ks = 1
        out = asm_gemm(a3, b3, trans_b=True, out_f32=True, ksplit=ks)
    if Np != N:
        out = out[:, :N].contiguous()
    if alpha != 1.0:
        out.mul_(alpha)
    if bias is not None or act != "none":
        from .activation import bias_act
        b32 = bias.float().reshape(-1) if bias is not None else None
        out = bias_act(out, b32, act) if N % 8 == 0 else _ref_act(out + (b32 if b32 is not None else 0),
                                                                   ACTS[act])
    if resid is not None:
        out.add_(resid.reshape(M, N).float())
    return out


def wgrad_f32(x2, dy2, out=None):
    """fp32 x2[T, K]ᵀ · dy2[T, N] (weight gradient) on the split path: the reduction (token) dim
    stacked as [x_hi; x_lo; x_hi] · [dy_hi; dy_hi; dy_lo] — one TN GEMM, no transposes. ``out``
    (f32 [K, N], contiguous): accumulated into (main_grad += …) by the GEMM epilogue."""
    T, K = x2.shape
    N = dy2.shape[1]
    if K % 8 == 0 and N % 8 == 0 and (out is None or out.is_contiguous()):
        Tp = _ceil(T, 64)
        x3 = split3(x2, "hlh", 1, Rp=Tp)
        d3 = split3(dy2, "hhl", 1, Rp=Tp)
        ks = pick_ksplit(K, N, 3 * Tp)
        if not asm_supported(x3, d3, trans_a=True, ksplit=ks):
            ks = 1
        if out is not None:
            return asm_gemm(x3, d3, trans_a=True, out=out, accumulate=True, ksplit=ks)
        return asm_gemm(x3, d3, trans_a=True, out_f32=True, ksplit=ks)
    g = gemm_nt_f32(x2.t().contiguous(), dy2.t().contiguous())
    return out.add_(g) if out is not None else g


def _ceil(x, m):
    return -(-x // m) * m


def _is_weight(t):
    """Parameters and the framework's cached weight copies (``linear.transposed``): their padded
    operand images may be cached across calls."""
    return isinstance(t, torch.nn.Parameter) or getattr(t, "_piamd_weight", False)


def _kc(t, Kp, rows=None, cache=False):
    """[R, K] operand → K-contiguous, 16-B aligned, K zero-padded to Kp (and rows to ``rows``).
    ``cache``: a weight's padded image is kept on the tensor, keyed by its version and the
    parameter epoch (optimizer writes), so an off-grid inference weight is padded once, not per
    call."""
    R, K = t.shape
    R2 = rows or R
    if Kp == K and R2 == R and t.stride(-1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0 \
            and t.stride(0) < (1 << 22) and (R == 1 or t.stride(0) >= K):
        return t
    key = None
    if cache and _is_weight(t):
        from .linear import _PARAM_EPOCH
        key = (_PARAM_EPOCH[0], t._version, t.data_ptr(), Kp, R2)
        c = getattr(t, "_piamd_pad", None)
        if c is not None and c[0] == key:
            return c[1]
    o = torch.zeros((R2, Kp), dtype=t.dtype, device=t.device) if (Kp != K or R2 != R) else \
        torch.empty((R2, Kp), dtype=t.dtype, device=t.device)
    o[:R, :K].copy_(t.detach())
    if key is not None:
        t._piamd_pad = (key, o)
    return o


def use_small(M, N, K):
    """Skinny kernel vs the 256×256-tile assembly GEMM (graph-timed sweep,
    profiles/small_gemm_tune_r4.jsonl): the skinny kernel for ≤ 64 rows, for ≤ 128 rows unless K
    is very long, and up to 512 rows for small weights (N·K ≤ 2048²); the asm GEMM with split-K
    beyond (e.g. M=256 N=6144 K=2048: 29 µs vs 35 µs)."""
    if M <= 64:
        return True
    if M <= 128 and K < 8192:
        return True
    return M <= 512 and N * K <= 2048 * 2048


_FUSED_ACTS = ("none", "gelu_tanh", "gelu", "relu")


def gemm_nt(a, b, alpha=1.0, bias=None, act="none", resid=None, out_f32=False):
    """C[M, N] = act(alpha·a[M, K]·b[N, K]ᵀ + bias) (+ resid): the 2-D product every framework
    matmul lowers to, on the framework's own kernels (skinny kernel for few rows, assembly GEMM
    otherwise). bf16 / fp16 operands of one dtype; any K (zero-padded to the kernels' 64-multiple)
    and any N (padded to a multiple of 4)."""
    if a.dtype == torch.float32:
        return gemm_nt_f32(a, b, alpha, bias, act, resid)
    M, K = a.shape
    N = b.shape[0]
    half = a.dtype
    small = use_small(M, N, K)
    Kp = max(64 if small else 128, _ceil(K, 64))
    Np = _ceil(N, 4) if small else (N if N % 4 == 0 else _ceil(N, 8))
    a2 = _kc(a, Kp)
    b2 = _kc(b, Kp, Np, cache=True)
    if bias is not None:
        bias = bias.to(half).reshape(-1)
        if Np != N:
            bias = torch.nn.functional.pad(bias, (0, Np - N))
        bias = bias.contiguous()
    r2 = None
    if resid is not None:
        r2 = resid.reshape(M, N).to(half)
        if Np != N:
            r2 = torch.nn.functional.pad(r2, (0, Np - N))
        if r2.stride(-1) != 1:
            r2 = r2.contiguous()
    if small:
        out = small_gemm(a2, b2, out_f32=out_f32, alpha=alpha, bias=bias, act=act, resid=r2)
    else:
        out = _asm_nt(a2, b2, alpha, bias, act, out_f32)
        if r2 is not None:
            out.add_(r2)
    return out if Np == N else out[:, :N].contiguous()


def _asm_nt(a, b, alpha, bias, act, out_f32):
    M, K = a.shape
    N = b.shape[0]
    ks = pick_ksplit(M, N, K)
    fused = (not out_f32 and alpha == 1.0 and act in _FUSED_ACTS and ks == 1
             and (bias is not None or act != "none"))
    if fused:
        return asm_gemm(a, b, trans_b=True, epi="bias_act", act=act, bias=bias)
    if not asm_supported(a, b, trans_b=True, ksplit=ks):
        ks = 1
    out = asm_gemm(a, b, trans_b=True, out_f32=out_f32, ksplit=ks)
    if alpha != 1.0:
        out.mul_(alpha)
    if bias is not None or act != "none":
        from .activation import bias_act
        out = bias_act(out, bias, act)
    return out


def _bcast_batch(x, y):
    """Broadcast the batch dims of ≥ 3-D operands → ([Bt, ·, ·] x, [Bt, ·, ·] y, batch shape)."""
    bx, by = x.shape[:-2], y.shape[:-2]
    bs = torch.broadcast_shapes(bx, by)
    def to3(t, bt):
        if bt == bs:
            return t.reshape(-1, *t.shape[-2:])
        if all(d == 1 for d in bt):  # a single matrix broadcast over the batch: stride 0
            return t.reshape(t.shape[-2:])
        return t.expand(*bs, *t.shape[-2:]).reshape(-1, *t.shape[-2:])
    return to3(x, bx), to3(y, by), bs


def bmm(x, y, transpose_x=False, transpose_y=False, alpha=1.0):
    """Batched C[i] = alpha·op(x[i])·op(y[i]) (x / y 3-D, or 2-D broadcast over the batch) as ONE
    batched assembly-GEMM launch (operand layouts handled by the kernel's four layout variants)."""
    nb = max(x.shape[0] if x.dim() == 3 else 1, y.shape[0] if y.dim() == 3 else 1)
    M = x.shape[-1] if transpose_x else x.shape[-2]
    K = x.shape[-2] if transpose_x else x.shape[-1]
    N = y.shape[-2] if transpose_y else y.shape[-1]
    if x.dtype == torch.float32:  # split-bf16: [nb·M, 3Kp] · [nb·N, 3Kp]ᵀ as one batched launch
        xa = (x.transpose(-1, -2) if transpose_x else x).expand(nb, M, K) if x.dim() == 3 or nb > 1 else \
            (x.transpose(-1, -2) if transpose_x else x)
        yb = (y if transpose_y else y.transpose(-1, -2))
        yb = yb.expand(nb, N, K) if (yb.dim() == 3 or nb > 1) else yb
        Kp = _ceil(K, 64)
        Np = _ceil(N, 4)
        A = split3(xa.reshape(-1, K), "hlh", 0, Cp=Kp).view(-1, M, 3 * Kp) if xa.dim() == 3 else \
            split3(xa, "hlh", 0, Cp=Kp)
        B = split3(yb.reshape(-1, K), "hhl", 0, Cp=Kp).view(-1, N, 3 * Kp) if yb.dim() == 3 else \
            split3(yb, "hhl", 0, Cp=Kp)
        if Np != N:
            B = torch.nn.functional.pad(B, (0, 0, 0, Np - N))
        if A.dim() == 2:
            A = A.unsqueeze(0)
        out = asm_gemm(A, B, trans_b=True, out_f32=True)
        if Np != N:
            out = out[..., :N].contiguous()
        if alpha != 1.0:
            out.mul_(alpha)
        return out

    def ok(t, inner_contig):
        return (t.stride(-1) == 1 and t.stride(-2) % 8 == 0 and t.data_ptr() % 16 == 0
                and t.stride(-2) < (1 << 22) and inner_contig
                and (t.dim() == 2 or t.shape[0] == 1 or t.stride(0) % 8 == 0))

    def sep(t):  # batch slices must not overlap (or broadcast one matrix: stride 0)
        return t.dim() == 2 or t.shape[0] == 1 or t.stride(0) == 0 or t.shape[-2] * t.stride(-2) <= t.stride(0)
    native = (K % 64 == 0 and K >= 128 and N % 4 == 0
              and ok(x, not transpose_x or M % 8 == 0) and ok(y, transpose_y or N % 8 == 0)
              and sep(x) and sep(y))
    if native:
        out = asm_gemm(x, y, trans_a=transpose_x, trans_b=transpose_y)
    else:  # K-contiguous, K-padded copies: [nb, M, Kp] · [nb, N, Kp]ᵀ
        Kp = max(128, _ceil(K, 64))
        Np = _ceil(N, 4)
        xa = x.transpose(-1, -2) if transpose_x else x
        yb = y if transpose_y else y.transpose(-1, -2)
        A = torch.zeros((*xa.shape[:-1], Kp), dtype=x.dtype, device=x.device)
        A[..., :K].copy_(xa)
        B = torch.zeros((*yb.shape[:-2], Np, Kp), dtype=y.dtype, device=y.device)
        B[..., :N, :K].copy_(yb)
        out = asm_gemm(A, B, trans_b=True)
        if Np != N:
            out = out[..., :N].contiguous()
    if out.dim() == 2:
        out = out.unsqueeze(0).expand(nb, M, N).contiguous() if nb > 1 else out.unsqueeze(0)
    if alpha != 1.0:
        out.mul_(alpha)
    return out


def split_nk(w, transpose):
    """Cached "hhl" split of an fp32 right operand as [N, 3·Kp]: of ``w`` itself when it is
    stored [N, K] (``transpose``), else of ``wᵀ`` (a Paddle [in, out] weight). Kept on the tensor,
    refreshed when it changed (autograd version / flat-optimizer epoch)."""
    from .linear import _PARAM_EPOCH
    key = (_PARAM_EPOCH[0], w._version)
    attr = "_piamd_split_n" if transpose else "_piamd_split_t"
    c = getattr(w, attr, None)
    if c is not None and c[0] == key:
        return c[1]
    src = w.detach() if transpose else w.detach().t()
    b3 = split3(src, "hhl", 0)
    setattr(w, attr, (key, b3))
    return b3


def _b_nk(y, transpose_y):
    """2-D right operand as [N, K] K-contiguous: the stored matrix when transposed, else the
    cached transposed copy (weights: transposed once, refreshed when they change)."""
    if transpose_y:
        return y
    from .linear import transposed
    if y.is_contiguous():
        return transposed(y)
    return y.t().contiguous()


def matmul_fwd(x, y, transpose_x=False, transpose_y=False, alpha=1.0):
    """paddle.matmul semantics (broadcast batch dims, 1-D operands) on the own kernels; the caller
    checked ``own_dtype(x, y)``."""
    xs, ys = x.dim(), y.dim()
    if xs == 1:
        x = x.unsqueeze(0)
        transpose_x = False
    if ys == 1:
        y = y.unsqueeze(1)
        transpose_y = False
    if y.dim() == 2 and not (transpose_x and x.dim() > 2):
        xa = x.transpose(-1, -2) if transpose_x else x
        lead = xa.shape[:-1]
        a2 = xa.reshape(-1, xa.shape[-1])
        if a2.dtype == torch.float32:
            out = gemm_nt_f32(a2, alpha=alpha, b3=split_nk(y, transpose_y))
        else:
            out = gemm_nt(a2, _b_nk(y, transpose_y), alpha=alpha)
        out = out.reshape(*lead, out.shape[-1])
    else:
        if x.dim() == 2 and y.dim() > 2:
            x = x.expand(*y.shape[:-2], *x.shape)
        x3, y3, bs = _bcast_batch(x, y)
        out = bmm(x3, y3, transpose_x, transpose_y, alpha)
        out = out.reshape(*bs, *out.shape[-2:])
    if xs == 1:
        out = out.squeeze(-2)
    if ys == 1:
        out = out.squeeze(-1)
    return out


def _sum_to(g, shape):
    if tuple(g.shape) == tuple(shape):
        return g
    while g.dim() > len(shape):
        g = g.sum(0)
    for i, d in enumerate(shape):
        if d == 1 and g.shape[i] != 1:
            g = g.sum(i, keepdim=True)
    return g


class _MatmulFn(torch.autograd.Function):
    """paddle.matmul on the own kernels with its gradients on the own kernels too (reference
    `phi/kernels/impl/matmul_grad_kernel_impl.h`): dX = dOut·Yᵀ, dY = Xᵀ·dOut, transposes folded
    into the GEMM flags, broadcast batch dims summed."""

    @staticmethod
    def forward(ctx, x, y, tx, ty, alpha):
        ctx.save_for_backward(x, y)
        ctx.tx, ctx.ty, ctx.alpha = tx, ty, alpha
        return matmul_fwd(x, y, tx, ty, alpha)

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        tx, ty, alpha = ctx.tx, ctx.ty, ctx.alpha
        g = g.contiguous()
        xs, ys = x.dim(), y.dim()
        x2 = x.unsqueeze(0) if xs == 1 else x
        y2 = y.unsqueeze(1) if ys == 1 else y
        g2 = g
        if xs == 1:
            g2 = g2.unsqueeze(-2)
        if ys == 1:
            g2 = g2.unsqueeze(-1)
        dx = dy = None
        if ctx.needs_input_grad[0]:
            # X' = op(x): dX' = g·op(y)ᵀ; dx = dX' or dX'ᵀ
            if tx:
                dx = matmul_fwd(y2, g2, ty, True, alpha)  # (g·Y'ᵀ)ᵀ = Y'·gᵀ
            else:
                dx = matmul_fwd(g2, y2, False, not ty, alpha)
            dx = _sum_to(dx, x2.shape)
            if xs == 1:
                dx = dx.squeeze(0)
        if ctx.needs_input_grad[1]:
            if ty:
                dy = matmul_fwd(g2, x2, True, tx, alpha)  # (X'ᵀ·g)ᵀ = gᵀ·X'
            else:
                dy = matmul_fwd(x2, g2, not tx, False, alpha)
            dy = _sum_to(dy, y2.shape)
            if ys == 1:
                dy = dy.squeeze(1)
        return dx, dy, None, None, None


def matmul(x, y, transpose_x=False, transpose_y=False, alpha=1.0):
    """``paddle.matmul`` / ``bmm`` / static ``matmul_v2`` / ``matmul`` / ``mul``: bf16 / fp16 CUDA
    operands run the framework's own GEMMs (forward and backward), fp32 CUDA operands the same
    kernels as split-bf16 products (``gemm_nt_f32``), or the autocast dtype under AMP O1; CPU
    tensors take the PyTorch reference."""
    if (x.is_cuda and y.is_cuda and x.dtype == torch.float32 and y.dtype == torch.float32
            and torch.is_autocast_enabled("cuda")):
        # AMP O1 (paddle.amp.auto_cast → torch autocast): matmul is a white-list op — fp32
        # operands run in the autocast dtype on the own 16-bit GEMMs (casts differentiable)
        dt = torch.get_autocast_dtype("cuda")
        x, y = x.to(dt), y.to(dt)
    if ((own_dtype(x, y) or own_f32(x, y)) and x.dim() >= 1 and y.dim() >= 1
            and x.numel() and y.numel()):
        if torch.is_grad_enabled() and (x.requires_grad or y.requires_grad):
            return _MatmulFn.apply(x, y, transpose_x, transpose_y, alpha)
        return matmul_fwd(x, y, transpose_x, transpose_y, alpha)
    if transpose_x and x.dim() > 1:
        x = x.transpose(-1, -2)
    if transpose_y and y.dim() > 1:
        y = y.transpose(-1, -2)
    out = torch.matmul(x, y)
    return out * alpha if alpha != 1.0 else out
