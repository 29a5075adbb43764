"""ctypes binding of the in-tree HIP kernel library ``_lib/libpiamd_kernels.so``.

The library is loaded lazily, *after* ``import torch`` so that its ``libamdhip64.so.7`` dependency
resolves to the HIP runtime torch already mapped (one runtime, one set of streams). Every launch
goes onto torch's current HIP stream, so the kernels compose with hipBLASLt GEMMs, RCCL
collectives on side streams and ``torch.cuda.CUDAGraph`` (hipGraph) capture.

Dispatch rule used by every op module: a tensor on the GPU runs the HIP kernel and FAILS LOUDLY
if the library is missing; CPU tensors take the PyTorch reference path (used by the CPU test tier
and as the numerics reference of the GPU tests).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from .. import _build

_LIB = None
_LOCK = threading.Lock()

c_void_p, c_int, c_float, c_ll, c_u64 = (ctypes.c_void_p, ctypes.c_int, ctypes.c_float,
                                         ctypes.c_longlong, ctypes.c_uint64)

# name -> argtypes (restype is int = hipError_t unless listed in _RESTYPES)
_SIGS = {
    # dtype, x, bias, residual, gamma, beta, y, residual_out, mean, rstd, rows, N, eps, p, seed,
    # offset, flags (bit0 = RMSNorm), stream
    "piamd_layernorm_fwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_u64,
                            c_u64, c_int, c_void_p],
    # dtype, dy, h, gamma, mean, rstd, dres_in, dres, dx, dgamma, dbeta, dbias, ws, rows, N, p,
    # seed, offset, accum_mask, flags, stream
    "piamd_layernorm_bwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                            c_float, c_u64, c_u64, c_int, c_int, c_void_p],
    "piamd_colsum": [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
    "piamd_adamw_flat": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_ll, c_float,
                         c_void_p, c_float, c_float, c_float, c_float, c_float, c_float, c_void_p,
                         c_float, c_void_p],
    "piamd_momentum_flat": [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_ll, c_float,
                            c_void_p, c_float, c_float, c_int, c_void_p, c_void_p],
    "piamd_sumsq": [c_void_p, c_int, c_ll, c_void_p, c_void_p, c_int, c_void_p],
    "piamd_xent_stats": [c_int, c_void_p, c_void_p, c_int, c_int, c_ll, c_int, c_void_p, c_void_p,
                         c_void_p, c_void_p],
    "piamd_xent_bwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_int, c_ll,
                       c_int, c_void_p, c_void_p],
    "piamd_bias_act_fwd": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p],
    "piamd_bias_act_bwd_grid": [c_int],
    "piamd_bias_act_bwd": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_int, c_int, c_int, c_void_p],
    "piamd_softmax_fwd": [c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_float,
                          c_void_p],
    "piamd_softmax_bwd": [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p],
    "piamd_dropout": [c_int, c_void_p, c_void_p, c_ll, c_float, c_u64, c_u64, c_void_p],
    "piamd_qkv_prep": [c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                       c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p],
    # qkv, ldq, bias, prep, rot, neox, base, kc, vc, lens, B, Hq, Hk, D, maxS, chunk, nsplit,
    # mask, ldm, scale, part, cnt, out, ldo, stream
    "piamd_decode_attn": [c_void_p, c_ll, c_void_p, c_int, c_int, c_int, c_float, c_void_p,
                          c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                          c_void_p, c_ll, c_float, c_void_p, c_void_p, c_void_p, c_ll, c_void_p],
    # bits, x, ldx, wp, scale, bias, y, ldy, ws, cnt, M, N, K, KS, act, stream
    "piamd_wo_gemm": [c_int, c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_ll,
                      c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "piamd_conv_wprep": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                         c_int, c_int, c_void_p],
    "piamd_wo_gemm_ex": [c_int, c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_ll,
                         c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                         c_void_p, c_float, c_void_p, c_ll, c_void_p],
    "piamd_wo_dequant": [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
}


_RESTYPES = {"piamd_layernorm_bwd_ws": ctypes.c_longlong, "piamd_dconv2d_wgrad_parts": ctypes.c_longlong,
             "piamd_group_norm_ws": ctypes.c_longlong}


class FaArgs(ctypes.Structure):
    """Mirror of ``struct FaArgs`` (csrc/kernels/flash_attn.h)."""
    _fields_ = ([(n, c_void_p) for n in ("q", "k", "v", "o", "lse", "dout", "delta", "dq", "dk", "dv",
                                        "mask", "cu_q", "cu_k")]
                + [(n, c_int) for n in ("B", "Sq", "Sk", "Hq", "Hk", "D", "ltot", "causal")]
                + [(n, c_ll) for n in ("sqb", "sqs", "sqh", "skb", "sks", "skh", "svb", "svs", "svh",
                                       "sob", "sos", "soh", "smb", "smh", "smq")]
                + [("scale", ctypes.c_float), ("p_drop", ctypes.c_float), ("seed", c_u64),
                   ("offset", c_u64), ("map", c_int), ("ds", c_void_p)])


class MegaArgs(ctypes.Structure):
    """Mirror of ``struct MegaArgs`` (csrc/kernels/decode_mega.hip)."""
    _fields_ = ([("layers", c_void_p)] + [(n, c_int) for n in ("nl", "maxS", "nsplit", "act")]
                + [("eps", ctypes.c_float), ("scale_log2", ctypes.c_float)]
                + [(n, c_void_p) for n in ("resid", "rbuf", "qn", "kvn", "part", "h", "bar", "err",
                                        "pos", "trace")] + [("late_dma", c_int), ("loader", c_int)]
                + [("rot", c_int), ("neox", c_int), ("log2_base", ctypes.c_float), ("w8", c_int),
                   ("nb", c_int), ("mm", c_int)])


_SIGS["piamd_decode_mega"] = [ctypes.POINTER(MegaArgs), c_int, c_int, c_int, c_int, c_int, c_void_p]
_SIGS["piamd_decode_mega_shape_supported"] = [c_int] * 7
_SIGS["piamd_decode_mega_batch_supported"] = [c_int] * 8
_SIGS["piamd_decode_mega_variant_supported"] = [c_int] * 9


class HeadArgs(ctypes.Structure):
    """Mirror of ``struct HeadArgs`` (csrc/kernels/decode_mega.hip)."""
    _fields_ = ([(n, c_void_p) for n in ("y", "g", "b")] + [("eps", ctypes.c_float), ("V", c_int)]
                + [(n, c_void_p) for n in ("w", "best", "cnt", "out", "done")]
                + [("eos", ctypes.c_longlong), ("pad", ctypes.c_longlong)]
                + [(n, c_void_p) for n in ("pos", "tok", "wemb", "pemb")]
                + [("P", c_int), ("resid", c_void_p)])


_SIGS["piamd_decode_head_greedy"] = [ctypes.POINTER(HeadArgs), c_int, c_void_p]
_SIGS["piamd_decode_mega_supported"] = []
_SIGS["piamd_fa_fwd"] = [ctypes.POINTER(FaArgs), c_int, c_void_p]
_SIGS["piamd_fa_bwd"] = [ctypes.POINTER(FaArgs), c_int, c_void_p]
_SIGS["piamd_layernorm_bwd_ws"] = [c_int, c_int]


def lib_path() -> str:
    # PIAMD_KERNEL_LIB: load another build of the kernel library (A/B timing of a kernel edit)
    return os.environ.get("PIAMD_KERNEL_LIB") or _build.KERNEL_LIB


def _load():
    global _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(
                f"paddle_infer_amd HIP kernel library not built ({path}); run "
                "`python -m paddle_infer_amd._build` (or __graft_entry__.build()).")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _LIB = lib
        return _LIB


def lib():
    return _LIB if _LIB is not None else _load()


def available() -> bool:
    try:
        lib()
        return True
    except (RuntimeError, OSError):
        return False


def has(name: str) -> bool:
    return hasattr(lib(), name)


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def call(name: str, *args) -> None:
    fn = getattr(lib(), name)
    err = fn(*args)
    if err != 0:
        raise RuntimeError(f"{name} failed with hipError {err}")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def dtype_code(t: torch.Tensor, fp16: bool = False) -> int:
    """Kernel dtype code: 0 = f32, 1 = bf16, 2 = fp16 (only for kernels built for it: ``fp16=True``)."""
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    if fp16 and t.dtype == torch.float16:
        return 2
    raise TypeError(f"unsupported dtype {t.dtype} for this HIP kernel "
                    f"({'bf16/fp16/f32' if fp16 else 'bf16/f32'} only)")


# GPU ops that had to leave the HIP path: (op, reason) -> count. Each (op, reason) warns once;
# tests assert this stays empty on the shapes/dtypes the kernels claim.
FALLBACKS: dict = {}


def fallback(op: str, reason: str) -> None:
    """Record (and warn once about) a GPU op that runs its PyTorch reference instead of HIP."""
    key = (op, reason)
    if key not in FALLBACKS:
        import warnings
        warnings.warn(f"paddle_infer_amd: {op} runs the PyTorch reference on GPU ({reason})",
                      RuntimeWarning, stacklevel=3)
    FALLBACKS[key] = FALLBACKS.get(key, 0) + 1


def main_grad(p):
    """The flat-buffer gradient view of a parameter (set by the training engine), else None."""
    return None if p is None else getattr(p, "main_grad", None)


def fire(p):
    """Signal the engine that ``p``'s gradient is complete (bucketed collective trigger)."""
    hook = getattr(p, "_grad_ready", None)
    if hook is not None:
        hook(p)


_SIGS["piamd_nan_inf_check"] = [c_int, c_void_p, c_ll, c_void_p, c_int, c_void_p]
# a, lda, trans_a, b, ldb, trans_b, c, ldc, c_f32, accumulate, M, N, K, epi, act, bias, aux, ldaux,
# ksplit, ws, f16, batch, sa, sb, sc, stream
_SIGS["piamd_agemm"] = [c_void_p, c_ll, c_int, c_void_p, c_ll, c_int, c_void_p, c_ll, c_int, c_int,
                        c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_ll, c_int, c_void_p,
                        c_int, c_int, c_ll, c_ll, c_ll, c_void_p]
_SIGS["piamd_agemm2"] = _SIGS["piamd_agemm"][:-1] + [c_void_p, c_void_p]  # ..., colsum, stream
_SIGS["piamd_colsum_parts"] = [c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]
_SIGS["piamd_agemm_load"] = [ctypes.c_char_p]
# f16, a, lda, b, ldb, c, ldc, c_f32, M, N, K, mb, nb, wn, depth, ks, alpha, bias, act, resid, ldr,
# ws, cnt, stream
_SIGS["piamd_small_gemm"] = [c_int, c_void_p, c_ll, c_void_p, c_ll, c_void_p, c_ll, c_int, c_int,
                             c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p,
                             c_int, c_void_p, c_ll, c_void_p, c_void_p, c_void_p]
# ... + ln_c1, ln_b2 (f32 [N] or null), ln_eps, ln_stats (f32 [M][2] out or null), rln_stats
# (f32 [M][2] or null), rln_g, rln_b (16-bit [N]: LayerNorm of a raw residual), stream
_SIGS["piamd_small_gemm_ln"] = _SIGS["piamd_small_gemm"][:-1] + [c_void_p, c_void_p, c_float, c_void_p,
                                                                 c_void_p, c_void_p, c_void_p, c_void_p]
_SIGS["piamd_agemm_loaded"] = []
_SIGS["piamd_fa_asm_load"] = [ctypes.c_char_p]
_SIGS["piamd_viterbi_decode"] = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
_SIGS["piamd_fa_asm_loaded"] = []
_SIGS["piamd_fa_asm_enable"] = [ctypes.c_int]
_SIGS["piamd_fa_asm_applies"] = [ctypes.c_void_p]
_SIGS["piamd_fa_fwd_nw"] = [ctypes.c_int]
_SIGS["piamd_transpose_bf16"] = [c_void_p, c_void_p, c_int, c_int, c_void_p]
# src, ld, dst, R, C, Rp, Cp, lo_mask, axis, stream
_SIGS["piamd_split3_f32"] = [c_void_p, c_ll, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p]
_SIGS["piamd_moe_gemm"] = [c_void_p, c_ll, c_void_p, c_ll, c_ll,
                                c_int, c_void_p, c_int, c_int, c_void_p,
                                c_ll, c_int, c_int, c_int, c_int,
                                c_int, c_void_p, c_void_p, c_ll, c_void_p]
_SIGS["piamd_moe_wgrad"] = [c_void_p, c_ll, c_void_p, c_ll, c_void_p,
                                 c_int, c_void_p, c_ll, c_int, c_int,
                                 c_int, c_int, c_void_p]
_SIGS["piamd_wo_moe_gemm"] = [c_int, c_void_p, c_ll, c_void_p, c_ll,
                                   c_void_p, c_void_p, c_void_p, c_int,
                                   c_int, c_void_p, c_ll, c_int, c_int,
                                   c_int, c_void_p]
# ids, w, start, vlocal, p, pos, S, out, T, H, stream
_SIGS["piamd_embedding_fwd"] = [c_void_p, c_void_p, c_ll, c_int, c_void_p, c_void_p, c_int,
                                c_void_p, c_ll, c_int, c_void_p]
# sorted, order, dy, dw, dw_f32, start, vlocal, T, H, accumulate, stream
_SIGS["piamd_embedding_bwd"] = [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_ll, c_int, c_ll,
                                c_int, c_int, c_void_p]
_SIGS["piamd_pos_embedding_bwd"] = [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                    c_void_p]
# logits, bf16, cum, seq_lens, stop, end_ids, step_ids, last_cache, last_offs, bs, beam, V,
# max_seq_len, max_dec_len, fuse, early, penalty, P, part, ids, cum_out, cache, offs, parent,
# stop_out, sl_out, st_out, stream
_SIGS["piamd_argmax_rows"] = [c_void_p, c_ll, c_int, c_int, c_int, c_void_p, c_void_p]
_SIGS["piamd_beam_search_softmax"] = ([c_void_p, c_int] + [c_void_p] * 7 + [c_int] * 7
                                      + [c_float, c_int] + [c_void_p] * 10)
# x, ldx, wq, ldw, xs, xs_const, ws, bias, y, ldy, M, N, K, act, stream
_SIGS["piamd_gemm_i8"] = [c_void_p, c_ll, c_void_p, c_ll, c_void_p, c_float, c_void_p, c_void_p,
                          c_void_p, c_ll, c_int, c_int, c_int, c_int, c_void_p]
_SIGS["piamd_quant_rows"] = [c_void_p, c_ll, c_void_p, c_ll, c_void_p, c_float, c_int, c_int,
                             c_void_p]
# x, w_ohwi, zero, y, N, H, W, C, OH, OW, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w, Kout, act,
# bias, tile_n, ksplit, ws, f16, stream
_SIGS["piamd_conv2d_fwd"] = [c_void_p] * 4 + [c_int] * 16 + [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]
# ... flags, stats (f32 [3][Kout][ceil(M/256)] per-tile BN statistics, nullable), stream
_SIGS["piamd_conv2d_fwd2"] = ([c_void_p] * 4 + [c_int] * 16
                              + [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p])
# ... stats, dst_h, dst_w, rs_h, rs_w, ph, pw (phase write into a larger output), stream
_SIGS["piamd_conv2d_fwd3"] = ([c_void_p] * 4 + [c_int] * 16
                              + [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p] + [c_int] * 6 + [c_void_p])
# dtype, nhwc, x, res, y, N, C, S, gamma, beta, run_mean, run_var, mean, rstd, momentum, eps,
# training, act, ws, stream
_SIGS["piamd_bn_fwd"] = ([c_int, c_int] + [c_void_p] * 3 + [c_int] * 3 + [c_void_p] * 6
                         + [c_float, c_float, c_int, c_int, c_void_p, c_void_p])
# dtype, nhwc, dy, y, x, dx, dres, N, C, S, gamma, mean, rstd, dgamma, dbeta, training, act, ws, stream
_SIGS["piamd_bn_set_parts"] = [c_ll, c_int]
_SIGS["piamd_maxpool_fwd_nhwc"] = [c_void_p] * 3 + [c_int] * 13 + [c_void_p]
_SIGS["piamd_maxpool_bwd_nhwc"] = [c_void_p] * 3 + [c_int] * 13 + [c_void_p]
# pool_nd.hip: dtype, x|dy, y|idx, idx|dx, N, C, I[3], O[3], K[3], S[3], P[3], mode, adaptive,
# exclusive, divisor, stream
_SIGS["piamd_pool_nd_fwd"] = ([c_int] + [c_void_p] * 3 + [c_int] * 2 + [ctypes.POINTER(c_int)] * 5
                              + [c_int] * 4 + [c_void_p])
_SIGS["piamd_pool_nd_bwd"] = _SIGS["piamd_pool_nd_fwd"]
# groupnorm.hip: fwd (dtype, x, y, gamma, beta, mean, rstd, ws, N, C, HW, G, eps, stream),
# bwd (dtype, dy, x, gamma, mean, rstd, dx, dgamma, dbeta, ws, N, C, HW, G, stream)
_SIGS["piamd_group_norm_ws"] = [c_int, c_int, c_int]
_SIGS["piamd_group_norm_fwd"] = [c_int] + [c_void_p] * 7 + [c_int, c_int, c_ll, c_int, c_float, c_void_p]
_SIGS["piamd_group_norm_bwd"] = [c_int] + [c_void_p] * 9 + [c_int, c_int, c_ll, c_int, c_void_p]
_SIGS["piamd_group_norm_apply"] = [c_int] + [c_void_p] * 6 + [c_int, c_int, c_ll, c_int, c_void_p]
# embedding.hip, any dtype: fwd (dtype, ids, w, start, vlocal, p, pos, S, out, T, H, stream),
# bwd (dtype, sorted, order, dy, dw_f32, start, vlocal, T, H, accumulate, stream)
_SIGS["piamd_embedding_fwd_dt"] = [c_int, c_void_p, c_void_p, c_ll, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                   c_ll, c_int, c_void_p]
_SIGS["piamd_embedding_bwd_dt"] = [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_ll, c_int,
                                   c_int, c_void_p]
# dtype, x|dy, y|dx(f32), N, C, I[3], O[3], scale[3], mode, align_corners, stream
_SIGS["piamd_interp_fwd"] = ([c_int] + [c_void_p] * 2 + [c_int] * 2 + [ctypes.POINTER(c_int)] * 2
                             + [ctypes.POINTER(c_float), c_int, c_int, c_void_p])
_SIGS["piamd_interp_bwd"] = _SIGS["piamd_interp_fwd"]
# dtype, x, grid, y, N, C, IH, IW, OH, OW, mode, pad, align_corners, stream
_SIGS["piamd_grid_sample_fwd"] = [c_int] + [c_void_p] * 3 + [c_int] * 9 + [c_void_p]
# dtype, dy, x, grid, dx(f32), dgrid(f32), N, C, IH, IW, OH, OW, mode, pad, align_corners, stream
_SIGS["piamd_grid_sample_bwd"] = [c_int] + [c_void_p] * 5 + [c_int] * 9 + [c_void_p]
_SIGS["piamd_bn_bwd"] = ([c_int, c_int] + [c_void_p] * 5 + [c_int] * 3 + [c_void_p] * 5
                         + [c_int, c_int, c_void_p, c_void_p])
_SIGS["piamd_bn_fwd2"] = ([c_int, c_int] + [c_void_p] * 3 + [c_int] * 3 + [c_void_p] * 6
                          + [c_float, c_float, c_int, c_int, c_void_p, c_void_p, c_void_p])
# ... ws, ss, part_t (channel-major conv statistics partials, nullable), P_t, stream
_SIGS["piamd_bn_fwd3"] = ([c_int, c_int] + [c_void_p] * 3 + [c_int] * 3 + [c_void_p] * 6
                          + [c_float, c_float, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p])
_SIGS["piamd_bn_bwd2"] = ([c_int, c_int] + [c_void_p] * 5 + [c_int] * 3 + [c_void_p] * 5
                          + [c_int, c_int, c_void_p, c_void_p, c_void_p])
# SyncBatchNorm: dtype, nhwc, x, N, C, S, ws, out[3][C], stream
_SIGS["piamd_bn_local_stats"] = [c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]
# dtype, nhwc, dy, y, x, N, C, S, mean, rstd, act, ws, ss, out[2][C], stream
_SIGS["piamd_bn_bwd_local_sums"] = ([c_int, c_int] + [c_void_p] * 3 + [c_int] * 3 + [c_void_p] * 2
                                    + [c_int, c_void_p, c_void_p, c_void_p, c_void_p])
# dtype, nhwc, dy, y, x, dx, dres, N, C, S, gamma, mean, rstd, act, sums, Mtot, ws, ss, stream
_SIGS["piamd_bn_bwd_apply_sums"] = ([c_int, c_int] + [c_void_p] * 5 + [c_int] * 3 + [c_void_p] * 3
                                    + [c_int, c_void_p, c_float, c_void_p, c_void_p, c_void_p])
# in, w, bias, out, N, H, W, Cin, OH, OW, Cout, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w,
# cin_g, cout_g, transposed, dtype, stream
_SIGS["piamd_dconv2d"] = [c_void_p] * 4 + [c_int] * 19 + [c_void_p]
# x, dy, d, ws, parts, N, H, W, Cin, OH, OW, Cout, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w,
# cin_g, cout_g, dtype, stream
_SIGS["piamd_dconv2d_wgrad"] = [c_void_p] * 4 + [c_int] * 19 + [c_void_p]
_SIGS["piamd_dconv2d_wgrad_parts"] = [c_int] * 18
# x, dy, zero, d, N, H, W, C, OH, OW, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w, Kout, tile_n,
# ksplit, ws, accumulate, f16, stream
_SIGS["piamd_conv2d_wgrad"] = [c_void_p] * 4 + [c_int] * 17 + [c_void_p, c_int, c_int, c_void_p]
# op, meta, fmeta, chunk_off, T, total_chunks, lr, mu, nesterov, beta1, beta2, eps, bc1, bc2_sqrt,
# grad_scale, stream
_SIGS["piamd_multi_tensor_update"] = ([c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float,
                                       c_float, c_int] + [c_float] * 5 + [c_void_p, c_void_p])
# in, out, rows, N, inverse, scale, stream
_SIGS["piamd_fft_c2c"] = [c_void_p, c_void_p, c_ll, c_int, c_int, c_float, c_void_p]
