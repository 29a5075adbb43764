"""Import of weight-only checkpoints quantized by the reference (CUTLASS sm80 byte order).

The reference's ``weight_quantize`` does not store the int8 / int4 weight row-major: for its
CUTLASS mixed-input GEMM it permutes the bytes (reference
`phi/kernels/impl/weight_quantize_kernel_gpu_impl.h:25` ``weight_permute_kernel_wint8`` for int8,
`phi/kernels/fusion/cutlass/cutlass_kernels/cutlass_preprocessors.cu`
``preprocess_weights_for_mixed_gemm`` — row permutation for the ldmatrix B fragments, sub-byte
transpose to column-major, 64-row × 4-column tile interleave, +bias and nibble interleave — for
int4) and stores each value with an unsigned offset (q + 128 / q + 8). This framework's weight-only
kernels read an MI355X MFMA-tile order instead (`ops/inference.py` ``_pack``; `infer.hip`). A
reference ``.pdiparams`` read as-is would therefore compute garbage silently.

Here the reference layouts are reproduced as element-level index maps (``sm80_int8_index`` is the
kernel's own index arithmetic; ``sm80_int4_perm`` composes the four preprocessing steps on element
ids), which gives both directions: :func:`ref_weight_quantize` (what the reference emits — used by
the tests) and :func:`import_ref_weight` (reference bytes → row-major q → MI355X tile order).
:func:`canonical_weight` is what the static weight-only ops call on every weight they receive:
it detects the reference layout from the stored bit patterns (the offset storage turns q = 0 into
the pattern −128 / nibble −8, which this framework's quantizer never emits; and a symmetric
quantization puts most values near 0, which read without the offset pile up at the range ends) unless
``PIAMD_WO_LAYOUT`` = ``mi355x`` / ``sm80`` pins it, and re-packs once per weight (cached).
"""
from __future__ import annotations

import os

import numpy as np
import torch


# ------------------------------------------------------------------------------- index maps
def sm80_int8_index(K: int, N: int) -> np.ndarray:
    """dest[i] for source element i = k·N + n of the row-major int8 [K, N] weight (the reference's
    ``weight_permute_kernel_wint8`` arithmetic, vectorised)."""
    lin = np.arange(K * N, dtype=np.int64)
    k, n = lin // N, lin % N
    km = k % 16
    e1 = km - km // 8 * 8
    e2 = km // 8
    pk = e1 + e2 + (e2 + 1) % 2 * km * 2 // 2 + e1 * e2 + k // 16 * 16
    return pk % 64 + pk // 64 * 128 + 64 * (n % 2) + K * 2 * (n // 2)


def sm80_int4_perm(K: int, N: int) -> np.ndarray:
    """P with out_elem[j] = in_elem[P[j]]: in = row-major [K, N] int4 elements, out = the element
    sequence of the preprocessed buffer (byte b holds elements 2b (low nibble), 2b + 1)."""
    assert K % 64 == 0 and N % 4 == 0, "int4 reference layout needs K % 64 == 0 and N % 4 == 0"
    ids = np.arange(K * N, dtype=np.int64).reshape(K, N)
    # 1. permute_B_rows_for_mixed_gemm (int4: 32-row tiles, ELTS_PER_REG = 8)
    t = np.arange(32)
    read = 8 * ((t % 8) // 2) + t % 2 + 2 * (t // 8)
    rows = np.arange(K) // 32 * 32 + read[np.arange(K) % 32]
    ids = ids[rows]
    # 2. subbyte_transpose: [K, N] row-major → column-major ([N][K])
    cm = ids.T.copy()                                     # cm[n, k]
    # 3. interleave_column_major_tensor: 32-bit words (8 elements along K), 64-row tiles,
    #    4 columns interleaved
    nvr = K // 8                                          # vec rows per column
    words = cm.reshape(N, nvr, 8)
    out_words = np.empty((N // 4, nvr * 4, 8), dtype=np.int64)
    vr = np.arange(nvr)
    base = vr // 8 * 8
    for rc in range(N):
        wc = rc // 4
        wr = 4 * base + 8 * (rc % 4) + vr % 8
        out_words[wc, wr] = words[rc, vr]
    seq = out_words.reshape(-1, 8)
    # 4. add_bias_and_interleave_int4s: nibble d of each 32-bit word ← nibble (2d | 2(d−4)+1)
    src = np.array([0, 2, 4, 6, 1, 3, 5, 7])
    return seq[:, src].reshape(-1)


# --------------------------------------------------------------------------- ref quantize
def ref_weight_quantize(w_kn: torch.Tensor, algo: str = "weight_only_int8"):
    """What the reference's ``weight_quantize`` (sm80) returns for a float weight [K, N]:
    (int8 bytes [N, K] (int8) or [N/2, K] (int4) in the CUTLASS order, scale [N])."""
    w = w_kn.detach().float().cpu()
    K, N = w.shape
    if algo == "weight_only_int8":
        amax = w.abs().amax(0)
        scale = amax / 127.0
        q = torch.round(torch.clamp(w / amax.clamp_min(1e-30) * 127.0, -127, 127)).to(torch.int32)
        dest = torch.from_numpy(sm80_int8_index(K, N))
        out = torch.empty(K * N, dtype=torch.int32)
        out[dest] = (q.reshape(-1) + 128) & 255
        return out.to(torch.uint8).view(torch.int8).reshape(N, K), scale
    assert algo == "weight_only_int4", algo
    scale = w.abs().amax(0) / 8.0
    q = torch.clamp(torch.round(w / scale.clamp_min(1e-30)), -8, 7).to(torch.int64)
    perm = torch.from_numpy(sm80_int4_perm(K, N))
    el = (q.reshape(-1)[perm] + 8) & 15
    el = el.reshape(-1, 2)
    b = (el[:, 0] | (el[:, 1] << 4)).to(torch.uint8)
    return b.view(torch.int8).reshape(N // 2, K), scale


def ref_to_rowmajor(wb: torch.Tensor, K: int, N: int, bits: int) -> torch.Tensor:
    """Reference bytes → row-major int8 q [K, N] (values in the signed range)."""
    raw = wb.detach().cpu().contiguous().view(torch.uint8).reshape(-1).to(torch.int64)
    if bits == 8:
        dest = torch.from_numpy(sm80_int8_index(K, N))
        return (raw[dest] - 128).to(torch.int8).reshape(K, N)
    el = torch.stack([raw & 15, raw >> 4], -1).reshape(-1) - 8
    perm = torch.from_numpy(sm80_int4_perm(K, N))
    q = torch.empty(K * N, dtype=torch.int64)
    q[perm] = el
    return q.to(torch.int8).reshape(K, N)


def import_ref_weight(wb: torch.Tensor, scale: torch.Tensor, algo: str = "weight_only_int8"):
    """Reference-layout weight → this framework's packed MFMA-tile weight (same logical shape,
    same device); the scale's semantics are unchanged (w ≈ q · scale[n])."""
    from ..ops.inference import _pack
    bits = 4 if algo in ("weight_only_int4", "int4") else 8
    N = scale.numel()
    K = wb.shape[-1]
    q = ref_to_rowmajor(wb, K, N, bits)
    packed = _pack(q.t().contiguous(), bits)  # uint8 bytes
    return packed.view(wb.dtype).reshape(wb.shape).to(wb.device)


# ------------------------------------------------------------------------------ detection
def _ext_fraction(wb: torch.Tensor, bits: int, sample: int = 1 << 16) -> float:
    """Fraction of values whose magnitude, read in THIS framework's convention, is ≥ ¾ of the
    range. Ours (symmetric per-channel quantization of a bell-shaped weight): ≪ 5 %; reference
    bytes (offset by +128 / +8): most values sit near the ends."""
    raw = wb.detach().reshape(-1)
    if raw.numel() > sample:
        raw = raw[torch.linspace(0, raw.numel() - 1, sample, device=raw.device).long()]
    u = raw.cpu().view(torch.uint8).to(torch.int64)
    if bits == 8:
        v = torch.where(u >= 128, u - 256, u)
        return float((v.abs() >= 96).float().mean())
    el = torch.cat([u & 15, u >> 4])
    v = torch.where(el >= 8, el - 16, el)
    return float((v.abs() >= 6).float().mean())


def _has_sentinel(wb: torch.Tensor, bits: int) -> bool:
    """This framework's quantizer never emits −128 (int8: clamp ±127) nor the nibble −8 (int4:
    scale = absmax/7); in the reference's offset storage those bit patterns are q = 0, which every
    real weight matrix contains."""
    u = wb.detach().reshape(-1).view(torch.uint8)
    if bits == 8:
        return bool((u == 128).any())
    # int4: a −8 can still be a column's extreme in a re-packed reference q (scale absmax/8), ≈ 1/K
    # of the values; the reference's zeros are far more frequent (≥ 1/16 even for uniform weights)
    n8 = ((u & 15) == 8).sum() + ((u >> 4) == 8).sum()
    return bool(n8.item() > 0.03 * 2 * u.numel())


def is_ref_layout(wb: torch.Tensor, bits: int) -> bool:
    mode = os.environ.get("PIAMD_WO_LAYOUT", "auto")
    if mode == "sm80":
        return True
    if mode == "mi355x":
        return False
    return _has_sentinel(wb, bits) or _ext_fraction(wb, bits) > 0.5


def canonical_weight(wb: torch.Tensor, scale: torch.Tensor, weight_dtype: str = "int8"):
    """The weight in MI355X tile order: reference-layout weights are re-packed once (cached on the
    tensor, invalidated by an in-place reload)."""
    if wb is None or wb.dtype not in (torch.int8, torch.uint8):
        return wb
    bits = 4 if weight_dtype in ("int4", "weight_only_int4") else 8
    key = (wb.data_ptr(), wb._version)
    c = getattr(wb, "_piamd_canon", None)
    if c is not None and c[0] == key:
        return c[1]
    out = import_ref_weight(wb, scale, "weight_only_int4" if bits == 4 else "weight_only_int8") \
        if is_ref_layout(wb, bits) else wb
    try:
        wb._piamd_canon = (key, out)
    except (AttributeError, RuntimeError):
        pass
    return out
