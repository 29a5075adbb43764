"""Deferred LayerNorm for post-LN encoders at few rows (BERT-style inference at small batches).

A post-LN layer ends every sub-block with ``y = LN(fc(x) + resid)``
(`fused_fc_elementwise_layernorm`, reference `fused/fused_fc_elementwise_layernorm_op.cu:64`) and
``y`` feeds exactly two places: the next GEMM (QKV / FFN1) and the next residual add. At a few
hundred rows the LayerNorm is its own launch (~5.4 µs, 17 % of BERT-Large batch 1). Here the producer skips it
and hands on the RAW rows ``h`` with the LayerNorm attached (:class:`Deferred`):

* the consuming GEMM folds the LayerNorm into its weights (``ops.gemm.ln_fold``: W∘γ, Σ_k, bias +
  W·β) and computes each row's (mean, rstd) on the matrix cores from the raw rows it loads anyway
  (``gemm_small.hip`` LN mode), writing the statistics out;
* the consuming residual epilogue (the next ``fused_fc_elementwise_layernorm``) adds
  (h − mean)·rstd·γ + β with those statistics instead of a materialised ``y``.

So a layer runs 5 launches instead of 7 (QKV, attention, out, FFN1, FFN2). The inference pass
``ln_defer_pass`` marks a producer ``defer_ln`` only when every consumer of its output is one of
these fold-aware ops and the output is not fetched; at run time a producer defers only on the
skinny-GEMM path (≤ ``DEFER_MAX_M`` rows, 16-bit CUDA), and any consumer that cannot fold (e.g. a
large batch routed to the assembly GEMM) materialises ``y`` once through the LayerNorm kernel.
The program's semantics are unchanged (the native engine ignores the attribute).
"""
from __future__ import annotations

import os

import torch

# rows up to which producers defer (BERT-Large fp16: batch 2 (256 rows) 1.957 -> 1.787 ms deferred;
# batch 4 (512 rows) 2.501 -> 2.789 ms, so 512 stays on the LayerNorm kernel; profiles/bert_fp16_r6.txt)
DEFER_MAX_M = int(os.environ.get("PIAMD_LN_DEFER_MAX_M", "256"))
ENABLED = os.environ.get("PIAMD_LN_DEFER", "1") != "0"


class Deferred:
    """LayerNorm (γ, β, eps) owed on a tensor of raw rows; ``stats`` (f32 [M, 2] mean / rstd) once
    a folding GEMM has computed them, ``mat`` the materialised LN output if one was needed."""
    __slots__ = ("gamma", "beta", "eps", "stats", "filled", "mat")

    def __init__(self, gamma, beta, eps, rows, device):
        self.gamma, self.beta, self.eps = gamma, beta, float(eps)
        self.stats = torch.empty((rows, 2), dtype=torch.float32, device=device)
        self.filled = False
        self.mat = None


def of(x):
    return getattr(x, "_piamd_ln", None) if isinstance(x, torch.Tensor) else None


def can_defer(x2, M: int, N: int) -> bool:
    """A producer's [M, N] output computed from ``x2`` may stay raw: 16-bit CUDA rows on the
    skinny path."""
    return (ENABLED and x2.is_cuda and x2.dtype in (torch.bfloat16, torch.float16)
            and M <= DEFER_MAX_M and N % 64 == 0)


def _as(t, dtype):
    """``t`` in ``dtype``, the converted copy cached on ``t`` (LayerNorm parameters may stay f32
    under mixed precision; a stable copy keeps the weight fold cached)."""
    if t.dtype == dtype and t.is_contiguous():
        return t
    key = (t.data_ptr(), t._version, dtype)
    c = getattr(t, "_piamd_as", None)
    if c is not None and c[0] == key:
        return c[1]
    o = t.to(dtype).contiguous()
    if not (t.is_cuda and torch.cuda.is_current_stream_capturing()):
        try:
            t._piamd_as = (key, o)
        except (AttributeError, RuntimeError):
            pass
    return o


def defer(h, gamma, beta, eps):
    """Attach the owed LayerNorm to ``h`` (returned)."""
    rows = h.numel() // h.shape[-1]
    h._piamd_ln = Deferred(_as(gamma.reshape(-1), h.dtype), _as(beta.reshape(-1), h.dtype), eps, rows,
                           h.device)
    return h


def materialize(x):
    """``x`` itself, or LN(x) (computed once) when ``x`` carries a deferred LayerNorm."""
    d = of(x)
    if d is None:
        return x
    if d.mat is None:
        from .. import ops
        d.mat = ops.layer_norm(x, d.gamma, d.beta, d.eps)
    return d.mat


def _fold(wk, d, bias):
    """Cached (W∘γ, c1, b2) of K-contiguous weight ``wk`` [N, K] for deferred LN ``d`` (+ bias),
    keyed by the operands' identities and versions (an in-place reload refreshes it)."""
    from ..ops.gemm import ln_fold
    from ..ops.linear import _PARAM_EPOCH
    key = (_PARAM_EPOCH[0], wk.data_ptr(), wk._version, d.gamma.data_ptr(), d.gamma._version,
           d.beta.data_ptr(), d.beta._version, bias.data_ptr() if bias is not None else 0,
           bias._version if bias is not None else 0)
    cache = getattr(wk, "_piamd_lnfold", None)
    if cache is not None and cache[0] == key:
        return cache[1]
    if wk.is_cuda and torch.cuda.is_current_stream_capturing():
        return None  # a fold built inside a capture would only exist at replay
    f = ln_fold(wk, d.gamma, d.beta, bias)
    try:
        wk._piamd_lnfold = (key, f)
    except (AttributeError, RuntimeError):
        pass
    return f


def linear(x, w, bias, act="none", weight_out_in=False):
    """``act(LN(x)·W + bias)`` for a deferred ``x`` ([..., K]; W [K, N], or [N, K] with
    ``weight_out_in``) on the LN-folding skinny GEMM; the row statistics land in the deferral for
    the residual consumer. None when this call cannot fold (the caller materialises)."""
    from ..ops.gemm import small_gemm, use_small
    from ..ops.linear import transposed
    d = of(x)
    if d is None or x.dtype != w.dtype or w.dim() != 2:
        return None
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    N = w.shape[0] if weight_out_in else w.shape[1]
    if (M > DEFER_MAX_M or not use_small(M, N, K) or K % 64 or N % 4 or not x2.is_contiguous()
            or (bias is not None and bias.numel() != N)):
        return None
    wk = w if weight_out_in else transposed(w)
    f = _fold(wk, d, bias.reshape(-1) if bias is not None else None)
    if f is None:
        return None
    wf, c1, b2 = f
    y = small_gemm(x2, wf, act=act, ln=(c1, b2, d.eps), ln_stats=d.stats)
    d.filled = True
    return y.reshape(*x.shape[:-1], N)


def resid_args(y, M):
    """For a residual ``y``: (tensor to add, resid_ln tuple or None). A deferred ``y`` whose
    statistics a folding GEMM already produced is added raw with its LayerNorm in the epilogue;
    otherwise it is materialised."""
    d = of(y)
    if d is None:
        return y, None
    if d.filled and d.stats.shape[0] == M:
        return y, (d.stats, d.gamma, d.beta)
    return materialize(y), None
