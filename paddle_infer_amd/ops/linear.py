"""Linear with Paddle weight layout ``[in, out]`` and gradient-accumulation fusion.

Parity: ``paddle.nn.functional.linear`` (`python/paddle/nn/functional/common.py`) and
``fused_matmul_bias`` / ``fused_linear`` (`incubate/nn/functional/fused_matmul_bias.py`,
`fluid/operators/fused/fused_gemm_epilogue_op.cu`).

Every GEMM of a bf16 / fp16 linear on the GPU runs on the framework's own kernels
(``ops.gemm.gemm_nt``): the hand-scheduled assembly GEMM (`csrc/asm/gemm_gen.py`) for products with
many rows, the skinny MFMA kernel (`csrc/kernels/gemm_small.hip`) for few rows (inference,
prefill). Forward ``x·Wtᵀ`` with the bias (and activation) in the epilogue, data gradient
``dy·Wᵀ``, and weight gradient ``xᵀ·dy`` accumulated straight into ``main_grad`` (a view into the
framework's flat gradient buffer) with split-K when the tile grid is small — the weight gradient is
never materialised as a separate tensor, and the parameter's ``_grad_ready`` hook (the bucketed
reduce-scatter/all-reduce trigger) fires right after. ``PIAMD_GEMM=blas`` routes the same products
to hipBLASLt (A/B comparisons). fp32 linears (Paddle's default dtype) run the same kernels as
split-bf16 products (`ops.gemm.gemm_nt_f32` / `wgrad_f32`); under AMP O1 an fp32 weight is cast to
the autocast dtype first.

Weight layout for the forward GEMM: on gfx950 hipBLASLt is 12-21 % faster when BOTH operands are
contiguous along the reduction dim (`x @ Wtᵀ` with ``Wt = [out, in]``) than on Paddle's ``x @ W``
(measured on every GPT-1.3B shape, `tools/bench_gemm_layouts.py`, `profiles/gemm_layouts_r1.txt`),
while the input-gradient GEMM ``dy @ Wᵀ`` is fastest on the ``[in, out]`` layout. Training therefore
keeps a bf16 ``[out, in]`` copy of each weight (`transposed`, one LDS-tiled HIP transpose per weight
per optimizer step, refreshed lazily on first use after the weights change) for the forward only.
"""
from __future__ import annotations

import torch


import os

_GEMM_IMPL = [os.environ.get("PIAMD_GEMM", "asm")]


def set_gemm_impl(impl: str) -> None:
    """"asm" (default: the framework's assembly GEMM) or "blas" (hipBLASLt)."""
    assert impl in ("asm", "blas"), impl
    _GEMM_IMPL[0] = impl


def _asm(a, b, trans_a=False, trans_b=False, ksplit=1):
    if _GEMM_IMPL[0] != "asm" or not a.is_cuda:
        return False
    from .gemm import asm_supported
    return asm_supported(a, b, trans_a, trans_b, ksplit)


def _own(*ts):
    from .gemm import own_dtype
    return _GEMM_IMPL[0] == "asm" and own_dtype(*ts)


def _own32(*ts):
    """fp32 CUDA operands on the own GEMMs as split-bf16 products (`ops.gemm.gemm_nt_f32`)."""
    from .gemm import own_f32
    return _GEMM_IMPL[0] == "asm" and own_f32(*ts)


def mm_nt(x2, w_nk, bias=None, act="none"):
    """y[M, N] = act(x2[M, K] · w_nkᵀ + bias), both operands K-contiguous."""
    if _own(x2, w_nk) and (bias is None or bias.dtype == x2.dtype):
        from .gemm import gemm_nt
        return gemm_nt(x2, w_nk, bias=bias, act=act)
    if act != "none":
        from .activation import bias_act
        return bias_act(mm_nt(x2, w_nk), bias, act)
    if bias is not None:
        return torch.addmm(bias, x2, w_nk.t())
    return torch.mm(x2, w_nk.t())


def wgrad_into(out, x2, dy2):
    """out[K, N] += x2[T, K]ᵀ · dy2[T, N] (weight gradient into main_grad; split-K on small grids).
    Token counts off the assembly kernel's 64-multiple take the own kernels on K-contiguous copies."""
    from .gemm import asm_gemm, gemm_nt, pick_ksplit
    if out.dtype == torch.float32 and _own32(x2, dy2):
        from .gemm import wgrad_f32
        wgrad_f32(x2, dy2, out=out)
        return out
    if out.is_contiguous() and out.dtype in (torch.bfloat16, torch.float32, torch.float16) \
            and dy2.is_contiguous() and (out.dtype != torch.float16 or x2.dtype == torch.float16):
        ks = pick_ksplit(out.shape[0], out.shape[1], x2.shape[0])
        if not _asm(x2, dy2, trans_a=True, ksplit=ks):
            ks = 1
        if _asm(x2, dy2, trans_a=True, ksplit=ks) and (out.dtype == torch.float32 or out.dtype == x2.dtype):
            asm_gemm(x2, dy2, trans_a=True, out=out, accumulate=True, ksplit=ks)
            return out
        if _own(x2, dy2):
            out.add_(gemm_nt(x2.t().contiguous(), dy2.t().contiguous(), out_f32=out.dtype == torch.float32))
            return out
    out.addmm_(x2.t(), dy2)
    return out


def _fire(p):
    hook = getattr(p, "_grad_ready", None)
    if hook is not None:
        hook(p)


_PARAM_EPOCH = [0]
TRANSPOSED_MIN_ROWS = 1024  # training: below this the per-step re-transpose is not repaid
# inference weights are transposed once (cached until they change), and hipBLASLt's TN kernels
# beat NN down to small M too: 128-row BERT-Large projections 13.4 -> 10.8 us (N=K=1024),
# 19.5 -> 11.9 us (K=4096) — `tools/bench_small_m_linear.py`, `profiles/small_m_linear_r2.txt`
INFER_TRANSPOSED_MIN_ROWS = 16


def bump_param_epoch():
    """Called by optimizers that write parameters outside autograd's version counter (the flat
    AdamW kernels): invalidates every cached transposed weight."""
    _PARAM_EPOCH[0] += 1


def transposed(w):
    """Cached contiguous ``wᵀ`` (bf16 / fp16 2-D CUDA weights; the HIP transpose moves 16-bit
    words, so it serves both), refreshed when the parameter changed."""
    key = (_PARAM_EPOCH[0], w._version)
    c = getattr(w, "_piamd_t", None)
    if c is not None and c[0] == key:
        return c[1]
    R, C = w.shape
    buf = c[1] if c is not None else torch.empty((C, R), dtype=w.dtype, device=w.device)
    buf._piamd_weight = True            # ops.gemm may cache a padded image of it ...
    buf.__dict__.pop("_piamd_pad", None)  # ... which this rewrite (no version bump) invalidates
    if R % 8 == 0 and C % 8 == 0:
        from . import _lib
        _lib.call("piamd_transpose_bf16", w.data_ptr(), buf.data_ptr(), R, C, _lib.stream())
    else:
        buf.copy_(w.detach().t())
    w._piamd_t = (key, buf)
    return buf


def _use_transposed(x2, w, min_rows=None):
    min_rows = TRANSPOSED_MIN_ROWS if min_rows is None else min_rows
    return (x2.is_cuda and w.dim() == 2 and w.dtype in (torch.bfloat16, torch.float16)
            and x2.dtype == w.dtype and x2.shape[0] >= min_rows and w.is_contiguous()
            and not getattr(w, "_piamd_no_t", False))


class _LinearFn(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")  # backward replays the forward's autocast state
    def forward(ctx, x, w, b):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if _use_transposed(x2, w) or (_own(x2, w) and w.dim() == 2 and w.is_contiguous()):
            y = mm_nt(x2, transposed(w), b)
        elif w.dim() == 2 and _own32(x2, w) and (b is None or b.dtype == torch.float32):
            from .gemm import gemm_nt_f32, split_nk
            y = gemm_nt_f32(x2, bias=b, b3=split_nk(w, False))
        elif b is not None:
            y = torch.addmm(b, x2, w)
        else:
            y = torch.mm(x2, w)
        ctx.save_for_backward(x2, w)
        ctx.has_b = b is not None
        ctx.bias = b
        ctx.shp = shp
        return y.view(*shp[:-1], w.shape[1])

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[1])
        dx = input_grad(dy2, w).view(ctx.shp) if ctx.needs_input_grad[0] else None
        dw = weight_grad(x2, dy2, w) if ctx.needs_input_grad[1] else None
        db = bias_grad(dy2, ctx.bias) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db


def input_grad(dy2, w):
    """dX = dY · Wᵀ for a [in, out] weight on the own GEMMs (16-bit or split-bf16 fp32)."""
    dy2c = dy2.contiguous() if w.is_contiguous() else dy2
    if _own32(dy2c, w):
        from .gemm import gemm_nt_f32, split_nk
        return gemm_nt_f32(dy2c, b3=split_nk(w, True))
    if w.is_contiguous() and dy2c.dtype == w.dtype:
        return mm_nt(dy2c, w)
    return torch.mm(dy2, w.t())


def weight_grad(x2, dy2, w):
    """dW = Xᵀ · dY: accumulated straight into ``w.main_grad`` (then the grad-ready hook fires,
    None returned) or returned as a tensor."""
    mg = getattr(w, "main_grad", None)
    if mg is not None:
        wgrad_into(mg, x2, dy2.contiguous())
        _fire(w)
        return None
    if _own(x2, dy2):
        dw = torch.zeros_like(w)
        wgrad_into(dw, x2, dy2.contiguous())
        return dw
    if _own32(x2, dy2):
        from .gemm import wgrad_f32
        return wgrad_f32(x2.contiguous(), dy2.contiguous())
    return torch.mm(x2.t(), dy2)


def bias_grad(dy2, b):
    """dB = Σ_rows dY into ``b.main_grad`` (HIP column sums; None returned) or as a tensor."""
    bmg = getattr(b, "main_grad", None)
    if bmg is not None and dy2.is_cuda and dy2.dtype == bmg.dtype:
        colsum_into(dy2, bmg, accumulate=True)
        _fire(b)
        return None
    return dy2.sum(0)





def linear_bias_act(x, weight, bias, act="gelu", weight_out_in=False):
    """Inference ``act(x @ weight + bias)`` as ONE own GEMM with the bias + activation in its
    epilogue on the cached K-contiguous weight (``ops.gemm.gemm_nt``: assembly-GEMM epilogue for
    many rows — bias / bias+ReLU / bias+GELU(tanh); exact-erf GELU and SiLU as GEMM + one HIP
    bias-act pass — and the skinny-kernel epilogue, every activation, for few rows). Parity: the
    reference's ``fused_gemm_epilogue`` / ``fc`` + act (`fused_gemm_epilogue_op.cu:229`). "gelu"
    is the exact erf form (phi GeluFunctor), "gelu_tanh" the tanh approximation. Falls back to
    GEMM + HIP bias-act when autograd is live. ``weight_out_in``: ``weight`` is stored
    ``[out, in]`` (already K-contiguous)."""
    from .activation import bias_act
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    n_out = weight.shape[0] if weight_out_in else weight.shape[1]
    if (bias is not None and bias.dtype == x2.dtype and not torch.is_grad_enabled()
            and _own(x2, weight) and weight.dim() == 2
            and (weight_out_in or weight.is_contiguous())):
        from .gemm import gemm_nt
        wk = weight if weight_out_in else transposed(weight)
        y = gemm_nt(x2, wk, bias=bias, act=act)
        return y.view(*shp[:-1], n_out)
    if weight_out_in:
        return bias_act(torch.nn.functional.linear(x, weight), bias, act)
    return bias_act(linear(x, weight, None), bias, act)


def colsum_into(x2, out, accumulate=True):
    """out[N] (+)= Σ_rows x2[rows, N] via the HIP column-sum kernel (bias gradients)."""
    from . import _lib
    rows, N = x2.shape
    G = max(1, min(256, rows // 16))
    part = torch.empty((G, N), device=x2.device, dtype=torch.float32)
    _lib.call("piamd_colsum", _lib.dtype_code(x2, fp16=True), x2.data_ptr(), out.data_ptr(), part.data_ptr(),
              G, rows, N, int(accumulate), _lib.stream())


def _recordable(fn):
    from ..static.framework import recordable
    return recordable("linear")(fn)


@_recordable
def linear(x, weight, bias=None):
    """y = x @ weight (+ bias); weight is ``[in_features, out_features]``. Under CUDA autocast an
    fp32 weight is cast to the autocast dtype here (differentiably: its gradient flows back to the
    fp32 parameter), so the product runs on the own 16-bit GEMMs instead of the library's
    mixed-dtype path (e.g. the classifier of an AMP-trained ResNet / MobileNet)."""
    if (x.is_cuda and weight.dtype == torch.float32 and torch.is_autocast_enabled("cuda")
            and getattr(weight, "main_grad", None) is None):  # main_grad weights keep the fused path
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return linear(x.to(dt), weight.to(dt), bias.to(dt) if bias is not None else None)
    if torch.is_grad_enabled() and (weight.requires_grad or getattr(weight, "main_grad", None) is not None):
        return _LinearFn.apply(x, weight, bias)
    # inference weights: same K-contiguous cached copy + bias-in-epilogue GEMM as training
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if _own(x2, weight) and weight.dim() == 2 and weight.is_contiguous():
        ok_b = bias is None or bias.dtype == x2.dtype
        y = mm_nt(x2, transposed(weight), bias if ok_b else None)
        if not ok_b:
            y = y + bias
        return y.view(*shp[:-1], weight.shape[1])
    if weight.dim() == 2 and _own32(x2, weight) and (bias is None or bias.dtype == torch.float32):
        from .gemm import gemm_nt_f32, split_nk
        return gemm_nt_f32(x2, bias=bias, b3=split_nk(weight, False)).view(*shp[:-1], weight.shape[1])
    if not _use_transposed(x2, weight, INFER_TRANSPOSED_MIN_ROWS):
        if bias is not None and bias.dtype == x2.dtype and x2.dim() == 2:
            return torch.addmm(bias, x2, weight).view(*shp[:-1], weight.shape[1])
        y = torch.matmul(x, weight)
        return y + bias if bias is not None else y
    wf = transposed(weight).t()
    y = torch.addmm(bias, x2, wf) if bias is not None and bias.dtype == x2.dtype else torch.mm(x2, wf)
    if bias is not None and bias.dtype != x2.dtype:
        y = y + bias
    return y.view(*shp[:-1], weight.shape[1])


# FFN1 bias gradient from the FFN2 data-gradient GEMM's epilogue (asm *cs kernels); PIAMD_FUSED_DB1=0
# restores the separate column-sum pass (A/B)
FUSED_DB1 = [os.environ.get("PIAMD_FUSED_DB1", "1") != "0"]


class _FusedMLPFn(torch.autograd.Function):
    """``m = act(x·W1 + b1)·W2`` with the elementwise work inside the GEMM epilogues (reference
    ``fused_feedforward`` / ``FusedFeedForward`` and the cublasLt GELU_AUX / DGELU epilogues of
    `fused_gemm_epilogue_op.cu`):

    * forward — FFN1 GEMM writes ``pre = bf16(x·W1 + b1)`` (saved) AND ``a = act(pre)``;
    * backward — the FFN2 data-gradient GEMM writes ``d_pre = (dm·W2ᵀ) ⊙ act'(pre)`` directly;
      ``db1`` is one column-sum pass over ``d_pre``; weight gradients go straight into
      ``main_grad``. No separate bias+activation kernels in either direction."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, w1, b1, w2, act):
        from .gemm import asm_gemm
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        pre = torch.empty((x2.shape[0], w1.shape[1]), dtype=x2.dtype, device=x2.device)
        a = asm_gemm(x2, transposed(w1), trans_b=True, epi="bias_act", act=act, bias=b1, aux=pre)
        m = mm_nt(a, transposed(w2))
        ctx.save_for_backward(x2, pre, a, w1, b1, w2)
        ctx.act, ctx.shp = act, shp
        return m.view(*shp[:-1], w2.shape[1])

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dm):
        from .gemm import asm_gemm, colsum_parts
        x2, pre, a, w1, b1, w2 = ctx.saved_tensors
        dm2 = dm.reshape(-1, w2.shape[1]).contiguous()
        # db1 = Σ_rows dpre comes out of the same epilogue (per-128-row-band column sums):
        # no separate column-sum pass over the [T, F] data gradient
        bmg = getattr(b1, "main_grad", None) if ctx.needs_input_grad[2] else None
        cs = None
        if ctx.needs_input_grad[2] and FUSED_DB1[0]:
            cs = torch.empty(((dm2.shape[0] + 127) // 128, w2.shape[0]), dtype=torch.float32,
                             device=dm2.device)
        dpre = asm_gemm(dm2, w2, trans_b=True, epi="dact", act=ctx.act, aux=pre, colsum=cs)
        dw1 = db1 = dw2 = None
        if ctx.needs_input_grad[3]:
            mg = getattr(w2, "main_grad", None)
            if mg is not None:
                wgrad_into(mg, a, dm2)
                _fire(w2)
            else:
                dw2 = wgrad_into(torch.zeros_like(w2), a, dm2)
        if ctx.needs_input_grad[2]:
            if cs is not None:
                if bmg is not None:
                    colsum_parts(cs, bmg, accumulate=True)
                    _fire(b1)
                else:
                    db1 = cs.sum(0).to(b1.dtype)
            elif bmg is not None and bmg.dtype == dpre.dtype:
                colsum_into(dpre, bmg, accumulate=True)
                _fire(b1)
            else:
                db1 = dpre.float().sum(0).to(b1.dtype)
        if ctx.needs_input_grad[1]:
            mg = getattr(w1, "main_grad", None)
            if mg is not None:
                wgrad_into(mg, x2, dpre)
                _fire(w1)
            else:
                dw1 = wgrad_into(torch.zeros_like(w1), x2, dpre)
        dx = mm_nt(dpre, w1).view(ctx.shp) if ctx.needs_input_grad[0] else None
        return dx, dw1, db1, dw2, None


def fused_mlp_supported(x, w1, b1, w2, act):
    """The fused path: bf16 CUDA tensors, GELU(tanh)/ReLU, assembly-GEMM shapes (hidden and FFN
    widths multiples of 64), transposable weights."""
    if not (x.is_cuda and _GEMM_IMPL[0] == "asm" and act in ("gelu_tanh", "relu")
            and x.dtype == torch.bfloat16 and w1.dtype == w2.dtype == x.dtype
            and b1 is not None and b1.dtype == x.dtype and w1.dim() == 2 and w2.dim() == 2
            and w1.is_contiguous() and w2.is_contiguous()
            and not getattr(w1, "_piamd_no_t", False) and not getattr(w2, "_piamd_no_t", False)):
        return False
    H, Fd = w1.shape
    T = x.numel() // H
    # the FFN2 data-gradient GEMM reduces over w2's output width: it needs the asm K contract too
    O = w2.shape[1]
    return H % 64 == 0 and Fd % 64 == 0 and w2.shape == (Fd, O) and O % 64 == 0 \
        and T > 0 and H >= 128 and Fd >= 128 and O >= 128


def fused_mlp(x, w1, b1, w2, act="gelu_tanh"):
    """``act(x @ w1 + b1) @ w2`` (weights ``[in, out]``; no output bias)."""
    if fused_mlp_supported(x, w1, b1, w2, act):
        return _FusedMLPFn.apply(x, w1, b1, w2, act)
    from .activation import bias_act
    return linear(bias_act(linear(x, w1), b1, act), w2)
