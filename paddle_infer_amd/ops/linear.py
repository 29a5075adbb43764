"""Linear with Paddle weight layout ``[in, out]`` and gradient-accumulation fusion.

Parity: ``paddle.nn.functional.linear`` (`python/paddle/nn/functional/common.py`) and
``fused_matmul_bias`` / ``fused_linear`` (`incubate/nn/functional/fused_matmul_bias.py`,
`fluid/operators/fused/fused_gemm_epilogue_op.cu`).

Plain GEMMs go to hipBLASLt through ``torch.matmul``/``addmm`` (bias fused as the GEMM epilogue).
When a weight carries a ``main_grad`` buffer (a view into the framework's flat gradient buffer),
the backward accumulates ``xᵀ·dy`` straight into it with ``addmm_`` (β = 1) — the weight gradient is
never materialised as a separate tensor, and the parameter's ``_grad_ready`` hook (the bucketed
reduce-scatter/all-reduce trigger) fires right after.
"""
from __future__ import annotations

import torch


def _fire(p):
    hook = getattr(p, "_grad_ready", None)
    if hook is not None:
        hook(p)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if b is not None:
            y = torch.addmm(b, x2, w)
        else:
            y = torch.mm(x2, w)
        ctx.save_for_backward(x2, w)
        ctx.has_b = b is not None
        ctx.bias = b
        ctx.shp = shp
        return y.view(*shp[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(dy2, w.t()).view(ctx.shp)
        dw = db = None
        mg = getattr(w, "main_grad", None)
        if ctx.needs_input_grad[1]:
            if mg is not None:
                mg.addmm_(x2.t(), dy2)
                _fire(w)
            else:
                dw = torch.mm(x2.t(), dy2)
        if ctx.has_b and ctx.needs_input_grad[2]:
            b = ctx.bias
            bmg = getattr(b, "main_grad", None)
            if bmg is not None and dy2.is_cuda and dy2.dtype == bmg.dtype:
                colsum_into(dy2, bmg, accumulate=True)
                _fire(b)
            else:
                db = dy2.sum(0)
        return dx, dw, db


def colsum_into(x2, out, accumulate=True):
    """out[N] (+)= Σ_rows x2[rows, N] via the HIP column-sum kernel (bias gradients)."""
    from . import _lib
    rows, N = x2.shape
    G = max(1, min(256, rows // 16))
    part = torch.empty((G, N), device=x2.device, dtype=torch.float32)
    _lib.call("piamd_colsum", _lib.dtype_code(x2), x2.data_ptr(), out.data_ptr(), part.data_ptr(),
              G, rows, N, int(accumulate), _lib.stream())


def _recordable(fn):
    from ..static.framework import recordable
    return recordable("linear")(fn)


@_recordable
def linear(x, weight, bias=None):
    """y = x @ weight (+ bias); weight is ``[in_features, out_features]``."""
    if weight.requires_grad or getattr(weight, "main_grad", None) is not None:
        return _LinearFn.apply(x, weight, bias)
    y = torch.matmul(x, weight)
    return y + bias if bias is not None else y
