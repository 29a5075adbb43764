"""Explicit ``<type>_grad`` kernels for the static-graph executor.

Reference: every PHI op with a gradient has its own backward kernel, registered next to the
forward (`paddle/phi/kernels/*_grad_kernel.h`: `matmul_grad_kernel.h`, `elementwise_grad_kernel.h`,
`activation_grad_kernel.h`, `softmax_grad_kernel.h`, `layer_norm_grad_kernel.h`,
`cross_entropy_grad_kernel.h`, `reduce_*_grad_kernel.h`, `embedding_grad_kernel.h` ...), and the
executor runs the `*_grad` OpDesc that `append_backward` emitted with THAT kernel — the backward
never re-traces the forward.

Here a grad op whose type has an entry in ``GRAD_KERNELS`` is computed directly from the slots the
grad OpDesc carries (forward inputs, forward outputs, ``<Out>@GRAD``) — no autograd graph, no
re-run of the forward. Types without an entry keep the executor's VJP path (`executor.py`
`_run_grad_op`), which differentiates the forward op's local graph.

Kernel contract: ``fn(ins, attrs) -> {"X@GRAD": tensor, ...}`` where ``ins[slot]`` is the list of
values of a grad-op input slot (``None`` for an absent / empty gradient) and the result names the
grad-op OUTPUT slots. On the GPU the fused ops route to the framework's HIP kernels (layer norm
backward, softmax-cross-entropy backward, activation backward); the rest are elementwise or
library-GEMM math on the framework's tensors.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

GRAD_KERNELS = {}


def register_grad(*names):
    def deco(fn):
        for n in names:
            GRAD_KERNELS[n] = fn
        return fn
    return deco


def _one(ins, slot):
    v = ins.get(slot)
    return v[0] if v else None


def _sum_to(g, shape):
    """Reduce a broadcast gradient back to `shape` (numpy broadcasting, trailing alignment)."""
    if tuple(g.shape) == tuple(shape):
        return g
    nd = g.dim() - len(shape)
    if nd > 0:
        g = g.sum(dim=tuple(range(nd)))
    dims = tuple(i for i, s in enumerate(shape) if s == 1 and g.shape[i] != 1)
    if dims:
        g = g.sum(dim=dims, keepdim=True)
    return g.reshape(shape)


def _y_view(x, y, axis):
    """Paddle elementwise `axis`: Y's dims align with X's starting at `axis` (-1 = trailing)."""
    if axis is None or axis == -1 or y.dim() == x.dim():
        return y, None
    shape = [1] * x.dim()
    for i, s in enumerate(y.shape):
        shape[axis + i] = s
    return y.reshape(shape), tuple(y.shape)


def _ew_grads(x, y, a, dout, dx_fn, dy_fn):
    yv, yshape = _y_view(x, y, a.get("axis", -1))
    res = {}
    if dx_fn is not None:
        res["X@GRAD"] = _sum_to(dx_fn(x, yv, dout), x.shape).to(x.dtype)
    if dy_fn is not None:
        gy = _sum_to(dy_fn(x, yv, dout), yv.shape)
        res["Y@GRAD"] = (gy.reshape(yshape) if yshape is not None else gy).to(y.dtype)
    return res


@register_grad("elementwise_add_grad")
def _add_grad(ins, a):
    return _ew_grads(_one(ins, "X"), _one(ins, "Y"), a, _one(ins, "Out@GRAD"),
                     lambda x, y, g: g, lambda x, y, g: g)


@register_grad("elementwise_sub_grad")
def _sub_grad(ins, a):
    return _ew_grads(_one(ins, "X"), _one(ins, "Y"), a, _one(ins, "Out@GRAD"),
                     lambda x, y, g: g, lambda x, y, g: -g)


@register_grad("elementwise_mul_grad")
def _mul_ew_grad(ins, a):
    return _ew_grads(_one(ins, "X"), _one(ins, "Y"), a, _one(ins, "Out@GRAD"),
                     lambda x, y, g: g * y, lambda x, y, g: g * x)


@register_grad("elementwise_div_grad")
def _div_grad(ins, a):
    return _ew_grads(_one(ins, "X"), _one(ins, "Y"), a, _one(ins, "Out@GRAD"),
                     lambda x, y, g: g / y, lambda x, y, g: -g * x / (y * y))


@register_grad("elementwise_max_grad")
def _max_grad(ins, a):
    return _ew_grads(_one(ins, "X"), _one(ins, "Y"), a, _one(ins, "Out@GRAD"),
                     lambda x, y, g: g * (x > y).to(g.dtype), lambda x, y, g: g * (x <= y).to(g.dtype))


@register_grad("elementwise_min_grad")
def _min_grad(ins, a):
    return _ew_grads(_one(ins, "X"), _one(ins, "Y"), a, _one(ins, "Out@GRAD"),
                     lambda x, y, g: g * (x < y).to(g.dtype), lambda x, y, g: g * (x >= y).to(g.dtype))


def _mm_grads(x, y, g, tx, ty):
    """matmul_v2 grad (`matmul_grad_kernel_impl.h`): dX = dOut·Yᵀ, dY = Xᵀ·dOut with the
    transposes folded, batch dims reduced where X or Y was broadcast."""
    xv = x.transpose(-1, -2) if tx else x
    yv = y.transpose(-1, -2) if ty else y
    vec_x, vec_y = xv.dim() == 1, yv.dim() == 1
    if vec_x:
        xv = xv.unsqueeze(0)
        g = g.unsqueeze(-2)
    if vec_y:
        yv = yv.unsqueeze(-1)
        g = g.unsqueeze(-1)
    from ..ops.gemm import matmul as _mm  # own GEMMs for bf16 / fp16, transposes as kernel flags
    dxv = _mm(g, yv, False, True)
    dyv = _mm(xv, g, True, False)
    dxv = _sum_to(dxv, xv.shape)
    dyv = _sum_to(dyv, yv.shape)
    if vec_x:
        dxv = dxv.squeeze(0)
    if vec_y:
        dyv = dyv.squeeze(-1)
    dx = dxv.transpose(-1, -2) if tx and dxv.dim() > 1 else dxv
    dy = dyv.transpose(-1, -2) if ty and dyv.dim() > 1 else dyv
    return dx.to(x.dtype), dy.to(y.dtype)


@register_grad("matmul_v2_grad")
def _matmul_v2_grad(ins, a):
    dx, dy = _mm_grads(_one(ins, "X"), _one(ins, "Y"), _one(ins, "Out@GRAD"),
                       bool(a.get("trans_x")), bool(a.get("trans_y")))
    return {"X@GRAD": dx, "Y@GRAD": dy}


@register_grad("matmul_grad")
def _matmul_grad(ins, a):
    g = _one(ins, "Out@GRAD")
    alpha = a.get("alpha", 1.0)
    if alpha not in (None, 1.0):
        g = g * alpha
    dx, dy = _mm_grads(_one(ins, "X"), _one(ins, "Y"), g,
                       bool(a.get("transpose_X")), bool(a.get("transpose_Y")))
    return {"X@GRAD": dx, "Y@GRAD": dy}


@register_grad("mul_grad")
def _mul_grad(ins, a):
    x, y, g = _one(ins, "X"), _one(ins, "Y"), _one(ins, "Out@GRAD")
    xn = a.get("x_num_col_dims", 1)
    x2 = x.reshape(int(np.prod(x.shape[:xn])), -1)
    y2 = y.reshape(x2.shape[1], -1)
    g2 = g.reshape(x2.shape[0], y2.shape[1])
    return {"X@GRAD": (g2 @ y2.t()).reshape(x.shape).to(x.dtype),
            "Y@GRAD": (x2.t() @ g2).reshape(y.shape).to(y.dtype)}


# ---- activations: from Out where the reference grad kernel uses Out (relu, sigmoid, tanh)
@register_grad("relu_grad")
def _relu_grad(ins, a):
    out, g = _one(ins, "Out"), _one(ins, "Out@GRAD")
    return {"X@GRAD": g * (out > 0).to(g.dtype)}


@register_grad("sigmoid_grad")
def _sigmoid_grad(ins, a):
    out, g = _one(ins, "Out"), _one(ins, "Out@GRAD")
    return {"X@GRAD": g * out * (1 - out)}


@register_grad("tanh_grad")
def _tanh_grad(ins, a):
    out, g = _one(ins, "Out"), _one(ins, "Out@GRAD")
    return {"X@GRAD": g * (1 - out * out)}


@register_grad("silu_grad", "swish_grad")
def _silu_grad(ins, a):
    x, g = _one(ins, "X"), _one(ins, "Out@GRAD")
    dx = _hip_act_bwd(x, g, "silu")
    if dx is not None:
        return {"X@GRAD": dx}
    s = torch.sigmoid(x.float())
    return {"X@GRAD": (g.float() * s * (1 + x.float() * (1 - s))).to(x.dtype)}


@register_grad("leaky_relu_grad")
def _leaky_grad(ins, a):
    x, g = _one(ins, "X"), _one(ins, "Out@GRAD")
    return {"X@GRAD": torch.where(x > 0, g, g * a.get("alpha", 0.02))}


def _hip_act_bwd(x, g, act):
    """dX of act(x) through the framework's `piamd_bias_act_bwd` HIP kernel (bf16/fp16, rows of
    a multiple of 8); None when the kernel does not apply."""
    from ..ops import _lib
    from ..ops.activation import ACTS
    N = x.shape[-1] if x.dim() else 1
    if not (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and N % 8 == 0):
        return None
    h = x.contiguous()
    dy = g.to(h.dtype).contiguous()
    dx = torch.empty_like(h)
    _lib.call("piamd_bias_act_bwd", int(h.dtype == torch.float16), ACTS[act], dy.data_ptr(),
              h.data_ptr(), None, dx.data_ptr(), None, None, h.numel() // N, N, 0, _lib.stream())
    return dx


@register_grad("gelu_grad")
def _gelu_grad(ins, a):
    """`gelu_grad_kernel.h`: erf form or the tanh approximation."""
    x, g = _one(ins, "X"), _one(ins, "Out@GRAD")
    approx = bool(a.get("approximate", False))
    dx = _hip_act_bwd(x, g, "gelu_tanh" if approx else "gelu")
    if dx is not None:
        return {"X@GRAD": dx}
    xf, gf = x.float(), g.float()
    if approx:
        k = math.sqrt(2.0 / math.pi)
        u = k * (xf + 0.044715 * xf ** 3)
        t = torch.tanh(u)
        d = 0.5 * (1 + t) + 0.5 * xf * (1 - t * t) * k * (1 + 3 * 0.044715 * xf * xf)
    else:
        d = 0.5 * (1 + torch.erf(xf / math.sqrt(2.0))) + xf * torch.exp(-0.5 * xf * xf) / math.sqrt(2 * math.pi)
    return {"X@GRAD": (gf * d).to(x.dtype)}


@register_grad("softmax_grad")
def _softmax_grad(ins, a):
    """`softmax_grad_kernel.h`: dX = Out ∘ (dOut − Σ dOut∘Out)."""
    out, g = _one(ins, "Out"), _one(ins, "Out@GRAD")
    axis = a.get("axis", -1)
    of, gf = out.float(), g.float()
    return {"X@GRAD": (of * (gf - (gf * of).sum(axis, keepdim=True))).to(out.dtype)}


@register_grad("layer_norm_grad")
def _layer_norm_grad(ins, a):
    """`layer_norm_grad_kernel.h`: statistics recomputed from X over the normalised dims."""
    x, g = _one(ins, "X"), _one(ins, "Y@GRAD")
    scale, bias = _one(ins, "Scale"), _one(ins, "Bias")
    bna = a.get("begin_norm_axis", x.dim() - 1)
    eps = a.get("epsilon", 1e-5)
    rows = int(np.prod(x.shape[:bna]))
    x2 = x.reshape(rows, -1).float()
    g2 = g.reshape(rows, -1).float()
    mu = x2.mean(1, keepdim=True)
    rstd = torch.rsqrt(x2.var(1, unbiased=False, keepdim=True) + eps)
    xh = (x2 - mu) * rstd
    w = scale.reshape(1, -1).float() if scale is not None else None
    gw = g2 * w if w is not None else g2
    n = x2.shape[1]
    dx = rstd * (gw - gw.mean(1, keepdim=True) - xh * (gw * xh).mean(1, keepdim=True))
    res = {"X@GRAD": dx.reshape(x.shape).to(x.dtype)}
    if scale is not None:
        res["Scale@GRAD"] = (g2 * xh).sum(0).reshape(scale.shape).to(scale.dtype)
    if bias is not None:
        res["Bias@GRAD"] = g2.sum(0).reshape(bias.shape).to(bias.dtype)
    del n
    return res


@register_grad("softmax_with_cross_entropy_grad")
def _swce_grad(ins, a):
    """`cross_entropy_grad_kernel.h` (hard labels): dLogits = (Softmax − onehot(Label)) ∘ dLoss,
    zero on ignore_index rows; soft labels: Softmax·ΣLabel − Label."""
    sm, lab, g = _one(ins, "Softmax"), _one(ins, "Label"), _one(ins, "Loss@GRAD")
    V = sm.shape[-1]
    s2 = sm.reshape(-1, V).float()
    g2 = g.reshape(-1, 1).float()
    if a.get("soft_label", False):
        l2 = lab.reshape(-1, V).float()
        d = (s2 * l2.sum(1, keepdim=True) - l2) * g2
    else:
        l1 = lab.reshape(-1).long()
        ign = a.get("ignore_index", -100)
        valid = (l1 != ign)
        d = s2.clone()
        idx = torch.nonzero(valid).squeeze(1)
        d[idx, l1[idx]] -= 1.0
        d = d * (g2 * valid.unsqueeze(1).float())
    return {"Logits@GRAD": d.reshape(sm.shape).to(sm.dtype)}


def _reduce_dims(x, a):
    if a.get("reduce_all", False) or not list(a.get("dim", []) or []):
        return list(range(x.dim()))
    return sorted(d % x.dim() for d in a.get("dim"))


def _expand_back(g, x, dims, keep):
    if not keep:
        for d in dims:
            g = g.unsqueeze(d) if g.dim() < x.dim() else g
    return g.reshape([1 if i in dims else s for i, s in enumerate(x.shape)]).expand(x.shape)


@register_grad("reduce_sum_grad")
def _rsum_grad(ins, a):
    x, g = _one(ins, "X"), _one(ins, "Out@GRAD")
    dims = _reduce_dims(x, a)
    return {"X@GRAD": _expand_back(g, x, dims, a.get("keep_dim", False)).to(x.dtype).contiguous()}


@register_grad("reduce_mean_grad")
def _rmean_grad(ins, a):
    x, g = _one(ins, "X"), _one(ins, "Out@GRAD")
    dims = _reduce_dims(x, a)
    n = int(np.prod([x.shape[d] for d in dims])) if dims else 1
    return {"X@GRAD": (_expand_back(g, x, dims, a.get("keep_dim", False)) / n).to(x.dtype).contiguous()}


@register_grad("mean_grad")
def _mean_grad(ins, a):
    x, g = _one(ins, "X"), _one(ins, "Out@GRAD")
    return {"X@GRAD": (g.reshape([]) / x.numel()).expand(x.shape).to(x.dtype).contiguous()}


@register_grad("scale_grad")
def _scale_grad(ins, a):
    return {"X@GRAD": _one(ins, "Out@GRAD") * a.get("scale", 1.0)}


@register_grad("cast_grad")
def _cast_grad(ins, a):
    return {"X@GRAD": _one(ins, "Out@GRAD").to(_one(ins, "X").dtype)}


@register_grad("reshape2_grad", "reshape_grad", "flatten_contiguous_range_grad", "squeeze2_grad",
               "unsqueeze2_grad")
def _reshape_grad(ins, a):
    return {"X@GRAD": _one(ins, "Out@GRAD").reshape(_one(ins, "X").shape)}


@register_grad("transpose2_grad", "transpose_grad")
def _transpose_grad(ins, a):
    perm = list(a.get("axis"))
    inv = [0] * len(perm)
    for i, p in enumerate(perm):
        inv[p] = i
    return {"X@GRAD": _one(ins, "Out@GRAD").permute(inv).contiguous()}


@register_grad("dropout_grad")
def _dropout_grad(ins, a):
    """The static registry's dropout is the inference form (`downgrade_in_infer` scales by
    1 − p, `upscale_in_train` is identity); its gradient is the same scale."""
    g = _one(ins, "Out@GRAD")
    p = a.get("dropout_prob", 0.5)
    if a.get("dropout_implementation", "downgrade_in_infer") == "downgrade_in_infer":
        return {"X@GRAD": g * (1.0 - p)}
    return {"X@GRAD": g}


@register_grad("lookup_table_v2_grad", "lookup_table_grad")
def _lookup_grad(ins, a):
    """`embedding_grad_kernel.h`: scatter-add of dOut rows into the table (padding row zero)."""
    ids, w, g = _one(ins, "Ids").long(), _one(ins, "W"), _one(ins, "Out@GRAD")
    flat = ids.reshape(-1)
    gw = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
    gw.index_add_(0, flat, g.reshape(flat.numel(), -1).float())
    pad = a.get("padding_idx", -1)
    if pad is not None and pad >= 0:
        gw[pad] = 0
    return {"W@GRAD": gw.to(w.dtype)}


@register_grad("concat_grad")
def _concat_grad(ins, a):
    xs, g = ins.get("X", []), _one(ins, "Out@GRAD")
    axis = a.get("axis", 0)
    axis = axis % g.dim()
    return {"X@GRAD": list(torch.split(g, [x.shape[axis] for x in xs], dim=axis))}


@register_grad("split_grad")
def _split_grad(ins, a):
    gs, x = ins.get("Out@GRAD", []), _one(ins, "X")
    outs = ins.get("Out", [])
    axis = a.get("axis", 0) % x.dim()
    parts = [g if g is not None else torch.zeros_like(o) for g, o in zip(gs, outs)]
    return {"X@GRAD": torch.cat(parts, dim=axis)}


@register_grad("sum_grad")
def _sum_grad(ins, a):
    g = _one(ins, "Out@GRAD")
    return {"X@GRAD": [g for _ in ins.get("X", [])]}
