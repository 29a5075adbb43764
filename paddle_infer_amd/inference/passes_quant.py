"""Load-time passes for quantized (QAT / PTQ-exported) programs.

Reference: `paddle/fluid/framework/ir/delete_weight_dequant_linear_op_pass.cc` (an int8 weight
feeding ``dequantize_linear`` is dequantized once at load) and `delete_quant_dequant_linear_op_pass.cc`.
On the reference's plain GPU path neither pass runs, so every Run dequantizes the int8 weights
again before an fp32 cuBLAS GEMM.

``delete_weight_dequant_linear_op_pass`` here goes one step further on the matmul family: an int8
weight [K, N] with per-output-channel (quant_axis 1) or per-tensor scales that feeds ``matmul_v2`` /
``matmul`` / ``mul`` / ``fc`` as the right operand becomes ONE ``weight_only_linear`` op on the
int8 weight-only MFMA GEMM (`csrc/kernels/infer.hip` wo_gemm: the int8 values are MFMA-tile packed,
the dequantisation runs in the GEMM main loop, the fc bias / activation in its epilogue) — the
weight stays int8 in memory. Any other consumer (conv2d, transposed matmul, per-K-row scales) gets
the dequantized float weight as a new persistable parameter (constant folding).
"""
from __future__ import annotations

import torch

from .passes import Graph, _new, _out, _pop, _typed

_MM = ("matmul_v2", "matmul", "mul", "fc")


def _int_grid(w):
    """True when the weight holds integer grid values (int8 storage or integral floats)."""
    if not w.is_floating_point():
        return True
    return bool(torch.equal(w, torch.round(w)))


def _weight_slot(op):
    return "W" if op.type == "fc" else "Y"


def _mm_ok(op, name):
    """``op`` uses ``name`` as a plain [K, N] right operand (no transposes / alpha)."""
    if op.type not in _MM or _pop(op, _weight_slot(op)) != name:
        return False
    a = op.attrs
    if op.type == "matmul_v2":
        return not a.get("trans_x", False) and not a.get("trans_y", False)
    if op.type == "matmul":
        return (not a.get("transpose_X", False) and not a.get("transpose_Y", False)
                and float(a.get("alpha", 1.0)) == 1.0)
    if op.type == "mul":
        return int(a.get("y_num_col_dims", 1)) == 1
    return True


def delete_weight_dequant_linear_op_pass(g: Graph):
    n = 0
    for op in list(_typed(g.ops)):
        if op.type != "dequantize_linear":
            continue
        wn, sn = _pop(op, "X"), _pop(op, "Scale")
        out = _out(op, "Y")
        if not (g.is_param(wn) and g.is_param(sn)) or out in g.keep:
            continue
        w = g.param(wn)
        scale = g.param(sn).float().reshape(-1)
        bits = int(op.attrs.get("bit_length", 8))
        axis = int(op.attrs.get("quant_axis", 0))
        rng = float(2 ** (bits - 1) - 1)
        cons = g.consumers(out)
        mm = (len(cons) == 1 and _mm_ok(cons[0], out) and w.dim() == 2 and bits == 8 and _int_grid(w)
              and (axis == 1 or scale.numel() == 1))
        K, N = (w.shape if w.dim() == 2 else (0, 0))
        rep = _wo_rewrite(g, cons[0], wn, w, scale, rng, N) if (mm and N % 32 == 0 and K % 64 == 0) else None
        if rep is not None:
            g.replace([op, cons[0]], rep)
        else:
            wf = w.float()
            y = wf * (scale.reshape(()) if (axis < 0 or scale.numel() == 1) else
                      scale.reshape([-1 if d == axis else 1 for d in range(w.dim())])) / rng
            fold = wn + "@dequant"
            g.program.params[fold] = y.contiguous()
            g.ops.remove(op)
            for o in g.ops:
                if o.paddle_inputs:
                    for k, v in o.paddle_inputs.items():
                        o.paddle_inputs[k] = [fold if x == out else x for x in v]
            g.program._version += 1
        n += 1
    return n


def _wo_rewrite(g, c, wn, w, scale, rng, N):
    """The weight_only_linear op replacing consumer ``c`` (None: keep the float fold)."""
    from ..ops.inference import _pack
    xname = _pop(c, "Input") if c.type == "fc" else _pop(c, "X")
    xs = _shape_of(g, xname)
    attrs = {"weight_dtype": "int8", "act_method": "none"}
    ins = {"x": [xname]}
    if c.type == "fc":
        act = c.attrs.get("activation_type", "") or ""
        if act not in ("", "relu", "gelu", "silu", "swish"):
            return None
        if xs and int(c.attrs.get("in_num_col_dims", 1)) != len(xs) - 1:
            return None
        attrs["act_method"] = act or "none"
        if c.paddle_inputs.get("Bias"):
            ins["bias"] = [_pop(c, "Bias")]
    elif c.type == "mul" and xs and int(c.attrs.get("x_num_col_dims", 1)) != len(xs) - 1:
        return None
    q = w.to(torch.float32).round().clamp(-128, 127).to(torch.int8)  # [K, N]
    s = (scale.expand(N) if scale.numel() == 1 else scale) / rng
    pw, ps = wn + "@wo_int8", wn + "@wo_scale"
    g.program.params[pw] = _pack(q.t().contiguous(), 8)
    g.program.params[ps] = s.contiguous().float()
    ins["weight"], ins["weight_scale"] = [pw], [ps]
    return _new(g.block, "weight_only_linear", ins, {"out": [_out(c)]}, attrs)


def _shape_of(g, name):
    v = g.block.vars.get(name) if hasattr(g.block, "vars") else None
    shp = getattr(v, "shape", None)
    return list(shp) if shp is not None else []


QUANT_PASSES = {"delete_weight_dequant_linear_op_pass": delete_weight_dequant_linear_op_pass}
