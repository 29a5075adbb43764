"""The rest of the reference GPU pass list (`paddle/fluid/inference/api/paddle_pass_builder.cc`,
GpuPassStrategy) that is not a TensorRT / cuDNN-placement pass:

  is_test_pass                        is_test = True on every op that has the attribute
                                      (`framework/ir/is_test_pass.cc`)
  simplify_with_basic_ops_pass        dropout(is_test) → scale / removed (`simplify_with_basic_ops_pass.cc`)
  constant_folding_pass               ops whose inputs are all persistable → evaluated once, the
                                      result becomes a parameter (`constant_folding_pass.cc`)
  gpu_cpu_map_matmul_v2_to_mul_pass   matmul_v2(X, W 2-D param, no transpose) → mul
  gpu_cpu_map_matmul_v2_to_matmul_pass  remaining matmul_v2 → matmul (transpose_X/Y, alpha 1)
  gpu_cpu_map_matmul_to_mul_pass      matmul(α = 1, no transpose, W 2-D param) → mul
  gpu_cpu_squeeze2_matmul_fuse_pass   squeeze2 [N,C,1,1]→[N,C] + matmul/matmul_v2(W) → mul(x_num_col_dims=1)
  gpu_cpu_reshape2_matmul_fuse_pass   reshape2 [N,C,1,1]→[N,C] + matmul(W) → mul
  gpu_cpu_flatten2_matmul_fuse_pass   flatten2 / flatten_contiguous_range(axis 1) + matmul(W) → mul
  matmul_scale_fuse_pass              matmul_v2(X, W param) + scale(s, bias 0) → matmul_v2(X, s·W)
  conv_elementwise_add_fuse_pass      conv2d + elementwise_add(bias, axis 1) → conv2d(Bias)
  conv_eltwiseadd_bn_fuse_pass        conv2d + elementwise_add(bias) + batch_norm → conv2d(W', b')
  conv_elementwise_add_act_fuse_pass  conv2d + add(bias) + act → conv2d_fusion(activation)
  conv_elementwise_add2_act_fuse_pass conv2d + add(bias) + add(residual) + act → conv2d_fusion(ResidualData)
  transpose_flatten_concat_fuse_pass  N × (transpose2 → flatten2) → concat  ⇒ fusion_transpose_flatten_concat

The matmul→mul maps exist in the reference so the later fc_fuse_pass sees one op form; here they
feed the same fc_fuse_pass (which accepts mul). The conv fusions land on the framework's own conv
kernels (`static/ops_registry.py` conv2d / conv2d_fusion → `ops/conv.py`).
"""
from __future__ import annotations

import numpy as np
import torch

from .passes import Graph, _new, _out, _pop, _typed

_CONV = ("conv2d", "depthwise_conv2d")
_FUSION_ACTS = ("relu", "relu6", "sigmoid", "tanh", "leaky_relu", "swish", "silu", "gelu")


def is_test_pass(g: Graph):
    n = 0
    for op in _typed(g.ops):
        if "is_test" in op.attrs and not op.attrs["is_test"]:
            op.attrs["is_test"] = True
            n += 1
    if n:
        g.program._version += 1
    return n


def simplify_with_basic_ops_pass(g: Graph):
    from .passes import delete_dropout_op_pass
    return delete_dropout_op_pass(g)


_NO_FOLD = {"feed", "fetch", "fill_constant", "uniform_random", "gaussian_random", "randint",
            "assign_value", "c_broadcast", "c_allreduce_sum", "dropout", "while", "conditional_block"}


def constant_folding_pass(g: Graph):
    """Evaluate ops whose every input is a parameter (persistable and loaded) once, at analysis
    time, with the op's registry kernel; the outputs become parameters and the op is removed."""
    from ..static.ops_registry import REGISTRY
    n = 0
    changed = True
    while changed:
        changed = False
        for op in list(_typed(g.ops)):
            if op.type in _NO_FOLD or op.type.endswith("_grad") or op.type not in REGISTRY:
                continue
            names = [x for v in op.paddle_inputs.values() for x in v if x]
            if not names or not all(g.is_param(x) for x in names):
                continue
            outs = [x for v in op.paddle_outputs.values() for x in v if x]
            if not outs or any(o in g.keep for o in outs):
                continue
            ins = {k: [g.param(x) for x in v] for k, v in op.paddle_inputs.items()}
            try:
                with torch.no_grad():
                    res = REGISTRY[op.type](ins, op.attrs)
            except Exception:
                continue
            for slot, onames in op.paddle_outputs.items():
                vals = res.get(slot)
                if vals is None:
                    continue
                vals = vals if isinstance(vals, (list, tuple)) else [vals]
                for o, v in zip(onames, vals):
                    if o and isinstance(v, torch.Tensor):
                        g.program.params[o] = v.detach()
                        var = g.block.vars.get(o)
                        if var is not None:
                            var.persistable = True
            g.ops.remove(op)
            g.program._version += 1
            n += 1
            changed = True
    return n


def _param2d(g, name):
    return name is not None and g.is_param(name) and g.param(name).dim() == 2


def gpu_cpu_map_matmul_v2_to_mul_pass(g: Graph):
    n = 0
    for op in list(_typed(g.ops)):
        if op.type != "matmul_v2" or op.attrs.get("trans_x") or op.attrs.get("trans_y"):
            continue
        y = _pop(op, "Y")
        if not _param2d(g, y):
            continue
        xv = g.block.vars.get(_pop(op, "X"))
        nd = len(xv.declared_shape) if xv is not None and xv.declared_shape else 2
        g.replace([op], _new(g.block, "mul", {"X": [_pop(op, "X")], "Y": [y]}, {"Out": [_out(op)]},
                             {"x_num_col_dims": max(1, nd - 1), "y_num_col_dims": 1}))
        n += 1
    return n


def gpu_cpu_map_matmul_v2_to_matmul_pass(g: Graph):
    n = 0
    for op in list(_typed(g.ops)):
        if op.type != "matmul_v2":
            continue
        g.replace([op], _new(g.block, "matmul", {"X": [_pop(op, "X")], "Y": [_pop(op, "Y")]},
                             {"Out": [_out(op)]},
                             {"transpose_X": bool(op.attrs.get("trans_x")),
                              "transpose_Y": bool(op.attrs.get("trans_y")), "alpha": 1.0}))
        n += 1
    return n


def gpu_cpu_map_matmul_to_mul_pass(g: Graph):
    n = 0
    for op in list(_typed(g.ops)):
        if op.type != "matmul" or op.attrs.get("transpose_X") or op.attrs.get("transpose_Y") \
                or float(op.attrs.get("alpha", 1.0)) != 1.0:
            continue
        y = _pop(op, "Y")
        if not _param2d(g, y):
            continue
        xv = g.block.vars.get(_pop(op, "X"))
        nd = len(xv.declared_shape) if xv is not None and xv.declared_shape else 2
        g.replace([op], _new(g.block, "mul", {"X": [_pop(op, "X")], "Y": [y]}, {"Out": [_out(op)]},
                             {"x_num_col_dims": max(1, nd - 1), "y_num_col_dims": 1}))
        n += 1
    return n


def _shape_then_matmul(g: Graph, first_types, ok):
    """<first>(X) → matmul|matmul_v2(·, W 2-D param, plain) ⇒ mul(X, W, x_num_col_dims=1)."""
    n = 0
    for op in list(_typed(g.ops)):
        if op.type not in first_types or op not in g.ops or not ok(op):
            continue
        out = _out(op)
        cons = g.consumers(out)
        if len(cons) != 1 or not g.single_use(out):
            continue
        mm = cons[0]
        if mm.func is not None or mm.type not in ("matmul", "matmul_v2") or _pop(mm, "X") != out:
            continue
        if mm.attrs.get("trans_x") or mm.attrs.get("trans_y") or mm.attrs.get("transpose_X") \
                or mm.attrs.get("transpose_Y") or float(mm.attrs.get("alpha", 1.0)) != 1.0:
            continue
        y = _pop(mm, "Y")
        if not _param2d(g, y):
            continue
        g.replace([op, mm], _new(g.block, "mul", {"X": [_pop(op, "X")], "Y": [y]}, {"Out": [_out(mm)]},
                                 {"x_num_col_dims": 1, "y_num_col_dims": 1}))
        n += 1
    return n


def _rank(g, name):
    v = g.block.vars.get(name)
    return len(v.declared_shape) if v is not None and v.declared_shape else None


def gpu_cpu_squeeze2_matmul_fuse_pass(g: Graph):
    return _shape_then_matmul(g, ("squeeze2",), lambda op: _rank(g, _pop(op, "X")) == 4
                              and sorted(int(a) % 4 for a in op.attrs.get("axes", [])) == [2, 3])


def gpu_cpu_reshape2_matmul_fuse_pass(g: Graph):
    def ok(op):
        shp = list(op.attrs.get("shape", []))
        return _rank(g, _pop(op, "X")) == 4 and len(shp) == 2 and shp[0] in (0, -1) \
            and not op.paddle_inputs.get("Shape") and not op.paddle_inputs.get("ShapeTensor")
    return _shape_then_matmul(g, ("reshape2",), ok)


def gpu_cpu_flatten2_matmul_fuse_pass(g: Graph):
    def ok(op):
        if op.type == "flatten2":
            return int(op.attrs.get("axis", 1)) == 1
        return int(op.attrs.get("start_axis", 1)) == 1 and int(op.attrs.get("stop_axis", -1)) in (-1, 3) \
            and _rank(g, _pop(op, "X")) in (None, 4, 2, 3)
    return _shape_then_matmul(g, ("flatten2", "flatten_contiguous_range"), ok)


def matmul_scale_fuse_pass(g: Graph):
    n = 0
    for mm in list(_typed(g.ops)):
        if mm.type != "matmul_v2" or mm not in g.ops:
            continue
        y = _pop(mm, "Y")
        if not g.is_param(y):
            continue
        out = _out(mm)
        cons = g.consumers(out)
        if len(cons) != 1 or not g.single_use(out) or cons[0].func is not None or cons[0].type != "scale":
            continue
        sc = cons[0]
        if float(sc.attrs.get("bias", 0.0)) != 0.0 or sc.paddle_inputs.get("ScaleTensor"):
            continue
        s = float(sc.attrs.get("scale", 1.0))
        w = g.param(y)
        wn = f"{y}@scaled{len(g.program.params)}"
        g.program.params[wn] = (w.float() * s).to(w.dtype)
        g.block.create_var(wn, list(w.shape), "float32", persistable=True)
        g.replace([mm, sc], _new(g.block, "matmul_v2", {"X": [_pop(mm, "X")], "Y": [wn]}, {"Out": [_out(sc)]},
                                 dict(mm.attrs)))
        n += 1
    return n


def _conv_bias_add(g, conv):
    """conv's single consumer when it is elementwise_add(conv_out, 1-D bias param, axis 1)."""
    out = _out(conv, "Output")
    cons = g.consumers(out)
    if len(cons) != 1 or not g.single_use(out):
        return None, None
    add = cons[0]
    if add.func is not None or add.type != "elementwise_add" or _pop(add, "X") != out:
        return None, None
    b = _pop(add, "Y")
    if not g.is_param(b) or g.param(b).dim() != 1 or int(add.attrs.get("axis", 1)) not in (1, -1) \
            or g.param(b).shape[0] != g.param(_pop(conv, "Filter")).shape[0]:
        return None, None
    if int(add.attrs.get("axis", 1)) == -1 and (_rank(g, out) or 4) == 4:
        return None, None  # trailing alignment would add over W, not over channels
    return add, b


def _plain_conv(g, op):
    return op.type in _CONV and not op.paddle_inputs.get("Bias") and g.is_param(_pop(op, "Filter")) \
        and op.attrs.get("data_format", "NCHW") in ("NCHW", "AnyLayout")


def conv_elementwise_add_act_fuse_pass(g: Graph):
    n = 0
    for conv in list(_typed(g.ops)):
        if conv not in g.ops or not _plain_conv(g, conv):
            continue
        add, b = _conv_bias_add(g, conv)
        if add is None:
            continue
        a_out = _out(add)
        cons = g.consumers(a_out)
        if len(cons) != 1 or not g.single_use(a_out) or cons[0].func is not None or cons[0].type not in _FUSION_ACTS:
            continue
        act = cons[0]
        attrs = dict(conv.attrs)
        attrs["activation"] = act.type
        ins = dict(conv.paddle_inputs)
        ins["Bias"] = [b]
        g.replace([conv, add, act], _new(g.block, "conv2d_fusion", ins, {"Output": [_out(act)]}, attrs))
        n += 1
    return n


def conv_elementwise_add2_act_fuse_pass(g: Graph):
    n = 0
    for conv in list(_typed(g.ops)):
        if conv not in g.ops or not _plain_conv(g, conv):
            continue
        add, b = _conv_bias_add(g, conv)
        if add is None:
            continue
        a_out = _out(add)
        cons = g.consumers(a_out)
        if len(cons) != 1 or not g.single_use(a_out) or cons[0].func is not None \
                or cons[0].type != "elementwise_add":
            continue
        add2 = cons[0]
        res = _pop(add2, "Y") if _pop(add2, "X") == a_out else _pop(add2, "X")
        if res is None or g.producer(res) is None and not g.is_param(res):
            pass
        r_out = _out(add2)
        cons2 = g.consumers(r_out)
        if len(cons2) != 1 or not g.single_use(r_out) or cons2[0].func is not None or cons2[0].type not in _FUSION_ACTS:
            continue
        act = cons2[0]
        attrs = dict(conv.attrs)
        attrs["activation"] = act.type
        ins = dict(conv.paddle_inputs)
        ins["Bias"] = [b]
        ins["ResidualData"] = [res]
        g.replace([conv, add, add2, act], _new(g.block, "conv2d_fusion", ins, {"Output": [_out(act)]}, attrs))
        n += 1
    return n


def conv_elementwise_add_fuse_pass(g: Graph):
    n = 0
    for conv in list(_typed(g.ops)):
        if conv not in g.ops or not _plain_conv(g, conv):
            continue
        add, b = _conv_bias_add(g, conv)
        if add is None:
            continue
        ins = dict(conv.paddle_inputs)
        ins["Bias"] = [b]
        g.replace([conv, add], _new(g.block, conv.type, ins, {"Output": [_out(add)]}, dict(conv.attrs)))
        n += 1
    return n


def conv_eltwiseadd_bn_fuse_pass(g: Graph):
    n = 0
    for conv in list(_typed(g.ops)):
        if conv not in g.ops or not _plain_conv(g, conv):
            continue
        add, b = _conv_bias_add(g, conv)
        if add is None:
            continue
        a_out = _out(add)
        cons = g.consumers(a_out)
        if len(cons) != 1 or not g.single_use(a_out) or cons[0].func is not None or cons[0].type != "batch_norm":
            continue
        bn = cons[0]
        names = [_pop(bn, s) for s in ("Scale", "Bias", "Mean", "Variance")]
        if not all(x is not None and g.is_param(x) for x in names):
            continue
        gamma, beta, mean, var = (g.param(x).float() for x in names)
        std = torch.sqrt(var + float(bn.attrs.get("epsilon", 1e-5)))
        wname = _pop(conv, "Filter")
        w = g.param(wname)
        k = len(g.program.params)
        wn, bnm = f"{wname}@eabn{k}", f"{b}@eabn{k}"
        g.program.params[wn] = (w.float() * (gamma / std).reshape(-1, 1, 1, 1)).to(w.dtype)
        g.program.params[bnm] = ((g.param(b).float() - mean) * gamma / std + beta).to(w.dtype)
        g.block.create_var(wn, list(w.shape), "float32", persistable=True)
        g.block.create_var(bnm, [w.shape[0]], "float32", persistable=True)
        ins = dict(conv.paddle_inputs)
        ins["Filter"] = [wn]
        ins["Bias"] = [bnm]
        g.replace([conv, add, bn], _new(g.block, conv.type, ins, {"Output": [_out(bn, "Y")]}, dict(conv.attrs)))
        n += 1
    return n


def transpose_flatten_concat_fuse_pass(g: Graph):
    n = 0
    for cat in list(_typed(g.ops)):
        if cat.type != "concat" or cat not in g.ops or cat.paddle_inputs.get("AxisTensor"):
            continue
        xs = cat.paddle_inputs.get("X", [])
        if len(xs) < 2:
            continue
        chain, trans_axis, flat_axis, srcs = [], None, None, []
        for x in xs:
            fl = g.producer(x)
            if fl is None or fl.func is not None or fl.type != "flatten2" or not g.single_use(x):
                break
            t_out = _pop(fl, "X")
            tr = g.producer(t_out)
            if tr is None or tr.func is not None or tr.type != "transpose2" or not g.single_use(t_out):
                break
            ta, fa = list(tr.attrs.get("axis", [])), int(fl.attrs.get("axis", 1))
            if trans_axis is None:
                trans_axis, flat_axis = ta, fa
            if ta != trans_axis or fa != flat_axis:
                break
            chain += [tr, fl]
            srcs.append(_pop(tr, "X"))
        else:
            g.replace(chain + [cat], _new(g.block, "fusion_transpose_flatten_concat", {"X": srcs},
                                          {"Out": [_out(cat)]},
                                          {"trans_axis": trans_axis, "flatten_axis": flat_axis,
                                           "concat_axis": int(cat.attrs.get("axis", 0))}))
            n += 1
    return n


EXTRA_PASSES = {f.__name__: f for f in (
    is_test_pass, simplify_with_basic_ops_pass, constant_folding_pass,
    gpu_cpu_map_matmul_v2_to_mul_pass, gpu_cpu_map_matmul_v2_to_matmul_pass, gpu_cpu_map_matmul_to_mul_pass,
    gpu_cpu_squeeze2_matmul_fuse_pass, gpu_cpu_reshape2_matmul_fuse_pass, gpu_cpu_flatten2_matmul_fuse_pass,
    matmul_scale_fuse_pass, conv_elementwise_add_fuse_pass, conv_eltwiseadd_bn_fuse_pass,
    conv_elementwise_add_act_fuse_pass, conv_elementwise_add2_act_fuse_pass,
    transpose_flatten_concat_fuse_pass)}

np  # noqa
