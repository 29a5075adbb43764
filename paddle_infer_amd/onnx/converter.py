"""Paddle ProgramDesc (reference op types) → ONNX graph converter.

Parity: the reference's ``paddle.onnx.export`` delegates to paddle2onnx, which walks an inference
ProgramDesc and maps every Paddle op onto ONNX operators (`paddle2onnx/mapper/*`). This module does
the same over the ``.pdmodel`` our ``jit.save`` writes (``static/lowering.py`` lowers every recorded
op to a reference Paddle op type first), targeting ONNX opset 13 (default domain). Ops with no
ONNX form (training-only ops, the HIP weight-only kernel) raise ``ONNXConvertError`` naming the op.
"""
from __future__ import annotations

import math

import numpy as np

from . import proto as P


class ONNXConvertError(ValueError):
    pass


class _G:
    """Graph under construction: nodes, initializers, var metadata of the Paddle block."""

    def __init__(self, block, params, opset):
        self.block, self.params, self.opset = block, params, opset
        self.nodes, self.inits, self._n = [], [], 0
        self.vars = {}
        for vd in block.get("vars", []):
            td = vd.get("type", {}).get("lod_tensor", {}).get("tensor", {})
            self.vars[vd["name"]] = (list(td.get("dims", [])), td.get("data_type", 5),
                                     bool(vd.get("persistable")))
        self.dtype_over = {}  # var -> ONNX dtype where a conversion changed it (shape → int64)

    # ---- metadata ------------------------------------------------------------------------------
    def dims(self, v):
        return list(self.vars.get(v, ([], 5, False))[0])

    def rank(self, v):
        return len(self.dims(v))

    def onnx_dtype(self, v):
        if v in self.dtype_over:
            return self.dtype_over[v]
        return P.PADDLE2ONNX.get(self.vars.get(v, ([], 5, False))[1], 1)

    def np_dtype(self, v):
        return P.ONNX2NP.get(self.onnx_dtype(v), np.dtype(np.float32))

    # ---- builders ------------------------------------------------------------------------------
    def name(self, hint):
        self._n += 1
        return f"{hint}__onnx{self._n}"

    def const(self, arr, hint="const"):
        n = self.name(hint)
        self.inits.append(P.tensor(n, np.asarray(arr)))
        return n

    def ints(self, vals, hint="ints"):
        return self.const(np.asarray(vals, dtype=np.int64), hint)

    def scalar_like(self, v, value, hint="s"):
        return self.const(np.asarray(value, dtype=self.np_dtype(v)), hint)

    def node(self, op, inputs, outputs=None, **attrs):
        outs = outputs if outputs is not None else [self.name(op.lower())]
        self.nodes.append({"op_type": op, "input": list(inputs), "output": list(outs),
                           "name": self.name(op), "attribute": [P.attr(k, v) for k, v in attrs.items()
                                                                if v is not None]})
        return outs[0] if len(outs) == 1 else outs


def _ins(op, slot):
    for s in op.get("inputs", []):
        if s.get("parameter") == slot:
            return list(s.get("arguments", []))
    return []


def _outs(op, slot):
    for s in op.get("outputs", []):
        if s.get("parameter") == slot:
            return list(s.get("arguments", []))
    return []


def _attrs(op):
    from ..static.io import _attr_value
    return {a["name"]: _attr_value(a) for a in op.get("attrs", [])}


MAPPERS = {}


def mapper(*types):
    def deco(fn):
        for t in types:
            MAPPERS[t] = fn
        return fn
    return deco


# ---------------------------------------------------------------------------------- elementwise
_BIN = {"elementwise_add": "Add", "elementwise_sub": "Sub", "elementwise_mul": "Mul",
        "elementwise_div": "Div", "elementwise_pow": "Pow", "elementwise_max": "Max",
        "elementwise_min": "Min"}


def _bcast_y(g, x, y, axis):
    rx, ry = g.rank(x), g.rank(y)
    if axis is None or axis == -1 or axis == rx - ry or ry == 0:
        return y
    extra = rx - axis - ry
    if extra <= 0:
        return y
    return g.node("Unsqueeze", [y, g.ints(list(range(ry, ry + extra)))])


@mapper(*_BIN)
def _m_binary(g, op, a):
    x, y = _ins(op, "X")[0], _ins(op, "Y")[0]
    g.node(_BIN[op["type"]], [x, _bcast_y(g, x, y, a.get("axis", -1))], _outs(op, "Out"))


@mapper("scale")
def _m_scale(g, op, a):
    x, out = _ins(op, "X")[0], _outs(op, "Out")[0]
    s, b = float(a.get("scale", 1.0)), float(a.get("bias", 0.0))
    cur = x
    if not a.get("bias_after_scale", True) and b != 0.0:
        cur = g.node("Add", [cur, g.scalar_like(x, b)])
        b = 0.0
    if s != 1.0:
        cur = g.node("Mul", [cur, g.scalar_like(x, s)]) if b != 0.0 else g.node(
            "Mul", [cur, g.scalar_like(x, s)], [out])
    if b != 0.0:
        g.node("Add", [cur, g.scalar_like(x, b)], [out])
    elif s == 1.0:
        g.node("Identity", [cur], [out])


@mapper("pow")
def _m_pow(g, op, a):
    x = _ins(op, "X")[0]
    g.node("Pow", [x, g.scalar_like(x, float(a.get("factor", 1.0)))], _outs(op, "Out"))


_UN = {"relu": "Relu", "tanh": "Tanh", "sigmoid": "Sigmoid", "exp": "Exp", "log": "Log",
       "sqrt": "Sqrt", "abs": "Abs", "floor": "Floor", "sin": "Sin", "cos": "Cos", "erf": "Erf",
       "reciprocal": "Reciprocal", "assign": "Identity", "logical_not": "Not"}


@mapper(*_UN)
def _m_unary(g, op, a):
    g.node(_UN[op["type"]], _ins(op, "X"), _outs(op, "Out"))


@mapper("rsqrt")
def _m_rsqrt(g, op, a):
    g.node("Reciprocal", [g.node("Sqrt", _ins(op, "X"))], _outs(op, "Out"))


@mapper("square")
def _m_square(g, op, a):
    x = _ins(op, "X")[0]
    g.node("Mul", [x, x], _outs(op, "Out"))


@mapper("silu")
def _m_silu(g, op, a):
    x = _ins(op, "X")[0]
    g.node("Mul", [x, g.node("Sigmoid", [x])], _outs(op, "Out"))


@mapper("relu6")
def _m_relu6(g, op, a):
    x = _ins(op, "X")[0]
    g.node("Clip", [x, g.scalar_like(x, 0.0), g.scalar_like(x, 6.0)], _outs(op, "Out"))


@mapper("hard_swish")
def _m_hswish(g, op, a):
    x = _ins(op, "X")[0]
    t = g.node("Clip", [g.node("Add", [x, g.scalar_like(x, 3.0)]), g.scalar_like(x, 0.0),
                        g.scalar_like(x, 6.0)])
    g.node("Div", [g.node("Mul", [x, t]), g.scalar_like(x, 6.0)], _outs(op, "Out"))


@mapper("leaky_relu")
def _m_leaky(g, op, a):
    g.node("LeakyRelu", _ins(op, "X"), _outs(op, "Out"), alpha=float(a.get("alpha", 0.02)))


@mapper("clip")
def _m_clip(g, op, a):
    x = _ins(op, "X")[0]
    g.node("Clip", [x, g.scalar_like(x, a.get("min", -3.4e38)), g.scalar_like(x, a.get("max", 3.4e38))],
           _outs(op, "Out"))


@mapper("gelu")
def _m_gelu(g, op, a):
    x, out = _ins(op, "X")[0], _outs(op, "Out")[0]
    if a.get("approximate", False):
        x3 = g.node("Mul", [g.node("Mul", [x, x]), x])
        inner = g.node("Mul", [g.node("Add", [x, g.node("Mul", [x3, g.scalar_like(x, 0.044715)])]),
                               g.scalar_like(x, math.sqrt(2.0 / math.pi))])
        t = g.node("Tanh", [inner])
    else:
        t = g.node("Erf", [g.node("Mul", [x, g.scalar_like(x, 1.0 / math.sqrt(2.0))])])
    h = g.node("Mul", [x, g.node("Add", [t, g.scalar_like(x, 1.0)])])
    g.node("Mul", [h, g.scalar_like(x, 0.5)], [out])


_CMP = {"greater_equal": "GreaterOrEqual", "greater_than": "Greater", "less_equal": "LessOrEqual",
        "less_than": "Less", "equal": "Equal", "logical_and": "And", "logical_or": "Or"}


@mapper(*_CMP)
def _m_cmp(g, op, a):
    g.node(_CMP[op["type"]], [_ins(op, "X")[0], _ins(op, "Y")[0]], _outs(op, "Out"))


@mapper("not_equal")
def _m_ne(g, op, a):
    g.node("Not", [g.node("Equal", [_ins(op, "X")[0], _ins(op, "Y")[0]])], _outs(op, "Out"))


@mapper("where")
def _m_where(g, op, a):
    g.node("Where", [_ins(op, "Condition")[0], _ins(op, "X")[0], _ins(op, "Y")[0]], _outs(op, "Out"))


# ---------------------------------------------------------------------------------- creation / cast
@mapper("fill_any_like")
def _m_fill_like(g, op, a):
    x, out = _ins(op, "X")[0], _outs(op, "Out")[0]
    dt = a.get("dtype", -1)
    npdt = g.np_dtype(x) if dt in (-1, None) else P.ONNX2NP[P.PADDLE2ONNX[dt]]
    g.node("ConstantOfShape", [g.node("Shape", [x])], [out],
           value=P.tensor("value", np.asarray([a.get("value", 0.0)], dtype=npdt)))


@mapper("fill_constant")
def _m_fill_const(g, op, a):
    npdt = P.ONNX2NP[P.PADDLE2ONNX[a.get("dtype", 5)]]
    arr = np.full([int(d) for d in a.get("shape", [1])], a.get("value", 0.0), dtype=npdt)
    g.node("Identity", [g.const(arr, "fill")], _outs(op, "Out"))


@mapper("cast")
def _m_cast(g, op, a):
    out = _outs(op, "Out")[0]
    to = P.PADDLE2ONNX[a.get("out_dtype", 5)]
    g.dtype_over[out] = to
    g.node("Cast", _ins(op, "X"), [out], to=to)


@mapper("shape")
def _m_shape(g, op, a):
    out = _outs(op, "Out")[0]
    g.dtype_over[out] = 7
    g.node("Shape", _ins(op, "Input"), [out])


# ---------------------------------------------------------------------------------- shape ops
@mapper("reshape2")
def _m_reshape(g, op, a):
    x, out = _ins(op, "X")[0], _outs(op, "Out")[0]
    st = _ins(op, "Shape") or _ins(op, "ShapeTensor")
    if st:
        s = st[0] if g.onnx_dtype(st[0]) == 7 else g.node("Cast", [st[0]], to=7)
        g.node("Reshape", [x, s], [out])
    else:
        g.node("Reshape", [x, g.ints(a.get("shape", []), "shape")], [out])


@mapper("transpose2")
def _m_transpose(g, op, a):
    g.node("Transpose", _ins(op, "X"), _outs(op, "Out"), perm=list(a.get("axis", [])))


@mapper("unsqueeze2")
def _m_unsqueeze(g, op, a):
    g.node("Unsqueeze", [_ins(op, "X")[0], g.ints(a.get("axes", []))], _outs(op, "Out"))


@mapper("squeeze2")
def _m_squeeze(g, op, a):
    x = _ins(op, "X")[0]
    axes = a.get("axes", [])
    if axes:
        g.node("Squeeze", [x, g.ints(axes)], _outs(op, "Out"))
    else:
        g.node("Squeeze", [x], _outs(op, "Out"))


@mapper("flatten_contiguous_range")
def _m_flatten(g, op, a):
    x = _ins(op, "X")[0]
    d = g.dims(x)
    s, e = a.get("start_axis", 1) % len(d), a.get("stop_axis", -1) % len(d)
    tail = d[e + 1:]
    if any(t < 0 for t in tail):
        raise ONNXConvertError("flatten_contiguous_range with a dynamic trailing dim")
    g.node("Reshape", [x, g.ints([0] * s + [-1] + tail)], _outs(op, "Out"))


@mapper("concat")
def _m_concat(g, op, a):
    g.node("Concat", _ins(op, "X"), _outs(op, "Out"), axis=int(a.get("axis", 0)))


@mapper("stack")
def _m_stack(g, op, a):
    ax = int(a.get("axis", 0))
    xs = _ins(op, "X")
    ax = ax if ax >= 0 else ax + g.rank(xs[0]) + 1
    us = [g.node("Unsqueeze", [x, g.ints([ax])]) for x in xs]
    g.node("Concat", us, _outs(op, "Y"), axis=ax)


@mapper("split")
def _m_split(g, op, a):
    x, outs = _ins(op, "X")[0], _outs(op, "Out")
    ax = int(a.get("axis", 0)) % max(1, g.rank(x))
    secs = list(a.get("sections", []) or [])
    if not secs:
        n = int(a.get("num", len(outs)))
        size = g.dims(x)[ax]
        if size < 0:
            raise ONNXConvertError("split of a dynamic dim into equal parts")
        secs = [size // n] * n
    if -1 in secs:
        size = g.dims(x)[ax]
        secs[secs.index(-1)] = size - (sum(secs) + 1)
    g.node("Split", [x, g.ints(secs)], outs, axis=ax)


def _slice(g, x, a, steps=None):
    axes = list(a.get("axes", []))
    starts = g.ints(a.get("starts", []))
    ends = g.ints([min(int(e), 2 ** 62) for e in a.get("ends", [])])
    ins = [x, starts, ends, g.ints(axes)]
    if steps is not None:
        ins.append(g.ints(steps))
    return g.node("Slice", ins)


@mapper("slice")
def _m_slice(g, op, a):
    y = _slice(g, _ins(op, "Input")[0], a)
    dec = list(a.get("decrease_axis", []) or [])
    if dec:
        g.node("Squeeze", [y, g.ints(dec)], _outs(op, "Out"))
    else:
        g.node("Identity", [y], _outs(op, "Out"))


@mapper("strided_slice")
def _m_strided_slice(g, op, a):
    y = _slice(g, _ins(op, "Input")[0], a, steps=list(a.get("strides", [])))
    dec = list(a.get("decrease_axis", []) or [])
    if dec:
        g.node("Squeeze", [y, g.ints(dec)], _outs(op, "Out"))
    else:
        g.node("Identity", [y], _outs(op, "Out"))


@mapper("expand_v2")
def _m_expand(g, op, a):
    shape = [1 if int(s) < 0 else int(s) for s in a.get("shape", [])]
    g.node("Expand", [_ins(op, "X")[0], g.ints(shape)], _outs(op, "Out"))


@mapper("expand_as_v2")
def _m_expand_as(g, op, a):
    y = _ins(op, "Y")
    tgt = g.node("Shape", [y[0]]) if y else g.ints(a.get("target_shape", []))
    g.node("Expand", [_ins(op, "X")[0], tgt], _outs(op, "Out"))


_RED = {"reduce_mean": "ReduceMean", "reduce_sum": "ReduceSum", "reduce_max": "ReduceMax",
        "reduce_min": "ReduceMin", "reduce_prod": "ReduceProd"}


@mapper(*_RED)
def _m_reduce(g, op, a):
    x = _ins(op, "X")[0]
    keep = int(bool(a.get("keep_dim", False)))
    axes = list(range(g.rank(x))) if a.get("reduce_all") or not a.get("dim") else list(a["dim"])
    kind = _RED[op["type"]]
    if kind == "ReduceSum":  # opset 13: axes is an input
        g.node(kind, [x, g.ints(axes)], _outs(op, "Out"), keepdims=keep)
    else:
        g.node(kind, [x], _outs(op, "Out"), axes=axes, keepdims=keep)


@mapper("softmax")
def _m_softmax(g, op, a):
    g.node("Softmax", _ins(op, "X"), _outs(op, "Out"), axis=int(a.get("axis", -1)))


# ---------------------------------------------------------------------------------- nn
@mapper("matmul_v2", "matmul")
def _m_matmul(g, op, a):
    x, y = _ins(op, "X")[0], _ins(op, "Y")[0]

    def tr(v, flag):
        if not flag:
            return v
        r = g.rank(v)
        perm = list(range(r - 2)) + [r - 1, r - 2]
        return g.node("Transpose", [v], perm=perm)
    tx = a.get("trans_x", a.get("transpose_X", False))
    ty = a.get("trans_y", a.get("transpose_Y", False))
    out = _outs(op, "Out")[0]
    alpha = float(a.get("alpha", 1.0))
    if alpha != 1.0:
        m = g.node("MatMul", [tr(x, tx), tr(y, ty)])
        g.node("Mul", [m, g.scalar_like(x, alpha)], [out])
    else:
        g.node("MatMul", [tr(x, tx), tr(y, ty)], [out])


@mapper("layer_norm")
def _m_layer_norm(g, op, a):
    x, out = _ins(op, "X")[0], _outs(op, "Y")[0]
    r = g.rank(x)
    bna = int(a.get("begin_norm_axis", r - 1))
    axes = list(range(bna, r))
    mean = g.node("ReduceMean", [x], axes=axes, keepdims=1)
    d = g.node("Sub", [x, mean])
    var = g.node("ReduceMean", [g.node("Mul", [d, d])], axes=axes, keepdims=1)
    y = g.node("Div", [d, g.node("Sqrt", [g.node("Add", [var, g.scalar_like(x, float(a.get("epsilon", 1e-5)))])])])
    nshape = g.dims(x)[bna:]
    for slot, opn in (("Scale", "Mul"), ("Bias", "Add")):
        p = _ins(op, slot)
        if p:
            pv = p[0]
            if len(axes) > 1:
                pv = g.node("Reshape", [pv, g.ints(nshape)])
            y = g.node(opn, [y, pv])
    g.node("Identity", [y], [out])


@mapper("lookup_table_v2", "lookup_table")
def _m_embedding(g, op, a):
    g.node("Gather", [_ins(op, "W")[0], _ins(op, "Ids")[0]], _outs(op, "Out"), axis=0)


@mapper("dropout")
def _m_dropout(g, op, a):
    x, out = _ins(op, "X")[0], _outs(op, "Out")[0]
    if a.get("dropout_implementation", "upscale_in_train") == "downgrade_in_infer":
        g.node("Mul", [x, g.scalar_like(x, 1.0 - float(a.get("dropout_prob", 0.5)))], [out])
    else:
        g.node("Identity", [x], [out])


def _pads(a, nd=2):
    p = [int(v) for v in a.get("paddings", [0] * nd)]
    if len(p) == nd:
        return p + p
    # Paddle 4-element order: [top, bottom, left, right] → ONNX [top, left, bottom, right]
    return [p[0], p[2], p[1], p[3]]


@mapper("conv2d", "depthwise_conv2d")
def _m_conv(g, op, a):
    if a.get("data_format", "NCHW") not in ("NCHW", "AnyLayout"):
        raise ONNXConvertError("conv2d data_format NHWC")
    algo = a.get("padding_algorithm", "EXPLICIT")
    kw = {"strides": list(a.get("strides", [1, 1])), "dilations": list(a.get("dilations", [1, 1])),
          "group": int(a.get("groups", 1))}
    if algo == "SAME":
        kw["auto_pad"] = "SAME_UPPER"
    elif algo == "VALID":
        kw["pads"] = [0, 0, 0, 0]
    else:
        kw["pads"] = _pads(a)
    g.node("Conv", [_ins(op, "Input")[0], _ins(op, "Filter")[0]], _outs(op, "Output"), **kw)


@mapper("batch_norm")
def _m_bn(g, op, a):
    ins = [_ins(op, s)[0] for s in ("X", "Scale", "Bias", "Mean", "Variance")]
    g.node("BatchNormalization", ins, [_outs(op, "Y")[0]], epsilon=float(a.get("epsilon", 1e-5)))


@mapper("pool2d")
def _m_pool(g, op, a):
    x, out = _ins(op, "X")[0], _outs(op, "Out")[0]
    mx = a.get("pooling_type", "max") == "max"
    k = [int(v) for v in a.get("ksize", [1, 1])]
    if a.get("global_pooling") or (a.get("adaptive") and k == [1, 1]):
        g.node("GlobalMaxPool" if mx else "GlobalAveragePool", [x], [out])
        return
    if a.get("adaptive"):
        d = g.dims(x)[2:]
        if any(v < 0 or v % o for v, o in zip(d, k)):
            raise ONNXConvertError("adaptive pool2d with a non-divisible / dynamic input size")
        k = [v // o for v, o in zip(d, k)]
        kw = {"kernel_shape": k, "strides": k}
    else:
        kw = {"kernel_shape": k, "strides": list(a.get("strides", k)), "pads": _pads(a),
              "ceil_mode": int(bool(a.get("ceil_mode", False)))}
    if mx:
        g.node("MaxPool", [x], [out], **kw)
    else:
        g.node("AveragePool", [x], [out], count_include_pad=0 if a.get("exclusive", True) else 1, **kw)


def _causal_mask(g, scores, like):
    """additive causal mask (0 / -inf) broadcast over [.., Sq, Sk] scores."""
    shp = g.node("Shape", [scores])
    sq = g.node("Gather", [shp, g.ints(-2)], axis=0)
    sk = g.node("Gather", [shp, g.ints(-1)], axis=0)
    one = g.ints(1)
    rows = g.node("Range", [g.ints(0), sq, one])
    cols = g.node("Range", [g.ints(0), sk, one])
    # key j is visible to query i iff j <= i + (Sk - Sq)
    off = g.node("Sub", [sk, sq])
    lim = g.node("Unsqueeze", [g.node("Add", [rows, off]), g.ints([1])])
    bad = g.node("Greater", [g.node("Unsqueeze", [cols, g.ints([0])]), lim])
    return g.node("Where", [bad, g.scalar_like(like, -1e30), g.scalar_like(like, 0.0)])


@mapper("flash_attn")
def _m_flash(g, op, a):
    q, k, v = (_ins(op, s)[0] for s in ("q", "k", "v"))
    out = _outs(op, "out")[0]
    D = g.dims(q)[-1]
    if D < 0:
        raise ONNXConvertError("flash_attn with a dynamic head dim")
    qt = g.node("Transpose", [q], perm=[0, 2, 1, 3])
    kt = g.node("Transpose", [k], perm=[0, 2, 3, 1])
    vt = g.node("Transpose", [v], perm=[0, 2, 1, 3])
    s = g.node("Mul", [g.node("MatMul", [qt, kt]), g.scalar_like(q, 1.0 / math.sqrt(D))])
    m = _ins(op, "attn_mask")
    if m:
        s = g.node("Add", [s, m[0]])
    if a.get("causal", False):
        s = g.node("Add", [s, _causal_mask(g, s, q)])
    p = g.node("Softmax", [s], axis=-1)
    g.node("Transpose", [g.node("MatMul", [p, vt])], [out], perm=[0, 2, 1, 3])


@mapper("fused_softmax_mask")
def _m_sm_mask(g, op, a):
    g.node("Softmax", [g.node("Add", [_ins(op, "X")[0], _ins(op, "Mask")[0]])], _outs(op, "Out"), axis=-1)


@mapper("fused_softmax_mask_upper_triangle")
def _m_sm_causal(g, op, a):
    x = _ins(op, "X")[0]
    g.node("Softmax", [g.node("Add", [x, _causal_mask(g, x, x)])], _outs(op, "Out"), axis=-1)


# ---------------------------------------------------------------------------------- driver
def program_to_onnx(desc: dict, params: dict, opset_version: int = 13,
                    producer: str = "paddle_infer_amd") -> dict:
    """ModelProto (as a dict for ``proto.encode_model``) of an inference ProgramDesc ``desc``
    (``static.proto.decode('ProgramDesc', ...)``) with persistable values ``params``."""
    if opset_version < 13:
        raise ONNXConvertError(f"opset_version {opset_version} < 13 is not supported (use 13+)")
    block = desc["blocks"][0]
    g = _G(block, params, opset_version)
    feeds, fetches = {}, {}
    for op in block.get("ops", []):
        t = op["type"]
        a = _attrs(op)
        if t == "feed":
            feeds[int(a.get("col", 0))] = _outs(op, "Out")[0]
            continue
        if t == "fetch":
            fetches[int(a.get("col", 0))] = _ins(op, "X")[0]
            continue
        fn = MAPPERS.get(t)
        if fn is None:
            raise ONNXConvertError(f"Paddle op '{t}' has no ONNX mapping")
        fn(g, op, a)
    used = set()
    for n in g.nodes:
        used.update(n["input"])
    inits = []
    for name in sorted(used):
        if name in params:
            arr = np.asarray(params[name])
            if arr.dtype == np.uint16:  # bf16 storage → f32
                arr = (arr.astype(np.uint32) << 16).view(np.float32)
            inits.append(P.tensor(name, arr))
    graph = {"name": "paddle_infer_amd_graph", "node": g.nodes, "initializer": inits + g.inits,
             "input": [P.value_info(feeds[i], g.onnx_dtype(feeds[i]), g.dims(feeds[i]))
                       for i in sorted(feeds)],
             "output": [P.value_info(fetches[i], g.onnx_dtype(fetches[i]), g.dims(fetches[i]))
                        for i in sorted(fetches)]}
    return {"ir_version": 8, "producer_name": producer, "producer_version": "2",
            "opset_import": [{"domain": "", "version": int(opset_version)}], "graph": graph}
