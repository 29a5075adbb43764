"""Lower recorded ops (torch / framework callables captured by ``jit.to_static`` / static
capture) into Paddle OpDescs with the reference op types, slot names and attributes, so
``jit.save`` / ``save_inference_model`` write a ``.pdmodel`` that contains only Paddle ops —
loadable by the reference's ProgramDesc tooling and executed here through the Paddle-op registry
(``ops_registry.py``), which the inference IR passes then fuse back onto the HIP kernels.

Parity: the op definitions of the reference (`paddle/phi/api/yaml/ops.yaml`,
`legacy_ops.yaml`, `paddle/fluid/operators/*_op.cc`): matmul_v2 / elementwise_* / scale /
layer_norm / gelu / softmax / lookup_table_v2 / reshape2 / transpose2 / slice / split / concat /
cast / conv2d / batch_norm / pool2d / flash_attn / dropout / where / compare + logical ops /
fill_any_like / shape / softmax_with_cross_entropy / fused_softmax_mask(_upper_triangle) /
weight_only_linear.

Each lowering returns a list of ``(type, inputs, outputs, attrs)``; intermediate names come from
``ctx.tmp()``. An op no rule covers raises ``LoweringError`` (save refuses to write a non-Paddle
op) unless the caller opted into ``allow_custom_ops``.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import proto
from .framework import SymDim, VarRef, symbolize
from ..framework.dtype import dtype_name


class LoweringError(ValueError):
    pass


class _Ctx:
    def __init__(self, block, op):
        self.block, self.op = block, op
        self.new_vars = []  # (name, dims, dtype code)
        self._tmp = {}
        self._n = 0

    def tmp(self, like=None, dims=None, dtype=None):
        self._n += 1
        name = f"{self.op.output_names()[0] if self.op.output_names() else 'lower'}.lower_{self._n}"
        if like is not None:
            dims = dims if dims is not None else self.dims(like)
            dtype = dtype if dtype is not None else self.dtype_code(like)
        self.new_vars.append((name, list(dims or [-1]), 5 if dtype is None else dtype))
        self._tmp[name] = self.new_vars[-1]
        return name

    def var(self, name):
        return self.block.vars.get(name)

    def shape(self, name):
        """Symbolized shape (ints and SymDim) of a program variable."""
        if name in self._tmp:
            return [SymDim(-1, ()) if d < 0 else d for d in self._tmp[name][1]]
        v = self.var(name)
        with torch._C.DisableTorchFunctionSubclass():
            return [symbolize(int(s)) for s in v.shape]

    def dims(self, name):
        return [(-1 if isinstance(s, SymDim) else int(s)) for s in self.shape(name)]

    def ndim(self, name):
        return len(self.shape(name))

    def dtype_code(self, name):
        if name in self._tmp:
            return self._tmp[name][2]
        v = self.var(name)
        with torch._C.DisableTorchFunctionSubclass():
            return proto.VT[dtype_name(v.dtype)]


def _name(x):
    if isinstance(x, VarRef):
        return x.name
    raise LoweringError(f"expected a tensor operand, got {x!r}")


def _is_var(x):
    return isinstance(x, VarRef)


def _arg(op, i, key, default=None):
    if len(op.args) > i:
        return op.args[i]
    return op.kwargs.get(key, default)


def _outs(op):
    return op.output_names()


def _intlist(v, n=None):
    if isinstance(v, (list, tuple)):
        out = [int(e) for e in v]
    else:
        out = [int(v)] * (n or 1)
    return out


def _shape_attr(ctx, x, target):
    """Paddle reshape ``shape`` attr from a (possibly symbolic) target shape: symbolic dims equal
    to the input's dim at the same position become 0 (copy), one other symbolic dim becomes -1."""
    src = ctx.shape(x)
    out, infer = [], 0
    for i, s in enumerate(target):
        if isinstance(s, SymDim):
            if i < len(src) and isinstance(src[i], SymDim) and (src[i].k, src[i].exps) == (s.k, s.exps):
                out.append(0)
            else:
                out.append(-1)
                infer += 1
        else:
            out.append(int(s))
    if infer > 1 or out.count(-1) > 1:
        raise LoweringError(f"reshape to {target} needs more than one inferred dim")
    return out


# --------------------------------------------------------------------------- rules
RULES = {}


def rule(*keys):
    def deco(fn):
        for k in keys:
            RULES[k] = fn
        return fn
    return deco


def _binary(ptype):
    def fn(ctx, op):
        a, b = _arg(op, 0, "input"), _arg(op, 1, "other")
        out = _outs(op)[0]
        alpha = op.kwargs.get("alpha", 1)
        if _is_var(a) and _is_var(b):
            y = _name(b)
            res = []
            if alpha != 1:
                y2 = ctx.tmp(like=y)
                res.append(("scale", {"X": [y]}, {"Out": [y2]}, {"scale": float(alpha), "bias": 0.0,
                                                                  "bias_after_scale": True}))
                y = y2
            return res + [(ptype, {"X": [_name(a)], "Y": [y]}, {"Out": [out]}, {"axis": -1})]
        if _is_var(a) and isinstance(b, (int, float)):
            b = float(b)
            if ptype == "elementwise_add":
                s, bias = 1.0, b * alpha
            elif ptype == "elementwise_sub":
                s, bias = 1.0, -b * alpha
            elif ptype == "elementwise_mul":
                s, bias = b, 0.0
            elif ptype == "elementwise_div" and b != 0.0:
                s, bias = 1.0 / b, 0.0
            else:
                raise LoweringError(f"{ptype} with scalar {b}")
            return [("scale", {"X": [_name(a)]}, {"Out": [out]}, {"scale": s, "bias": bias,
                                                                 "bias_after_scale": True})]
        if _is_var(b) and isinstance(a, (int, float)) and ptype in ("elementwise_add", "elementwise_mul",
                                                                      "elementwise_sub"):
            if ptype == "elementwise_sub":  # a - b
                return [("scale", {"X": [_name(b)]}, {"Out": [out]}, {"scale": -1.0, "bias": float(a),
                                                                     "bias_after_scale": True})]
            s, bias = (1.0, float(a)) if ptype == "elementwise_add" else (float(a), 0.0)
            return [("scale", {"X": [_name(b)]}, {"Out": [out]}, {"scale": s, "bias": bias,
                                                                 "bias_after_scale": True})]
        raise LoweringError(f"{ptype} operands {a!r}, {b!r}")
    return fn


T = torch.Tensor
for _fns, _pt in (((torch.add, T.add, T.__add__, T.__radd__, T.add_), "elementwise_add"),
                  ((torch.sub, T.sub, T.__sub__), "elementwise_sub"),
                  ((torch.mul, T.mul, T.__mul__, T.__rmul__), "elementwise_mul"),
                  ((torch.div, torch.true_divide, T.div, T.__truediv__), "elementwise_div"),
                  ((torch.maximum,), "elementwise_max"), ((torch.minimum,), "elementwise_min")):
    RULES.update({f: _binary(_pt) for f in _fns})


@rule(T.__rsub__)
def _rsub(ctx, op):
    a, b = op.args[0], op.args[1]  # b - a
    if _is_var(a) and isinstance(b, (int, float)):
        return [("scale", {"X": [_name(a)]}, {"Out": [_outs(op)[0]]},
                 {"scale": -1.0, "bias": float(b), "bias_after_scale": True})]
    raise LoweringError("rsub")


@rule(T.__rtruediv__)
def _rdiv(ctx, op):
    a, b = op.args[0], op.args[1]  # b / a
    if _is_var(a) and isinstance(b, (int, float)):
        r = ctx.tmp(like=_name(a))
        return [("reciprocal", {"X": [_name(a)]}, {"Out": [r]}, {}),
                ("scale", {"X": [r]}, {"Out": [_outs(op)[0]]},
                 {"scale": float(b), "bias": 0.0, "bias_after_scale": True})]
    raise LoweringError("rtruediv")


@rule(T.__neg__, torch.neg, T.neg)
def _neg(ctx, op):
    return [("scale", {"X": [_name(op.args[0])]}, {"Out": [_outs(op)[0]]},
             {"scale": -1.0, "bias": 0.0, "bias_after_scale": True})]


@rule(torch.pow, T.pow, T.__pow__)
def _pow(ctx, op):
    x, e = op.args[0], op.args[1]
    if _is_var(x) and isinstance(e, (int, float)):
        return [("pow", {"X": [_name(x)]}, {"Out": [_outs(op)[0]]}, {"factor": float(e)})]
    return _binary("elementwise_pow")(ctx, op)


_UNARY = {torch.relu: "relu", F.relu: "relu", T.relu: "relu", torch.tanh: "tanh", T.tanh: "tanh",
          F.tanh: "tanh", torch.sigmoid: "sigmoid", T.sigmoid: "sigmoid", F.sigmoid: "sigmoid",
          F.silu: "silu", torch.exp: "exp", T.exp: "exp", torch.log: "log", T.log: "log",
          torch.sqrt: "sqrt", T.sqrt: "sqrt", torch.rsqrt: "rsqrt", T.rsqrt: "rsqrt",
          torch.abs: "abs", T.abs: "abs", F.relu6: "relu6", F.hardswish: "hard_swish",
          torch.square: "square", torch.floor: "floor", torch.sin: "sin", torch.cos: "cos",
          torch.erf: "erf", T.contiguous: "assign", T.clone: "assign", torch.clone: "assign",
          T.detach: "assign", torch.logical_not: "logical_not", T.logical_not: "logical_not",
          T.__invert__: "logical_not"}


def _unary(ctx, op):
    return [(_UNARY[op.func], {"X": [_name(op.args[0])]}, {"Out": [_outs(op)[0]]}, {})]


RULES.update({f: _unary for f in _UNARY})


@rule(torch.clamp, T.clamp, torch.clip, T.clip)
def _clamp(ctx, op):
    """Reference `clip` op (phi clip_kernel): min / max attributes, one side may be open."""
    lo, hi = _arg(op, 1, "min", None), _arg(op, 2, "max", None)
    if _is_var(lo) or _is_var(hi):
        raise LoweringError("clamp with tensor bounds")
    big = 3.4e38
    return [("clip", {"X": [_name(op.args[0])]}, {"Out": [_outs(op)[0]]},
             {"min": float(-big if lo is None else lo), "max": float(big if hi is None else hi)})]


@rule(F.leaky_relu)
def _leaky(ctx, op):
    return [("leaky_relu", {"X": [_name(op.args[0])]}, {"Out": [_outs(op)[0]]},
             {"alpha": float(_arg(op, 1, "negative_slope", 0.01))})]


@rule(F.gelu)
def _gelu_t(ctx, op):
    return [("gelu", {"X": [_name(op.args[0])]}, {"Out": [_outs(op)[0]]},
             {"approximate": op.kwargs.get("approximate", "none") == "tanh"})]


_CMP = {T.ge: "greater_equal", torch.ge: "greater_equal", T.__ge__: "greater_equal",
        T.gt: "greater_than", torch.gt: "greater_than", T.__gt__: "greater_than",
        T.le: "less_equal", torch.le: "less_equal", T.__le__: "less_equal",
        T.lt: "less_than", torch.lt: "less_than", T.__lt__: "less_than",
        T.eq: "equal", torch.eq: "equal", T.__eq__: "equal",
        T.ne: "not_equal", torch.ne: "not_equal", T.__ne__: "not_equal",
        T.__and__: "logical_and", torch.logical_and: "logical_and", T.logical_and: "logical_and",
        T.__or__: "logical_or", torch.logical_or: "logical_or", T.logical_or: "logical_or"}


def _cmp(ctx, op):
    a, b = op.args[0], op.args[1]
    ptype = _CMP[op.func]
    res = []
    if not _is_var(b):  # scalar operand: materialise it
        if not isinstance(b, (int, float, bool)):
            raise LoweringError(f"{ptype} operand {b!r}")
        t = ctx.tmp(dims=[1], dtype=ctx.dtype_code(_name(a)))
        res.append(("fill_constant", {}, {"Out": [t]},
                    {"shape": [1], "value": float(b), "dtype": ctx.dtype_code(_name(a))}))
        b = VarRef(t)
    return res + [(ptype, {"X": [_name(a)], "Y": [_name(b)]}, {"Out": [_outs(op)[0]]}, {"axis": -1})]


RULES.update({f: _cmp for f in _CMP})


@rule(torch.where)
def _where(ctx, op):
    c, x, y = op.args[:3]
    res, names = [], []
    ref = _name(x) if _is_var(x) else _name(y)
    for v in (x, y):
        if _is_var(v):
            names.append(_name(v))
        else:
            t = ctx.tmp(like=ref)
            res.append(("fill_any_like", {"X": [ref]}, {"Out": [t]}, {"value": float(v), "dtype": -1}))
            names.append(t)
    return res + [("where", {"Condition": [_name(c)], "X": [names[0]], "Y": [names[1]]},
                   {"Out": [_outs(op)[0]]}, {})]


@rule(torch.zeros_like, torch.ones_like, torch.full_like)
def _fill_like(ctx, op):
    x = _name(op.args[0])
    val = {torch.zeros_like: 0.0, torch.ones_like: 1.0}.get(op.func)
    if val is None:
        val = float(_arg(op, 1, "fill_value"))
    dt = op.kwargs.get("dtype")
    return [("fill_any_like", {"X": [x]}, {"Out": [_outs(op)[0]]},
             {"value": val, "dtype": proto.VT[dtype_name(dt)] if dt is not None else -1})]


@rule(T.to, T.float, T.half, T.bfloat16, T.int, T.long, T.bool, T.type)
def _cast(ctx, op):
    x = _name(op.args[0])
    fixed = {T.float: torch.float32, T.half: torch.float16, T.bfloat16: torch.bfloat16,
             T.int: torch.int32, T.long: torch.int64, T.bool: torch.bool}.get(op.func)
    dt = fixed
    if dt is None:
        for a in list(op.args[1:]) + list(op.kwargs.values()):
            if isinstance(a, torch.dtype):
                dt = a
    out = _outs(op)[0]
    if dt is None:
        return [("assign", {"X": [x]}, {"Out": [out]}, {})]
    return [("cast", {"X": [x]}, {"Out": [out]},
             {"in_dtype": ctx.dtype_code(x), "out_dtype": proto.VT[dtype_name(dt)]})]


@rule(torch.matmul, T.matmul, T.__matmul__, torch.mm, T.mm, torch.bmm, T.bmm)
def _matmul(ctx, op):
    return [("matmul_v2", {"X": [_name(op.args[0])], "Y": [_name(op.args[1])]},
             {"Out": [_outs(op)[0]]}, {"trans_x": False, "trans_y": False})]


@rule(F.linear)
def _torch_linear(ctx, op):
    x, w, b = _arg(op, 0, "input"), _arg(op, 1, "weight"), _arg(op, 2, "bias")
    out = _outs(op)[0]
    if b is None:
        return [("matmul_v2", {"X": [_name(x)], "Y": [_name(w)]}, {"Out": [out]},
                 {"trans_x": False, "trans_y": True})]
    t = ctx.tmp(like=out)
    return [("matmul_v2", {"X": [_name(x)], "Y": [_name(w)]}, {"Out": [t]},
             {"trans_x": False, "trans_y": True}),
            ("elementwise_add", {"X": [t], "Y": [_name(b)]}, {"Out": [out]}, {"axis": -1})]


def _linear_ops(ctx, x, w, b, out):
    if b is None:
        return [("matmul_v2", {"X": [x], "Y": [w]}, {"Out": [out]}, {"trans_x": False, "trans_y": False})]
    t = ctx.tmp(like=out)
    return [("matmul_v2", {"X": [x], "Y": [w]}, {"Out": [t]}, {"trans_x": False, "trans_y": False}),
            ("elementwise_add", {"X": [t], "Y": [b]}, {"Out": [out]}, {"axis": -1})]


@rule("linear")
def _fw_linear(ctx, op):
    x, w, b = _arg(op, 0, "x"), _arg(op, 1, "weight"), _arg(op, 2, "bias")
    return _linear_ops(ctx, _name(x), _name(w), _name(b) if b is not None else None, _outs(op)[0])


@rule(T.reshape, torch.reshape, T.view)
def _reshape(ctx, op):
    x = _name(op.args[0])
    shape = op.args[1:] if len(op.args) > 2 or not isinstance(op.args[1], (list, tuple)) else op.args[1]
    if op.kwargs.get("shape") is not None:
        shape = op.kwargs["shape"]
    if any(isinstance(s, torch.dtype) for s in shape):
        raise LoweringError("view(dtype)")
    out = _outs(op)[0]
    return [("reshape2", {"X": [x]}, {"Out": [out], "XShape": [ctx.tmp(dims=[-1])]},
             {"shape": _shape_attr(ctx, x, shape)})]


@rule(T.view_as, T.reshape_as)
def _view_as(ctx, op):
    x, other = _name(op.args[0]), _name(op.args[1])
    s = ctx.tmp(dims=[ctx.ndim(other)], dtype=2)
    return [("shape", {"Input": [other]}, {"Out": [s]}, {}),
            ("reshape2", {"X": [x], "Shape": [s]}, {"Out": [_outs(op)[0]], "XShape": [ctx.tmp(dims=[-1])]},
             {"shape": []})]


@rule(T.permute, torch.permute)
def _permute(ctx, op):
    x = _name(op.args[0])
    perm = op.args[1:] if len(op.args) > 2 or not isinstance(op.args[1], (list, tuple)) else op.args[1]
    if "dims" in op.kwargs:
        perm = op.kwargs["dims"]
    nd = ctx.ndim(x)
    return [("transpose2", {"X": [x]}, {"Out": [_outs(op)[0]], "XShape": [ctx.tmp(dims=[-1])]},
             {"axis": [int(p) % nd for p in perm]})]


@rule(T.transpose, torch.transpose, T.t, torch.t)
def _transpose(ctx, op):
    x = _name(op.args[0])
    nd = ctx.ndim(x)
    if op.func in (T.t, torch.t):
        d0, d1 = 0, 1
    else:
        d0, d1 = int(_arg(op, 1, "dim0")) % nd, int(_arg(op, 2, "dim1")) % nd
    perm = list(range(nd))
    perm[d0], perm[d1] = perm[d1], perm[d0]
    return [("transpose2", {"X": [x]}, {"Out": [_outs(op)[0]], "XShape": [ctx.tmp(dims=[-1])]},
             {"axis": perm})]


@rule(T.unsqueeze, torch.unsqueeze)
def _unsqueeze(ctx, op):
    x = _name(op.args[0])
    d = int(_arg(op, 1, "dim"))
    if d < 0:
        d += ctx.ndim(x) + 1
    return [("unsqueeze2", {"X": [x]}, {"Out": [_outs(op)[0]], "XShape": [ctx.tmp(dims=[-1])]},
             {"axes": [d]})]


@rule(T.squeeze, torch.squeeze)
def _squeeze(ctx, op):
    x = _name(op.args[0])
    d = _arg(op, 1, "dim")
    axes = [] if d is None else _intlist(d)
    return [("squeeze2", {"X": [x]}, {"Out": [_outs(op)[0]], "XShape": [ctx.tmp(dims=[-1])]},
             {"axes": axes})]


@rule(torch.flatten, T.flatten)
def _flatten(ctx, op):
    x = _name(op.args[0])
    nd = ctx.ndim(x)
    s, e = int(_arg(op, 1, "start_dim", 0)), int(_arg(op, 2, "end_dim", -1))
    return [("flatten_contiguous_range", {"X": [x]},
             {"Out": [_outs(op)[0]], "XShape": [ctx.tmp(dims=[-1])]},
             {"start_axis": s % nd, "stop_axis": e % nd})]


@rule(torch.cat, torch.concat)
def _cat(ctx, op):
    xs = _arg(op, 0, "tensors")
    return [("concat", {"X": [_name(t) for t in xs]}, {"Out": [_outs(op)[0]]},
             {"axis": int(_arg(op, 1, "dim", 0))})]


@rule(torch.stack)
def _stack(ctx, op):
    xs = _arg(op, 0, "tensors")
    return [("stack", {"X": [_name(t) for t in xs]}, {"Y": [_outs(op)[0]]},
             {"axis": int(_arg(op, 1, "dim", 0))})]


@rule(torch.split, T.split, torch.chunk, T.chunk)
def _split(ctx, op):
    x = _name(op.args[0])
    nd = ctx.ndim(x)
    spec = op.args[1]
    axis = int(_arg(op, 2, "dim", 0)) % nd
    outs = _outs(op)
    if op.func in (torch.chunk, T.chunk):
        return [("split", {"X": [x]}, {"Out": outs}, {"axis": axis, "num": int(spec), "sections": []})]
    if isinstance(spec, (list, tuple)):
        return [("split", {"X": [x]}, {"Out": outs}, {"axis": axis, "num": 0, "sections": _intlist(spec)})]
    size = ctx.shape(x)[axis]
    if isinstance(size, SymDim):
        raise LoweringError("split of a symbolic dim by chunk size")
    secs = [int(spec)] * (int(size) // int(spec)) + ([int(size) % int(spec)] if int(size) % int(spec) else [])
    return [("split", {"X": [x]}, {"Out": outs}, {"axis": axis, "num": 0, "sections": secs})]


@rule(T.__getitem__)
def _getitem(ctx, op):
    x = _name(op.args[0])
    idx = op.args[1]
    idx = idx if isinstance(idx, tuple) else (idx,)
    shape = ctx.shape(x)
    axes, starts, ends, dec, strides = [], [], [], [], []
    d = 0
    nd = len(shape)
    for i, it in enumerate(idx):
        if it is Ellipsis:
            d = nd - (len(idx) - i - 1)
            continue
        if it is None:
            raise LoweringError("indexing with None")
        if isinstance(it, int):
            axes.append(d)
            starts.append(it)
            ends.append(it + 1 if it != -1 else 2 ** 31 - 1)
            strides.append(1)
            dec.append(d)
        elif isinstance(it, slice):
            if it.start is None and it.stop is None and it.step in (None, 1):
                d += 1
                continue
            st = 0 if it.start is None else it.start
            en = 2 ** 31 - 1 if it.stop is None else it.stop
            if isinstance(st, SymDim) or isinstance(en, SymDim) or not isinstance(st, int) \
                    or not isinstance(en, int):
                raise LoweringError("slice bound is symbolic / a tensor")
            axes.append(d)
            starts.append(st)
            ends.append(en)
            strides.append(1 if it.step is None else int(it.step))
        else:
            raise LoweringError(f"advanced indexing {it!r}")
        d += 1
    out = _outs(op)[0]
    if not axes:
        return [("assign", {"X": [x]}, {"Out": [out]}, {})]
    if any(s != 1 for s in strides):
        return [("strided_slice", {"Input": [x]}, {"Out": [out]},
                 {"axes": axes, "starts": starts, "ends": ends, "strides": strides,
                  "decrease_axis": dec, "infer_flags": [1] * len(axes)})]
    return [("slice", {"Input": [x]}, {"Out": [out]},
             {"axes": axes, "starts": starts, "ends": ends, "decrease_axis": dec,
              "infer_flags": [1] * len(axes)})]


@rule(T.expand)
def _expand(ctx, op):
    x = _name(op.args[0])
    shape = op.args[1:] if len(op.args) > 2 or not isinstance(op.args[1], (list, tuple)) else op.args[1]
    out = []
    for s in shape:
        out.append(-1 if isinstance(s, SymDim) else int(s))
    return [("expand_v2", {"X": [x]}, {"Out": [_outs(op)[0]]}, {"shape": out})]


@rule(T.expand_as)
def _expand_as(ctx, op):
    x, y = _name(op.args[0]), _name(op.args[1])
    return [("expand_as_v2", {"X": [x], "Y": [y]}, {"Out": [_outs(op)[0]]},
             {"target_shape": ctx.dims(y)})]


@rule(torch.mean, T.mean, torch.sum, T.sum, torch.amax, torch.amin)
def _reduce(ctx, op):
    ptype = {torch.mean: "reduce_mean", T.mean: "reduce_mean", torch.sum: "reduce_sum",
             T.sum: "reduce_sum", torch.amax: "reduce_max", torch.amin: "reduce_min"}[op.func]
    x = _name(op.args[0])
    dim = _arg(op, 1, "dim")
    keep = bool(_arg(op, 2, "keepdim", False))
    if isinstance(dim, torch.dtype):
        raise LoweringError("reduce with dtype")
    if dim is None:
        return [(ptype, {"X": [x]}, {"Out": [_outs(op)[0]]}, {"dim": [], "keep_dim": keep,
                                                              "reduce_all": True})]
    return [(ptype, {"X": [x]}, {"Out": [_outs(op)[0]]},
             {"dim": _intlist(dim), "keep_dim": keep, "reduce_all": False})]


@rule(torch.max, T.max, torch.min, T.min)
def _max_min(ctx, op):
    """Full reduce (``torch.max(x)``) or elementwise against a second tensor; the
    (values, indices) form with a dim has no single Paddle op."""
    is_max = op.func in (torch.max, T.max)
    x = _name(op.args[0])
    other = _arg(op, 1, "other") if len(op.args) > 1 or "other" in op.kwargs else None
    if other is None and "dim" not in op.kwargs:
        return [("reduce_max" if is_max else "reduce_min", {"X": [x]}, {"Out": [_outs(op)[0]]},
                 {"dim": [], "keep_dim": False, "reduce_all": True})]
    if other is not None and not isinstance(other, int):
        return [("elementwise_max" if is_max else "elementwise_min", {"X": [x], "Y": [_name(other)]},
                 {"Out": [_outs(op)[0]]}, {"axis": -1})]
    raise LoweringError("max/min along a dim returns (values, indices)")


@rule(F.softmax, torch.softmax, T.softmax)
def _softmax(ctx, op):
    return [("softmax", {"X": [_name(op.args[0])]}, {"Out": [_outs(op)[0]]},
             {"axis": int(_arg(op, 1, "dim", -1))})]


@rule(F.layer_norm)
def _torch_ln(ctx, op):
    x = _name(op.args[0])
    ns = _intlist(_arg(op, 1, "normalized_shape"))
    w, b = _arg(op, 2, "weight"), _arg(op, 3, "bias")
    eps = float(_arg(op, 4, "eps", 1e-5))
    return [_ln_desc(ctx, x, w, b, eps, _outs(op)[0], ctx.ndim(x) - len(ns))]


def _ln_desc(ctx, x, w, b, eps, out, bna=None):
    ins = {"X": [x]}
    if w is not None:
        ins["Scale"] = [_name(w)]
    if b is not None:
        ins["Bias"] = [_name(b)]
    bna = ctx.ndim(x) - 1 if bna is None else bna
    return ("layer_norm", ins, {"Y": [out], "Mean": [ctx.tmp(dims=[-1])],
                                "Variance": [ctx.tmp(dims=[-1])]},
            {"epsilon": eps, "begin_norm_axis": bna})


@rule("layer_norm")
def _fw_ln(ctx, op):
    x = _name(_arg(op, 0, "x"))
    return [_ln_desc(ctx, x, _arg(op, 1, "weight"), _arg(op, 2, "bias"),
                     float(_arg(op, 3, "eps", 1e-5)), _outs(op)[0])]


@rule("skip_layernorm")
def _fw_add_ln(ctx, op):
    """fused_add_layer_norm(x, residual, w, b, eps, x_bias, dropout_p, training) -> (LN(h), h)."""
    x, res = _name(_arg(op, 0, "x")), _arg(op, 1, "residual")
    w, b = _arg(op, 2, "weight"), _arg(op, 3, "bias")
    eps = float(_arg(op, 4, "eps", 1e-5))
    xb = _arg(op, 5, "x_bias")
    p, training = float(_arg(op, 6, "dropout_p", 0.0)), _arg(op, 7, "training", True)
    y, h = _outs(op)
    res_ops, cur = [], x
    if xb is not None:
        t = ctx.tmp(like=x)
        res_ops.append(("elementwise_add", {"X": [cur], "Y": [_name(xb)]}, {"Out": [t]}, {"axis": -1}))
        cur = t
    if p > 0 and training:
        t = ctx.tmp(like=x)
        res_ops.append(("dropout", {"X": [cur]}, {"Out": [t], "Mask": [ctx.tmp(dims=[-1], dtype=20)]},
                        {"dropout_prob": p, "is_test": False,
                         "dropout_implementation": "upscale_in_train"}))
        cur = t
    if res is not None:
        res_ops.append(("elementwise_add", {"X": [_name(res)], "Y": [cur]}, {"Out": [h]}, {"axis": -1}))
    else:
        res_ops.append(("assign", {"X": [cur]}, {"Out": [h]}, {}))
    res_ops.append(_ln_desc(ctx, h, w, b, eps, y))
    return res_ops


def _rms_desc(ctx, x, w, eps, out):
    sq, ms, r, n = (ctx.tmp(like=x) for _ in range(4))
    ops = [("elementwise_mul", {"X": [x], "Y": [x]}, {"Out": [sq]}, {"axis": -1}),
           ("reduce_mean", {"X": [sq]}, {"Out": [ms]}, {"dim": [-1], "keep_dim": True,
                                                         "reduce_all": False}),
           ("scale", {"X": [ms]}, {"Out": [r]}, {"scale": 1.0, "bias": eps, "bias_after_scale": True}),
           ("rsqrt", {"X": [r]}, {"Out": [n]}, {})]
    if w is None:
        return ops + [("elementwise_mul", {"X": [x], "Y": [n]}, {"Out": [out]}, {"axis": -1})]
    t = ctx.tmp(like=x)
    return ops + [("elementwise_mul", {"X": [x], "Y": [n]}, {"Out": [t]}, {"axis": -1}),
                  ("elementwise_mul", {"X": [t], "Y": [_name(w)]}, {"Out": [out]}, {"axis": -1})]


@rule("rms_norm")
def _fw_rms(ctx, op):
    return _rms_desc(ctx, _name(_arg(op, 0, "x")), _arg(op, 1, "weight"),
                     float(_arg(op, 2, "eps", 1e-6)), _outs(op)[0])


_ACT_OPS = {0: None, 1: ("gelu", {"approximate": True}), 2: ("gelu", {"approximate": False}),
            3: ("relu", {}), 4: ("silu", {})}
_ACT_NAMES = {"none": 0, "identity": 0, "gelu_tanh": 1, "gelu": 2, "relu": 3, "silu": 4, "swish": 4}


@rule("fused_bias_act")
def _fw_bias_act(ctx, op):
    x, b = _name(_arg(op, 0, "x")), _arg(op, 1, "bias")
    act = _ACT_OPS[_ACT_NAMES[_arg(op, 2, "act", "gelu")]]
    out = _outs(op)[0]
    res, cur = [], x
    if b is not None:
        t = out if act is None else ctx.tmp(like=x)
        res.append(("elementwise_add", {"X": [x], "Y": [_name(b)]}, {"Out": [t]}, {"axis": -1}))
        cur = t
    if act is None:
        return res or [("assign", {"X": [x]}, {"Out": [out]}, {})]
    return res + [(act[0], {"X": [cur]}, {"Out": [out]}, dict(act[1]))]


@rule("gelu")
def _fw_gelu(ctx, op):
    return [("gelu", {"X": [_name(op.args[0])]}, {"Out": [_outs(op)[0]]},
             {"approximate": bool(_arg(op, 1, "approximate", False))})]


@rule("dropout", F.dropout)
def _dropout(ctx, op):
    x = _name(op.args[0])
    p = float(_arg(op, 1, "p", 0.5))
    training = _arg(op, 2, "training", True)
    return [("dropout", {"X": [x]}, {"Out": [_outs(op)[0]], "Mask": [ctx.tmp(dims=[-1], dtype=20)]},
             {"dropout_prob": p, "is_test": not training,
              "dropout_implementation": "upscale_in_train"})]


def _flash_desc(ctx, q, k, v, out, causal, scale, mask, p, training):
    D = ctx.dims(q)[-1]
    res = []
    if scale is not None and abs(float(scale) - 1.0 / math.sqrt(D)) > 1e-12:
        qs = ctx.tmp(like=q)  # flash_attn has no scale attr: fold the ratio into q
        res.append(("scale", {"X": [q]}, {"Out": [qs]},
                    {"scale": float(scale) * math.sqrt(D), "bias": 0.0, "bias_after_scale": True}))
        q = qs
    ins = {"q": [q], "k": [k], "v": [v]}
    if mask is not None:
        ins["attn_mask"] = [_name(mask)]
    res.append(("flash_attn", ins,
                {"out": [out], "softmax": [ctx.tmp(dims=[-1])], "softmax_lse": [ctx.tmp(dims=[-1])],
                 "seed_offset": [ctx.tmp(dims=[2], dtype=3)]},
                {"dropout": float(p), "causal": bool(causal), "return_softmax": False,
                 "is_test": not training, "rng_name": ""}))
    return res


@rule("flash_attn")
def _fw_flash(ctx, op):
    q, k, v = (_name(_arg(op, i, n)) for i, n in enumerate(("q", "k", "v")))
    return _flash_desc(ctx, q, k, v, _outs(op)[0], _arg(op, 3, "causal", False), _arg(op, 4, "scale"),
                       _arg(op, 5, "attn_mask"), float(_arg(op, 6, "dropout_p", 0.0)),
                       _arg(op, 7, "training", True))


@rule("flash_attn_packed")
def _fw_flash_packed(ctx, op):
    qkv = _name(_arg(op, 0, "qkv"))
    hq = int(_arg(op, 1, "num_heads"))
    hk = _arg(op, 2, "num_kv_heads") or hq
    dims = ctx.dims(qkv)
    q = ctx.tmp(like=qkv, dims=dims[:2] + [hq, dims[3]])
    k = ctx.tmp(like=qkv, dims=dims[:2] + [int(hk), dims[3]])
    v = ctx.tmp(like=qkv, dims=dims[:2] + [int(hk), dims[3]])
    return ([("split", {"X": [qkv]}, {"Out": [q, k, v]}, {"axis": 2, "num": 0,
                                                          "sections": [hq, int(hk), int(hk)]})]
            + _flash_desc(ctx, q, k, v, _outs(op)[0], _arg(op, 3, "causal", True), _arg(op, 4, "scale"),
                          None, float(_arg(op, 5, "dropout_p", 0.0)), _arg(op, 6, "training", True)))


@rule("softmax_mask_fuse")
def _fw_softmax_mask(ctx, op):
    x, mask = _name(op.args[0]), _arg(op, 1, "mask")
    scale, causal = float(_arg(op, 2, "scale", 1.0)), bool(_arg(op, 3, "causal", False))
    res, cur = [], x
    if scale != 1.0:
        t = ctx.tmp(like=x)
        res.append(("scale", {"X": [x]}, {"Out": [t]}, {"scale": scale, "bias": 0.0,
                                                        "bias_after_scale": True}))
        cur = t
    out = _outs(op)[0]
    if causal:
        if mask is not None:
            t = ctx.tmp(like=x)
            res.append(("elementwise_add", {"X": [cur], "Y": [_name(mask)]}, {"Out": [t]}, {"axis": -1}))
            cur = t
        return res + [("fused_softmax_mask_upper_triangle", {"X": [cur]}, {"Out": [out]}, {})]
    if mask is not None:
        return res + [("fused_softmax_mask", {"X": [cur], "Mask": [_name(mask)]}, {"Out": [out]}, {})]
    return res + [("softmax", {"X": [cur]}, {"Out": [out]}, {"axis": -1})]


@rule(F.scaled_dot_product_attention)
def _sdpa(ctx, op):
    # [B, H, S, D] layout: transpose into flash_attn's [B, S, H, D] and back
    q, k, v = (_name(op.args[i]) for i in range(3))
    mask = _arg(op, 3, "attn_mask")
    causal = bool(op.kwargs.get("is_causal", False))
    scale = op.kwargs.get("scale")
    res, tr = [], []
    for t in (q, k, v):
        d = ctx.dims(t)
        n = ctx.tmp(like=t, dims=[d[0], d[2], d[1], d[3]])
        res.append(("transpose2", {"X": [t]}, {"Out": [n], "XShape": [ctx.tmp(dims=[-1])]},
                    {"axis": [0, 2, 1, 3]}))
        tr.append(n)
    o = ctx.tmp(like=tr[0])
    res += _flash_desc(ctx, tr[0], tr[1], tr[2], o, causal, scale, mask, 0.0, False)
    res.append(("transpose2", {"X": [o]}, {"Out": [_outs(op)[0]], "XShape": [ctx.tmp(dims=[-1])]},
                {"axis": [0, 2, 1, 3]}))
    return res


@rule(F.embedding)
def _embedding(ctx, op):
    ids, w = _name(op.args[0]), _name(op.args[1])
    pad = _arg(op, 2, "padding_idx")
    return [("lookup_table_v2", {"Ids": [ids], "W": [w]}, {"Out": [_outs(op)[0]]},
             {"padding_idx": -1 if pad is None else int(pad)})]


@rule(torch.conv2d, F.conv2d)
def _conv2d(ctx, op):
    x, w = _name(op.args[0]), _name(op.args[1])
    b = _arg(op, 2, "bias")
    st = _intlist(_arg(op, 3, "stride", 1), 2)
    pad = _arg(op, 4, "padding", 0)
    dil = _intlist(_arg(op, 5, "dilation", 1), 2)
    groups = int(_arg(op, 6, "groups", 1))
    if isinstance(pad, str):
        attrs_pad = {"paddings": [0, 0], "padding_algorithm": pad.upper()}
    else:
        attrs_pad = {"paddings": _intlist(pad, 2), "padding_algorithm": "EXPLICIT"}
    out = _outs(op)[0]
    conv_out = out if b is None else ctx.tmp(like=out)
    res = [("conv2d", {"Input": [x], "Filter": [w]}, {"Output": [conv_out]},
            dict(strides=st, dilations=dil, groups=groups, data_format="NCHW", **attrs_pad))]
    if b is not None:
        res.append(("elementwise_add", {"X": [conv_out], "Y": [_name(b)]}, {"Out": [out]}, {"axis": 1}))
    return res


@rule(F.batch_norm)
def _batch_norm(ctx, op):
    x, rm, rv = _name(op.args[0]), _arg(op, 1, "running_mean"), _arg(op, 2, "running_var")
    w, b = _arg(op, 3, "weight"), _arg(op, 4, "bias")
    training = bool(_arg(op, 5, "training", False))
    mom, eps = float(_arg(op, 6, "momentum", 0.1)), float(_arg(op, 7, "eps", 1e-5))
    if rm is None or w is None or b is None:
        raise LoweringError("batch_norm without running stats / affine params")
    out = _outs(op)[0]
    return [("batch_norm", {"X": [x], "Scale": [_name(w)], "Bias": [_name(b)], "Mean": [_name(rm)],
                            "Variance": [_name(rv)]},
             {"Y": [out], "MeanOut": [_name(rm)], "VarianceOut": [_name(rv)],
              "SavedMean": [ctx.tmp(dims=[-1])], "SavedVariance": [ctx.tmp(dims=[-1])]},
             {"epsilon": eps, "momentum": 1.0 - mom, "is_test": not training, "data_layout": "NCHW",
              "use_global_stats": not training})]


@rule(F.max_pool2d, F.avg_pool2d, F.adaptive_avg_pool2d, F.adaptive_max_pool2d)
def _pool(ctx, op):
    x = _name(op.args[0])
    out = _outs(op)[0]
    if op.func in (F.adaptive_avg_pool2d, F.adaptive_max_pool2d):
        k = _intlist(_arg(op, 1, "output_size"), 2)
        ptype = "avg" if op.func is F.adaptive_avg_pool2d else "max"
        return [("pool2d", {"X": [x]}, {"Out": [out]},
                 {"pooling_type": ptype, "ksize": k, "adaptive": True, "global_pooling": False,
                  "strides": [1, 1], "paddings": [0, 0], "ceil_mode": False, "exclusive": True,
                  "data_format": "NCHW", "padding_algorithm": "EXPLICIT"})]
    k = _intlist(_arg(op, 1, "kernel_size"), 2)
    st = _arg(op, 2, "stride")
    st = k if st is None or st == [] else _intlist(st, 2)
    pd = _intlist(_arg(op, 3, "padding", 0), 2)
    if op.func is F.max_pool2d:
        ceil = bool(_arg(op, 5, "ceil_mode", False))
        excl = True
    else:
        ceil = bool(_arg(op, 4, "ceil_mode", False))
        excl = not bool(_arg(op, 5, "count_include_pad", True))
    return [("pool2d", {"X": [x]}, {"Out": [out]},
             {"pooling_type": "max" if op.func is F.max_pool2d else "avg", "ksize": k, "strides": st,
              "paddings": pd, "ceil_mode": ceil, "exclusive": excl, "adaptive": False,
              "global_pooling": False, "data_format": "NCHW", "padding_algorithm": "EXPLICIT"})]


@rule("softmax_with_cross_entropy")
def _fw_xent(ctx, op):
    logits, labels = _name(op.args[0]), _name(op.args[1])
    ign = int(_arg(op, 2, "ignore_index", -100))
    lab2 = ctx.tmp(like=labels, dims=ctx.dims(labels) + [1])
    loss2 = ctx.tmp(like=logits, dims=ctx.dims(labels) + [1])
    return [("unsqueeze2", {"X": [labels]}, {"Out": [lab2], "XShape": [ctx.tmp(dims=[-1])]},
             {"axes": [ctx.ndim(labels)]}),
            ("softmax_with_cross_entropy", {"Logits": [logits], "Label": [lab2]},
             {"Softmax": [ctx.tmp(like=logits)], "Loss": [loss2]},
             {"soft_label": False, "ignore_index": ign, "axis": -1, "numeric_stable_mode": True}),
            ("squeeze2", {"X": [loss2]}, {"Out": [_outs(op)[0]], "XShape": [ctx.tmp(dims=[-1])]},
             {"axes": [ctx.ndim(labels)]})]


@rule("weight_only_linear")
def _fw_wol(ctx, op):
    x, w = _name(_arg(op, 0, "x")), _name(_arg(op, 1, "weight"))
    b, s = _arg(op, 2, "bias"), _arg(op, 3, "weight_scale")
    wd = _arg(op, 4, "weight_dtype", "int8")
    ins = {"x": [x], "weight": [w]}
    if b is not None:
        ins["bias"] = [_name(b)]
    if s is not None:
        ins["weight_scale"] = [_name(s)]
    act = _arg(op, 5, "act_method", "none")
    if _arg(op, 6, "ln") is not None or _arg(op, 7, "resid") is not None:
        raise LoweringError("weight_only_linear with fused ln / resid (decode-only form)")
    return [("weight_only_linear", ins, {"out": [_outs(op)[0]]},
             {"weight_dtype": str(wd), "act_method": str(act)})]


# --------------------------------------------------------------------------- driver
def rule_for(op):
    r = RULES.get(op.func) if op.func is not None else None
    if r is None:
        r = RULES.get(op.type)
    return r


def lower(block, op):
    """-> (list of (type, inputs, outputs, attrs), new temp vars) for one recorded op."""
    r = rule_for(op)
    if r is None:
        raise LoweringError(f"no Paddle op lowering for recorded op '{op.type}' "
                            f"({getattr(op.func, '__qualname__', op.func)!r})")
    ctx = _Ctx(block, op)
    try:
        descs = r(ctx, op)
    except LoweringError:
        raise
    except (TypeError, IndexError, KeyError, ValueError, AttributeError) as e:
        raise LoweringError(f"cannot lower '{op.type}' ({op.func!r}): {e}") from e
    return descs, ctx.new_vars


def attr_desc(name, v):
    """Python value -> framework.proto OpDesc.Attr dict with the natural Paddle type."""
    A = proto.ATTR
    if isinstance(v, bool):
        return {"name": name, "type": A["BOOLEAN"], "b": v}
    if isinstance(v, int):
        if -2 ** 31 <= v < 2 ** 31:
            return {"name": name, "type": A["INT"], "i": v}
        return {"name": name, "type": A["LONG"], "l": v}
    if isinstance(v, float):
        return {"name": name, "type": A["FLOAT"], "f": v}
    if isinstance(v, str):
        return {"name": name, "type": A["STRING"], "s": v}
    if isinstance(v, (list, tuple)):
        if all(isinstance(e, bool) for e in v) and v:
            return {"name": name, "type": A["BOOLEANS"], "bools": list(v)}
        if all(isinstance(e, int) and not isinstance(e, bool) for e in v):
            return {"name": name, "type": A["INTS"], "ints": list(v)}
        if all(isinstance(e, (int, float)) for e in v):
            return {"name": name, "type": A["FLOATS"], "floats": [float(e) for e in v]}
        if all(isinstance(e, str) for e in v):
            return {"name": name, "type": A["STRINGS"], "strings": list(v)}
    raise LoweringError(f"attribute {name}={v!r} has no Paddle attr type")
