"""Paddle operator registry: slot-based kernels for Paddle op types.

Parity: the reference's op definitions (`paddle/fluid/operators/*_op.cc`, `paddle/phi/ops/`,
`phi/api/yaml/legacy_ops.yaml`) — same op type names, input/output slot names and attributes —
so programs produced by Paddle (``feed`` / ``matmul_v2`` / ``elementwise_add`` / ``layer_norm`` /
``conv2d`` / ``fc`` ...) execute here, and the inference IR passes (`inference/passes.py`) can
rewrite subgraphs into the fused types registered below (``fc``, ``skip_layernorm``,
``fused_bias_act``, ``flash_attn_packed``), which dispatch to the hand-written HIP kernels.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import proto
from .framework import VarRef

REGISTRY = {}
INPLACE_OUT_OPS = {"write_to_array"}
MISSING_OK_OPS = {"select_input", "c_broadcast"}
DEVICE = [torch.device("cpu")]  # device of the running Executor (creation ops allocate there)


def register(*names):
    def deco(fn):
        for n in names:
            REGISTRY[n] = fn
        return fn
    return deco


def _dt(code):
    inv = {v: k for k, v in proto.VT.items()}
    from ..framework.dtype import to_torch_dtype
    return to_torch_dtype(inv.get(int(code), "float32"))


def _bcast(x, y, axis):
    if axis is None or axis == -1 or y.dim() == x.dim():
        return y
    shape = [1] * x.dim()
    for i, s in enumerate(y.shape):
        shape[axis + i] = s
    return y.reshape(shape)


def run_paddle_op(op, sub, env, scope):
    fn = REGISTRY.get(op.type)
    if fn is None:
        raise NotImplementedError(f"Paddle op '{op.type}' has no kernel in paddle_infer_amd")
    if op.type in MISSING_OK_OPS:  # e.g. select_input: the branch not taken never wrote its var
        def get(n):
            try:
                return sub(VarRef(n))
            except KeyError:
                return None
        ins = {k: [get(n) for n in v] for k, v in op.paddle_inputs.items()}
    else:
        ins = {k: [sub(VarRef(n)) for n in v] for k, v in op.paddle_inputs.items()}
    if op.type in INPLACE_OUT_OPS:  # ops that update their output variable in place (arrays)
        ins["__out__"] = [env.get(n) for n in op.paddle_outputs.get("Out", [])]
    outs = fn(ins, op.attrs)
    for slot, names in op.paddle_outputs.items():
        vals = outs.get(slot)
        if vals is None:
            continue
        vals = vals if isinstance(vals, (list, tuple)) else [vals]
        for n, v in zip(names, vals):
            env[n] = v


# matmul-family ops lower to ops.gemm.matmul: bf16 / fp16 on the framework's own GEMMs (skinny
# MFMA kernel / assembly GEMM / batched assembly GEMM), transposes folded into the kernel layouts
@register("matmul_v2")
def _matmul_v2(ins, a):
    from ..ops.gemm import matmul as _mm
    return {"Out": _mm(ins["X"][0], ins["Y"][0], bool(a.get("trans_x")), bool(a.get("trans_y")))}


@register("matmul")
def _matmul(ins, a):
    from ..ops.gemm import matmul as _mm
    alpha = a.get("alpha", 1.0)
    return {"Out": _mm(ins["X"][0], ins["Y"][0], bool(a.get("transpose_X")),
                       bool(a.get("transpose_Y")), 1.0 if alpha is None else float(alpha))}


@register("mul")
def _mul(ins, a):
    from ..ops.gemm import matmul as _mm
    x, y = ins["X"][0], ins["Y"][0]
    xn = a.get("x_num_col_dims", 1)
    x2 = x.reshape(int(np.prod(x.shape[:xn])), -1)
    out = _mm(x2, y.reshape(x2.shape[1], -1))
    return {"Out": out.reshape(*x.shape[:xn], -1)}


for _name, _f in [("elementwise_add", torch.add), ("elementwise_sub", torch.sub),
                  ("elementwise_mul", torch.mul), ("elementwise_div", torch.true_divide),
                  ("elementwise_pow", torch.pow), ("elementwise_max", torch.maximum),
                  ("elementwise_min", torch.minimum)]:
    register(_name)(lambda ins, a, _f=_f: {"Out": _f(ins["X"][0], _bcast(ins["X"][0], ins["Y"][0], a.get("axis", -1)))})

for _name, _f in [("relu", F.relu), ("sigmoid", torch.sigmoid), ("tanh", torch.tanh), ("silu", F.silu),
                  ("swish", F.silu), ("hard_swish", F.hardswish), ("relu6", F.relu6), ("exp", torch.exp),
                  ("sqrt", torch.sqrt), ("rsqrt", torch.rsqrt), ("abs", torch.abs), ("log", torch.log),
                  ("floor", torch.floor), ("assign", lambda t: t.clone()), ("square", torch.square)]:
    register(_name)(lambda ins, a, _f=_f: {"Out": _f(ins["X"][0])})


@register("gelu")
def _gelu(ins, a):
    from .. import ops
    return {"Out": ops.gelu(ins["X"][0], bool(a.get("approximate", False)))}


@register("leaky_relu")
def _leaky(ins, a):
    return {"Out": F.leaky_relu(ins["X"][0], a.get("alpha", 0.02))}


@register("softmax")
def _softmax(ins, a):
    x = ins["X"][0]
    axis = a.get("axis", -1)
    if axis in (-1, x.dim() - 1):
        from .. import ops
        return {"Out": ops.fused_softmax_mask(x)}
    return {"Out": torch.softmax(x, axis)}


@register("layer_norm")
def _layer_norm(ins, a):
    from .. import ops
    x = ins["X"][0]
    bna = a.get("begin_norm_axis", x.dim() - 1)
    scale = ins.get("Scale", [None])[0] if ins.get("Scale") else None
    bias = ins.get("Bias", [None])[0] if ins.get("Bias") else None
    if bna == x.dim() - 1:
        y = ops.layer_norm(x, scale, bias, a.get("epsilon", 1e-5))
    else:
        y = F.layer_norm(x, x.shape[bna:], scale.reshape(x.shape[bna:]) if scale is not None else None,
                         bias.reshape(x.shape[bna:]) if bias is not None else None, a.get("epsilon", 1e-5))
    return {"Y": y}


@register("skip_layernorm")
def _skip_ln(ins, a):
    from .. import ops
    y, _ = ops.fused_add_layer_norm(ins["X"][0], ins["Y"][0], ins["Scale"][0], ins["Bias"][0],
                                    a.get("epsilon", 1e-5), None, 0.0, False, need_residual=False)
    return {"Out": y}


@register("batch_norm")
def _bn(ins, a):
    y = F.batch_norm(ins["X"][0], ins["Mean"][0], ins["Variance"][0], ins["Scale"][0], ins["Bias"][0],
                     False, 0.0, a.get("epsilon", 1e-5))
    return {"Y": y}


def _pads(p, nd):
    p = list(p or [0] * nd)
    if len(p) == 2 * nd and all(p[2 * i] == p[2 * i + 1] for i in range(nd)):
        p = p[0::2]
    return p


def _conv_padding(a):
    pad = a.get("padding_algorithm", "EXPLICIT")
    return "same" if pad == "SAME" else (0 if pad == "VALID" else _pads(a.get("paddings"), 2))


@register("conv2d", "depthwise_conv2d")
def _conv2d(ins, a):
    """Through the framework's conv dispatch (`nn.functional.conv2d`): GPU tensors run the own
    HIP conv kernels (`ops/conv.py` conv2d_any), CPU the reference path."""
    from ..nn import functional as PF
    x, w = ins["Input"][0], ins["Filter"][0]
    y = PF.conv2d(x, w, ins["Bias"][0] if ins.get("Bias") else None, a.get("strides", [1, 1]),
                  _conv_padding(a), a.get("dilations", [1, 1]), a.get("groups", 1),
                  a.get("data_format", "NCHW") if a.get("data_format") in ("NCHW", "NHWC") else "NCHW")
    return {"Output": y}


_FUSION_ACTS = {"relu": F.relu, "relu6": F.relu6, "sigmoid": torch.sigmoid, "tanh": torch.tanh,
                "leaky_relu": F.leaky_relu, "swish": F.silu, "silu": F.silu, "gelu": F.gelu,
                "identity": None, "": None}


@register("conv2d_fusion", "fused_conv2d_add_act")
def _conv2d_fusion(ins, a):
    """Reference `fused/conv_fusion_op.cc` (conv2d_fusion): Output = act(conv(Input, Filter) +
    Bias [+ ResidualData]); the target of conv_elementwise_add(2)_act_fuse_pass."""
    y = _conv2d(ins, a)["Output"]
    if ins.get("ResidualData") and ins["ResidualData"][0] is not None:
        y = y + ins["ResidualData"][0]
    fn = _FUSION_ACTS.get(a.get("activation", "relu"), None)
    return {"Output": fn(y) if fn is not None else y}


@register("conv2d_transpose")
def _conv2d_t(ins, a):
    from ..nn import functional as PF
    y = PF.conv2d_transpose(ins["Input"][0], ins["Filter"][0], None, a.get("strides", [1, 1]),
                            _pads(a.get("paddings"), 2), a.get("output_padding") or 0,
                            a.get("groups", 1), a.get("dilations", [1, 1]))
    return {"Output": y}


@register("pool2d")
def _pool2d(ins, a):
    x = ins["X"][0]
    k = a.get("ksize", [1, 1])
    if a.get("global_pooling"):
        k = list(x.shape[2:])
    if a.get("adaptive"):
        fn = F.adaptive_avg_pool2d if a.get("pooling_type", "max") == "avg" else F.adaptive_max_pool2d
        return {"Out": fn(x, k)}
    st, pd = a.get("strides", k), _pads(a.get("paddings"), 2)
    if a.get("pooling_type", "max") == "max":
        return {"Out": F.max_pool2d(x, k, st, pd, ceil_mode=bool(a.get("ceil_mode")))}
    return {"Out": F.avg_pool2d(x, k, st, pd, bool(a.get("ceil_mode")), not a.get("exclusive", True))}


@register("reshape2", "reshape")
def _reshape(ins, a):
    x = ins["X"][0]
    shape = list(a.get("shape", []))
    if ins.get("Shape"):
        shape = [int(v) for v in ins["Shape"][0].tolist()]
    shape = [x.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return {"Out": x.reshape(shape)}


@register("transpose2", "transpose")
def _transpose(ins, a):
    return {"Out": ins["X"][0].permute(*a.get("axis"))}


@register("flatten2", "flatten")
def _flatten2(ins, a):
    """Reference `flatten_op.cc` (flatten2): [d0..d(axis-1)] x [d(axis)..] as a 2-D tensor."""
    x = ins["X"][0]
    ax = int(a.get("axis", 1))
    lead = int(np.prod(x.shape[:ax])) if ax > 0 else 1
    return {"Out": x.reshape(lead, -1)}


@register("fusion_transpose_flatten_concat")
def _fusion_tfc(ins, a):
    """Reference `fused/fusion_transpose_flatten_concat_op.cc`: per input transpose(trans_axis) →
    flatten(flatten_axis) → concat(concat_axis)."""
    ax, fa = list(a.get("trans_axis")), int(a.get("flatten_axis", 1))
    parts = []
    for x in ins["X"]:
        t = x.permute(ax)
        lead = int(np.prod(t.shape[:fa])) if fa > 0 else 1
        parts.append(t.reshape(lead, -1))
    return {"Out": torch.cat(parts, int(a.get("concat_axis", 0)))}


@register("flatten_contiguous_range")
def _flatten(ins, a):
    return {"Out": torch.flatten(ins["X"][0], a.get("start_axis", 1), a.get("stop_axis", -1))}


@register("squeeze2")
def _squeeze(ins, a):
    x = ins["X"][0]
    axes = [ax % x.dim() for ax in a.get("axes", [])] or [i for i, s in enumerate(x.shape) if s == 1]
    for ax in sorted(axes, reverse=True):
        if x.shape[ax] == 1:
            x = x.squeeze(ax)
    return {"Out": x}


@register("unsqueeze2")
def _unsqueeze(ins, a):
    x = ins["X"][0]
    for ax in sorted(a.get("axes", [])):
        x = x.unsqueeze(ax)
    return {"Out": x}


@register("concat")
def _concat(ins, a):
    return {"Out": torch.cat(ins["X"], a.get("axis", 0))}


@register("split")
def _split(ins, a):
    x = ins["X"][0]
    axis = a.get("axis", 0)
    sec = a.get("sections") or []
    if sec:
        if -1 in sec:
            sec = list(sec)
            sec[sec.index(-1)] = x.shape[axis] - sum(s for s in sec if s != -1)
        return {"Out": list(torch.split(x, sec, axis))}
    return {"Out": list(torch.chunk(x, a.get("num", 1), axis))}


@register("slice")
def _slice(ins, a):
    x = ins["Input"][0]
    sl = [slice(None)] * x.dim()
    for ax, s, e in zip(a.get("axes", []), a.get("starts", []), a.get("ends", [])):
        sl[ax] = slice(s, min(e, x.shape[ax]) if e > 0 else e)
    out = x[tuple(sl)]
    for ax in sorted(a.get("decrease_axis", []) or [], reverse=True):
        out = out.squeeze(ax)
    return {"Out": out}


@register("scale")
def _scale(ins, a):
    x = ins["X"][0]
    s, b = a.get("scale", 1.0), a.get("bias", 0.0)
    return {"Out": x * s + b if a.get("bias_after_scale", True) else (x + b) * s}


@register("cast")
def _cast(ins, a):
    return {"Out": ins["X"][0].to(_dt(a.get("out_dtype", 5)))}


@register("dropout")
def _dropout(ins, a):
    x = ins["X"][0]
    p = a.get("dropout_prob", 0.5)
    if a.get("dropout_implementation", "downgrade_in_infer") == "downgrade_in_infer":
        return {"Out": x * (1.0 - p)}
    return {"Out": x}


@register("lookup_table_v2", "lookup_table")
def _lookup(ins, a):
    ids = ins["Ids"][0].long()
    if ids.dim() > 1 and ids.shape[-1] == 1 and a.get("_squeeze_last", False):
        ids = ids.squeeze(-1)
    # Paddle semantics (reference `embedding_kernel.cu`): padding rows read as zeros; on the GPU the
    # own gather kernels (`paddle_infer_amd.nn.functional.embedding` → ops/embedding.py)
    from ..nn import functional as PF
    pad = a.get("padding_idx")
    return {"Out": PF.embedding(ids, ins["W"][0], pad if pad is not None and pad >= 0 else None)}


@register("fill_constant")
def _fill(ins, a):
    return {"Out": torch.full(a.get("shape", [1]), a.get("value", 0.0), dtype=_dt(a.get("dtype", 5)),
                              device=DEVICE[-1])}


for _name, _f in [("reduce_mean", torch.mean), ("reduce_sum", torch.sum), ("reduce_max", torch.amax),
                  ("reduce_min", torch.amin)]:
    def _mk(_f=_f):
        def op(ins, a):
            x = ins["X"][0]
            if a.get("reduce_all") or not a.get("dim"):
                out = _f(x)
                return {"Out": out.reshape([1] * x.dim()) if a.get("keep_dim") else out}
            return {"Out": _f(x, dim=tuple(a["dim"]), keepdim=bool(a.get("keep_dim")))}
        return op
    register(_name)(_mk())


@register("arg_max")
def _argmax(ins, a):
    return {"Out": torch.argmax(ins["X"][0], a.get("axis", -1), bool(a.get("keepdims")))}


@register("top_k_v2")
def _topk(ins, a):
    v, i = torch.topk(ins["X"][0], a.get("k", 1), a.get("axis", -1), a.get("largest", True))
    return {"Out": v, "Indices": i}


@register("softmax_with_cross_entropy")
def _swce(ins, a):
    lg, lab = ins["Logits"][0], ins["Label"][0]
    loss = F.cross_entropy(lg.reshape(-1, lg.shape[-1]).float(), lab.reshape(-1).long(),
                           ignore_index=a.get("ignore_index", -100), reduction="none")
    return {"Loss": loss.reshape(*lab.shape[:-1], 1) if lab.dim() == lg.dim() else loss,
            "Softmax": torch.softmax(lg, -1)}


# ---------------------------------------------------------------- fused (IR-pass targets)
from ..inference import ln_defer as _ln_defer  # noqa: E402


def _tanh_small_ok(x2, w, b):
    """fc + tanh on the skinny GEMM's tanh epilogue: 16-bit CUDA rows it takes, with a bias."""
    if not (x2.is_cuda and x2.dtype in (torch.bfloat16, torch.float16) and w.dim() == 2 and w.dtype == x2.dtype
            and b is not None and b.dtype == x2.dtype and b.numel() == w.shape[1]):
        return False
    from ..ops.gemm import use_small
    M, K = x2.shape
    N = w.shape[1]
    return use_small(M, N, K) and K % 64 == 0 and N % 4 == 0 and w.is_contiguous()


@register("fc")
def _fc(ins, a):
    """Reference `fc_op.cc`: Out = act(Input @ W + Bias) (in_num_col_dims flattening)."""
    from ..ops.linear import linear
    from .. import ops
    x, w = ins["Input"][0], ins["W"][0]
    b = ins["Bias"][0] if ins.get("Bias") else None
    nc = a.get("in_num_col_dims", x.dim() - 1)
    act = a.get("activation_type", "")
    if _ln_defer.of(x) is not None:  # raw rows of a post-LN producer: LayerNorm folded in here
        y = (_ln_defer.linear(x, w, b, act or "none") if nc == x.dim() - 1
             and act in ("", "gelu", "relu", "gelu_tanh") else None)
        if y is not None:
            return {"Out": y}
        x = _ln_defer.materialize(x)
    x2 = x.reshape(int(np.prod(x.shape[:nc])), -1)
    if act in ("gelu", "relu", "silu", "gelu_tanh") and x2.is_cuda and x2.dtype in (torch.bfloat16,
                                                                                    torch.float16):
        from ..ops.linear import linear_bias_act
        y = linear_bias_act(x2, w, b, act) if b is not None else ops.bias_act(linear(x2, w, None), b, act)
    elif act == "tanh" and _tanh_small_ok(x2, w, b):  # e.g. the BERT pooler: tanh in the epilogue
        from ..ops.gemm import small_gemm
        from ..ops.linear import transposed
        y = small_gemm(x2.contiguous(), transposed(w), bias=b.reshape(-1), act="tanh")
    elif act in ("gelu", "relu", "silu", "gelu_tanh") and x2.is_cuda and x2.dtype == torch.float32:
        y = ops.bias_act(linear(x2, w, None), b, act)  # split-bf16 GEMM + the f32 bias-act kernel
    else:
        y = linear(x2, w, b)
        if act:
            y = {"relu": F.relu, "gelu": F.gelu, "silu": F.silu, "tanh": torch.tanh,
                 "sigmoid": torch.sigmoid}[act](y)
    return {"Out": y.reshape(*x.shape[:nc], -1)}


@register("fused_bias_act")
def _fused_bias_act(ins, a):
    from .. import ops
    return {"Out": ops.bias_act(ins["X"][0], ins["Bias"][0] if ins.get("Bias") else None,
                                a.get("act_method", "gelu"))}


@register("flash_attn_packed")
def _flash_packed(ins, a):
    from .. import ops
    qkv = ins["QKV"][0]
    return {"Out": ops.flash_attention_packed(qkv, a["num_heads"], a.get("num_kv_heads") or a["num_heads"],
                                              causal=bool(a.get("causal", False)), scale=a.get("scale"))}


@register("fused_embedding_eltwise_layernorm")
def _emb_ln(ins, a):
    """Reference `fused_embedding_eltwise_layernorm_op`: LN(Σ_i Emb_i[Ids_i])."""
    from .. import ops
    acc = None
    for ids, w in zip(ins["Ids"], ins["Embs"]):
        ids = ids.long()
        if ids.dim() > 1 and ids.shape[-1] == 1:
            ids = ids.squeeze(-1)
        e = F.embedding(ids, w)
        acc = e if acc is None else acc + e
    return {"Out": ops.layer_norm(acc, ins["Scale"][0], ins["Bias"][0], a.get("epsilon", 1e-5))}


# ---------------------------------------------------------------- ops emitted by lowering.py
for _name, _f in [("greater_equal", torch.ge), ("greater_than", torch.gt), ("less_equal", torch.le),
                  ("less_than", torch.lt), ("equal", torch.eq), ("not_equal", torch.ne),
                  ("logical_and", torch.logical_and), ("logical_or", torch.logical_or),
                  ("logical_xor", torch.logical_xor)]:
    register(_name)(lambda ins, a, _f=_f: {"Out": _f(ins["X"][0], _bcast(ins["X"][0], ins["Y"][0], a.get("axis", -1)))})

for _name, _f in [("logical_not", torch.logical_not), ("reciprocal", torch.reciprocal),
                  ("sin", torch.sin), ("cos", torch.cos), ("erf", torch.erf)]:
    register(_name)(lambda ins, a, _f=_f: {"Out": _f(ins["X"][0])})


@register("where")
def _where(ins, a):
    return {"Out": torch.where(ins["Condition"][0].bool(), ins["X"][0], ins["Y"][0])}


@register("fill_any_like")
def _fill_any_like(ins, a):
    x = ins["X"][0]
    dt = a.get("dtype", -1)
    dt = x.dtype if dt in (-1, None) else _dt(dt)
    return {"Out": torch.full_like(x, a.get("value", 0.0), dtype=dt)}


@register("shape")
def _shape(ins, a):
    x = ins["Input"][0]
    return {"Out": torch.tensor(list(x.shape), dtype=torch.int32, device=x.device)}


@register("expand_v2")
def _expand_v2(ins, a):
    x = ins["X"][0]
    shape = list(a.get("shape", []))
    off = len(shape) - x.dim()
    shape = [x.shape[i - off] if s == -1 else s for i, s in enumerate(shape)]
    return {"Out": x.expand(shape)}


@register("expand_as_v2")
def _expand_as_v2(ins, a):
    x = ins["X"][0]
    if ins.get("Y"):
        return {"Out": x.expand_as(ins["Y"][0])}
    return {"Out": x.expand(a["target_shape"])}


@register("stack")
def _stack(ins, a):
    return {"Y": torch.stack(ins["X"], a.get("axis", 0))}


@register("pow")
def _pow(ins, a):
    return {"Out": torch.pow(ins["X"][0], a.get("factor", 1.0))}


@register("strided_slice")
def _strided_slice(ins, a):
    x = ins["Input"][0]
    sl = [slice(None)] * x.dim()
    for ax, s, e, st in zip(a["axes"], a["starts"], a["ends"], a["strides"]):
        sl[ax] = slice(s, min(e, x.shape[ax]) if e > 0 else e, st)
    out = x[tuple(sl)]
    for ax in sorted(a.get("decrease_axis", []) or [], reverse=True):
        out = out.squeeze(ax)
    return {"Out": out}


@register("fused_softmax_mask")
def _fsm(ins, a):
    from .. import ops
    x, m = ins["X"][0], ins["Mask"][0]
    if m.dim() == x.dim() and m.shape != x.shape:
        m = m.expand_as(x).contiguous()
    return {"Out": ops.fused_softmax_mask(x, m)}


@register("fused_softmax_mask_upper_triangle")
def _fsm_tri(ins, a):
    from .. import ops
    return {"Out": ops.fused_softmax_mask(ins["X"][0], None, 1.0, causal=True)}


def _flash_slots(ins, *names):
    for n in names:
        if ins.get(n):
            return ins[n][0]
    return None


@register("flash_attn")
def _flash_attn(ins, a):
    """Reference `ops.yaml: flash_attn` (q, k, v [B, S, H, D], optional attn_mask; dropout /
    causal / is_test attrs) — also the [B, H, S, D] ``layout`` form self_attention_fuse_pass emits."""
    from .. import ops
    q, k, v = (_flash_slots(ins, n, n.upper()) for n in ("q", "k", "v"))
    mask = _flash_slots(ins, "attn_mask")
    bhsd = a.get("layout", "bshd") == "bhsd"
    if bhsd:
        q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    p = 0.0 if a.get("is_test", True) else float(a.get("dropout", 0.0))
    o = ops.flash_attention(q, k, v, causal=bool(a.get("causal", False)), scale=a.get("scale"),
                            attn_mask=mask, dropout_p=p)
    o = o.transpose(1, 2) if bhsd else o
    return {"out": o, "Out": o}


@register("weight_only_linear")
def _wol(ins, a):
    from .. import ops
    b = ins["bias"][0] if ins.get("bias") else None
    x = ins["x"][0]
    xin = x
    if x.is_cuda and x.dtype != torch.bfloat16:  # the GPU weight-only GEMM takes bf16 activations
        xin = x.to(torch.bfloat16)
        b = b.to(torch.bfloat16) if b is not None else None
    from ..inference.ref_layout import canonical_weight  # reference (sm80) bytes → MI355X order
    wd = a.get("weight_dtype", "int8")
    w = canonical_weight(ins["weight"][0], ins["weight_scale"][0], wd)
    y = ops.weight_only_linear(xin, w, b, ins["weight_scale"][0], wd, a.get("act_method", "none"))
    return {"out": y.to(x.dtype) if y.dtype != x.dtype else y}


# ---------------------------------------------------------------- LLM / BERT fused inference ops
def _seq(ins, slot):
    return list(ins.get(slot) or [])


def _ring_group(a):
    """``ring_id`` of a tensor-parallel fused op → its process group (None: single rank / -1).
    Ring 0 is the world group (reference `c_comm_init` ring 0)."""
    import torch.distributed as dist
    ring = a.get("ring_id", -1)
    ring = -1 if ring is None else int(ring)
    if ring < 0 or not dist.is_initialized() or dist.get_world_size() == 1:
        return None
    from ..distributed.collective import get_group
    g = get_group(ring)
    if g is None:
        raise RuntimeError(f"ring_id {ring}: no communicator (create it with new_group first)")
    return getattr(g, "pg", None) or dist.group.WORLD


def _fmt_common(ins, a):
    """Slot → functional-argument mapping shared by the fused_multi_transformer variants
    (reference `fused_multi_transformer_op.cc:152-190`)."""
    time_step = None
    if ins.get("TimeStep"):
        ts = ins["TimeStep"][0]
        time_step = int(ts.reshape(-1)[0].item()) if ts.numel() == 1 else ts
    # RotaryPosEmb [2, B, 1, S, D] (cos | sin) with rotary_emb_dims = head-dim chunks; PreCaches:
    # per layer prefix K/V [2, B, H, P, D] (`fused_multi_transformer_op.cc:166,170`)
    rd = int(a.get("rotary_emb_dims", 0) or 0)
    rot = ins["RotaryPosEmb"][0] if ins.get("RotaryPosEmb") else None
    if rd and rot is None:
        raise ValueError("fused_multi_transformer: rotary_emb_dims != 0 needs the RotaryPosEmb input")
    ext = {}
    if rot is not None and rd:
        ext = dict(rotary_embs=rot, rotary_table_dims=rd)
    if ins.get("PreCaches") and any(t is not None for t in ins["PreCaches"]):
        ext["pre_caches"] = _seq(ins, "PreCaches")
    return dict(**ext,pre_layer_norm=bool(a.get("pre_layer_norm", True)), epsilon=float(a.get("epsilon", 1e-5)),
                cache_kvs=_seq(ins, "CacheKV") or None,
                beam_offset=ins["BeamCacheOffset"][0] if ins.get("BeamCacheOffset") else None,
                seq_lens=ins["SeqLengths"][0] if ins.get("SeqLengths") else None,
                time_step=time_step, attn_mask=ins["SrcMask"][0] if ins.get("SrcMask") else None,
                activation=a.get("act_method", "gelu"), trans_qkvw=bool(a.get("trans_qkvw", True)),
                rotary_emb_dims=0, causal=bool(a.get("causal", False)),
                group=_ring_group(a))


@register("fused_multi_transformer")
def _fused_multi_transformer(ins, a):
    """Reference `fused_multi_transformer_op.cc` / `.cu`: X, LnScale/LnBias, QKVW/QKVBias,
    OutLinearW/Bias, FFNLnScale/Bias, FFN1Weight/Bias, FFN2Weight/Bias (one entry per layer),
    optional CacheKV (updated in place → CacheKVOut), TimeStep (decode), SrcMask, SeqLengths."""
    from ..incubate.nn import functional as IF
    kw = _fmt_common(ins, a)
    out = IF.fused_multi_transformer(
        ins["X"][0], _seq(ins, "LnScale"), _seq(ins, "LnBias"), _seq(ins, "QKVW"), _seq(ins, "QKVBias"),
        _seq(ins, "OutLinearW"), _seq(ins, "OutLinearBias"), _seq(ins, "FFNLnScale"),
        _seq(ins, "FFNLnBias"), _seq(ins, "FFN1Weight"), _seq(ins, "FFN1Bias"), _seq(ins, "FFN2Weight"),
        _seq(ins, "FFN2Bias"), dropout_rate=0.0, training=False,
        num_kv_heads=a.get("num_kv_heads") or None, **kw)
    y, caches = (out if isinstance(out, tuple) else (out, None))
    return {"Out": y, "CacheKVOut": caches or []}


@register("fused_multi_transformer_weight_only")
def _fused_multi_transformer_wo(ins, a):
    """Reference `fused_multi_transformer_weight_only_op.cu`: the same slots plus the per-channel
    *WScale / *WeightScale inputs; weights packed int8 ([N, K]) or int4 ([N/2, K])."""
    from ..incubate.nn import functional as IF
    from ..inference.ref_layout import canonical_weight  # reference (sm80) bytes → MI355X order
    kw = _fmt_common(ins, a)
    kw.pop("trans_qkvw")
    wd = a.get("weight_dtype", "int8")

    def cw(slot, sslot):
        return [canonical_weight(w, s_, wd) for w, s_ in zip(_seq(ins, slot), _seq(ins, sslot))]
    out = IF.fused_multi_transformer_weight_only(
        ins["X"][0], _seq(ins, "LnScale"), _seq(ins, "LnBias"), cw("QKVW", "QKVWScale"), _seq(ins, "QKVWScale"),
        _seq(ins, "QKVBias"), cw("OutLinearW", "OutLinearWScale"), _seq(ins, "OutLinearWScale"),
        _seq(ins, "OutLinearBias"), _seq(ins, "FFNLnScale"), _seq(ins, "FFNLnBias"),
        cw("FFN1Weight", "FFN1WeightScale"), _seq(ins, "FFN1WeightScale"), _seq(ins, "FFN1Bias"),
        cw("FFN2Weight", "FFN2WeightScale"), _seq(ins, "FFN2WeightScale"), _seq(ins, "FFN2Bias"),
        weight_dtype=a.get("weight_dtype", "int8"), num_heads=a.get("num_heads"),
        num_kv_heads=a.get("num_kv_heads") or None, **kw)
    y, caches = (out if isinstance(out, tuple) else (out, None))
    return {"Out": y, "CacheKVOut": caches or []}


def _cached_view(w, shape):
    """A reshaped view of a weight kept on the weight itself, so per-weight caches (the
    K-contiguous transposed copy of ``ops.linear.transposed``) survive across runs."""
    v = getattr(w, "_piamd_view", None)
    if v is None or tuple(v.shape) != tuple(shape) or v.data_ptr() != w.data_ptr():
        v = w.reshape(shape)
        try:
            w._piamd_view = v
        except (AttributeError, RuntimeError):
            pass
    return v


@register("multihead_matmul")
def _multihead_matmul(ins, a):
    """Reference `fused/multihead_matmul_op.cu`: Input [B, S, E] · W [E, 3, E] + Bias [3, E],
    attention with the additive BiasQK mask ([B, H|1, S, S]), alpha-scaled; Out [B, S, E]."""
    from .. import ops
    from ..ops.linear import linear
    x, w, bias = ins["Input"][0], ins["W"][0], ins["Bias"][0]
    B, S, E = x.shape
    H = int(a["head_number"])
    D = E // H
    qkv = None
    if _ln_defer.of(x) is not None:  # QKV GEMM on the raw rows with the producer's LayerNorm folded
        qkv = _ln_defer.linear(x, _cached_view(w, (E, 3 * E)), bias.reshape(3 * E))
        if qkv is None:
            x = _ln_defer.materialize(x)
    if qkv is None:
        qkv = linear(x.reshape(B * S, E), _cached_view(w, (E, 3 * E)), bias.reshape(3 * E))
    qkv = qkv.reshape(B, S, 3, H, D)
    qkv = qkv.reshape(B, S, 3 * H, D)
    mask = ins["BiasQK"][0] if ins.get("BiasQK") else None
    scale = float(a.get("alpha", 1.0 / D ** 0.5))
    if mask is None:
        o = ops.flash_attention_packed(qkv, H, H, causal=False, scale=scale)
    else:
        o = ops.flash_attention(qkv[:, :, :H], qkv[:, :, H:2 * H], qkv[:, :, 2 * H:], False, scale,
                                attn_mask=mask)
    return {"Out": o.reshape(B, S, E)}


def _fc_resid_deferred(x2, w, b0, y, ins, a):
    """(fc(x2) + b0 + y as ONE skinny GEMM with y's own deferred LayerNorm applied in the epilogue,
    γ, β) — the output's LayerNorm is then deferred to its consumers; None when this call does
    not qualify."""
    from ..ops.gemm import small_gemm, use_small
    from ..ops.linear import transposed
    g, be = (ins["Scale"][0] if ins.get("Scale") else None), (ins["Bias1"][0] if ins.get("Bias1") else None)
    if g is None or be is None or w.dim() != 2 or x2.dtype != w.dtype or not x2.is_contiguous():
        return None
    M, K = x2.shape
    N = w.shape[1]
    if (not _ln_defer.can_defer(x2, M, N) or not use_small(M, N, K)
            or K % 64 or N % 4 or y.numel() != M * N):
        return None
    r, rln = _ln_defer.resid_args(y, M)
    r2 = r.reshape(M, N)
    if r2.dtype != x2.dtype or not r2.is_contiguous():
        return None
    b0 = _ln_defer._as(b0.reshape(-1), x2.dtype) if b0 is not None else None  # f32 under mixed precision
    return small_gemm(x2, transposed(w), bias=b0, resid=r2, resid_ln=rln), g, be


@register("fused_fc_elementwise_layernorm")
def _fc_eltwise_ln(ins, a):
    """Reference `fused/fused_fc_elementwise_layernorm_op.cu`:
    Out = LN(fc(X, W, Bias0) + Y; Scale, Bias1), fc flattening at x_num_col_dims."""
    from .. import ops
    from ..ops.linear import linear
    x, w, y = _ln_defer.materialize(ins["X"][0]), ins["W"][0], ins["Y"][0]
    b0 = ins["Bias0"][0] if ins.get("Bias0") else None
    nc = int(a.get("x_num_col_dims", x.dim() - 1))
    x2 = x.reshape(int(np.prod(x.shape[:nc])), -1)
    if a.get("defer_ln") and a.get("activation_type") in ("", None):
        r = _fc_resid_deferred(x2, w, b0, y, ins, a)
        if r is not None:  # raw fc + residual; the LayerNorm rides in the consumers (ln_defer)
            h = r[0].reshape(*x.shape[:nc], -1)
            return {"Out": _ln_defer.defer(h, r[1], r[2], float(a.get("epsilon", 1e-5)))}
    y = _ln_defer.materialize(y)
    h = linear(x2, w, b0).reshape(*x.shape[:nc], -1)
    if a.get("activation_type") == "relu":
        h = F.relu(h)
    out, _ = ops.fused_add_layer_norm(h, y, ins["Scale"][0] if ins.get("Scale") else None,
                                      ins["Bias1"][0] if ins.get("Bias1") else None,
                                      float(a.get("epsilon", 1e-5)), None, 0.0, False, need_residual=False)
    return {"Out": out}




# ------------------------------------------------------------------------ backward / optimizer ops
@register("sum")
def _sum(ins, a):
    xs = [x for x in ins["X"] if x is not None]
    out = xs[0]
    for x in xs[1:]:
        out = out + x
    return {"Out": out}


@register("fill_zeros_like")
def _fill_zeros_like(ins, a):
    return {"Out": torch.zeros_like(ins["X"][0])}


def _lr(ins):
    return ins["LearningRate"][0].reshape(()).float()


def _reg(p, g, a):
    # reference optimizer ops: regularization_method "l2_decay" adds coeff * param to the gradient
    if a.get("regularization_method") == "l2_decay" and a.get("regularization_coeff"):
        return g + float(a["regularization_coeff"]) * p
    return g


def _skip(ins):
    """SkipUpdate input (AMP: found_inf of this step): the optimizer op leaves every state as is."""
    s = ins.get("SkipUpdate")
    return bool(s and s[0] is not None and bool(s[0].reshape(-1)[0]))


@register("check_finite_and_unscale")
def _check_finite_and_unscale(ins, a):
    """Reference `amp/check_finite_and_unscale_op.cu`: Out = X / Scale, FoundInfinite = any
    inf/nan among all X (in place on the gradients)."""
    scale = ins["Scale"][0].reshape(()).float()
    inv = 1.0 / scale
    found = torch.zeros((), dtype=torch.bool, device=scale.device)
    outs = []
    for x in ins["X"]:
        found = found | ~torch.isfinite(x).all()
        outs.append(x.mul_(inv.to(x.dtype)) if not x.requires_grad else x * inv.to(x.dtype))
    return {"Out": outs, "FoundInfinite": found.reshape(1)}


@register("update_loss_scaling")
def _update_loss_scaling(ins, a):
    """Reference `amp/update_loss_scaling_op.cu`: on inf/nan zero the gradients, count bad steps and
    shrink the scale every decr_every_n_nan_or_inf of them; else count good steps and grow it every
    incr_every_n_steps (unless stop_update)."""
    found = bool(ins["FoundInfinite"][0].reshape(-1)[0])
    ls, good, bad = ins["PrevLossScaling"][0], ins["InGoodSteps"][0], ins["InBadSteps"][0]
    xs = ins["X"]
    if found:
        xs = [x.zero_() if not x.requires_grad else torch.zeros_like(x) for x in xs]
    if not a.get("stop_update", False):
        with torch.no_grad():
            if found:
                good.zero_()
                bad.add_(1)
                if int(bad.reshape(-1)[0]) >= int(a.get("decr_every_n_nan_or_inf", 2)):
                    ls.mul_(float(a.get("decr_ratio", 0.5))).clamp_(min=1.0)
                    bad.zero_()
            else:
                bad.zero_()
                good.add_(1)
                if int(good.reshape(-1)[0]) >= int(a.get("incr_every_n_steps", 1000)):
                    nxt = ls * float(a.get("incr_ratio", 2.0))
                    if bool(torch.isfinite(nxt).all()):
                        ls.copy_(nxt)
                    good.zero_()
    return {"Out": xs, "LossScaling": ls, "OutGoodSteps": good, "OutBadSteps": bad}


@register("sgd")
def _sgd(ins, a):
    """Reference `phi/kernels/gpu/sgd_kernel.cu`: ParamOut = Param - lr * Grad (in place)."""
    p, g = ins["Param"][0], ins["Grad"][0]
    if _skip(ins):
        return {"ParamOut": p}
    gf = _reg(p, g.to(p.dtype), a)
    p.sub_(_lr(ins).to(p.dtype) * gf)
    return {"ParamOut": p}


@register("momentum")
def _momentum(ins, a):
    """Reference `phi/kernels/impl/momentum_kernel_impl.h`: v = mu v + g; p -= lr (g + mu v) | lr v."""
    p, g, v = ins["Param"][0], ins["Grad"][0], ins["Velocity"][0]
    if _skip(ins):
        return {"ParamOut": p, "VelocityOut": v}
    mu = float(a.get("mu", 0.9))
    gf = _reg(p, g.float() * float(a.get("rescale_grad", 1.0)), a)
    v.mul_(mu).add_(gf)
    lr = _lr(ins)
    upd = gf + mu * v if a.get("use_nesterov") else v
    p.sub_((lr * upd).to(p.dtype))
    return {"ParamOut": p, "VelocityOut": v}


@register("adam", "adamw")
def _adam(ins, a):
    """Reference `phi/kernels/gpu/adam_kernel.cu` / `adamw_kernel.cu` (beta pow accumulators carried
    as [1] tensors, updated in place; AdamW decays the parameter by lr * coeff first)."""
    p, g = ins["Param"][0], ins["Grad"][0]
    m1, m2 = ins["Moment1"][0], ins["Moment2"][0]
    b1p, b2p = ins["Beta1Pow"][0], ins["Beta2Pow"][0]
    if _skip(ins):
        return {"ParamOut": p, "Moment1Out": m1, "Moment2Out": m2, "Beta1PowOut": b1p, "Beta2PowOut": b2p}
    b1, b2, eps = float(a.get("beta1", 0.9)), float(a.get("beta2", 0.999)), float(a.get("epsilon", 1e-8))
    lr = _lr(ins) * float(a.get("lr_ratio", 1.0))
    gf = _reg(p, g.float(), a)
    if a.get("with_decay") and a.get("coeff"):
        p.mul_((1.0 - lr * float(a["coeff"])).to(p.dtype))
    m1.mul_(b1).add_(gf, alpha=1 - b1)
    m2.mul_(b2).addcmul_(gf, gf, value=1 - b2)
    bc1 = 1 - b1p.reshape(()).float()
    bc2 = torch.sqrt(1 - b2p.reshape(()).float())
    step = lr * bc2 / bc1
    p.sub_((step * m1 / (m2.sqrt() + eps * bc2)).to(p.dtype))
    b1p.mul_(b1)
    b2p.mul_(b2)
    return {"ParamOut": p, "Moment1Out": m1, "Moment2Out": m2, "Beta1PowOut": b1p, "Beta2PowOut": b2p}


@register("clip")
def _clip_op(ins, a):
    return {"Out": torch.clamp(ins["X"][0], float(a.get("min", -3.4e38)), float(a.get("max", 3.4e38)))}


from . import ops_registry_ext  # noqa: E402,F401  (registers the extended op set)
from . import ops_registry_more  # noqa: E402,F401  (fused blocks, rnn, 3-D conv / pool, detection)
from . import ops_registry_model  # noqa: E402,F401  (quantization, fused BN+act, vocab-parallel CE, gate attention, beam search)
from . import ops_registry_tail  # noqa: E402,F401  (the long tail: math / linalg / losses / optimizers / collectives / RNN / detection / fork serving ops)
