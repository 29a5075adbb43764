"""Inference IR passes over Paddle-typed static Programs.

Parity: reference `paddle/fluid/framework/ir/*_pass.cc` and the GPU pass list of
`paddle/fluid/inference/api/paddle_pass_builder.cc` (GpuPassStrategy). Each pass pattern-matches
a chain of Paddle ops and rewrites it into one fused op whose kernel is registered in
`static/ops_registry.py` and runs the MI355X HIP kernels:

  delete_dropout_op_pass          dropout(is_test)                     → scale / (removed)
  identity_scale_op_clean_pass    scale(1, 0)                          → (removed)
  conv_bn_fuse_pass               conv2d + batch_norm                  → conv2d (folded W, b)
  fc_fuse_pass                    mul|matmul(_v2) + elementwise_add    → fc
  fc_act_fuse_pass                fc + relu|gelu|silu|tanh|sigmoid     → fc(activation_type)
  skip_layernorm_fuse_pass        elementwise_add + layer_norm         → skip_layernorm
  embedding_eltwise_layernorm_fuse_pass  lookup_table×N + adds + LN    → fused_embedding_eltwise_layernorm
  self_attention_fuse_pass        matmul(QKᵀ)[·α] + softmax + matmul(V) → flash_attn
  linear_bias_act_fuse_pass       traced linear(no bias) + fused_bias_act → one GEMM with the
                                  bias+act epilogue (`ops.linear.linear_bias_act`)

Passes only rewrite when every intermediate has exactly one consumer and is not fetched.
"""
from __future__ import annotations

import numpy as np
import torch

from ..static.framework import Operator

ACTS = ("relu", "gelu", "silu", "swish", "tanh", "sigmoid")


class Graph:
    """Minimal producer/consumer view of a Program's global block."""

    def __init__(self, program, fetch_names=()):
        self.program = program
        self.block = program.global_block()
        self.keep = set(fetch_names) | set(program.fetch_names)

    @property
    def ops(self):
        return self.block.ops

    def consumers(self, name):
        return [op for op in self.ops if name in op.input_names()]

    def producer(self, name):
        for op in self.ops:
            if name in op.output_names():
                return op
        return None

    def single_use(self, name):
        return name not in self.keep and len(self.consumers(name)) == 1

    def is_param(self, name):
        return name in self.program.params

    def param(self, name):
        return self.program.params[name]

    def replace(self, old_ops, new_op):
        idx = min(self.ops.index(o) for o in old_ops)
        for o in old_ops:
            self.ops.remove(o)
        self.ops.insert(idx, new_op)
        self.program._version += 1

    def bypass(self, op, x, out):
        """Remove an identity op ``out = op(x)``. Prefer renaming x's producer to write ``out``
        (keeps fetched names stable); else point out's consumers at ``x``. False if impossible."""
        prod = self.producer(x)
        if prod is not None and prod.func is None and prod.paddle_outputs is not None \
                and self.single_use(x):
            for k, v in prod.paddle_outputs.items():
                prod.paddle_outputs[k] = [out if n == x else n for n in v]
            self.ops.remove(op)
        elif out not in self.keep:
            self.ops.remove(op)
            for o in self.ops:
                if o.paddle_inputs:
                    for k, v in o.paddle_inputs.items():
                        o.paddle_inputs[k] = [x if n == out else n for n in v]
        else:
            return False
        self.program._version += 1
        return True


def _pop(op, slot):
    return (op.paddle_inputs or {}).get(slot, [None])[0]


def _out(op, slot="Out"):
    return (op.paddle_outputs or {}).get(slot, [None])[0]


def _new(block, type_, ins, outs, attrs):
    op = Operator(block, None, (), {}, None, type=type_, attrs=attrs)
    op.paddle_inputs, op.paddle_outputs = ins, outs
    return op


def _typed(ops):
    return [o for o in ops if o.func is None and o.paddle_inputs is not None]


# ----------------------------------------------------------------------------------- passes
def delete_dropout_op_pass(g: Graph):
    n = 0
    for op in list(_typed(g.ops)):
        if op.type != "dropout":
            continue
        impl = op.attrs.get("dropout_implementation", "downgrade_in_infer")
        x, out = _pop(op, "X"), _out(op)
        if impl == "upscale_in_train":
            if not g.bypass(op, x, out):
                continue
        else:
            p = float(op.attrs.get("dropout_prob", 0.5))
            g.replace([op], _new(g.block, "scale", {"X": [x]}, {"Out": [out]},
                                 {"scale": 1.0 - p, "bias": 0.0, "bias_after_scale": True}))
        n += 1
    return n


def identity_scale_op_clean_pass(g: Graph):
    n = 0
    for op in list(_typed(g.ops)):
        if op.type == "scale" and float(op.attrs.get("scale", 1.0)) == 1.0 and \
                float(op.attrs.get("bias", 0.0)) == 0.0 and not op.paddle_inputs.get("ScaleTensor"):
            if g.bypass(op, _pop(op, "X"), _out(op)):
                n += 1
    return n


def conv_bn_fuse_pass(g: Graph):
    n = 0
    for bn in list(_typed(g.ops)):
        if bn.type != "batch_norm":
            continue
        x = _pop(bn, "X")
        conv = g.producer(x)
        if conv is None or conv.func is not None or conv.type not in ("conv2d", "depthwise_conv2d") \
                or not g.single_use(x) or conv.paddle_inputs.get("Bias"):
            continue
        wname = _pop(conv, "Filter")
        if not g.is_param(wname):
            continue
        names = [_pop(bn, s) for s in ("Scale", "Bias", "Mean", "Variance")]
        if not all(g.is_param(nm) for nm in names):
            continue
        gamma, beta, mean, var = (g.param(nm).float() for nm in names)
        eps = float(bn.attrs.get("epsilon", 1e-5))
        std = torch.sqrt(var + eps)
        w = g.param(wname)
        new_w = (w.float() * (gamma / std).reshape(-1, 1, 1, 1)).to(w.dtype)
        new_b = (beta - mean * gamma / std).to(w.dtype)
        wn, bnm = wname + "@bnfused", names[1] + "@bnfused"
        g.program.params[wn] = new_w
        g.program.params[bnm] = new_b
        g.block.create_var(wn, list(new_w.shape), "float32", persistable=True)
        g.block.create_var(bnm, list(new_b.shape), "float32", persistable=True)
        ins = dict(conv.paddle_inputs)
        ins["Filter"] = [wn]
        ins["Bias"] = [bnm]
        fused = _new(g.block, conv.type, ins, {"Output": [_out(bn, "Y")]}, dict(conv.attrs))
        g.replace([conv, bn], fused)
        n += 1
    return n


def fc_fuse_pass(g: Graph):
    n = 0
    for mm in list(_typed(g.ops)):
        if mm.type not in ("mul", "matmul", "matmul_v2"):
            continue
        if mm not in g.ops:
            continue
        y = _pop(mm, "Y")
        if not g.is_param(y) or g.param(y).dim() != 2:
            continue
        if mm.type == "matmul_v2" and (mm.attrs.get("trans_x") or mm.attrs.get("trans_y")):
            continue
        if mm.type == "matmul" and (mm.attrs.get("transpose_X") or mm.attrs.get("transpose_Y")
                                    or float(mm.attrs.get("alpha", 1.0)) != 1.0):
            continue
        out = _out(mm)
        cons = g.consumers(out)
        if len(cons) != 1 or out in g.keep:
            continue
        add = cons[0]
        if add.func is not None or add.type != "elementwise_add":
            continue
        b = _pop(add, "Y") if _pop(add, "X") == out else _pop(add, "X")
        if not g.is_param(b) or g.param(b).dim() != 1:
            continue
        x = _pop(mm, "X")
        xv = g.block.vars.get(x)
        nd = len(xv.declared_shape) if xv is not None and xv.declared_shape else 2
        ncol = int(mm.attrs.get("x_num_col_dims", 1)) if mm.type == "mul" else nd - 1
        fused = _new(g.block, "fc", {"Input": [x], "W": [y], "Bias": [b]}, {"Out": [_out(add)]},
                     {"in_num_col_dims": ncol, "activation_type": ""})
        g.replace([mm, add], fused)
        n += 1
    return n


def fc_act_fuse_pass(g: Graph):
    n = 0
    for fc in list(_typed(g.ops)):
        if fc.type != "fc" or fc.attrs.get("activation_type") or fc not in g.ops:
            continue
        out = _out(fc)
        cons = g.consumers(out)
        if len(cons) != 1 or out in g.keep or cons[0].func is not None or cons[0].type not in ACTS:
            continue
        act = cons[0]
        if act.type == "gelu" and act.attrs.get("approximate"):
            kind = "gelu_tanh"
        else:
            kind = {"swish": "silu"}.get(act.type, act.type)
        attrs = dict(fc.attrs)
        attrs["activation_type"] = kind
        g.replace([fc, act], _new(g.block, "fc", dict(fc.paddle_inputs), {"Out": [_out(act)]}, attrs))
        n += 1
    return n


def skip_layernorm_fuse_pass(g: Graph):
    n = 0
    for add in list(_typed(g.ops)):
        if add.type != "elementwise_add" or add not in g.ops:
            continue
        x, y = _pop(add, "X"), _pop(add, "Y")
        if g.is_param(x) or g.is_param(y) or int(add.attrs.get("axis", -1)) != -1:
            continue
        xv, yv = g.block.vars.get(x), g.block.vars.get(y)
        if xv is None or yv is None or xv.declared_shape != yv.declared_shape:
            continue
        out = _out(add)
        cons = g.consumers(out)
        if len(cons) != 1 or out in g.keep or cons[0].func is not None or cons[0].type != "layer_norm":
            continue
        ln = cons[0]
        nd = len(xv.declared_shape or [])
        if int(ln.attrs.get("begin_norm_axis", nd - 1)) != nd - 1:
            continue
        for extra in ("Mean", "Variance"):
            nm = _out(ln, extra)
            if nm and (nm in g.keep or g.consumers(nm)):
                break
        else:
            fused = _new(g.block, "skip_layernorm",
                         {"X": [x], "Y": [y], "Scale": [_pop(ln, "Scale")], "Bias": [_pop(ln, "Bias")]},
                         {"Out": [_out(ln, "Y")]}, {"epsilon": float(ln.attrs.get("epsilon", 1e-5))})
            g.replace([add, ln], fused)
            n += 1
    return n


def embedding_eltwise_layernorm_fuse_pass(g: Graph):
    n = 0
    for ln in list(_typed(g.ops)):
        if ln.type != "layer_norm" or ln not in g.ops:
            continue
        chain, embs, ok = [], [], True

        def walk(name):
            nonlocal ok
            p = g.producer(name)
            if p is None or p.func is not None:
                ok = False
                return
            if p.type in ("lookup_table_v2", "lookup_table") and g.single_use(name):
                chain.append(p)
                embs.append((_pop(p, "Ids"), _pop(p, "W")))
            elif p.type == "elementwise_add" and g.single_use(name):
                chain.append(p)
                walk(_pop(p, "X"))
                walk(_pop(p, "Y"))
            else:
                ok = False
        walk(_pop(ln, "X"))
        if not ok or len(embs) < 2:
            continue
        fused = _new(g.block, "fused_embedding_eltwise_layernorm",
                     {"Ids": [i for i, _ in embs], "Embs": [w for _, w in embs],
                      "Scale": [_pop(ln, "Scale")], "Bias": [_pop(ln, "Bias")]},
                     {"Out": [_out(ln, "Y")]}, {"epsilon": float(ln.attrs.get("epsilon", 1e-5))})
        g.replace(chain + [ln], fused)
        n += 1
    return n


def self_attention_fuse_pass(g: Graph):
    """softmax(α·Q·Kᵀ [+ mask]) · V with Q/K/V in [B, H, S, D] → flash_attn (no-mask form)."""
    n = 0
    for sm in list(_typed(g.ops)):
        if sm.type != "softmax" or sm not in g.ops or int(sm.attrs.get("axis", -1)) != -1:
            continue
        s_in = _pop(sm, "X")
        prod = g.producer(s_in)
        alpha, scale_op = 1.0, None
        if prod is not None and prod.func is None and prod.type == "scale" and g.single_use(s_in) \
                and float(prod.attrs.get("bias", 0.0)) == 0.0:
            scale_op, alpha = prod, float(prod.attrs.get("scale", 1.0))
            s_in = _pop(prod, "X")
            prod = g.producer(s_in)
        if prod is None or prod.func is not None or prod.type not in ("matmul", "matmul_v2") \
                or not g.single_use(s_in):
            continue
        ty = prod.attrs.get("trans_y") if prod.type == "matmul_v2" else prod.attrs.get("transpose_Y")
        tx = prod.attrs.get("trans_x") if prod.type == "matmul_v2" else prod.attrs.get("transpose_X")
        if not ty or tx:
            continue
        if prod.type == "matmul":
            alpha *= float(prod.attrs.get("alpha", 1.0))
        p = _out(sm)
        cons = g.consumers(p)
        if len(cons) != 1 or p in g.keep:
            continue
        pv = cons[0]
        if pv.func is not None or pv.type not in ("matmul", "matmul_v2") or _pop(pv, "X") != p:
            continue
        if pv.attrs.get("trans_x") or pv.attrs.get("trans_y") or pv.attrs.get("transpose_X") \
                or pv.attrs.get("transpose_Y"):
            continue
        q, k, v = _pop(prod, "X"), _pop(prod, "Y"), _pop(pv, "Y")
        qv = g.block.vars.get(q)
        if qv is None or not qv.declared_shape or len(qv.declared_shape) != 4:
            continue
        old = [prod, sm, pv] + ([scale_op] if scale_op is not None else [])
        fused = _new(g.block, "flash_attn", {"Q": [q], "K": [k], "V": [v]}, {"Out": [_out(pv)]},
                     {"layout": "bhsd", "scale": alpha, "causal": False})
        g.replace(old, fused)
        n += 1
    return n


def linear_bias_act_fuse_pass(g: Graph):
    """Traced programs (``jit.save`` of dygraph models) record ``linear`` and ``fused_bias_act``
    as torch-callable ops; fold the pair into one epilogue GEMM."""
    from ..ops import linear as L
    from ..static.framework import VarRef
    n = 0
    for lin in list(g.ops):
        if lin.type != "linear" or lin.func is None or lin not in g.ops:
            continue
        args = tuple(lin.args) + (None,) * (3 - len(lin.args))
        if lin.kwargs or len(lin.args) > 3 or args[2] is not None:
            continue
        outs = lin.output_names()
        if len(outs) != 1 or not g.single_use(outs[0]):
            continue
        ba = g.consumers(outs[0])[0]
        if ba.type != "fused_bias_act" or ba.func is None or ba.kwargs:
            continue
        bargs = tuple(ba.args)
        if not bargs or not isinstance(bargs[0], VarRef) or bargs[0].name != outs[0]:
            continue
        bias = bargs[1] if len(bargs) > 1 else None
        act = bargs[2] if len(bargs) > 2 else "gelu"
        if not isinstance(bias, VarRef) or act not in L._EPILOGUE_ACTS:
            continue
        fused = Operator(g.block, L.linear_bias_act, (args[0], args[1], bias, act), {}, ba.outputs,
                         type="fc")
        g.replace([lin, ba], fused)
        n += 1
    return n


GPU_PASSES = [
    "delete_dropout_op_pass", "identity_scale_op_clean_pass", "conv_bn_fuse_pass",
    "embedding_eltwise_layernorm_fuse_pass", "self_attention_fuse_pass", "fc_fuse_pass",
    "fc_act_fuse_pass", "skip_layernorm_fuse_pass", "linear_bias_act_fuse_pass",
]

PASSES = {name: globals()[name] for name in GPU_PASSES}


def apply_passes(program, passes=None, fetch_names=(), debug=False):
    g = Graph(program, fetch_names)
    stats = {}
    for name in (passes if passes is not None else GPU_PASSES):
        fn = PASSES.get(name)
        if fn is None:
            continue
        stats[name] = fn(g)
        if debug:
            print(f"--- {name}: {stats[name]} rewrites")
    return stats


np  # noqa
