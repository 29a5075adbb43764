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
  identity_reshape_clean_pass     reshape2(X, Shape=shape(X))          → (removed)
  fused_multi_transformer_{encoder,decoder}[_fuse_qkv]_pass, multi_devices_* (fmt_passes.py)
                                  exported LLM layer ops (+ KV-cache concat, + mp collectives)
                                  → fused_multi_transformer with CacheKV / TimeStep / ring_id
  fused_multi_transformer_encoder_traced_pass  traced pre-LN causal layer → fused_multi_transformer
  fuse_multi_transformer_layer_pass     consecutive fused_multi_transformer → one multi-layer op
  multihead_matmul_fuse_pass      fc(QKV) + head split + attention + merge → multihead_matmul
  flash_attn_packed_fuse_pass     split(QKV) + flash_attn               → flash_attn_packed
  fc_elementwise_layernorm_fuse_pass  fc + residual add + layer_norm    → fused_fc_elementwise_layernorm
  ln_defer_pass                   post-LN fc+LN feeding only QKV / FFN1 GEMMs + residual adds
                                  → defer_ln (LayerNorm folded into the consumers at few rows)
  + the rest of the reference GPU list in passes_extra.py (is_test, simplify_with_basic_ops,
    constant_folding, gpu_cpu_* matmul maps / shape+matmul fusions, matmul_scale, conv + bias
    (+ residual) (+ act) → conv2d_fusion, conv + bias + bn, transpose_flatten_concat)

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




# ---------------------------------------------------------------- passes over lowered programs
def identity_reshape_clean_pass(g: Graph):
    """reshape2(X, Shape = shape(X)) → X (the view_as identities a traced program lowers to)."""
    n = 0
    for op in list(_typed(g.ops)):
        if op.type not in ("reshape2", "reshape") or op not in g.ops or not op.paddle_inputs.get("Shape"):
            continue
        x, sh = _pop(op, "X"), _pop(op, "Shape")
        sp = g.producer(sh)
        if sp is None or sp.func is not None or sp.type != "shape" or _pop(sp, "Input") != x:
            continue
        if g.bypass(op, x, _out(op)):
            if not g.consumers(sh) and sh not in g.keep:
                g.ops.remove(sp)
            n += 1
    return n


def _single_consumer(g, name, types):
    if name is None or name in g.keep:
        return None
    cons = g.consumers(name)
    if len(cons) != 1 or cons[0].func is not None or cons[0].type not in types:
        return None
    return cons[0]


def _split_qkv(g, split):
    """A 3-way split along the head axis whose outputs feed exactly one flash_attn as q, k, v."""
    outs = (split.paddle_outputs or {}).get("Out", [])
    if split.type != "split" or int(split.attrs.get("axis", -1)) != 2 or len(outs) != 3:
        return None
    secs = list(split.attrs.get("sections") or [])
    if len(secs) != 3:
        return None
    fa = _single_consumer(g, outs[0], ("flash_attn",))
    if fa is None or any(g.consumers(o) != [fa] for o in outs[1:]) or any(o in g.keep for o in outs):
        return None
    qn = (fa.paddle_inputs.get("q") or fa.paddle_inputs.get("Q") or [None])[0]
    kn = (fa.paddle_inputs.get("k") or fa.paddle_inputs.get("K") or [None])[0]
    vn = (fa.paddle_inputs.get("v") or fa.paddle_inputs.get("V") or [None])[0]
    if [qn, kn, vn] != outs or fa.attrs.get("layout", "bshd") != "bshd":
        return None
    if not fa.attrs.get("is_test", True) and float(fa.attrs.get("dropout", 0.0)) > 0:
        return None
    return fa, secs


def flash_attn_packed_fuse_pass(g: Graph):
    """split(qkv, axis 2) + flash_attn(q, k, v) → flash_attn_packed(QKV): attention reads Q/K/V
    straight out of the fused projection output (no split copies)."""
    n = 0
    for sp in list(_typed(g.ops)):
        if sp.type != "split" or sp not in g.ops:
            continue
        m = _split_qkv(g, sp)
        if m is None:
            continue
        fa, secs = m
        if fa.paddle_inputs.get("attn_mask") or secs[1] != secs[2]:
            continue
        out = (fa.paddle_outputs.get("out") or fa.paddle_outputs.get("Out"))[0]
        fused = _new(g.block, "flash_attn_packed", {"QKV": [_pop(sp, "X")]}, {"Out": [out]},
                     {"num_heads": int(secs[0]), "num_kv_heads": int(secs[1]),
                      "causal": bool(fa.attrs.get("causal", False))})
        g.replace([sp, fa], fused)
        n += 1
    return n


def _fc_of(g, op):
    """(input, W, Bias, activation) of an fc op, else None."""
    if op is None or op.func is not None or op.type != "fc":
        return None
    return _pop(op, "Input"), _pop(op, "W"), _pop(op, "Bias"), op.attrs.get("activation_type", "")


def _attn_chain(g, x, fc=None):
    """x → fc(qkv) → reshape2 [.., S, Hq+2Hk, D] → split → flash_attn → reshape2 [.., S, E]:
    (ops, qkv_fc, heads (hq, hk), D, flash op, attn-out name) or None."""
    fc = fc if fc is not None else _single_consumer(g, x, ("fc",))
    if fc is None or _fc_of(g, fc)[3] or not g.is_param(_pop(fc, "W")):
        return None
    r1 = _single_consumer(g, _out(fc), ("reshape2", "reshape"))
    if r1 is None or r1.paddle_inputs.get("Shape"):
        return None
    shp = list(r1.attrs.get("shape") or [])
    if len(shp) != 4:
        return None
    sp = _single_consumer(g, _out(r1), ("split",))
    m = _split_qkv(g, sp) if sp is not None else None
    if m is None:
        return None
    fa, secs = m
    fout = (fa.paddle_outputs.get("out") or fa.paddle_outputs.get("Out"))[0]
    r2 = _single_consumer(g, fout, ("reshape2", "reshape"))
    if r2 is None or r2.paddle_inputs.get("Shape") or len(r2.attrs.get("shape") or []) != 3:
        return None
    return [fc, r1, sp, fa, r2], fc, (int(secs[0]), int(secs[1])), int(shp[3]), fa, _out(r2)


def multihead_matmul_fuse_pass(g: Graph):
    """Reference `multihead_matmul_fuse_pass_v2/v3`: the BERT self-attention block (QKV fc →
    head split → attention [+ additive mask] → head merge) → one multihead_matmul op."""
    n = 0
    for fc in list(_typed(g.ops)):
        if fc.type != "fc" or fc not in g.ops:
            continue
        x = _pop(fc, "Input")
        chain = _attn_chain(g, x, fc)
        if chain is None:
            continue
        ops, _, (hq, hk), D, fa, out = chain
        if hq != hk or fa.attrs.get("causal"):
            continue
        w = _pop(fc, "W")
        E = g.param(w).shape[0]
        if hq * D != E:
            continue
        ins = {"Input": [x], "W": [w], "Bias": [_pop(fc, "Bias")]}
        if fa.paddle_inputs.get("attn_mask"):
            ins["BiasQK"] = fa.paddle_inputs["attn_mask"]
        fused = _new(g.block, "multihead_matmul", ins, {"Out": [out]},
                     {"head_number": hq, "alpha": 1.0 / float(np.sqrt(D))})
        g.replace(ops, fused)
        n += 1
    return n


def fc_elementwise_layernorm_fuse_pass(g: Graph):
    """Reference `fc_elementwise_layernorm_fuse_pass`: fc + elementwise_add(residual) +
    layer_norm → fused_fc_elementwise_layernorm (post-LN transformer blocks)."""
    n = 0
    for fc in list(_typed(g.ops)):
        if fc.type != "fc" or fc not in g.ops or fc.attrs.get("activation_type") not in ("", None):
            continue
        add = _single_consumer(g, _out(fc), ("elementwise_add",))
        if add is None or int(add.attrs.get("axis", -1)) != -1:
            continue
        y = _pop(add, "Y") if _pop(add, "X") == _out(fc) else _pop(add, "X")
        if g.is_param(y):
            continue
        ln = _single_consumer(g, _out(add), ("layer_norm",))
        if ln is None:
            continue
        if any(_out(ln, e) and (_out(ln, e) in g.keep or g.consumers(_out(ln, e)))
               for e in ("Mean", "Variance")):
            continue
        ins = {"X": [_pop(fc, "Input")], "W": [_pop(fc, "W")], "Y": [y],
               "Scale": [_pop(ln, "Scale")], "Bias1": [_pop(ln, "Bias")]}
        if _pop(fc, "Bias"):
            ins["Bias0"] = [_pop(fc, "Bias")]
        fused = _new(g.block, "fused_fc_elementwise_layernorm", ins, {"Out": [_out(ln, "Y")]},
                     {"x_num_col_dims": int(fc.attrs.get("in_num_col_dims", 1)),
                      "epsilon": float(ln.attrs.get("epsilon", 1e-5)), "begin_norm_axis": 1,
                      "activation_type": ""})
        g.replace([fc, add, ln], fused)
        n += 1
    return n


def _residual_add(g, base, other):
    """The unique elementwise_add consumer of ``other`` that adds the residual ``base``."""
    add = _single_consumer(g, other, ("elementwise_add",))
    if add is None or int(add.attrs.get("axis", -1)) != -1:
        return None
    if {_pop(add, "X"), _pop(add, "Y")} != {base, other}:
        return None
    return add


def fused_multi_transformer_encoder_traced_pass(g: Graph):
    """The traced-model form of `fused_multi_transformer_encoder_pass.cc` (the op-form passes over
    exported programs live in `fmt_passes.py`): one pre-LN decoder-only transformer layer as a
    ``jit.save``-traced program records it (after fc_fuse / self_attention_fuse) —
        ln1 = layer_norm(x); qkv = fc(ln1); attention (causal flash_attn over the head split);
        x2 = x + fc(attn); ln2 = layer_norm(x2); x3 = x2 + fc(fc(ln2, act))
    → one fused_multi_transformer op (the LLM inference kernels: fused LN prologues, packed QKV,
    flash / split-K decode attention over a KV cache, epilogue GEMMs)."""
    n = 0
    for ln1 in list(_typed(g.ops)):
        if ln1.type != "layer_norm" or ln1 not in g.ops:
            continue
        x = _pop(ln1, "X")
        chain = _attn_chain(g, _out(ln1, "Y"))
        if chain is None or len(g.consumers(_out(ln1, "Y"))) != 1:
            continue
        attn_ops, qkv_fc, (hq, hk), D, fa, attn_out = chain
        if not fa.attrs.get("causal") or fa.paddle_inputs.get("attn_mask"):
            continue
        ofc = _single_consumer(g, attn_out, ("fc",))
        if ofc is None or _fc_of(g, ofc)[3]:
            continue
        add1 = _residual_add(g, x, _out(ofc))
        if add1 is None:
            continue
        x2 = _out(add1)
        ln2s = [c for c in g.consumers(x2) if c.func is None and c.type == "layer_norm"]
        if len(ln2s) != 1 or len(g.consumers(x2)) != 2 or x2 in g.keep:
            continue
        ln2 = ln2s[0]
        f1 = _single_consumer(g, _out(ln2, "Y"), ("fc",))
        if f1 is None or _fc_of(g, f1)[3] not in ("gelu", "relu", "gelu_tanh", ""):
            continue
        f2 = _single_consumer(g, _out(f1), ("fc",))
        if f2 is None or _fc_of(g, f2)[3]:
            continue
        add2 = _residual_add(g, x2, _out(f2))
        if add2 is None:
            continue
        if len(g.consumers(x)) != 2:  # x feeds ln1 and the first residual add only
            continue
        eps1, eps2 = float(ln1.attrs.get("epsilon", 1e-5)), float(ln2.attrs.get("epsilon", 1e-5))
        if abs(eps1 - eps2) > 1e-12:
            continue
        wq = _pop(qkv_fc, "W")
        W = g.param(wq)
        E = W.shape[0]
        wn = wq + "@fmt"  # [E, Hq+2Hk, D] view: the trans_qkvw=False layout
        if wn not in g.program.params:
            g.program.params[wn] = W.reshape(E, hq + 2 * hk, D)
            g.block.create_var(wn, [E, hq + 2 * hk, D], "float32", persistable=True)
        act = _fc_of(g, f1)[3] or "none"
        ins = {"X": [x], "LnScale": [_pop(ln1, "Scale")], "LnBias": [_pop(ln1, "Bias")],
               "QKVW": [wn], "QKVBias": [_pop(qkv_fc, "Bias")], "OutLinearW": [_pop(ofc, "W")],
               "OutLinearBias": [_pop(ofc, "Bias")], "FFNLnScale": [_pop(ln2, "Scale")],
               "FFNLnBias": [_pop(ln2, "Bias")], "FFN1Weight": [_pop(f1, "W")],
               "FFN1Bias": [_pop(f1, "Bias")], "FFN2Weight": [_pop(f2, "W")], "FFN2Bias": [_pop(f2, "Bias")]}
        attrs = {"pre_layer_norm": True, "epsilon": eps1, "dropout_rate": 0.0, "is_test": True,
                 "dropout_implementation": "upscale_in_train", "act_method": act,
                 "trans_qkvw": False, "ring_id": -1, "causal": True}
        if hk != hq:
            attrs["num_kv_heads"] = hk
        fused = _new(g.block, "fused_multi_transformer", ins, {"Out": [_out(add2)]}, attrs)
        g.replace([ln1] + attn_ops + [ofc, add1, ln2, f1, f2, add2], fused)
        n += 1
    return n


_FMT_LIST_SLOTS = ("LnScale", "LnBias", "QKVW", "QKVBias", "OutLinearW", "OutLinearBias",
                   "FFNLnScale", "FFNLnBias", "FFN1Weight", "FFN1Bias", "FFN2Weight", "FFN2Bias",
                   "CacheKV", "QKVWScale", "OutLinearWScale", "FFN1WeightScale", "FFN2WeightScale")


def fuse_multi_transformer_layer_pass(g: Graph):
    """Reference `fuse_multi_transformer_layer_pass.cc`: consecutive single-layer
    fused_multi_transformer ops (Out of one = X of the next, same attrs) → ONE op whose weight
    slots list every layer (one launch sequence, one KV-cache list)."""
    n = 0
    changed = True
    while changed:
        changed = False
        for a in list(_typed(g.ops)):
            if a.type != "fused_multi_transformer" or a not in g.ops:
                continue
            b = _single_consumer(g, _out(a), ("fused_multi_transformer",))
            if b is None or _pop(b, "X") != _out(a):
                continue
            if {k: v for k, v in a.attrs.items()} != {k: v for k, v in b.attrs.items()}:
                continue
            ins = {"X": [_pop(a, "X")]}
            for slot in _FMT_LIST_SLOTS:
                va, vb = a.paddle_inputs.get(slot) or [], b.paddle_inputs.get(slot) or []
                if va or vb:
                    ins[slot] = list(va) + list(vb)
            for slot in ("TimeStep", "SrcMask", "SeqLengths", "BeamCacheOffset"):
                if a.paddle_inputs.get(slot):
                    ins[slot] = a.paddle_inputs[slot]
            outs = {"Out": [_out(b)]}
            ca, cb = (a.paddle_outputs.get("CacheKVOut") or []), (b.paddle_outputs.get("CacheKVOut") or [])
            if ca or cb:
                outs["CacheKVOut"] = list(ca) + list(cb)
            g.replace([a, b], _new(g.block, "fused_multi_transformer", ins, outs, dict(a.attrs)))
            n += 1
            changed = True
            break
    return n


# consumers that take a deferred LayerNorm (inference/ln_defer.py) and the input slots they take it in
_LN_DEFER_SLOTS = {"fc": ("Input",), "multihead_matmul": ("Input",), "fused_fc_elementwise_layernorm": ("Y",)}


def ln_defer_pass(g: Graph):
    """Post-LN chains at few rows: mark ``fused_fc_elementwise_layernorm`` ops whose output feeds
    only fold-aware consumers (the next QKV / FFN1 GEMM, the next residual epilogue) ``defer_ln``;
    at run time they hand on raw rows and the consumers apply the LayerNorm (``ln_defer``: weight
    fold + matrix-core row statistics, LN'd residual in the GEMM epilogue). Reference counterpart:
    the fused `fused_fc_elementwise_layernorm_op.cu` kernel, which still runs the LN per producer."""
    n = 0
    for op in _typed(g.ops):
        if op.type != "fused_fc_elementwise_layernorm" or op.attrs.get("activation_type") not in ("", None):
            continue
        out = _out(op)
        if not _pop(op, "Scale") or not _pop(op, "Bias1") or out in g.keep:
            continue
        cons = g.consumers(out)
        ok = bool(cons)
        for c in cons:
            slots = _LN_DEFER_SLOTS.get(c.type) if c.func is None and c.paddle_inputs else None
            if not slots or any(out in v and k not in slots for k, v in c.paddle_inputs.items()):
                ok = False
            elif c.type == "fc" and c.attrs.get("activation_type") not in ("", None, "gelu", "relu", "gelu_tanh"):
                ok = False
        if ok and not op.attrs.get("defer_ln"):
            op.attrs["defer_ln"] = True
            g.program._version += 1
            n += 1
    return n


from .fmt_passes import (  # noqa: E402
    PASS_ORDER as _FMT_ORDER,
    fused_multi_transformer_decoder_fuse_qkv_pass, fused_multi_transformer_decoder_pass,
    fused_multi_transformer_encoder_fuse_qkv_pass, multi_devices_fused_multi_transformer_decoder_fuse_qkv_pass,
    multi_devices_fused_multi_transformer_encoder_fuse_qkv_pass)
from .fmt_passes import fused_multi_transformer_encoder_pass_ops as fused_multi_transformer_encoder_pass  # noqa: E402

from .passes_extra import EXTRA_PASSES  # noqa: E402
from .passes_quant import QUANT_PASSES  # noqa: E402

globals().update(EXTRA_PASSES)
globals().update(QUANT_PASSES)

# Order follows the reference GpuPassStrategy: cleanups, the LLM layer passes, conv fusions, the
# matmul→mul maps (so fc_fuse sees one form), attention / fc / LN fusions, constant folding last.
GPU_PASSES = [
    "delete_weight_dequant_linear_op_pass",  # QAT exports: int8 weights onto the weight-only GEMM
    "is_test_pass", "simplify_with_basic_ops_pass",
    "delete_dropout_op_pass", "identity_scale_op_clean_pass", "identity_reshape_clean_pass",
    *_FMT_ORDER,  # the reference runs the LLM passes before the generic fc / attention fusions
    "conv_bn_fuse_pass", "conv_eltwiseadd_bn_fuse_pass", "embedding_eltwise_layernorm_fuse_pass",
    "self_attention_fuse_pass", "matmul_scale_fuse_pass",
    "gpu_cpu_squeeze2_matmul_fuse_pass", "gpu_cpu_reshape2_matmul_fuse_pass",
    "gpu_cpu_flatten2_matmul_fuse_pass", "gpu_cpu_map_matmul_v2_to_mul_pass",
    "gpu_cpu_map_matmul_v2_to_matmul_pass", "gpu_cpu_map_matmul_to_mul_pass",
    "fc_fuse_pass", "fc_act_fuse_pass", "fused_multi_transformer_encoder_traced_pass",
    "fuse_multi_transformer_layer_pass", "multihead_matmul_fuse_pass", "flash_attn_packed_fuse_pass",
    "fc_elementwise_layernorm_fuse_pass", "skip_layernorm_fuse_pass", "linear_bias_act_fuse_pass",
    "ln_defer_pass", "conv_elementwise_add2_act_fuse_pass", "conv_elementwise_add_act_fuse_pass",
    "conv_elementwise_add_fuse_pass", "transpose_flatten_concat_fuse_pass", "constant_folding_pass",
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
