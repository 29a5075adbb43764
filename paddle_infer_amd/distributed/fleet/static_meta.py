"""Static-graph Fleet meta-optimizers as Program rewrites (reference
`python/paddle/distributed/fleet/meta_optimizers/amp_optimizer.py:20`, `recompute_optimizer.py:20`,
`gradient_merge_optimizer.py:20`, `fp16_allreduce_optimizer.py:20`, `raw_program_optimizer.py`; the
rewrites themselves follow `fluid/contrib/mixed_precision/{fp16_utils,decorator}.py`,
`fluid/backward.py` ``_append_backward_ops_with_checkpoints_`` and `fluid/optimizer.py`
``GradientMergeOptimizer``):

* **amp** — ``cast`` ops in front of the white-list ops (matmul / mul / fc / linear / conv) feed them
  16-bit operands and a ``cast`` back in front of every black-list op (softmax-CE, reductions,
  norms) that would read a 16-bit value (``rewrite_program``). fp16 adds loss scaling as ops: the
  loss is multiplied by the persistable ``loss_scaling`` before backward; ``check_finite_and_unscale``
  divides every gradient by it and reports ``found_inf``; ``update_loss_scaling`` updates the scale
  (dynamic mode: good / bad step counters) and zeroes the gradients of a step with inf/nan; every
  optimizer op takes ``found_inf`` as ``SkipUpdate``.
* **recompute** — the forward ops between two consecutive checkpoints form a segment. Its ops run
  without keeping an autograd graph in the forward pass, and a copy of the segment (outputs renamed
  ``…@RECOMPUTE``) is emitted right before the segment's first grad op; the segment's grad ops read
  the copies, so its activations die after the forward pass (the executor's GC plan) and are
  recomputed from the checkpoints in backward. (Dropout inside a segment needs a fixed seed, as in
  the reference.)
* **gradient_merge** — every run adds each gradient into a persistable ``…@GRAD@MERGED``; a step
  counter selects every k-th run, whose ``conditional_block`` averages the merged gradients (``avg``),
  runs the data-parallel all-reduce and the optimizer ops, then zeroes the accumulators.
* **fp16_allreduce** — the data-parallel all-reduce moves fp16 copies of the gradients
  (``cast`` → ``c_allreduce_sum`` → ``cast`` back).
* data parallel — one ``c_allreduce_sum`` + ``scale`` 1/N per gradient ahead of the optimizer ops.
"""
from __future__ import annotations

import torch

from ...static.backward import BACKWARD, FORWARD, GRAD, OPTIMIZE, _persistable, op_role
from ...static.framework import Operator, Variable, VarRef
from ...static.proto import VT

AMP_WHITE = {"matmul_v2", "matmul", "mul", "fc", "linear", "conv2d", "depthwise_conv2d",
             "conv2d_transpose", "conv3d", "bmm", "mm", "fused_gemm_epilogue"}
AMP_BLACK = {"softmax_with_cross_entropy", "cross_entropy", "cross_entropy2", "mean", "reduce_mean",
             "reduce_sum", "sum", "exp", "log", "pow", "square", "sqrt", "layer_norm", "batch_norm",
             "softmax", "log_softmax", "sigmoid_cross_entropy_with_logits", "mse_loss", "cumsum",
             "elementwise_pow"}


def _mkop(block, type_, ins, outs, attrs, role):
    op = Operator(block, None, (), {}, None, type=type_, attrs=dict(attrs, op_role=role))
    op.paddle_inputs = {k: list(v) for k, v in ins.items()}
    op.paddle_outputs = {k: list(v) for k, v in outs.items()}
    return op


def _dtype(block, name):
    v = block.vars.get(name)
    if v is None:
        t = block.program.params.get(name)
        return t.dtype if t is not None else None
    with torch._C.DisableTorchFunctionSubclass():
        return v.dtype


def _new_var(block, name, like, dtype=None):
    with torch._C.DisableTorchFunctionSubclass():
        v = block.vars[like]
        meta = torch.empty(v.shape, dtype=dtype or v.dtype, device="meta")
    block.vars[name] = Variable(meta, name, block, False, False,
                                declared_shape=getattr(v, "declared_shape", None))
    return name


def rename_inputs(op, mapping):
    """Rename the INPUT references of ``op`` (traced args / kwargs and Paddle slots)."""
    if not mapping:
        return

    def ren(x):
        if isinstance(x, VarRef) and x.name in mapping:
            return VarRef(mapping[x.name])
        return x
    from torch.utils._pytree import tree_map
    op.args = tree_map(ren, op.args)
    op.kwargs = tree_map(ren, op.kwargs)
    if op.paddle_inputs:
        op.paddle_inputs = {k: [mapping.get(n, n) for n in v] for k, v in op.paddle_inputs.items()}


def _rename_outputs(op, mapping):
    def ren(x):
        if isinstance(x, VarRef) and x.name in mapping:
            return VarRef(mapping[x.name])
        return x
    from torch.utils._pytree import tree_map
    op.outputs = tree_map(ren, op.outputs)
    if op.paddle_outputs:
        op.paddle_outputs = {k: [mapping.get(n, n) for n in v] for k, v in op.paddle_outputs.items()}


def _copy_op(op):
    c = Operator(op.block, op.func, op.args, op.kwargs, op.outputs, type=op.type, attrs=dict(op.attrs))
    if op.paddle_inputs is not None:
        c.paddle_inputs = {k: list(v) for k, v in op.paddle_inputs.items()}
        c.paddle_outputs = {k: list(v) for k, v in (op.paddle_outputs or {}).items()}
    return c


def _bump(prog):
    prog._version = getattr(prog, "_version", 0) + 1


# ------------------------------------------------------------------------------------------ amp
def amp_rewrite_forward(block, dtype="bfloat16", white=None, black=None):
    """Insert the casts of ``rewrite_program``; returns the number of casts inserted."""
    white = (AMP_WHITE | set(white or ())) - set(black or ())
    black = AMP_BLACK | set(black or ())
    low = torch.bfloat16 if dtype == "bfloat16" else torch.float16
    code = VT[dtype]
    tag = "bf16" if dtype == "bfloat16" else "fp16"
    low_of = {}          # fp32 var -> its cast copy
    high_of = {}         # 16-bit var -> its fp32 cast copy
    low_vars = set()     # vars produced in 16-bit by white ops
    new_ops, n = [], 0
    for op in block.ops:
        if op_role(op) != FORWARD or op.type in ("cast", "feed", "fetch"):
            new_ops.append(op)
            continue
        ren = {}
        if op.type in white:
            for name in dict.fromkeys(op.input_names()):
                if name in low_vars or _dtype(block, name) != torch.float32:
                    continue
                c = low_of.get(name)
                if c is None:
                    c = low_of[name] = _new_var(block, f"{name}.cast_{tag}", name, low)
                    new_ops.append(_mkop(block, "cast", {"X": [name]}, {"Out": [c]},
                                         {"in_dtype": VT["float32"], "out_dtype": code}, FORWARD))
                    n += 1
                ren[name] = c
            rename_inputs(op, ren)
            low_vars.update(o for o in op.output_names() if _dtype(block, o) in (torch.float32, low))
        else:
            if op.type in black:
                for name in dict.fromkeys(op.input_names()):
                    if name not in low_vars:
                        continue
                    c = high_of.get(name)
                    if c is None:
                        c = high_of[name] = _new_var(block, f"{name}.cast_fp32", name, torch.float32)
                        new_ops.append(_mkop(block, "cast", {"X": [name]}, {"Out": [c]},
                                             {"in_dtype": code, "out_dtype": VT["float32"]}, FORWARD))
                        n += 1
                    ren[name] = c
                rename_inputs(op, ren)
            elif any(name in low_vars for name in op.input_names()):
                # gray op fed by a 16-bit value: its outputs follow the promoted dtype; a gray op
                # whose every float input is 16-bit stays 16-bit (reference gray-list rule)
                ins = [x for x in op.input_names() if _dtype(block, x) is not None and
                       (_dtype(block, x).is_floating_point)]
                if ins and all(x in low_vars or x in low_of.values() for x in ins):
                    low_vars.update(op.output_names())
        new_ops.append(op)
    block.ops[:] = new_ops
    for i, op in enumerate(block.ops):
        op.idx = i
    _bump(block.program)
    return n


def amp_scale_loss(block, loss, init_scaling):
    """scaled_loss = loss · loss_scaling (persistable [1] f32); returns (scaled Variable, name)."""
    prog = block.program
    ls = _persistable(prog, "loss_scaling_0", torch.tensor([float(init_scaling)], dtype=torch.float32))
    out = _new_var(block, loss.var_name + "@SCALED", loss.var_name)
    block.append_op(_mkop(block, "elementwise_mul", {"X": [loss.var_name], "Y": [ls]}, {"Out": [out]},
                          {"axis": -1}, FORWARD))
    return block.vars[out], ls


def _optimizer_ops(block):
    return [op for op in block.ops if op_role(op) == OPTIMIZE and op.paddle_inputs
            and "Grad" in op.paddle_inputs]


def amp_unscale_and_skip(block, ls, cfg, merged=False):
    """check_finite_and_unscale + update_loss_scaling ahead of the optimizer ops; every optimizer
    op skips its update on a step with inf/nan (SkipUpdate = found_inf). ``merged`` (gradient
    merge follows): the two ops take the OPTIMIZE role so ``gradient_merge_rewrite`` moves them
    into the every-k-steps block, where they act once on the merged gradients (reference
    GradientMergeOptimizer runs the AMP apply_gradients inside its conditional block)."""
    prog = block.program
    opt_ops = _optimizer_ops(block)
    grads = list(dict.fromkeys(op.paddle_inputs["Grad"][0] for op in opt_ops))
    found = _persistable(prog, "find_infinite_scale_0", torch.zeros([1], dtype=torch.bool))
    good = _persistable(prog, "num_good_steps_0", torch.zeros([1], dtype=torch.int32))
    bad = _persistable(prog, "num_bad_steps_0", torch.zeros([1], dtype=torch.int32))
    first = min(i for i, op in enumerate(block.ops) if op_role(op) == OPTIMIZE)
    # BACKWARD role: once per run; OPTIMIZE role under gradient merge: once per k runs
    role = OPTIMIZE if merged else BACKWARD
    new = [_mkop(block, "check_finite_and_unscale", {"X": grads, "Scale": [ls]},
                 {"Out": grads, "FoundInfinite": [found]}, {}, role)]
    if cfg.get("use_dynamic_loss_scaling", True):
        new.append(_mkop(block, "update_loss_scaling",
                         {"X": grads, "FoundInfinite": [found], "PrevLossScaling": [ls],
                          "InGoodSteps": [good], "InBadSteps": [bad]},
                         {"Out": grads, "LossScaling": [ls], "OutGoodSteps": [good], "OutBadSteps": [bad]},
                         {"incr_every_n_steps": int(cfg.get("incr_every_n_steps", 1000)),
                          "decr_every_n_nan_or_inf": int(cfg.get("decr_every_n_nan_or_inf", 2)),
                          "incr_ratio": float(cfg.get("incr_ratio", 2.0)),
                          "decr_ratio": float(cfg.get("decr_ratio", 0.5)), "stop_update": False},
                         role))
    block.ops[first:first] = new
    for op in opt_ops:
        op.paddle_inputs["SkipUpdate"] = [found]
    for i, op in enumerate(block.ops):
        op.idx = i
    _bump(prog)


# ------------------------------------------------------------------------------------ recompute
def recompute_rewrite(block, checkpoints):
    """Segments between consecutive checkpoints: forward ops run graph-free, a renamed copy runs
    ahead of the segment's grad ops. Returns the number of re-emitted ops."""
    ck = [c if isinstance(c, str) else c.var_name for c in checkpoints]
    fwd = [(i, op) for i, op in enumerate(block.ops) if op_role(op) == FORWARD]
    producer = {}
    for i, op in fwd:
        for o in op.output_names():
            producer.setdefault(o, i)
    pos = sorted({producer[c] for c in ck if c in producer})
    if len(pos) < 2:
        return 0
    ckset = set(ck)
    segments = []
    for a, b in zip(pos[:-1], pos[1:]):
        seg = [op for i, op in fwd if a < i <= b]
        if seg:
            segments.append(seg)
    grad_ops = [op for op in block.ops if op_role(op) == BACKWARD and getattr(op, "fwd_op", None) is not None]
    inserted = 0
    for seg in segments:
        ids = {id(op) for op in seg}
        produced = set()
        for op in seg:
            produced.update(op.output_names())
        # every value the segment produces (its closing checkpoint too) is re-produced under a new
        # name, so the forward values stay untouched for the ops outside the segment
        inner = {n: n + "@RECOMPUTE" for n in produced}
        if not inner:
            continue
        gseg = [g for g in grad_ops if id(g.fwd_op) in ids]
        if not gseg:
            continue
        at = min(block.ops.index(g) for g in gseg)
        copies = []
        for op in seg:
            op.attrs["_recompute_fwd"] = True   # original: no autograd graph kept (executor)
            c = _copy_op(op)
            rename_inputs(c, inner)
            _rename_outputs(c, inner)
            c.attrs.pop("_recompute_fwd", None)
            c.attrs["op_role"] = FORWARD
            c.attrs["_recompute_copy"] = True
            for n in op.output_names():
                if n in inner:
                    _new_var(block, inner[n], n)
            copies.append(c)
        block.ops[at:at] = copies
        inserted += len(copies)
        for g in gseg:
            rename_inputs(g, inner)
            g.fwd_op = next(c for o, c in zip(seg, copies) if o is g.fwd_op)
    for i, op in enumerate(block.ops):
        op.idx = i
    _bump(block.program)
    return inserted


# ------------------------------------------------------------------------- allreduce / merge
def _allreduce_ops(block, grads, world, fp16, role):
    ops = []
    for g in grads:
        tgt = g
        if fp16 and _dtype(block, g) == torch.float32:
            tgt = _new_var(block, g + "@FP16", g, torch.float16)
            ops.append(_mkop(block, "cast", {"X": [g]}, {"Out": [tgt]},
                             {"in_dtype": VT["float32"], "out_dtype": VT["float16"]}, role))
        ops.append(_mkop(block, "c_allreduce_sum", {"X": [tgt]}, {"Out": [tgt]},
                         {"ring_id": 0, "use_calc_stream": True}, role))
        if tgt != g:
            ops.append(_mkop(block, "cast", {"X": [tgt]}, {"Out": [g]},
                             {"in_dtype": VT["float16"], "out_dtype": VT["float32"]}, role))
        ops.append(_mkop(block, "scale", {"X": [g]}, {"Out": [g]},
                         {"scale": 1.0 / world, "bias": 0.0, "bias_after_scale": True}, role))
    return ops


def insert_dp_allreduce(block, world, fp16=False):
    """One (fp16-cast) c_allreduce_sum + scale 1/N per gradient ahead of the optimizer ops."""
    ops = block.ops
    first = next((i for i, op in enumerate(ops) if op_role(op) == OPTIMIZE), len(ops))
    grads = sorted({n for op in ops[first:] if op_role(op) == OPTIMIZE for n in op.input_names()
                    if n.endswith(GRAD)})
    block.ops[first:first] = _allreduce_ops(block, grads, world, fp16, BACKWARD)
    for i, op in enumerate(block.ops):
        op.idx = i
    _bump(block.program)


def gradient_merge_rewrite(block, k_steps, avg=True, world=1, fp16_allreduce=False):
    """Merge gradients over ``k_steps`` runs; the optimizer (and the all-reduce) run every k-th."""
    prog = block.program
    first = next(i for i, op in enumerate(block.ops) if op_role(op) == OPTIMIZE)
    tail = block.ops[first:]
    grads = sorted({n for op in tail for n in op.input_names() if n.endswith(GRAD)
                    and op.paddle_inputs is not None})
    merged = {}
    pre = []
    for g in grads:
        p = g[: -len(GRAD)]
        base = prog.params.get(p)
        if base is None:
            continue
        m = _persistable(prog, g + "@MERGED", torch.zeros_like(base, dtype=torch.float32))
        merged[g] = m
        pre.append(_mkop(block, "elementwise_add", {"X": [m], "Y": [g]}, {"Out": [m]}, {"axis": -1}, OPTIMIZE))
    step = _persistable(prog, "gradient_merge_step", torch.zeros([1], dtype=torch.int32))
    kv = _persistable(prog, "gradient_merge_k", torch.tensor([int(k_steps)], dtype=torch.int32))
    zero = _persistable(prog, "gradient_merge_zero", torch.zeros([1], dtype=torch.int32))
    cond = _new_var(block, "gradient_merge_cond", step, torch.bool)
    pre += [_mkop(block, "increment", {"X": [step]}, {"Out": [step]}, {"step": 1.0}, OPTIMIZE),
            _mkop(block, "elementwise_mod", {"X": [step], "Y": [kv]}, {"Out": [step]}, {"axis": -1}, OPTIMIZE),
            _mkop(block, "equal", {"X": [step], "Y": [zero]}, {"Out": [cond]}, {"axis": -1}, OPTIMIZE)]
    sub = prog._create_block(block.idx)
    body = []
    if avg and k_steps > 1:
        for g, m in merged.items():
            body.append(_mkop(sub, "scale", {"X": [m]}, {"Out": [m]},
                              {"scale": 1.0 / k_steps, "bias": 0.0, "bias_after_scale": True}, OPTIMIZE))
    if world > 1:
        body += _allreduce_ops(sub, list(merged.values()), world, fp16_allreduce, OPTIMIZE)
    for op in tail:
        rename_inputs(op, merged)
        if op.type in ("check_finite_and_unscale", "update_loss_scaling"):
            _rename_outputs(op, merged)  # unscale the merged gradients in place
        op.block = sub
        body.append(op)
    for g, m in merged.items():
        body.append(_mkop(sub, "fill_zeros_like", {"X": [m]}, {"Out": [m]}, {}, OPTIMIZE))
    sub.ops[:] = body
    for i, op in enumerate(sub.ops):
        op.idx = i
    produced_in = set()
    for op in body:
        produced_in.update(op.output_names())
    ext = sorted({n for op in body for n in op.input_names()} - (produced_in - set(merged.values())))
    cb = _mkop(block, "conditional_block", {"Cond": [cond], "Input": ext},
               {"Out": sorted(produced_in), "Scope": []},
               {"sub_block": sub.idx, "is_scalar_condition": True}, OPTIMIZE)
    block.ops[first:] = pre + [cb]
    for i, op in enumerate(block.ops):
        op.idx = i
    _bump(prog)
    return merged


Variable  # noqa
