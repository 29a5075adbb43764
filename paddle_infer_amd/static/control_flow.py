"""Control flow in static Programs: ``cond`` and ``while_loop`` as ops with sub-blocks.

Parity: reference `python/paddle/fluid/layers/control_flow.py` (``cond`` → two
``conditional_block`` ops + ``select_input``; ``while_loop`` → a ``while`` op whose sub-block
recomputes the condition) and the executor side `paddle/fluid/operators/controlflow/
{conditional_block_op,while_op}.cc`.

Here one ``cond`` op holds both branch blocks (attrs ``true_block`` / ``false_block`` + the branch
result names) and one ``while`` op holds a condition block and a body block with the loop-carried
variables. Tracing records each branch / body into its own sub-block (``Program._block_guard``);
the Executor evaluates the predicate on the device value (one host read per decision, as in the
reference) and runs only the chosen block. append_backward differentiates each control-flow op as
one op (``cond_grad`` / ``while_grad``: the VJP of the branch / iterations actually taken). On save
(`io._CFLowering`) they become the reference's own ops — ``conditional_block`` + ``select_input``
and ``while`` with sub-blocks — which `run_conditional_block` / `run_paddle_while` execute.
"""
from __future__ import annotations

import torch

from .framework import Operator, Variable, unique_name


def _as_var(prog, v):
    """A branch / loop value as a Program variable (real tensors and Python scalars become
    persistable constants)."""
    if isinstance(v, Variable):
        return v
    if isinstance(v, torch.Tensor):
        return prog.global_block().vars[prog.param_var(v)]
    if isinstance(v, (bool, int, float)):
        t = torch.tensor(v)
        return prog.global_block().vars[prog.param_var(t)]
    raise TypeError(f"control-flow value of type {type(v).__name__} is not a tensor")


def _meta(v):
    with torch._C.DisableTorchFunctionSubclass():
        return torch.empty(v.shape, dtype=v.dtype, device="meta")


def _external_reads(block):
    """Names read by the ops of ``block`` that the block does not produce itself."""
    made, ext = set(), []
    for op in block.ops:
        for n in op.input_names():
            if n not in made and n not in ext:
                ext.append(n)
        made.update(op.output_names())
        for k in ("true_block", "false_block", "cond_block", "body_block"):
            if k in op.attrs:  # nested control flow: its inputs are already listed on the op
                pass
    return ext


def _flatten(out):
    if isinstance(out, (list, tuple)):
        return list(out), type(out)
    return [out], None


def cond(pred, true_fn, false_fn):
    prog = pred.block.program
    parent = prog.current_block()
    tb, fb = prog._create_block(parent.idx), prog._create_block(parent.idx)
    with prog._block_guard(tb):
        t_out = true_fn() if true_fn is not None else None
    with prog._block_guard(fb):
        f_out = false_fn() if false_fn is not None else None
    if t_out is None and f_out is None:
        outs_t, outs_f, kind = [], [], None
    else:
        outs_t, kind = _flatten(t_out)
        outs_f, _ = _flatten(f_out)
        if len(outs_t) != len(outs_f):
            raise ValueError(f"cond branches return {len(outs_t)} vs {len(outs_f)} values")
    results, t_names, f_names, passthrough = [], [], [], {}
    for i, (a, b) in enumerate(zip(outs_t, outs_f)):
        if not isinstance(a, (Variable, torch.Tensor)) and not isinstance(b, (Variable, torch.Tensor)):
            if a is b or a == b:  # identical Python values in both branches
                passthrough[i] = a
                continue
        va, vb = _as_var(prog, a), _as_var(prog, b)
        ma, mb = _meta(va), _meta(vb)
        if ma.dtype != mb.dtype:
            raise TypeError(f"cond output {i}: dtype {ma.dtype} vs {mb.dtype}")
        name = unique_name("cond_out")
        meta = ma if ma.shape == mb.shape else torch.empty(
            [x if x == y else 1 for x, y in zip(ma.shape, mb.shape)] if ma.dim() == mb.dim() else ma.shape,
            dtype=ma.dtype, device="meta")
        parent.vars[name] = Variable(meta, name, parent, False, True)
        t_names.append(va.var_name)
        f_names.append(vb.var_name)
        results.append((i, parent.vars[name]))
    ext = [n for n in dict.fromkeys(_external_reads(tb) + _external_reads(fb) + t_names + f_names)
           if n not in {o for op in tb.ops + fb.ops for o in op.output_names()}]
    op = Operator(parent, None, (), {}, None, type="cond",
                  attrs={"true_block": tb.idx, "false_block": fb.idx, "true_outs": t_names,
                         "false_outs": f_names})
    op.paddle_inputs = {"Cond": [pred.var_name], "Input": ext}
    op.paddle_outputs = {"Out": [v.var_name for _, v in results]}
    parent.append_op(op)
    if kind is None and t_out is None:
        return None
    vals = [None] * len(outs_t)
    for i, v in passthrough.items():
        vals[i] = v
    for i, v in results:
        vals[i] = v
    return vals[0] if kind is None else kind(vals)


def while_loop(cond_fn, body_fn, loop_vars):
    prog = None
    for v in loop_vars:
        if isinstance(v, Variable):
            prog = v.block.program
            break
    parent = prog.current_block()
    init = [_as_var(prog, v) for v in loop_vars]
    carried = []
    for v in init:  # loop-carried names: the cond / body blocks read these
        n = unique_name("loop_var")
        parent.vars[n] = Variable(_meta(v), n, parent, False, True)
        carried.append(parent.vars[n])
    cb, bb = prog._create_block(parent.idx), prog._create_block(parent.idx)
    with prog._block_guard(cb):
        c = cond_fn(*carried)
    if not isinstance(c, Variable):
        raise TypeError("while_loop condition must be a boolean tensor inside a static program")
    with prog._block_guard(bb):
        nxt = body_fn(*carried)
    nxt, _ = _flatten(nxt)
    if len(nxt) != len(carried):
        raise ValueError(f"while_loop body returns {len(nxt)} values for {len(carried)} loop vars")
    nxt = [_as_var(prog, v) for v in nxt]
    outs = []
    for v in carried:
        n = unique_name("loop_out")
        parent.vars[n] = Variable(_meta(v), n, parent, False, True)
        outs.append(parent.vars[n])
    carried_names = {v.var_name for v in carried}
    made = {o for op in cb.ops + bb.ops for o in op.output_names()}
    ext = [n for n in dict.fromkeys(_external_reads(cb) + _external_reads(bb) + [v.var_name for v in nxt])
           if n not in made and n not in carried_names]
    op = Operator(parent, None, (), {}, None, type="while",
                  attrs={"cond_block": cb.idx, "body_block": bb.idx, "cond_out": c.var_name,
                         "carried": [v.var_name for v in carried], "body_outs": [v.var_name for v in nxt]})
    op.paddle_inputs = {"X": [v.var_name for v in init], "Input": ext}
    op.paddle_outputs = {"Out": [v.var_name for v in outs]}
    parent.append_op(op)
    return outs


def run_cond(executor, op, sub, env, scope, program):
    p = sub_value(op.paddle_inputs["Cond"][0], sub)
    take = bool(p.reshape(-1)[0].item()) if isinstance(p, torch.Tensor) else bool(p)
    blk = program.block(op.attrs["true_block" if take else "false_block"])
    for o in blk.ops:
        executor._run_op(o, sub, env, scope, program)
    srcs = op.attrs["true_outs" if take else "false_outs"]
    for dst, src in zip(op.paddle_outputs["Out"], srcs):
        env[dst] = sub_value(src, sub)


def run_while(executor, op, sub, env, scope, program, max_iters=10 ** 7):
    for dst, src in zip(op.attrs["carried"], op.paddle_inputs["X"]):
        env[dst] = sub_value(src, sub)
    cb, bb = program.block(op.attrs["cond_block"]), program.block(op.attrs["body_block"])
    for _ in range(max_iters):
        for o in cb.ops:
            executor._run_op(o, sub, env, scope, program)
        c = sub_value(op.attrs["cond_out"], sub)
        if not (bool(c.reshape(-1)[0].item()) if isinstance(c, torch.Tensor) else bool(c)):
            break
        for o in bb.ops:
            executor._run_op(o, sub, env, scope, program)
        new = [sub_value(n, sub) for n in op.attrs["body_outs"]]
        for dst, v in zip(op.attrs["carried"], new):
            env[dst] = v
    else:
        raise RuntimeError("while op exceeded max_iters")
    for dst, src in zip(op.paddle_outputs["Out"], op.attrs["carried"]):
        env[dst] = env[src]


def _truth(v):
    return bool(v.reshape(-1)[0].item()) if isinstance(v, torch.Tensor) else bool(v)


def run_paddle_while(executor, op, sub, env, scope, program, max_iters=10 ** 7):
    """Reference `controlflow/while_op.cc`: run ``sub_block`` while the Condition variable is
    true. The block updates the loop variables (and the condition) by name, in place — the
    Executor's environment is the scope the reference's step scopes read through."""
    cond = op.paddle_inputs["Condition"][0]
    blk = program.block(op.attrs["sub_block"])
    for _ in range(max_iters):
        if not _truth(sub_value(cond, sub)):
            return
        for o in blk.ops:
            executor._run_op(o, sub, env, scope, program)
    raise RuntimeError("while op exceeded max_iters")


def run_conditional_block(executor, op, sub, env, scope, program):
    """Reference `controlflow/conditional_block_op.cc`: run ``sub_block`` when the scalar Cond is
    true (``is_scalar_condition``) or, otherwise, when every Cond tensor is non-empty."""
    conds = [sub_value(n, sub) for n in op.paddle_inputs.get("Cond", [])]
    if op.attrs.get("is_scalar_condition", False):
        run = _truth(conds[0])
    else:
        run = all(isinstance(c, torch.Tensor) and c.numel() > 0 for c in conds)
    if run:
        for o in program.block(op.attrs["sub_block"]).ops:
            executor._run_op(o, sub, env, scope, program)


def sub_value(name, sub):
    from .framework import VarRef
    return sub(VarRef(name))
