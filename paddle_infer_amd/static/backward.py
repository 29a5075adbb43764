"""Static autodiff: ``append_backward`` / ``gradients`` and the optimizer pass of ``minimize``.

Parity: reference `python/paddle/fluid/backward.py:1569` (append_backward: walk the ops that lie
between the parameters and the loss in reverse, emit one ``<type>_grad`` op per forward op,
``fill_constant``-style seed for ``loss@GRAD``, renamed partial gradients
``x@GRAD@RENAME@k`` summed by a ``sum`` op when a variable feeds several ops — the reference's
``_addup_repetitive_outputs_``), ``gradients`` (:func:`gradients`), and
`python/paddle/optimizer/optimizer.py` ``_create_optimization_pass`` (one ``sgd`` / ``momentum`` /
``adam`` / ``adamw`` op per parameter with persistable accumulators ``<param>_moment1_0`` …, a
persistable learning-rate variable, the grad clip and L2 regularization appended as ops). Every
backward op carries ``op_role`` (reference `framework.py` OpRole: Forward 0, Backward 1,
Optimize 2, Loss 256).

Grad ops are Paddle-typed (slot dicts): the forward op's input slots + output slots +
``<out slot>@GRAD``  →  ``<in slot>@GRAD``, attributes copied from the forward op. For an op
recorded from a torch / framework callable the slots are ``X`` (its inputs) and ``Out`` (its
outputs). The Executor runs a grad op as the VJP of its forward op (`executor.py`
``_run_grad_op``): through the autograd graph the forward built in the same run, or, when that
graph is absent, by re-running the forward op on detached leaves. ``save_train_program``
(`io.py`) re-derives the backward over the lowered Paddle forward so a saved training program
holds only reference op types (``matmul_v2_grad``, ``elementwise_add_grad`` ...).
"""
from __future__ import annotations

import copy

import torch

from .framework import Operator, VarRef, Variable

FORWARD, BACKWARD, OPTIMIZE, LOSS = 0, 1, 2, 256
GRAD = "@GRAD"
_LEGACY = ("backward", "optimize")


def op_role(op):
    if op.type in _LEGACY:
        return BACKWARD if op.type == "backward" else OPTIMIZE
    return int(op.attrs.get("op_role", FORWARD)) & ~LOSS


def is_grad_op(op):
    return op.type.endswith("_grad") and op_role(op) == BACKWARD


def _trainable_params(program, parameter_list=None):
    names = []
    if parameter_list:
        for p in parameter_list:
            names.append(p if isinstance(p, str) else (p.var_name if isinstance(p, Variable) else program.param_var(p)))
        return names
    for name, t in program.params.items():
        if t.is_floating_point() and t.requires_grad:
            names.append(name)
    return names


def _meta_of(block, name):
    v = block.vars[name]
    with torch._C.DisableTorchFunctionSubclass():
        return torch.empty(v.shape, dtype=v.dtype, device="meta")


def _is_float(block, name):
    v = block.vars.get(name)
    if v is None:
        return False
    with torch._C.DisableTorchFunctionSubclass():
        return v.dtype.is_floating_point or v.dtype.is_complex


def _new_var(block, name, like):
    if name not in block.vars:
        block.vars[name] = Variable(_meta_of(block, like), name, block, False, True)
    return name


def _paddle_op(block, type_, ins, outs, attrs):
    op = Operator(block, None, (), {}, None, type=type_, attrs=attrs)
    op.paddle_inputs = {k: list(v) for k, v in ins.items()}
    op.paddle_outputs = {k: list(v) for k, v in outs.items()}
    return block.append_op(op)


def fwd_slots(op):
    """(input slots, output slots) of a forward op: Paddle slots, or X / Out for a recorded op."""
    if op.func is None and op.paddle_inputs is not None:
        return dict(op.paddle_inputs), dict(op.paddle_outputs or {})
    return {"X": op.input_names()}, {"Out": op.output_names()}


def build_backward(block, loss_name, wrt, stop=()):
    """Append the grad ops of ``loss_name`` w.r.t. the variables ``wrt`` to ``block``; returns the
    names in ``wrt`` that received a gradient (``<name>@GRAD``)."""
    stop = set(stop)
    fwd_ops = [op for op in block.ops if op_role(op) == FORWARD]
    dep = set(wrt)  # variables that depend on a differentiated variable
    for op in fwd_ops:
        if any(n in dep for n in op.input_names()):
            dep.update(o for o in op.output_names() if _is_float(block, o) and o not in stop)
    need = {loss_name}
    path = []  # forward ops between wrt and the loss, reverse program order
    for op in reversed(fwd_ops):
        if any(o in need for o in op.output_names()) and any(i in dep for i in op.input_names()):
            path.append(op)
            need.update(i for i in op.input_names() if i in dep)
    consumers = {}
    for op in path:
        for i in dict.fromkeys(op.input_names()):
            if i in dep and i in need:
                consumers[i] = consumers.get(i, 0) + 1
    pending = {loss_name: [loss_name + GRAD]}
    _new_var(block, loss_name + GRAD, loss_name)
    _paddle_op(block, "fill_any_like", {"X": [loss_name]}, {"Out": [loss_name + GRAD]},
               {"value": 1.0, "dtype": -1, "op_role": BACKWARD | LOSS})
    done = set()

    def finalize(name):
        parts = pending.get(name)
        if not parts:
            return ""
        if name not in done:
            done.add(name)
            if len(parts) > 1:
                _new_var(block, name + GRAD, name)
                _paddle_op(block, "sum", {"X": parts}, {"Out": [name + GRAD]}, {"op_role": BACKWARD})
        return name + GRAD

    for fop in path:
        ins, outs = fwd_slots(fop)
        out_g = {s: [finalize(o) if o in need else "" for o in names] for s, names in outs.items()}
        if not any(g for gs in out_g.values() for g in gs):
            continue
        in_g, seen = {}, set()
        for s, names in ins.items():
            gs = []
            for x in names:
                if x in dep and x in need and x not in seen:
                    seen.add(x)
                    k = len(pending.setdefault(x, []))
                    g = x + GRAD if consumers.get(x, 1) == 1 else f"{x}{GRAD}@RENAME@{k}"
                    pending[x].append(_new_var(block, g, x))
                    gs.append(g)
                else:
                    gs.append("")
            in_g[s + GRAD] = gs
        gins = dict(ins)
        gins.update(outs)
        gins.update({s + GRAD: gs for s, gs in out_g.items()})
        attrs = {k: v for k, v in fop.attrs.items() if k != "op_role"}
        attrs["op_role"] = BACKWARD
        gop = _paddle_op(block, fop.type + "_grad", gins, in_g, attrs)
        gop.fwd_op = fop
    return [w for w in wrt if finalize(w)]


def append_backward(loss, parameter_list=None, no_grad_set=None, callbacks=None, checkpoints=None):
    block = loss.block
    prog = block.program
    names = _trainable_params(prog, parameter_list)
    skip = set()
    if no_grad_set:
        skip = {n if isinstance(n, str) else n.var_name for n in no_grad_set}
        names = [n for n in names if n not in skip]
    got = build_backward(block, loss.var_name, names, stop=skip)
    prog._backward_info = {"loss": loss.var_name, "params": list(got), "stop": sorted(skip)}
    return [(block.vars[n], block.vars[n + GRAD]) for n in got]


def gradients(targets, inputs, target_gradients=None, no_grad_set=None):
    """Reference `fluid/backward.py` ``gradients``: d(sum targets)/d(inputs); ``None`` for an input
    the targets do not depend on."""
    t = targets[0] if isinstance(targets, (list, tuple)) else targets
    ins = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    names = [i.var_name if isinstance(i, Variable) else i for i in ins]
    block = t.block
    got = set(build_backward(block, t.var_name, names))
    block.program._grad_roots = set(getattr(block.program, "_grad_roots", set())) | set(names)
    return [block.vars[n + GRAD] if n in got else None for n in names]


# ------------------------------------------------------------------------ optimizer pass
class OptimizerSpec:
    """A dygraph optimizer captured at program-build time; bound to the Scope's parameters on the
    Executor's first run (optimizers without a static op form)."""

    def __init__(self, opt):
        self.opt = opt

    def bind(self, params):
        o = copy.copy(self.opt)
        o._parameter_list = params
        o._param_groups = None
        o._accumulators = {}
        o._master = {}
        o._step = 0
        if hasattr(o, "_flat"):
            o._flat = None
            if params and all(p.is_cuda for p in params):
                o._maybe_flat({})
        return o


def _persistable(prog, name, value):
    """A persistable program variable holding ``value`` (optimizer accumulator / LR)."""
    b = prog.global_block()
    t = value.detach().clone()
    prog.params[name] = t
    prog._param_of[id(t)] = name
    meta = torch.empty(t.shape, dtype=t.dtype, device="meta")
    b.vars[name] = Variable(meta, name, b, True, True, declared_shape=list(t.shape))
    prog._opt_vars = set(getattr(prog, "_opt_vars", ())) | {name}
    return name


def _static_grad_clip(block, clip, grads):
    """Grad clip as recorded ops on the gradient Variables (reference ClipGradBy*._static_clip)."""
    from ..nn import clip as _clip
    from .framework import _STATE
    prev = _STATE["static"]
    _STATE["static"] = True
    try:
        gv = [block.vars[g] for g in grads]
        if isinstance(clip, _clip.ClipGradByGlobalNorm):
            sq = [torch.sum(torch.square(g.float())) for g in gv]
            total = torch.sqrt(torch.stack(sq).sum())
            scale = clip.clip_norm / torch.clamp(total, min=clip.clip_norm)
            outs = [g * scale.to(g.dtype) for g in gv]
        elif isinstance(clip, _clip.ClipGradByNorm):
            outs = [g * torch.clamp(clip.clip_norm / (torch.sqrt(torch.sum(torch.square(g.float()))) + 1e-6),
                                    max=1.0).to(g.dtype) for g in gv]
        elif isinstance(clip, _clip.ClipGradByValue):
            outs = [torch.clamp(g, clip.min, clip.max) for g in gv]
        else:
            raise NotImplementedError(type(clip).__name__)
    finally:
        _STATE["static"] = prev
    return [o.var_name for o in outs]


def minimize(optimizer, loss, parameter_list=None, no_grad_set=None):
    from .. import optimizer as O
    pg = append_backward(loss, parameter_list, no_grad_set)
    block = loss.block
    prog = block.program
    names = [p.var_name for p, _ in pg]
    first = len(block.ops)
    kind = type(optimizer)
    static_form = kind in (O.SGD, O.Momentum, O.Adam, O.AdamW) and optimizer._param_groups is None \
        and (optimizer._grad_clip is None or type(optimizer._grad_clip).__name__ in (
            "ClipGradByGlobalNorm", "ClipGradByNorm", "ClipGradByValue"))
    if not static_form:
        op = Operator(block, None, tuple(VarRef(n + GRAD) for n in names), {}, None, type="optimize",
                      attrs={"optimizer": OptimizerSpec(optimizer), "params": names, "op_role": OPTIMIZE})
        block.append_op(op)
        return None, pg
    grads = [n + GRAD for n in names]
    if optimizer._grad_clip is not None:
        grads = _static_grad_clip(block, optimizer._grad_clip, grads)
    lr_name = f"learning_rate_{id(optimizer) % 100000}"
    _persistable(prog, lr_name, torch.tensor([optimizer.get_lr()], dtype=torch.float32))
    prog._lr_vars = dict(getattr(prog, "_lr_vars", {}))
    prog._lr_vars[lr_name] = optimizer
    wd = optimizer.regularization
    coeff = wd if isinstance(wd, (int, float)) else getattr(wd, "_coeff", 0.0) if wd is not None else 0.0
    for n, g in zip(names, grads):
        p = prog.params[n]
        ins = {"Param": [n], "Grad": [g], "LearningRate": [lr_name]}
        outs = {"ParamOut": [n]}
        attrs = {"op_role": OPTIMIZE}
        if kind is O.SGD:
            t = "sgd"
        elif kind is O.Momentum:
            t = "momentum"
            v = _persistable(prog, f"{n}_velocity_0", torch.zeros_like(p, dtype=torch.float32))
            ins["Velocity"], outs["VelocityOut"] = [v], [v]
            attrs.update(mu=float(optimizer._momentum), use_nesterov=bool(optimizer._nesterov),
                         rescale_grad=float(optimizer._rescale))
        else:
            t = "adamw" if kind is O.AdamW else "adam"
            m1 = _persistable(prog, f"{n}_moment1_0", torch.zeros_like(p, dtype=torch.float32))
            m2 = _persistable(prog, f"{n}_moment2_0", torch.zeros_like(p, dtype=torch.float32))
            b1 = _persistable(prog, f"{n}_beta1_pow_acc_0", torch.tensor([optimizer._beta1], dtype=torch.float32))
            b2 = _persistable(prog, f"{n}_beta2_pow_acc_0", torch.tensor([optimizer._beta2], dtype=torch.float32))
            ins.update(Moment1=[m1], Moment2=[m2], Beta1Pow=[b1], Beta2Pow=[b2])
            outs.update(Moment1Out=[m1], Moment2Out=[m2], Beta1PowOut=[b1], Beta2PowOut=[b2])
            attrs.update(beta1=optimizer._beta1, beta2=optimizer._beta2, epsilon=optimizer._epsilon)
            if kind is O.AdamW:
                c = optimizer._coeff_for(p) if hasattr(optimizer, "_coeff_for") else optimizer._wd
                fn = getattr(optimizer, "_apply_decay_param_fun", None)
                if fn is not None:
                    c = optimizer._wd if fn(getattr(p, "pd_name", n)) else 0.0
                attrs.update(coeff=float(c), with_decay=bool(c), lr_ratio=1.0)
        if kind is not O.AdamW and coeff:  # L2Decay: regularization_method on the op (reference)
            attrs.update(regularization_method="l2_decay", regularization_coeff=float(coeff))
        _paddle_op(block, t, ins, outs, attrs)
    for op in block.ops[first:]:
        op.attrs.setdefault("op_role", OPTIMIZE)
        op.attrs["op_role"] = OPTIMIZE
    return None, pg
