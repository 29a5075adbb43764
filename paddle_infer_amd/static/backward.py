"""Static autodiff: ``append_backward`` / ``gradients`` (reference `python/paddle/fluid/backward.py`).

Instead of emitting one grad op per forward op, the program gets a single ``backward`` op whose
execution runs autograd over the forward ops the Executor just ran (the forward is executed with
grad enabled when the program contains a backward op). Its outputs are the ``<param>@GRAD``
variables, consumed by ``optimize`` ops or fetched directly.
"""
from __future__ import annotations

import copy

import torch

from .framework import Operator, VarRef, Variable


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


def append_backward(loss, parameter_list=None, no_grad_set=None, callbacks=None, checkpoints=None):
    block = loss.block
    prog = block.program
    names = _trainable_params(prog, parameter_list)
    if no_grad_set:
        skip = {n if isinstance(n, str) else n.var_name for n in no_grad_set}
        names = [n for n in names if n not in skip]
    outs = []
    for n in names:
        g = n + "@GRAD"
        pv = block.vars[n]
        with torch._C.DisableTorchFunctionSubclass():
            meta = torch.empty(pv.shape, dtype=pv.dtype, device="meta")
        block.vars[g] = Variable(meta, g, block, False, True)
        outs.append(VarRef(g))
    op = Operator(block, None, (VarRef(loss.var_name),), {}, outs, type="backward",
                  attrs={"params": names})
    block.append_op(op)
    return [(block.vars[n], block.vars[n + "@GRAD"]) for n in names]


def gradients(targets, inputs, target_gradients=None, no_grad_set=None):
    t = targets[0] if isinstance(targets, (list, tuple)) else targets
    ins = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    pg = append_backward(t, parameter_list=[i.var_name if isinstance(i, Variable) else i for i in ins])
    return [g for _, g in pg]


class OptimizerSpec:
    """A dygraph optimizer captured at program-build time; bound to the Scope's parameters on the
    Executor's first run."""

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


def minimize(optimizer, loss, parameter_list=None, no_grad_set=None):
    pg = append_backward(loss, parameter_list, no_grad_set)
    block = loss.block
    names = [p.var_name for p, _ in pg]
    op = Operator(block, None, tuple(VarRef(n + "@GRAD") for n in names), {}, None, type="optimize",
                  attrs={"optimizer": OptimizerSpec(optimizer), "params": names})
    block.append_op(op)
    return None, pg
