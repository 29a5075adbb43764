"""Static-graph Executor (reference `python/paddle/fluid/executor.py`,
`paddle/fluid/framework/new_executor/standalone_executor.cc` / `interpretercore.cc`).

Plan (cached per program version) comes from the native runtime (`csrc/runtime/scheduler.cc`):
dependency-respecting instruction order + per-instruction GC list, so intermediates are released
right after their last consumer (the reference's eager-deletion GC). Persistable variables live in
the Scope across runs. Training programs contain ``backward`` (autograd over the recorded forward)
and ``optimize`` ops (a Paddle optimizer bound to the scope's parameters).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch
from torch.utils._pytree import tree_map

from .framework import (Program, SymDim, SYM_PRIMES, VarRef, Variable, default_main_program, default_startup_program,
                        global_scope)
from .. import _build

_RT = None


def runtime_lib():
    global _RT
    if _RT is None:
        path = _build.RUNTIME_LIB
        if not os.path.exists(path):
            _build.build(verbose=False)
        lib = ctypes.CDLL(path)
        P = ctypes.POINTER
        i32p, u8p, i64p = P(ctypes.c_int), P(ctypes.c_ubyte), P(ctypes.c_longlong)
        lib.piamd_plan.argtypes = [ctypes.c_int, ctypes.c_int, i32p, i32p, i32p, i32p, u8p, i32p,
                                   i32p, i32p, i32p]
        lib.piamd_plan.restype = ctypes.c_int
        lib.piamd_memplan.argtypes = [ctypes.c_int, i64p, i32p, i32p, ctypes.c_longlong, i64p]
        lib.piamd_memplan.restype = ctypes.c_longlong
        _RT = lib
    return _RT


def _arr(a, ct):
    a = np.ascontiguousarray(a, dtype={ctypes.c_int: np.int32, ctypes.c_ubyte: np.uint8,
                                       ctypes.c_longlong: np.int64}[ct])
    return a, a.ctypes.data_as(ctypes.POINTER(ct))


def build_plan(ops, keep_names):
    """Native dependency / GC plan for a list of Operators."""
    names = {}
    for op in ops:
        for n in op.input_names() + op.output_names():
            names.setdefault(n, len(names))
    in_ptr, in_idx, out_ptr, out_idx = [0], [], [0], []
    for op in ops:
        in_idx += [names[n] for n in op.input_names()]
        in_ptr.append(len(in_idx))
        out_idx += [names[n] for n in op.output_names()]
        out_ptr.append(len(out_idx))
    nv = len(names)
    keep = np.zeros(max(nv, 1), dtype=np.uint8)
    for n, i in names.items():
        if n in keep_names:
            keep[i] = 1
    nops = len(ops)
    lib = runtime_lib()
    a_ip, p_ip = _arr(in_ptr, ctypes.c_int)
    a_ii, p_ii = _arr(in_idx or [0], ctypes.c_int)
    a_op, p_op = _arr(out_ptr, ctypes.c_int)
    a_oi, p_oi = _arr(out_idx or [0], ctypes.c_int)
    a_k, p_k = _arr(keep, ctypes.c_ubyte)
    order = np.zeros(max(nops, 1), np.int32)
    free_ptr = np.zeros(nops + 1, np.int32)
    free_idx = np.zeros(max(nv, 1), np.int32)
    level = np.zeros(max(nops, 1), np.int32)
    P = ctypes.POINTER(ctypes.c_int)
    rc = lib.piamd_plan(nops, nv, p_ip, p_ii, p_op, p_oi, p_k, order.ctypes.data_as(P),
                        free_ptr.ctypes.data_as(P), free_idx.ctypes.data_as(P), level.ctypes.data_as(P))
    if rc != 0:
        raise RuntimeError(f"piamd_plan failed ({rc})")
    inv = {i: n for n, i in names.items()}
    frees = [[inv[int(v)] for v in free_idx[free_ptr[i]:free_ptr[i + 1]]] for i in range(nops)]
    return [int(i) for i in order[:nops]], frees, [int(x) for x in level[:nops]]


class Executor:
    def __init__(self, place=None):
        from .. import device as _d
        self.device = _d._resolve(place)
        self._plans = {}
        self._optims = {}

    def close(self):
        self._plans.clear()

    def _init_params(self, program, scope):
        for name, t in program.params.items():
            cur = scope.get(name)
            if cur is None:
                v = t.detach().to(self.device).clone()
                if t.is_floating_point() and t.requires_grad:
                    v.requires_grad_(True)
                scope.set(name, v)

    def run(self, program=None, feed=None, fetch_list=None, feed_var_name="feed",
            fetch_var_name="fetch", scope=None, return_numpy=True, use_program_cache=True,
            use_prune=False):
        program = program or default_main_program()
        scope = scope or global_scope()
        if hasattr(program, "_program"):  # CompiledProgram
            program = program._program
        self._init_params(program, scope)
        if program is default_startup_program() or not program.global_block().ops:
            return []
        fetch_list = fetch_list or []
        fetch_names = [f.var_name if isinstance(f, Variable) else str(f) for f in fetch_list]
        ops = program.global_block().ops
        key = (id(program), program._version, tuple(fetch_names))
        if key not in self._plans:
            keep = set(program.params) | set(fetch_names)
            self._plans[key] = build_plan(ops, keep)
        order, frees, _ = self._plans[key]
        env = {}
        for name, val in (feed or {}).items():
            t = val if isinstance(val, torch.Tensor) else torch.as_tensor(np.asarray(val))
            env[name] = t.to(self.device)
        training = any(op.type in ("backward", "optimize") for op in ops)
        bind = {}
        bvars = program.global_block().vars
        for name, t in env.items():
            v = bvars.get(name)
            ds = getattr(v, "declared_shape", None) or []
            for i, s in enumerate(ds):
                if (s is None or s < 0) and i < t.dim():
                    bind.setdefault(SYM_PRIMES[min(i, len(SYM_PRIMES) - 1)], int(t.shape[i]))

        def get(name):
            if name in env:
                return env[name]
            v = scope.get(name)
            if v is None:
                raise KeyError(f"variable {name} has no value (feed it or run the startup program)")
            return v

        dev = self.device

        def sub(x):
            if isinstance(x, VarRef):
                return get(x.name)
            if isinstance(x, SymDim):
                return x.resolve(bind)
            if isinstance(x, torch.device) and x.type == "meta":  # captured on meta tensors
                return dev
            return x

        with torch.set_grad_enabled(training):
            for pos, oi in enumerate(order):
                op = ops[oi]
                self._run_op(op, sub, env, scope, program)
                for n in frees[pos]:
                    if n not in fetch_names:
                        env.pop(n, None)
        outs = []
        for n in fetch_names:
            v = env[n] if n in env else scope.get(n)
            v = v.detach()
            outs.append(v.cpu().numpy() if return_numpy else v)
        return outs

    def _run_op(self, op, sub, env, scope, program):
        from .ops_registry import run_paddle_op
        if op.type == "backward":
            loss = sub(op.args[0])
            names = op.attrs["params"]
            params = [scope.get(n) for n in names]
            grads = torch.autograd.grad(loss, params, allow_unused=True)
            for n, g in zip(names, grads):
                env[n + "@GRAD"] = g if g is not None else torch.zeros_like(scope.get(n))
            return
        if op.type == "optimize":
            opt = self._optimizer_for(op, scope)
            with torch.no_grad():
                for n, p in zip(op.attrs["params"], opt._parameter_list):
                    p.grad = env[n + "@GRAD"]
                opt.step()
                for p in opt._parameter_list:
                    p.grad = None
            return
        if op.func is None:  # a Paddle-typed op loaded from a foreign .pdmodel
            from . import ops_registry
            ops_registry.DEVICE.append(self.device)
            try:
                run_paddle_op(op, sub, env, scope)
            finally:
                ops_registry.DEVICE.pop()
            return
        args = tree_map(sub, op.args)
        kwargs = tree_map(sub, op.kwargs)
        if op.attrs.get("is_test") and "dropout" in getattr(op.func, "__name__", ""):
            kwargs = dict(kwargs, training=False)
        out = op.func(*args, **kwargs)

        def assign(ref, val):
            if isinstance(ref, VarRef):
                env[ref.name] = val
        _zip_assign(op.outputs, out, assign)

    def _optimizer_for(self, op, scope):
        key = id(op)
        if key not in self._optims:
            spec = op.attrs["optimizer"]
            params = [scope.get(n) for n in op.attrs["params"]]
            self._optims[key] = spec.bind(params)
        return self._optims[key]


def _zip_assign(refs, vals, fn):
    if isinstance(refs, (list, tuple)):
        for r, v in zip(refs, vals):
            _zip_assign(r, v, fn)
    elif isinstance(refs, dict):
        for k in refs:
            _zip_assign(refs[k], vals[k], fn)
    else:
        fn(refs, vals)


class CompiledProgram:
    def __init__(self, program_or_graph, build_strategy=None):
        self._program = program_or_graph

    def with_data_parallel(self, loss_name=None, build_strategy=None, exec_strategy=None, places=None):
        return self


class BuildStrategy:
    def __init__(self):
        self.fuse_elewise_add_act_ops = False
        self.fuse_bn_act_ops = False
        self.enable_auto_fusion = False


class ExecutionStrategy:
    def __init__(self):
        self.num_threads = 1
