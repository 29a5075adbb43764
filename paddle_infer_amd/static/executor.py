"""Static-graph Executor (reference `python/paddle/fluid/executor.py`,
`paddle/fluid/framework/new_executor/standalone_executor.cc` / `interpretercore.cc`).

Plan (cached per program version) comes from the native runtime (`csrc/runtime/scheduler.cc`):
dependency-respecting instruction order + per-instruction GC list, so intermediates are released
right after their last consumer (the reference's eager-deletion GC). Persistable variables live in
the Scope across runs. Training programs (`backward.py`) hold one ``<type>_grad`` op per forward
op — run with its explicit grad kernel (`grad_kernels.py`, the reference `*_grad` PHI kernels)
when the program holds reference op types, else as the forward op's VJP (`_run_grad_op`) — plus ``sum`` ops for renamed partial gradients and
per-parameter optimizer ops (``sgd`` / ``momentum`` / ``adam`` / ``adamw``) that update the
persistable parameters and accumulators in place; the learning-rate variable of a program built
by ``minimize`` is refreshed from its optimizer / LRScheduler before each run (reference
`executor.py` ``_update_lr``).
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
        i32p, u8p = P(ctypes.c_int), P(ctypes.c_ubyte)
        lib.piamd_plan.argtypes = [ctypes.c_int, ctypes.c_int, i32p, i32p, i32p, i32p, u8p, i32p,
                                   i32p, i32p, i32p]
        lib.piamd_plan.restype = ctypes.c_int
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
        compiled = program if isinstance(program, CompiledProgram) else None
        if compiled is not None:
            program = compiled._program
            if (compiled._build_strategy.allow_cuda_graph_capture and self.device.type == "cuda"
                    and not compiled._data_parallel):
                from .backward import op_role, FORWARD
                if all(op_role(op) == FORWARD for op in program.global_block().ops):
                    return self._run_graph(compiled, program, feed, fetch_list, scope, return_numpy)
        self._init_params(program, scope)
        if program is default_startup_program() or not program.global_block().ops:
            return []
        from ..incubate.checkpoint import auto_checkpoint as _acp
        if _acp.current_range() is not None:  # register / restore inside train_epoch_range
            _acp._auto_checkpoint(self, program)
        fetch_list = fetch_list or []
        fetch_names = [f.var_name if isinstance(f, Variable) else str(f) for f in fetch_list]
        ops = program.global_block().ops
        key = (id(program), program._version, tuple(fetch_names))
        if key not in self._plans:
            keep = set(program.params) | set(fetch_names)
            self._plans[key] = build_plan(ops, keep)
        order, frees, _ = self._plans[key]
        skey = ("streams",) + key
        if skey not in self._plans:
            from .streams import stream_plan, COMM_OPS
            self._plans[skey] = stream_plan(ops, order) if any(op.type in COMM_OPS for op in ops) else None
        splan = self._plans[skey]
        env = {}
        for name, val in (feed or {}).items():
            t = val if isinstance(val, torch.Tensor) else torch.as_tensor(np.asarray(val))
            env[name] = t.to(self.device)
        from .backward import op_role, FORWARD
        training = any(op_role(op) != FORWARD for op in ops)
        for lr_name, opt in getattr(program, "_lr_vars", {}).items():
            cur = scope.get(lr_name)
            val = torch.tensor([float(opt.get_lr())], dtype=torch.float32, device=self.device)
            if cur is None:
                scope.set(lr_name, val)
            else:
                cur.copy_(val)
        for name in getattr(program, "_grad_roots", ()):
            if name in env and env[name].is_floating_point():
                env[name] = env[name].detach().requires_grad_(True)
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

        self._leafmap = {}
        self._cf_depth = 0
        self._training = training
        dp = buckets = None
        if compiled is not None and compiled._data_parallel and training:
            import torch.distributed as dist
            from ..distributed.collective import multi_rank
            if multi_rank():
                from .backward import op_role as _role, OPTIMIZE as _OPT, GRAD as _G
                dp = sorted({n for op in ops if _role(op) == _OPT for n in op.input_names()
                             if n.endswith(_G)})
                if compiled._build_strategy.fuse_all_reduce_ops:
                    bkey = ("dp_buckets",) + key
                    if bkey not in self._plans:
                        from .streams import GradBuckets
                        self._plans[bkey] = GradBuckets(ops, order, set(dp), _grad_nbytes(program),
                                                        world=dist.get_world_size())
                    buckets = self._plans[bkey]
        runner = None
        if splan is not None:
            from .streams import StreamRunner
            runner = StreamRunner(self.device, *splan)
            self.last_stream_runner = runner
        with torch.set_grad_enabled(training):
            for pos, oi in enumerate(order):
                op = ops[oi]
                if dp is not None:
                    from .backward import op_role as _role, OPTIMIZE as _OPT
                    if _role(op) == _OPT:
                        if buckets is not None:
                            buckets.wait(env)
                        else:
                            _allreduce_grads(env, dp, False)
                        dp = None
                if runner is not None:
                    runner.run(pos, oi, op, lambda: self._run_op(op, sub, env, scope, program), env)
                else:
                    self._run_op(op, sub, env, scope, program)
                if buckets is not None and dp is not None:
                    buckets.after(pos, env)
                for n in frees[pos]:
                    if n not in fetch_names:
                        env.pop(n, None)
            if runner is not None:
                runner.finish()
            if buckets is not None and dp is not None:  # no optimizer op ran: reduce anyway
                buckets.wait(env)
        for hook in getattr(program, "_post_run_hooks", ()) if training else ():
            hook(scope, program)  # e.g. static.ExponentialMovingAverage
        if training:  # persistable outputs (updated params / accumulators) back into the Scope
            for n in list(env):
                if n in program.params and n not in (feed or {}):
                    cur = scope.get(n)
                    val = env.pop(n)
                    if cur is None:
                        scope.set(n, val)
                    elif val is not cur:
                        with torch.no_grad():
                            cur.copy_(val)
        outs = []
        for n in fetch_names:
            v = env[n] if n in env else scope.get(n)
            v = v.detach()
            outs.append(v.cpu().numpy() if return_numpy else v)
        return outs

    def _run_graph(self, compiled, program, feed, fetch_list, scope, return_numpy):
        """Forward program replayed from a hipGraph: eager warm-up on the first call of a feed
        signature, capture on the second (static feed buffers, outputs kept by the graph pool),
        replay afterwards (feeds copied into the static buffers)."""
        feed = feed or {}
        fetch_list = fetch_list or []
        names = [f.var_name if isinstance(f, Variable) else str(f) for f in fetch_list]
        tens = {k: (v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))).to(self.device)
                for k, v in feed.items()}
        key = (id(program), program._version, tuple(names),
               tuple((k, tuple(t.shape), t.dtype) for k, t in sorted(tens.items())))
        ent = compiled._graphs.get(key)
        if ent is None:  # warm-up run (allocator, kernel first-launch costs) outside capture
            compiled._graphs[key] = "warm"
            outs = self.run(program, tens, fetch_list, scope=scope, return_numpy=False)
        elif ent == "warm":
            static = {k: t.clone() for k, t in tens.items()}
            self.run(program, static, fetch_list, scope=scope, return_numpy=False)  # prime plans
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                outs = self.run(program, static, fetch_list, scope=scope, return_numpy=False)
            compiled._graphs[key] = (g, static, outs)
            g.replay()
        else:
            g, static, outs = ent
            for k, t in tens.items():
                static[k].copy_(t)
            g.replay()
        return [o.cpu().numpy() if return_numpy else o.clone() for o in outs]

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
        from .backward import op_role, is_grad_op, OPTIMIZE, FORWARD
        if is_grad_op(op):
            self._run_grad_op(op, sub, env)
            return
        if (op.attrs.get("_recompute_fwd") and getattr(self, "_training", False)
                and not getattr(self, "_in_recompute", False)):
            # a recompute segment's forward op (fleet static recompute): no autograd graph is kept,
            # its outputs re-enter as leaves; the segment's copy re-produces them in backward
            self._in_recompute = True
            try:
                with torch.no_grad():
                    self._run_op(op, sub, env, scope, program)
            finally:
                self._in_recompute = False
            for n in op.output_names():
                t = env.get(n)
                if isinstance(t, torch.Tensor) and t.is_floating_point() and not t.requires_grad:
                    env[n] = t.detach().requires_grad_(True)
            return
        if getattr(self, "_training", False) and op_role(op) == FORWARD and not getattr(self, "_cf_depth", 0):
            # per-op autograd graphs: a forward op of a training program reads its differentiable
            # inputs through fresh leaves (views, no copy), so its grad op's VJP is exactly this
            # op's local Jacobian product (a grad w.r.t. one input never leaks through another).
            # A control-flow op is ONE such op: its sub-block ops run on a plain autograd graph
            # from these leaves (first read of each external input only — a loop may rebind the
            # name), and cond_grad / while_grad are the VJP through whatever path ran.
            leaves, orig = {}, {}
            ext = set(op.input_names())
            outer = sub

            def sub(x):  # noqa: F811
                v = outer(x)
                if isinstance(x, VarRef) and isinstance(v, torch.Tensor) and v.requires_grad and x.name in ext:
                    lf = leaves.get(x.name)
                    if lf is None:
                        lf = leaves[x.name] = v.detach().requires_grad_(True)
                        orig[x.name] = v
                        return lf
                    return lf if orig[x.name] is v else v
                return v
            for n in op.output_names():
                self._leafmap[n] = leaves
        if op.type in ("cond", "while", "conditional_block") and op.func is None:
            from . import control_flow as _cf
            if op.type == "conditional_block":
                fn = _cf.run_conditional_block
            elif op.type == "while":
                fn = _cf.run_paddle_while if "sub_block" in op.attrs else _cf.run_while
            else:
                fn = _cf.run_cond
            self._cf_depth = getattr(self, "_cf_depth", 0) + 1
            try:
                fn(self, op, sub, env, scope, program)
            finally:
                self._cf_depth -= 1
            return
        if op.func is None:  # a Paddle-typed op (loaded .pdmodel, IR pass, backward / optimizer pass)
            from . import ops_registry
            ops_registry.DEVICE.append(self.device)
            try:
                if op_role(op) == OPTIMIZE:
                    with torch.no_grad():
                        run_paddle_op(op, sub, env, scope)
                else:
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

    @staticmethod
    def _run_grad_kernel(op, val, env):
        """Run `op` with its explicit grad kernel (`grad_kernels.GRAD_KERNELS`) when it has one:
        the gradient comes from the grad OpDesc's slots alone (forward inputs / outputs and the
        output gradients), as the reference executor runs a `*_grad` PHI kernel. Returns False
        for types without a kernel (the VJP path below handles them)."""
        from .grad_kernels import GRAD_KERNELS
        fn = GRAD_KERNELS.get(op.type)
        if fn is None:
            return False
        fop = getattr(op, "fwd_op", None)
        if fop is not None and fop.func is not None:
            return False  # forward is a traced framework op: its grad op carries generic slots

        def get(n):
            if not n:
                return None
            if n in env:
                return env[n]
            try:
                return val(n)
            except KeyError:
                return None
        ins = {k: [get(n) for n in v] for k, v in op.paddle_inputs.items()}
        if any(t is None for k, v in ins.items() if not k.endswith("@GRAD") for t in v):
            return False  # a forward slot bound to a non-variable (a traced constant)
        for k, v in ins.items():  # an output gradient that never reached this op is zero
            if k.endswith("@GRAD") and any(t is None for t in v):
                fwd = ins.get(k[:-5], [])
                ins[k] = [t if t is not None else (torch.zeros_like(f) if isinstance(f, torch.Tensor) else None)
                          for t, f in zip(v, fwd)]
        if any(t is None for k, v in ins.items() if k.endswith("@GRAD") for t in v):
            return False
        with torch.no_grad():
            res = fn(ins, op.attrs)
        for slot, names in op.paddle_outputs.items():
            vals = res.get(slot)
            if vals is None:
                continue
            vals = vals if isinstance(vals, (list, tuple)) else [vals]
            for n, v in zip(names, vals):
                if n and v is not None:
                    env[n] = v.detach()
        return True

    def _run_grad_op(self, op, sub, env):
        """VJP of the grad op's forward op. Fast path: the op-local autograd graph its forward built
        in this run (the forward read its inputs through leaves, see `_run_op`). Otherwise the
        forward op is re-run on detached leaves (a forward that ran without a graph)."""
        from .ops_registry import REGISTRY
        ins, outs = op.paddle_inputs, op.paddle_outputs
        gslot = {k[:-5]: v for k, v in ins.items() if k.endswith("@GRAD")}
        fins = {k: v for k, v in ins.items() if not k.endswith("@GRAD") and k not in gslot}
        fouts = {k: ins.get(k, []) for k in gslot}
        xs = []
        for k, targets in outs.items():
            for x, g in zip(fins.get(k[:-5], []), targets):
                if g and x not in xs:
                    xs.append(x)
        if not xs:
            return

        def val(n):
            return env[n] if n in env else sub(VarRef(n))
        if self._run_grad_kernel(op, val, env):
            return
        gouts = []
        for k, onames in fouts.items():
            for o, g in zip(onames, gslot[k]):
                if g and (g in env):
                    gouts.append((o, env[g]))
        leaves = None
        for onames in fouts.values():
            for o in onames:
                leaves = self._leafmap.get(o, leaves) if hasattr(self, "_leafmap") else None
        ov = [env.get(o) for o, _ in gouts]
        fast = leaves is not None and all(isinstance(t, torch.Tensor) and t.grad_fn is not None for t in ov)
        xv = [leaves.get(x) if fast else val(x) for x in xs]
        with torch.enable_grad():
            if not fast:
                leaves = {x: (t.detach().requires_grad_(True) if isinstance(t, torch.Tensor) and t.is_floating_point() else t)
                          for x, t in zip(xs, xv)}

                def sub2(r):
                    if isinstance(r, VarRef) and r.name in leaves:
                        return leaves[r.name]
                    return sub(r)
                fop = getattr(op, "fwd_op", None)
                produced = {}
                if fop is not None and fop.func is not None:
                    args = tree_map(sub2, fop.args)
                    kwargs = tree_map(sub2, fop.kwargs)
                    res = fop.func(*args, **kwargs)
                    _zip_assign(fop.outputs, res, lambda r, v: produced.__setitem__(r.name, v) if isinstance(r, VarRef) else None)
                else:
                    fn = REGISTRY.get(op.type[:-5])
                    if fn is None:
                        raise NotImplementedError(f"no forward kernel for grad op {op.type}")
                    attrs = {k: v for k, v in op.attrs.items() if k != "op_role"}
                    res = fn({k: [sub2(VarRef(n)) for n in v] for k, v in fins.items()}, attrs)
                    for k, onames in fouts.items():
                        vals = res.get(k)
                        vals = vals if isinstance(vals, (list, tuple)) else [vals]
                        produced.update(zip(onames, vals))
                ov = [produced.get(o) for o, _ in gouts]
                xv = [leaves[x] for x in xs]
            pairs = [(o, g) for o, (_, g) in zip(ov, gouts) if isinstance(o, torch.Tensor) and o.requires_grad]
            diff = [i for i, t in enumerate(xv) if isinstance(t, torch.Tensor) and t.requires_grad]
            grads = [None] * len(xs)
            if pairs and diff:
                r = torch.autograd.grad([o for o, _ in pairs], [xv[i] for i in diff],
                                        [g.to(o.dtype) if g.dtype != o.dtype else g for o, g in pairs],
                                        allow_unused=True)
                for i, gr in zip(diff, r):
                    grads[i] = gr
        gmap = dict(zip(xs, grads))
        for k, targets in outs.items():
            for x, g in zip(fins.get(k[:-5], []), targets):
                if g:
                    gr = gmap.get(x)
                    env[g] = gr.detach() if gr is not None else torch.zeros_like(val(x)).detach()

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


class BuildStrategy:
    """Reference `paddle.static.BuildStrategy` (`framework/details/build_strategy.h`). Honoured:
    ``fuse_bn_act_ops`` / ``fuse_bn_add_act_ops`` (conv+bn folding), ``fuse_elewise_add_act_ops``
    / ``fuse_gemm_epilogue`` (fc + bias + activation fusions), ``enable_auto_fusion`` (the whole
    GPU pass list) on Paddle-typed inference programs; ``allow_cuda_graph_capture`` (forward
    programs on the GPU replayed from a captured hipGraph per feed signature);
    ``fuse_all_reduce_ops`` (data-parallel gradients all-reduced as ONE flat bucket per dtype).
    The rest are accepted for API compatibility (memory reuse is the executor's eager GC)."""

    def __init__(self):
        self.fuse_elewise_add_act_ops = False
        self.fuse_bn_act_ops = False
        self.fuse_bn_add_act_ops = False
        self.fuse_gemm_epilogue = False
        self.fuse_relu_depthwise_conv = False
        self.fuse_all_reduce_ops = True
        self.fuse_all_optimizer_ops = False
        self.enable_auto_fusion = False
        self.enable_inplace = True
        self.memory_optimize = True
        self.allow_cuda_graph_capture = False
        self.sync_batch_norm = False
        self.num_trainers = 1
        self.trainer_id = 0
        self.reduce_strategy = 0
        self.gradient_scale_strategy = 0
        self.debug_graphviz_path = ""

    def pass_list(self):
        if self.enable_auto_fusion:
            from ..inference.passes import GPU_PASSES
            return list(GPU_PASSES)
        ps = []
        if self.fuse_bn_act_ops or self.fuse_bn_add_act_ops:
            ps.append("conv_bn_fuse_pass")
        if self.fuse_elewise_add_act_ops or self.fuse_gemm_epilogue:
            ps += ["fc_fuse_pass", "fc_act_fuse_pass", "linear_bias_act_fuse_pass"]
        return ps


class ExecutionStrategy:
    """Reference `paddle.static.ExecutionStrategy` (accepted; one HIP stream per process)."""

    def __init__(self):
        self.num_threads = 1
        self.num_iteration_per_drop_scope = 100
        self.num_iteration_per_run = 1
        self.use_thread_barrier = False


class CompiledProgram:
    """Reference `python/paddle/fluid/compiler.py:CompiledProgram`: a program prepared once for
    repeated execution. Here: BuildStrategy fusion passes applied to a clone of a Paddle-typed
    forward program; ``with_data_parallel`` = one process per GPU (the launcher's world):
    gradients are averaged over the default group (RCCL on GPUs, gloo on CPUs) right before the
    first optimizer op of every run; ``allow_cuda_graph_capture`` replays forward runs from a
    hipGraph captured per (feed shapes/dtypes, fetch list)."""

    def __init__(self, program_or_graph, build_strategy=None):
        self._source = program_or_graph
        self._build_strategy = build_strategy or BuildStrategy()
        self._exec_strategy = ExecutionStrategy()
        self._data_parallel = False
        self._loss_name = None
        self._prepared = None
        self._graphs = {}

    @property
    def _program(self):
        if self._prepared is None:
            self._prepared = self._prepare()
        return self._prepared

    def _prepare(self):
        prog = self._source
        ps = self._build_strategy.pass_list()
        from .backward import op_role, FORWARD
        ops = prog.global_block().ops
        if ps and ops and all(op.func is None and op_role(op) == FORWARD for op in ops):
            from ..inference.passes import apply_passes
            prog = prog.clone()
            apply_passes(prog, ps, fetch_names=tuple(prog.fetch_names))
        return prog

    def with_data_parallel(self, loss_name=None, build_strategy=None, exec_strategy=None,
                           places=None, share_vars_from=None):
        self._data_parallel = True
        self._loss_name = loss_name
        if build_strategy is not None:
            self._build_strategy = build_strategy
            self._prepared = None
        if exec_strategy is not None:
            self._exec_strategy = exec_strategy
        return self


def _grad_nbytes(program):
    """Bytes of ``<param>@GRAD`` (bucket sizing of the data-parallel gradient all-reduce)."""
    def f(n):
        p = program.params.get(n[:-len("@GRAD")]) if n.endswith("@GRAD") else None
        return float(p.numel() * p.element_size()) if p is not None else 0.0
    return f


def _allreduce_grads(env, names, fused=True):
    """Average the named gradients over the default process group (one flat bucket per dtype)."""
    import torch.distributed as dist
    world = dist.get_world_size()
    ts = [env[n] for n in names if n in env and isinstance(env[n], torch.Tensor)]
    if not ts:
        return
    if not fused:
        for t in ts:
            dist.all_reduce(t)
            t.div_(world)
        return
    from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
    by_dtype = {}
    for t in ts:
        by_dtype.setdefault(t.dtype, []).append(t)
    for group in by_dtype.values():
        flat = _flatten_dense_tensors([t.detach() for t in group])
        dist.all_reduce(flat)
        flat.div_(world)
        for t, v in zip(group, _unflatten_dense_tensors(flat, group)):
            with torch.no_grad():
                t.copy_(v)
