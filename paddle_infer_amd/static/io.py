"""Static-graph model IO: ``.pdmodel`` (ProgramDesc protobuf) + ``.pdiparams`` (combined tensors).

Parity: reference `python/paddle/static/io.py` (save_inference_model / load_inference_model /
serialize_program / deserialize_program / save / load / load_program_state) and
`python/paddle/fluid/io.py`. Inference programs are pruned to the ops the fetch targets need and
framed by ``feed`` / ``fetch`` ops exactly like the reference; persistables are written sorted
by name in the combined LoDTensor stream.

Saving LOWERS every recorded op (torch / framework callables captured by ``jit.to_static`` or
static capture) into Paddle OpDescs with the reference's op types, slots and attributes
(`lowering.py`), so a written ``.pdmodel`` holds only Paddle ops and executes through the
Paddle-op registry (`ops_registry.py`). ``allow_custom_ops=True`` keeps an op no lowering covers in
its recorded form (two extra string attrs, ``op_callable`` + ``op_spec``); LOADING such an op only
resolves callables on an explicit allowlist (``resolve_func``) — a ``.pdmodel`` naming anything
else (``os.system``, ``builtins.eval``, ``torch.load`` ...) is rejected before any code runs.
"""
from __future__ import annotations

import copy
import json
import math
import os

import numpy as np
import torch

from . import proto
from .framework import Operator, Program, SymDim, VarRef, Variable
from ..framework.dtype import dtype_name, to_torch_dtype


# ------------------------------------------------------------------------ arg-spec (de)serialise
def _enc(x):
    if isinstance(x, VarRef):
        return {"$v": x.name}
    if isinstance(x, SymDim):
        return {"$sym": [x.k, [list(e) for e in x.exps]]}
    if isinstance(x, tuple):
        return {"$t": [_enc(v) for v in x]}
    if isinstance(x, list):
        return [_enc(v) for v in x]
    if isinstance(x, dict):
        return {"$d": {k: _enc(v) for k, v in x.items()}}
    if isinstance(x, slice):
        return {"$s": [_enc(x.start), _enc(x.stop), _enc(x.step)]}
    if x is Ellipsis:
        return {"$e": 1}
    if isinstance(x, torch.dtype):
        return {"$dt": dtype_name(x)}
    if isinstance(x, torch.device):
        return {"$dev": str(x)}
    if isinstance(x, (torch.memory_format, torch.layout)):
        return {"$mf": str(x)}
    if isinstance(x, torch.Size):
        return {"$t": list(x)}
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    if isinstance(x, float) and (math.isinf(x) or math.isnan(x)):
        return {"$f": repr(x)}
    return x


def _dec(x):
    if isinstance(x, list):
        return [_dec(v) for v in x]
    if isinstance(x, dict):
        if "$v" in x:
            return VarRef(x["$v"])
        if "$sym" in x:
            return SymDim(x["$sym"][0], x["$sym"][1])
        if "$t" in x:
            return tuple(_dec(v) for v in x["$t"])
        if "$d" in x:
            return {k: _dec(v) for k, v in x["$d"].items()}
        if "$s" in x:
            return slice(*[_dec(v) for v in x["$s"]])
        if "$e" in x:
            return Ellipsis
        if "$dt" in x:
            return to_torch_dtype(x["$dt"])
        if "$dev" in x:
            return torch.device(x["$dev"])
        if "$mf" in x:
            return getattr(torch, x["$mf"].replace("torch.", ""))
        if "$f" in x:
            return float(x["$f"])
    return x


def func_name(func):
    objcls = getattr(func, "__objclass__", None)
    if objcls is not None:
        return f"torch.Tensor.{func.__name__}"
    owner = getattr(func, "__self__", None)
    if isinstance(owner, type) and func.__name__ == "apply":  # autograd.Function.apply
        return f"{owner.__module__}.{owner.__qualname__}.apply"
    mod = getattr(func, "__module__", None)
    q = getattr(func, "__qualname__", None) or getattr(func, "__name__")
    if mod == "torch._tensor":
        return f"torch._tensor.{q}"
    name = f"{mod}.{q}" if mod else q
    try:
        r = _import_attr(name)
        if r is func or getattr(r, "__wrapped__", None) is func:  # recordable() wrappers
            return name
    except (AttributeError, ImportError, ValueError):
        pass
    import torch.nn.functional as F
    for prefix, ns in (("torch", torch), ("torch.nn.functional", F), ("torch.Tensor", torch.Tensor),
                       ("torch._C._nn", torch._C._nn), ("torch.special", torch.special),
                       ("torch.linalg", torch.linalg), ("torch.fft", torch.fft)):
        if getattr(ns, func.__name__, None) is func:
            return f"{prefix}.{func.__name__}"
    raise ValueError(f"cannot serialise op callable {func!r}")


def _import_attr(name):
    import importlib
    parts = name.split(".")
    for i in range(len(parts) - 1, 0, -1):
        try:
            obj = importlib.import_module(".".join(parts[:i]))
        except ImportError:
            continue
        for p in parts[i:]:
            obj = getattr(obj, p)
        return obj
    raise ValueError(name)


_ALLOWED = None
_ALLOWED_MODULE_PREFIXES = ("torch.", "paddle_infer_amd.")


def _allowlist():
    """Names of the only callables a loaded program may invoke: the torch ops the static capture
    can record (``torch.overrides.get_overridable_functions`` — tensor math only: no IO, no
    pickling, no process control) plus the framework's own recordable ops and autograd functions."""
    global _ALLOWED
    if _ALLOWED is None:
        import torch.overrides as ov
        allowed = {}
        for ns, fns in ov.get_overridable_functions().items():
            for fn in fns:
                try:
                    allowed[func_name(fn)] = fn
                except (ValueError, AttributeError, TypeError):
                    continue
        from .framework import _paddle_types
        for fn in _paddle_types():
            try:
                allowed[func_name(fn)] = fn
            except (ValueError, AttributeError, TypeError):
                continue
        _ALLOWED = allowed
    return _ALLOWED


def _framework_callable(name):
    """paddle_infer_amd recordable ops (``static.framework.recordable``) and autograd Functions."""
    import importlib
    parts = name.split(".")
    for i in range(len(parts) - 1, 0, -1):
        mod = ".".join(parts[:i])
        if not mod.startswith("paddle_infer_amd"):
            return None
        try:
            obj = importlib.import_module(mod)
        except ImportError:
            continue
        for p in parts[i:]:
            obj = getattr(obj, p, None)
            if obj is None:
                return None
        if getattr(obj, "_paddle_type", None) is not None:
            return obj
        owner = getattr(obj, "__self__", None)
        if isinstance(owner, type) and issubclass(owner, torch.autograd.Function) \
                and owner.__module__.startswith("paddle_infer_amd"):
            return obj
        return None
    return None


def resolve_func(name):
    """Resolve a stored ``op_callable`` name — ONLY from the allowlist (see ``_allowlist``)."""
    if not isinstance(name, str) or not name.startswith(_ALLOWED_MODULE_PREFIXES):
        raise ValueError(f"op_callable {name!r} is not an allowed operator")
    fn = _allowlist().get(name)
    if fn is None and name.startswith("paddle_infer_amd."):
        fn = _framework_callable(name)
    if fn is None:
        raise ValueError(f"op_callable {name!r} is not an allowed operator")
    return fn


# ------------------------------------------------------------------------ Program <-> desc
def _var_desc(v: Variable, is_param):
    shape = v.declared_shape if v.declared_shape is not None else list(v.shape)
    with torch._C.DisableTorchFunctionSubclass():
        dt = v.dtype
    return {"name": v.var_name,
            "type": {"type": proto.VT_LOD_TENSOR,
                     "lod_tensor": {"tensor": {"data_type": proto.VT[dtype_name(dt)],
                                               "dims": [(-1 if s is None else int(s)) for s in shape]},
                                    "lod_level": 0}},
            "persistable": bool(v.persistable_), "is_parameter": bool(is_param),
            "stop_gradient": bool(v.stop_gradient_)}


def _paddle_op_desc(type_, ins, outs, attrs):
    from .lowering import attr_desc
    return {"type": type_,
            "inputs": [{"parameter": k, "arguments": list(v)} for k, v in ins.items()],
            "outputs": [{"parameter": k, "arguments": list(v)} for k, v in outs.items()],
            "attrs": [attr_desc(k, v) for k, v in attrs.items()]}


def _typed_attr_descs(attrs):
    """Attrs of a Paddle-typed op (loaded from a Paddle program or built by a pass)."""
    from .lowering import attr_desc, LoweringError
    out = []
    for k, v in attrs.items():
        if v is None:
            continue
        try:
            out.append(attr_desc(k, v))
        except LoweringError:
            out.append({"name": k, "type": proto.ATTR["STRING"], "s": json.dumps(_enc(v))})
    return out


def _tensor_var_desc(name, like):
    """A fresh LoD-tensor var desc with the dims / dtype of the existing desc ``like``."""
    d = copy.deepcopy(like)
    d.update(name=name, persistable=False, is_parameter=False, stop_gradient=True)
    return d


VT_STEP_SCOPES = 11


class _CFLowering:
    """Emit the framework's ``cond`` / ``while`` ops as Paddle control flow (reference
    `python/paddle/fluid/layers/control_flow.py`): ``cond`` → ``logical_not`` + two
    ``conditional_block`` ops (``is_scalar_condition``) + one ``select_input`` per result (Mask =
    the predicate as int32, X = [false value, true value]); ``while_loop`` → ``assign`` of the
    initial values into the loop-carried vars, the condition block inlined before the loop, and a
    ``while`` op whose sub-block runs the body, copies the body results back into the carried vars
    (through temporaries, so a permutation of the carried vars is safe) and recomputes the
    condition. Sub-blocks get fresh indices in emission order."""

    def __init__(self, program, allow_custom_ops):
        import collections
        import types
        self.program, self.allow = program, allow_custom_ops
        self.view = types.SimpleNamespace(vars=collections.ChainMap(*[b.vars for b in program.blocks]))
        self.blocks = []        # emitted sub-block dicts (idx 1..)
        self.new_vars = {}      # name -> var desc (temps, lowering temporaries)
        self._n = 0

    def _tmp(self, stem, like=None, dims=None, dt=None):
        self._n += 1
        name = f"{stem}.cf_{self._n}"
        if like is not None and like in self.view.vars:
            self.new_vars[name] = _tensor_var_desc(name, _var_desc(self.view.vars[like], False))
        else:
            self.new_vars[name] = {"name": name, "type": {"type": proto.VT_LOD_TENSOR, "lod_tensor": {
                "tensor": {"data_type": dt, "dims": dims}, "lod_level": 0}},
                "persistable": False, "is_parameter": False, "stop_gradient": True}
        return name

    def _scope_var(self):
        self._n += 1
        name = f"_cf_scope.{self._n}"
        self.new_vars[name] = {"name": name, "type": {"type": VT_STEP_SCOPES}, "persistable": False}
        return name

    def _new_block(self, parent_idx):
        bd = {"idx": len(self.blocks) + 1, "parent_idx": parent_idx, "vars": [], "ops": []}
        self.blocks.append(bd)
        return bd

    def emit(self, ops, block_idx):
        """-> list of Paddle op descs for the recorded ``ops`` of one block."""
        from .lowering import lower, LoweringError
        out = []
        for op in ops:
            if op.type in ("backward", "optimize"):
                continue
            if op.func is None and op.type == "cond":
                out.extend(self._cond(op, block_idx))
                continue
            if op.func is None and op.type == "while":
                out.extend(self._while(op, block_idx))
                continue
            if op.func is None and op.paddle_inputs is not None:  # already a Paddle op
                d = {"type": op.type,
                     "inputs": [{"parameter": k, "arguments": list(v)} for k, v in op.paddle_inputs.items()],
                     "outputs": [{"parameter": k, "arguments": list(v)}
                                 for k, v in (op.paddle_outputs or {}).items()],
                     "attrs": _typed_attr_descs({k: v for k, v in op.attrs.items() if k != "sub_block"})}
                if "sub_block" in op.attrs:  # a loaded Paddle while / conditional_block: re-emit its block
                    sub = self._new_block(block_idx)
                    sub["ops"] = self.emit(self.program.block(op.attrs["sub_block"]).ops, sub["idx"])
                    d["attrs"].append({"name": "sub_block", "type": proto.ATTR["BLOCK"],
                                       "block_idx": sub["idx"]})
                out.append(d)
                continue
            if op.func is None:
                out.append(_recorded_op_desc(op))
                continue
            try:
                descs, new_vars = lower(self.view, op)
            except LoweringError:
                if not self.allow:
                    raise
                out.append(_recorded_op_desc(op))
                continue
            for name, dims, dt in new_vars:
                if name not in self.new_vars and name not in self.view.vars:
                    self.new_vars[name] = {"name": name, "type": {"type": proto.VT_LOD_TENSOR, "lod_tensor": {
                        "tensor": {"data_type": dt, "dims": dims}, "lod_level": 0}},
                        "persistable": False, "is_parameter": False, "stop_gradient": True}
            out.extend(_paddle_op_desc(*d) for d in descs)
        return out

    def _cond(self, op, block_idx):
        pred = op.paddle_inputs["Cond"][0]
        ins = op.paddle_inputs.get("Input", [])
        res = op.paddle_outputs.get("Out", [])
        t_outs, f_outs = op.attrs["true_outs"], op.attrs["false_outs"]
        not_pred = self._tmp("cond_not", like=pred)
        mask = self._tmp("cond_mask", dims=[1], dt=proto.VT["int32"])
        descs = [_paddle_op_desc("logical_not", {"X": [pred]}, {"Out": [not_pred]}, {})]
        for c, blk_key, outs in ((pred, "true_block", t_outs), (not_pred, "false_block", f_outs)):
            sub = self._new_block(block_idx)
            sub["ops"] = self.emit(self.program.block(op.attrs[blk_key]).ops, sub["idx"])
            d = _paddle_op_desc("conditional_block", {"Cond": [c], "Input": ins},
                                {"Out": list(outs), "Scope": [self._scope_var()]},
                                {"is_scalar_condition": True})
            d["attrs"].append({"name": "sub_block", "type": proto.ATTR["BLOCK"], "block_idx": sub["idx"]})
            descs.append(d)
        descs.append(_paddle_op_desc("cast", {"X": [pred]}, {"Out": [mask]},
                                     {"in_dtype": proto.VT["bool"], "out_dtype": proto.VT["int32"]}))
        for r, t, f in zip(res, t_outs, f_outs):
            descs.append(_paddle_op_desc("select_input", {"X": [f, t], "Mask": [mask]}, {"Out": [r]}, {}))
        return descs

    def _while(self, op, block_idx):
        a = op.attrs
        init, outs = op.paddle_inputs["X"], op.paddle_outputs["Out"]
        carried, body_outs = a["carried"], a["body_outs"]
        cond_ops = self.program.block(a["cond_block"]).ops
        descs = [_paddle_op_desc("assign", {"X": [s]}, {"Out": [d]}, {}) for s, d in zip(init, carried)]
        descs += self.emit(cond_ops, block_idx)
        sub = self._new_block(block_idx)
        body = self.emit(self.program.block(a["body_block"]).ops, sub["idx"])
        tmps = [self._tmp("loop_next", like=c) for c in carried]
        body += [_paddle_op_desc("assign", {"X": [s]}, {"Out": [t]}, {}) for s, t in zip(body_outs, tmps)]
        body += [_paddle_op_desc("assign", {"X": [t]}, {"Out": [c]}, {}) for t, c in zip(tmps, carried)]
        body += self.emit(cond_ops, sub["idx"])
        sub["ops"] = body
        reads = list(dict.fromkeys(op.paddle_inputs.get("Input", []) + list(carried)))
        d = _paddle_op_desc("while", {"X": reads, "Condition": [a["cond_out"]]},
                            {"Out": list(carried), "StepScopes": [self._scope_var()]}, {"is_test": True})
        d["attrs"].append({"name": "sub_block", "type": proto.ATTR["BLOCK"], "block_idx": sub["idx"]})
        descs.append(d)
        descs += [_paddle_op_desc("assign", {"X": [c]}, {"Out": [o]}, {}) for c, o in zip(carried, outs)]
        return descs


def _recorded_op_desc(op):
    """An op no Paddle lowering covers, kept in recorded (callable) form."""
    attrs = [{"name": k, "type": proto.ATTR["STRING"], "s": json.dumps(_enc(v))}
             for k, v in op.attrs.items() if k not in ("optimizer",)]
    if op.func is not None:
        attrs.append({"name": "op_callable", "type": proto.ATTR["STRING"], "s": func_name(op.func)})
        attrs.append({"name": "op_spec", "type": proto.ATTR["STRING"],
                      "s": json.dumps({"args": _enc(op.args), "kwargs": _enc(op.kwargs),
                                       "outputs": _enc(op.outputs)})})
    return {"type": op.type, "inputs": [{"parameter": "X", "arguments": op.input_names()}],
            "outputs": [{"parameter": "Out", "arguments": op.output_names()}], "attrs": attrs}


def _desc_names(op_descs, blocks):
    names = set()
    for od in list(op_descs) + [o for bd in blocks for o in bd["ops"]]:
        for x in od["inputs"] + od["outputs"]:
            names.update(x["arguments"])
    return names


def program_to_desc(program: Program, feed_names=None, fetch_names=None, ops=None,
                    paddle_ops=True, allow_custom_ops=False):
    """``paddle_ops``: lower recorded ops to Paddle OpDescs (`lowering.py`); an op no rule covers
    raises ``LoweringError`` unless ``allow_custom_ops`` keeps it in recorded (callable) form.
    ``cond`` / ``while`` become Paddle ``conditional_block`` / ``while`` ops with sub-blocks
    (`_CFLowering`)."""
    from .lowering import LoweringError
    b = program.global_block()
    ops = b.ops if ops is None else ops
    if not paddle_ops and any(op.type in ("cond", "while") and op.func is None for op in ops):
        raise LoweringError("cond / while are serialised as Paddle control-flow ops only (paddle_ops=True)")
    op_descs = []
    if feed_names:
        for i, n in enumerate(feed_names):
            op_descs.append({"type": "feed", "inputs": [{"parameter": "X", "arguments": ["feed"]}],
                             "outputs": [{"parameter": "Out", "arguments": [n]}],
                             "attrs": [{"name": "col", "type": proto.ATTR["INT"], "i": i}]})
    cf = _CFLowering(program, allow_custom_ops)
    if paddle_ops:
        op_descs.extend(cf.emit(ops, 0))
    else:
        op_descs.extend(_recorded_op_desc(op) for op in ops if op.type not in ("backward", "optimize"))
    if fetch_names:
        for i, n in enumerate(fetch_names):
            op_descs.append({"type": "fetch", "inputs": [{"parameter": "X", "arguments": [n]}],
                             "outputs": [{"parameter": "Out", "arguments": ["fetch"]}],
                             "attrs": [{"name": "col", "type": proto.ATTR["INT"], "i": i}]})
    used = set()
    for op in ops:
        used.update(op.input_names())
        used.update(op.output_names())
    used.update(feed_names or [])
    used.update(fetch_names or [])
    used |= _desc_names(op_descs, cf.blocks)
    allv = cf.view.vars
    vars_ = [_var_desc(allv[n], n in program.params) for n in sorted(used) if n in allv]
    seen = {v["name"] for v in vars_}
    vars_ += [d for n, d in cf.new_vars.items() if n not in seen]
    if feed_names:
        vars_.append({"name": "feed", "type": {"type": proto.VT_FEED}, "persistable": True})
    if fetch_names:
        vars_.append({"name": "fetch", "type": {"type": proto.VT_FETCH}, "persistable": True})
    return {"blocks": [{"idx": 0, "parent_idx": -1, "vars": vars_, "ops": op_descs}] + cf.blocks,
            "version": {"version": 0}}


def _attr_value(a):
    t = a.get("type", 0)
    return {0: a.get("i"), 1: a.get("f"), 2: a.get("s"), 3: a.get("ints", []), 4: a.get("floats", []),
            5: a.get("strings", []), 6: a.get("b"), 7: a.get("bools", []), 8: a.get("block_idx"),
            9: a.get("l"), 10: a.get("blocks_idx", []), 11: a.get("longs", []),
            12: a.get("float64s", []), 13: a.get("var_name"), 14: a.get("vars_name", []),
            15: a.get("float64")}.get(t)


CONTROL_FLOW_OPS = ("while", "conditional_block")


def desc_to_program(desc: dict):
    """Every block of the ProgramDesc (sub-blocks of ``while`` / ``conditional_block`` keep their
    indices, so BLOCK attributes stay valid). Op types with no kernel are rejected HERE, at load
    (reference: the predictor refuses an unregistered op when it builds the program)."""
    from .ops_registry import REGISTRY
    prog = Program()
    feeds, fetches = [], []
    np_dt = {v: k for k, v in proto.VT.items()}
    blocks = sorted(desc["blocks"], key=lambda d: d.get("idx", 0))
    for bd in blocks[1:]:
        prog._create_block(bd.get("parent_idx", 0))
    unknown = set()
    for bd in blocks:
        b = prog.block(bd.get("idx", 0))
        for vd in bd.get("vars", []):
            ty = vd.get("type", {})
            if ty.get("type") != proto.VT_LOD_TENSOR:
                continue
            td = ty.get("lod_tensor", {}).get("tensor", {})
            v = b.create_var(vd["name"], td.get("dims", [1]) or [1], np_dt.get(td.get("data_type", 5), "float32"),
                             persistable=vd.get("persistable", False),
                             stop_gradient=vd.get("stop_gradient", True))
            v.declared_shape = td.get("dims", [])
        for od in bd.get("ops", []):
            ins = {x["parameter"]: x.get("arguments", []) for x in od.get("inputs", [])}
            outs = {x["parameter"]: x.get("arguments", []) for x in od.get("outputs", [])}
            attrs = {a["name"]: _attr_value(a) for a in od.get("attrs", [])}
            if od["type"] == "feed":
                feeds.append((attrs.get("col", len(feeds)), outs["Out"][0]))
                continue
            if od["type"] == "fetch":
                fetches.append((attrs.get("col", len(fetches)), ins["X"][0]))
                continue
            if "op_callable" in attrs:
                spec = json.loads(attrs.pop("op_spec"))
                func = resolve_func(attrs.pop("op_callable"))
                extra = {k: _dec(json.loads(v)) for k, v in attrs.items() if isinstance(v, str)}
                op = Operator(b, func, _dec(spec["args"]), _dec(spec["kwargs"]), _dec(spec["outputs"]),
                              type=od["type"], attrs=extra)
            else:
                t = od["type"]
                # <type>_grad ops run as the VJP of their forward op (static/executor.py)
                if t not in REGISTRY and t not in CONTROL_FLOW_OPS and not t.endswith("_grad"):
                    unknown.add(t)
                op = Operator(b, None, (), {}, None, type=od["type"], attrs=attrs)
                op.paddle_inputs, op.paddle_outputs = ins, outs
            b.append_op(op)
    if unknown:
        raise NotImplementedError(
            f"program uses Paddle op type(s) with no kernel in paddle_infer_amd: {sorted(unknown)}")
    prog.feed_names = [n for _, n in sorted(feeds)]
    prog.fetch_names = [n for _, n in sorted(fetches)]
    return prog


def serialize_program(feed_vars, fetch_vars, program=None, **kwargs):
    from .framework import default_main_program
    program = program or default_main_program()
    feeds = [v.var_name if isinstance(v, Variable) else v for v in _as_list(feed_vars)]
    fetches = [v.var_name if isinstance(v, Variable) else v for v in _as_list(fetch_vars)]
    ops = prune(program, fetches)
    return proto.encode("ProgramDesc", program_to_desc(
        program, feeds, fetches, ops, allow_custom_ops=bool(kwargs.get("allow_custom_ops", False))))


def deserialize_program(data: bytes):
    return desc_to_program(proto.decode("ProgramDesc", data))


def _as_list(x):
    return list(x) if isinstance(x, (list, tuple)) else [x]


def prune(program, fetch_names):
    from .backward import op_role, FORWARD
    ops = [op for op in program.global_block().ops if op_role(op) == FORWARD]
    need = set(fetch_names)
    keep = []
    for op in reversed(ops):
        outs = set(op.output_names())
        if outs & need:
            keep.append(op)
            need.update(op.input_names())
    return list(reversed(keep))


# ------------------------------------------------------------------------ params
def serialize_persistables(feed_vars, fetch_vars, executor=None, program=None, names=None):
    from .framework import default_main_program, global_scope
    program = program or default_main_program()
    scope = global_scope()
    names = sorted(names if names is not None else program.params.keys())
    out = bytearray()
    for n in names:
        t = scope.get(n)
        t = program.params[n] if t is None else t
        t = t.detach().cpu()
        if t.dtype == torch.bfloat16:
            arr, vt = t.view(torch.int16).numpy().view(np.uint16), proto.VT["bfloat16"]
        else:
            arr, vt = t.numpy(), proto.VT[dtype_name(t.dtype)]
        out += proto.tensor_to_stream(arr, vt)
    return bytes(out)


def deserialize_persistables(program, data: bytes, executor=None, names=None):
    from .framework import global_scope
    names = sorted(names if names is not None else [
        n for n, v in program.global_block().vars.items() if v.persistable_])
    pos = 0
    scope = global_scope()
    dev = executor.device if executor is not None else torch.device("cpu")
    for n in names:
        arr, vt, pos = proto.tensor_from_stream(data, pos)
        if vt == proto.VT["bfloat16"]:
            t = torch.from_numpy(arr.view(np.int16)).view(torch.bfloat16)
        else:
            t = torch.from_numpy(arr)
        program.params[n] = t
        scope.set(n, t.to(dev))
    return program


def save_inference_model(path_prefix, feed_vars, fetch_vars, executor, program=None, **kwargs):
    from .framework import default_main_program
    program = program or default_main_program()
    d = os.path.dirname(path_prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    fetches = [v.var_name if isinstance(v, Variable) else v for v in _as_list(fetch_vars)]
    ops = prune(program, fetches)
    used = set()
    for op in ops:
        used.update(op.input_names())
    pnames = sorted(n for n in program.params if n in used)
    with open(path_prefix + ".pdmodel", "wb") as f:
        f.write(serialize_program(feed_vars, fetch_vars, program,
                                  allow_custom_ops=kwargs.get("allow_custom_ops", False)))
    with open(path_prefix + ".pdiparams", "wb") as f:
        f.write(serialize_persistables(feed_vars, fetch_vars, executor, program, pnames))


def load_inference_model(path_prefix, executor, model_filename=None, params_filename=None, **kw):
    mf = model_filename or path_prefix + ".pdmodel"
    pf = params_filename or path_prefix + ".pdiparams"
    with open(mf, "rb") as f:
        prog = deserialize_program(f.read())
    if os.path.exists(pf):
        with open(pf, "rb") as f:
            deserialize_persistables(prog, f.read(), executor)
    fetch_vars = [prog.global_block().vars[n] for n in prog.fetch_names]
    return [prog, list(prog.feed_names), fetch_vars]


def train_program_desc(program):
    """ProgramDesc of a TRAINING program holding only reference op types: the recorded forward is
    lowered to Paddle ops (`lowering.py`), the backward is re-derived over those Paddle ops
    (``matmul_v2_grad`` / ``elementwise_add_grad`` / ``sum`` ... with ``op_role`` 1, `backward.py`),
    and the optimize phase (grad-clip ops lowered, ``sgd`` / ``momentum`` / ``adam`` / ``adamw``
    ops as built by ``minimize``) follows with ``op_role`` 2."""
    from .backward import op_role, FORWARD, OPTIMIZE, build_backward
    info = getattr(program, "_backward_info", None)
    if info is None:
        raise ValueError("program has no backward (append_backward / minimize was not called)")
    b = program.global_block()
    fwd = [op for op in b.ops if op_role(op) == FORWARD]
    opt = [op for op in b.ops if op_role(op) == OPTIMIZE]
    if any(op.type == "optimize" for op in opt):
        raise ValueError("this optimizer has no static op form (sgd / momentum / adam / adamw)")
    lp = desc_to_program(program_to_desc(program, ops=fwd))
    lp.params = dict(program.params)
    lb = lp.global_block()
    for n in program.params:
        if n in lb.vars:
            lb.vars[n].persistable_ = True
    build_backward(lb, info["loss"], info["params"], info.get("stop", ()))
    d = program_to_desc(lp)
    dopt = program_to_desc(program, ops=opt)
    for od in dopt["blocks"][0]["ops"]:
        if not any(a["name"] == "op_role" for a in od["attrs"]):
            od["attrs"].append({"name": "op_role", "type": proto.ATTR["INT"], "i": OPTIMIZE})
    blk = d["blocks"][0]
    have = {v["name"] for v in blk["vars"]}
    for v in dopt["blocks"][0]["vars"]:
        if v["name"] not in have:
            have.add(v["name"])
            blk["vars"].append(v)
    blk["ops"].extend(dopt["blocks"][0]["ops"])
    return d


def _opt_names(program):
    """Persistables that are not model parameters (optimizer accumulators, learning rate)."""
    return sorted(getattr(program, "_opt_vars", ()))


def save(program, model_path, protocol=4, **configs):
    """Reference `python/paddle/static/io.py` ``save``: ``.pdparams`` (parameters), ``.pdopt``
    (optimizer accumulators + learning rate) and ``.pdmodel`` (the whole program; a training
    program through :func:`train_program_desc`)."""
    from ..framework.io import save as _save
    from .framework import global_scope
    scope = global_scope()
    d = os.path.dirname(model_path)
    if d:
        os.makedirs(d, exist_ok=True)
    opt = set(_opt_names(program))
    state = {n: (scope.get(n) if scope.get(n) is not None else t) for n, t in program.params.items()}
    _save({n: t for n, t in state.items() if n not in opt}, model_path + ".pdparams")
    _save({n: t for n, t in state.items() if n in opt}, model_path + ".pdopt")
    desc = train_program_desc(program) if getattr(program, "_backward_info", None) else program_to_desc(program)
    with open(model_path + ".pdmodel", "wb") as f:
        f.write(proto.encode("ProgramDesc", desc))


def load(program, model_path, executor=None, var_list=None):
    """Reference ``paddle.static.load``: parameters and optimizer state into ``program``'s
    persistables (and the global Scope)."""
    from ..framework.io import load as _load
    state = dict(_load(model_path + ".pdparams"))
    if os.path.exists(model_path + ".pdopt"):
        state.update(_load(model_path + ".pdopt"))
    set_program_state(program, state, executor)


def load_program_state(model_path, var_list=None):
    from ..framework.io import load as _load
    return _load(model_path + ".pdparams" if not model_path.endswith(".pdparams") else model_path)


def set_program_state(program, state_dict, executor=None):
    from .framework import global_scope
    scope = global_scope()
    b = program.global_block()
    for n, v in state_dict.items():
        if n in program.params or n in b.vars:
            t = torch.as_tensor(v)
            program.params[n] = t
            cur = scope.get(n)
            if cur is not None:
                with torch.no_grad():
                    cur.copy_(t.to(cur.dtype))
            elif executor is not None:
                t = t.to(executor.device).clone()
                if t.is_floating_point() and (n + "@GRAD") in b.vars:
                    t.requires_grad_(True)
                scope.set(n, t)
