"""Static-graph IR: Program / Block / Variable / Operator, program_guard, data, Scope.

Parity: reference `python/paddle/fluid/framework.py` (Program, Block, Variable, Operator,
program_guard, default_main_program / default_startup_program, name_scope) and
`paddle/fluid/framework/{program_desc,block_desc,op_desc,var_desc,scope}.cc`.

Capture mechanism (MI355X-native, no per-op builder code): a static ``Variable`` is a
``torch.Tensor`` subclass backed by a *meta* tensor (shape/dtype only, no memory). Every torch
call that touches one is intercepted by ``__torch_function__``: the call is replayed on meta
tensors for shape/dtype inference, the outputs become new Variables, and an ``Operator``
recording the function, its argument structure (Variables → var refs, real tensors → persistable
parameter vars) and outputs is appended to the current block. So the whole ``paddle.*`` / ``nn``
API (including fused HIP ops, whose reference compositions run on meta tensors) builds programs
unchanged. Paddle op types are attached where a mapping exists (``matmul_v2``,
``elementwise_add``, ``layer_norm`` ...) for ``.pdmodel`` interop and IR passes.
"""
from __future__ import annotations

import contextlib
import itertools

import torch
from torch.utils._pytree import tree_map

from ..framework.dtype import to_torch_dtype, dtype_name

_STATE = {"static": False}
_uid = itertools.count()


def unique_name(prefix="tmp"):
    return f"{prefix}_{next(_uid)}"


class VarRef:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"VarRef({self.name})"


# Dynamic (None / -1) dims of `data` vars are traced with a sentinel prime extent per position;
# every int recorded into an op that the sentinel divides becomes a SymDim resolved at run time
# from the fed shapes (the reference keeps -1 dims in VarDesc and infers shapes per run).
SYM_PRIMES = (9973, 9967, 9949, 9941, 9931, 9929)


class SymDim:
    __slots__ = ("k", "exps")

    def __init__(self, k, exps):
        self.k, self.exps = int(k), tuple((int(p), int(e)) for p, e in exps)

    def resolve(self, bind):
        v = self.k
        for p, e in self.exps:
            v *= bind.get(p, p) ** e
        return v

    def __repr__(self):
        return f"SymDim({self.k}, {self.exps})"


def symbolize(v):
    if isinstance(v, bool) or not isinstance(v, int) or v < SYM_PRIMES[-1]:
        return v
    exps, k = [], v
    for p in SYM_PRIMES:
        e = 0
        while k % p == 0:
            k //= p
            e += 1
        if e:
            exps.append((p, e))
    return SymDim(k, exps) if exps else v


class Variable(torch.Tensor):
    """Symbolic tensor of a static Program (meta-backed)."""

    @staticmethod
    def __new__(cls, meta, name, block, persistable=False, stop_gradient=True, declared_shape=None):
        v = torch.Tensor._make_subclass(cls, meta, False)
        v.var_name = name
        v.block = block
        v.persistable_ = persistable
        v.stop_gradient_ = stop_gradient
        v.declared_shape = declared_shape
        return v

    @property
    def name(self):
        return self.var_name

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in _PASSTHROUGH:
            with torch._C.DisableTorchFunctionSubclass():
                return func(*args, **kwargs)
        return _record(func, args, kwargs)

    def __repr__(self):
        with torch._C.DisableTorchFunctionSubclass():
            return f"Variable(name={self.var_name}, shape={list(self.shape)}, dtype={self.dtype})"

    def __hash__(self):
        return id(self)

    def numpy(self):
        raise RuntimeError("static Variable has no value; fetch it with Executor.run")


_PASSTHROUGH = set()
for _n in ["shape", "dtype", "device", "ndim", "requires_grad", "is_cuda", "is_leaf", "grad_fn",
           "layout", "names", "is_sparse", "is_quantized", "is_meta", "data_ptr"]:
    _a = getattr(torch.Tensor, _n, None)
    if _a is not None:
        _PASSTHROUGH.add(getattr(_a, "__get__", _a))
for _n in ["dim", "size", "numel", "element_size", "__len__", "is_floating_point", "is_complex",
           "__format__", "__repr__", "__hash__", "stride", "storage_offset", "is_contiguous",
           "__reduce_ex__", "nelement", "type"]:
    _a = getattr(torch.Tensor, _n, None)
    if _a is not None:
        _PASSTHROUGH.add(_a)


# Paddle op-type names for common torch functions (interop / IR passes / .pdmodel readability)
def _paddle_types():
    import torch.nn.functional as F
    T = torch.Tensor
    m = {
        torch.matmul: "matmul_v2", T.matmul: "matmul_v2", T.__matmul__: "matmul_v2",
        torch.mm: "matmul_v2", torch.bmm: "matmul_v2", F.linear: "linear",
        torch.add: "elementwise_add", T.add: "elementwise_add", T.__add__: "elementwise_add",
        T.__radd__: "elementwise_add", torch.sub: "elementwise_sub", T.sub: "elementwise_sub",
        T.__sub__: "elementwise_sub", T.__rsub__: "elementwise_sub", torch.mul: "elementwise_mul",
        T.mul: "elementwise_mul", T.__mul__: "elementwise_mul", T.__rmul__: "elementwise_mul",
        torch.true_divide: "elementwise_div", torch.div: "elementwise_div", T.div: "elementwise_div",
        T.__truediv__: "elementwise_div", torch.pow: "elementwise_pow", T.pow: "elementwise_pow",
        T.__pow__: "elementwise_pow", torch.relu: "relu", F.relu: "relu", F.gelu: "gelu",
        torch.sigmoid: "sigmoid", torch.tanh: "tanh", F.silu: "silu", torch.softmax: "softmax",
        F.softmax: "softmax", T.softmax: "softmax", F.log_softmax: "log_softmax",
        F.layer_norm: "layer_norm", F.batch_norm: "batch_norm", F.group_norm: "group_norm",
        F.conv2d: "conv2d", F.conv1d: "conv1d", F.conv_transpose2d: "conv2d_transpose",
        F.max_pool2d: "pool2d", F.avg_pool2d: "pool2d", F.adaptive_avg_pool2d: "pool2d",
        F.embedding: "lookup_table_v2", F.dropout: "dropout", torch.reshape: "reshape2",
        T.reshape: "reshape2", T.view: "reshape2", T.permute: "transpose2", torch.permute: "transpose2",
        T.transpose: "transpose2", torch.transpose: "transpose2", torch.cat: "concat",
        torch.stack: "stack", torch.split: "split", T.split: "split", torch.flatten: "flatten_contiguous_range",
        T.flatten: "flatten_contiguous_range", torch.mean: "reduce_mean", T.mean: "reduce_mean",
        torch.sum: "reduce_sum", T.sum: "reduce_sum", T.__getitem__: "slice", T.to: "cast",
        torch.exp: "exp", torch.log: "log", torch.sqrt: "sqrt", torch.rsqrt: "rsqrt",
        F.cross_entropy: "softmax_with_cross_entropy", torch.where: "where", T.unsqueeze: "unsqueeze2",
        torch.unsqueeze: "unsqueeze2", T.squeeze: "squeeze2", torch.squeeze: "squeeze2",
        F.scaled_dot_product_attention: "fused_attention", T.contiguous: "assign", T.clone: "assign",
        torch.tril: "tril_triu", torch.triu: "tril_triu", T.masked_fill: "masked_fill",
        torch.argmax: "arg_max", torch.topk: "top_k_v2", T.expand: "expand_v2", torch.clamp: "clip",
        T.float: "cast", T.half: "cast", T.bfloat16: "cast", T.__neg__: "scale", torch.neg: "scale",
    }
    return m


_TYPES = None


def _has_variable(args, kwargs):
    for a in args:
        if isinstance(a, Variable):
            return True
        if isinstance(a, (list, tuple)) and any(isinstance(b, Variable) for b in a):
            return True
    return any(isinstance(v, Variable) for v in kwargs.values())


def recordable(paddle_op_type):
    """Make a framework op (``ops.*``) record ITSELF into a static Program when called on
    Variables, so the Executor later dispatches on the real tensors (HIP kernel on GPU) instead of
    freezing whichever branch the meta-tensor trace took."""
    import functools

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            if _has_variable(args, kwargs):
                return _record(fn, args, kwargs)
            return fn(*args, **kwargs)
        fn._paddle_type = paddle_op_type
        wrapper._paddle_type = paddle_op_type
        return wrapper
    return deco


def paddle_type(func):
    global _TYPES
    t = getattr(func, "_paddle_type", None)
    if t is not None:
        return t
    if _TYPES is None:
        _TYPES = _paddle_types()
    try:
        return _TYPES.get(func, "torch_op")
    except TypeError:
        return "torch_op"


def func_qualname(func):
    mod = getattr(func, "__module__", None) or ""
    q = getattr(func, "__qualname__", None) or getattr(func, "__name__", repr(func))
    if isinstance(func, type(torch.Tensor.add)) or mod in ("", None) or "method" in type(func).__name__:
        objcls = getattr(func, "__objclass__", None)
        if objcls is not None:
            return f"torch.Tensor.{func.__name__}"
    return f"{mod}.{q}" if mod else q


class Operator:
    def __init__(self, block, func, args, kwargs, outputs, type=None, attrs=None):  # noqa: A002
        self.block = block
        self.func = func
        self.args = args          # structure with VarRef leaves
        self.kwargs = kwargs
        self.outputs = outputs    # structure with VarRef leaves (or None)
        self.type = type or (paddle_type(func) if func is not None else "custom")
        self.attrs = dict(attrs or {})
        self.idx = None
        self.paddle_inputs = None   # slot -> [var names] for Paddle-typed ops (no torch callable)
        self.paddle_outputs = None

    def input_names(self):
        names = []

        def visit(x):
            if isinstance(x, VarRef):
                names.append(x.name)
            return x
        tree_map(visit, (self.args, self.kwargs))
        for v in (self.paddle_inputs or {}).values():
            names.extend(v)
        return names

    def output_names(self):
        names = []

        def visit(x):
            if isinstance(x, VarRef):
                names.append(x.name)
            return x
        tree_map(visit, self.outputs)
        for v in (self.paddle_outputs or {}).values():
            names.extend(v)
        return names

    def __repr__(self):
        return f"Op({self.type}: {self.input_names()} -> {self.output_names()})"


_OP_DEVICE = [None]  # static.device_guard: op_device attribute of the ops being recorded


class Block:
    def __init__(self, program, idx=0, parent_idx=-1):
        self.program, self.idx, self.parent_idx = program, idx, parent_idx
        self.vars = {}
        self.ops = []

    def var(self, name):
        return self.vars[name]

    def has_var(self, name):
        return name in self.vars

    def create_var(self, name=None, shape=(1,), dtype="float32", persistable=False, stop_gradient=True):
        name = name or unique_name("var")
        meta = torch.empty([SYM_PRIMES[min(i, len(SYM_PRIMES) - 1)] if (s is None or s < 0) else int(s)
                            for i, s in enumerate(shape)],
                           dtype=to_torch_dtype(dtype), device="meta")
        v = Variable(meta, name, self, persistable, stop_gradient, declared_shape=list(shape))
        self.vars[name] = v
        return v

    def append_op(self, op):
        if _OP_DEVICE[0] is not None and "op_device" not in op.attrs:
            op.attrs["op_device"] = _OP_DEVICE[0]
        op.idx = len(self.ops)
        self.ops.append(op)
        self.program._version += 1
        return op

    @property
    def all_parameters(self):
        return [v for v in self.vars.values() if v.persistable_ and v.var_name in self.program.params]


class Program:
    def __init__(self):
        self.blocks = [Block(self, 0)]
        self.params = {}       # persistable var name -> real tensor (initial value)
        self._param_of = {}    # id(real tensor) -> var name
        self._version = 0
        self.random_seed = 0
        self.feed_names = []
        self.fetch_names = []

    def global_block(self):
        return self.blocks[0]

    def current_block(self):
        return self.blocks[getattr(self, "_cur_block", 0)]

    def _create_block(self, parent_idx=None):
        """A sub-block (body of a control-flow op: reference `Program._create_block`)."""
        parent = self._cur_block if parent_idx is None and hasattr(self, "_cur_block") else (parent_idx or 0)
        b = Block(self, len(self.blocks), parent)
        self.blocks.append(b)
        return b

    @contextlib.contextmanager
    def _block_guard(self, block):
        """Record ops into ``block`` (tracing a control-flow branch / loop body)."""
        prev = getattr(self, "_cur_block", 0)
        self._cur_block = block.idx
        try:
            yield block
        finally:
            self._cur_block = prev

    def block(self, idx):
        return self.blocks[idx]

    @property
    def num_blocks(self):
        return len(self.blocks)

    def list_vars(self):
        return list(self.global_block().vars.values())

    def all_parameters(self):
        return self.global_block().all_parameters

    def clone(self, for_test=False):
        import copy
        p = Program()
        p.params = self.params
        p._param_of = dict(self._param_of)
        b = p.global_block()
        src = self.global_block()
        b.vars = dict(src.vars)
        if for_test:
            from .backward import op_role, FORWARD
            b.ops = [op for op in src.ops if op_role(op) == FORWARD]
        else:
            b.ops = list(src.ops)
            for k in ("_backward_info", "_lr_vars", "_grad_roots", "_opt_vars"):
                if hasattr(self, k):
                    setattr(p, k, getattr(self, k))
        p.feed_names, p.fetch_names = list(self.feed_names), list(self.fetch_names)
        if for_test:
            for op in b.ops:
                if op.type == "dropout" or "dropout" in getattr(op.func, "__name__", ""):
                    op.attrs["is_test"] = True
        copy  # noqa
        return p

    def to_string(self, throw_on_error=False, with_details=False):
        lines = [f"Program(vars={len(self.global_block().vars)}, ops={len(self.global_block().ops)})"]
        for op in self.global_block().ops:
            lines.append("  " + repr(op))
        return "\n".join(lines)

    __str__ = to_string

    def param_var(self, tensor):
        """Persistable var holding a real tensor (parameter / buffer / constant)."""
        key = id(tensor)
        name = self._param_of.get(key)
        if name is None:
            name = getattr(tensor, "pd_name", None) or unique_name("param")
            while name in self.params:
                name = unique_name(name)
            self._param_of[key] = name
            self.params[name] = tensor
            b = self.global_block()
            meta = torch.empty(tensor.shape, dtype=tensor.dtype, device="meta")
            b.vars[name] = Variable(meta, name, b, True, not tensor.requires_grad,
                                    declared_shape=list(tensor.shape))
        return name


_MAIN = [Program()]
_STARTUP = [Program()]


def default_main_program():
    return _MAIN[-1]


def default_startup_program():
    return _STARTUP[-1]


@contextlib.contextmanager
def program_guard(main_program, startup_program=None):
    _MAIN.append(main_program)
    _STARTUP.append(startup_program or Program())
    prev = _STATE["static"]
    _STATE["static"] = True
    try:
        yield
    finally:
        _MAIN.pop()
        _STARTUP.pop()
        _STATE["static"] = prev


@contextlib.contextmanager
def name_scope(prefix=None):
    yield


def data(name, shape, dtype="float32", lod_level=0):
    prog = default_main_program()
    v = prog.global_block().create_var(name, shape, dtype, persistable=False, stop_gradient=True)
    if name not in prog.feed_names:
        prog.feed_names.append(name)
    return v


def _record(func, args, kwargs):
    # a torch method replaced by a Paddle-signature adapter (framework/tensor_patch.py) arrives
    # here as the ORIGINAL method; record the adapter (the name every op table keys on) — it
    # forwards torch-form calls unchanged when the Executor replays the op
    from ..framework.tensor_patch import ADAPTER_OF
    func = ADAPTER_OF.get(func, func)
    prog = None

    def find(x):
        nonlocal prog
        if isinstance(x, Variable) and prog is None:
            prog = x.block.program
        return x
    tree_map(find, (args, kwargs))
    prog = prog or default_main_program()
    block = prog.current_block()

    def to_meta(x):
        if isinstance(x, Variable):
            return x.as_subclass(torch.Tensor)
        if isinstance(x, torch.Tensor):
            return torch.empty(x.shape, dtype=x.dtype, device="meta") if x.device.type != "meta" else x
        return x

    def to_ref(x):
        if isinstance(x, Variable):
            return VarRef(x.var_name)
        if isinstance(x, torch.Tensor):
            return VarRef(prog.param_var(x))
        if isinstance(x, torch.Size):
            return tuple(symbolize(int(v)) for v in x)
        return symbolize(x)

    margs = tree_map(to_meta, args)
    mkw = tree_map(to_meta, kwargs)
    with torch._C.DisableTorchFunctionSubclass():
        out = func(*margs, **mkw)

    def wrap(o):
        if isinstance(o, torch.Tensor):
            name = unique_name("tmp")
            v = Variable(o if o.device.type == "meta" else o.to("meta"), name, block, False, False)
            block.vars[name] = v
            return v
        return o
    outs = tree_map(wrap, out)
    out_refs = tree_map(lambda o: VarRef(o.var_name) if isinstance(o, Variable) else o, outs)
    op = Operator(block, func, tree_map(to_ref, args), tree_map(to_ref, kwargs), out_refs)
    block.append_op(op)
    return outs


class Scope:
    """name → tensor (reference `paddle/fluid/framework/scope.h`)."""

    def __init__(self):
        self.vars = {}

    def var(self, name):
        return self.vars.setdefault(name, None)

    def find_var(self, name):
        return _ScopeVar(self, name) if name in self.vars else None

    def get(self, name):
        return self.vars.get(name)

    def set(self, name, t):
        self.vars[name] = t


class _ScopeVar:
    def __init__(self, scope, name):
        self.scope, self.name = scope, name

    def get_tensor(self):
        return self.scope.vars[self.name]


_GLOBAL_SCOPE = Scope()


def global_scope():
    return _GLOBAL_SCOPE


@contextlib.contextmanager
def scope_guard(scope):
    global _GLOBAL_SCOPE
    old = _GLOBAL_SCOPE
    _GLOBAL_SCOPE = scope
    try:
        yield
    finally:
        _GLOBAL_SCOPE = old


class InputSpec:
    """Reference `python/paddle/static/input.py:InputSpec`."""

    def __init__(self, shape, dtype="float32", name=None, stop_gradient=False):
        self.shape, self.dtype, self.name, self.stop_gradient = list(shape), dtype, name, stop_gradient

    def __repr__(self):
        return f"InputSpec(shape={self.shape}, dtype={self.dtype}, name={self.name})"

    @classmethod
    def from_tensor(cls, t, name=None):
        return cls(list(t.shape), dtype_name(t.dtype), name)


dtype_name  # noqa
