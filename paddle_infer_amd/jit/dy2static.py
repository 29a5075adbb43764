"""``paddle.jit.dy2static``: AST conversion of Python control flow for ``jit.to_static``.

Parity: reference `python/paddle/fluid/dygraph/dygraph_to_static/` — ``program_translator.py:1001``
(convert a dygraph function's source), ``ifelse_transformer.py`` (an ``if`` becomes
``convert_ifelse(pred, true_fn, false_fn, ...)`` over the variables its branches assign),
``loop_transformer.py`` (``while`` / ``for ... in range`` become ``convert_while_loop``),
``logical_transformer.py`` (``and`` / ``or`` / ``not`` in conditions) and
``convert_operators.py`` (the run-time helpers below).

At run time every helper keeps plain Python semantics for Python values and concrete tensors
(one host read of a tensor predicate, as dygraph does); on static ``Variable``s (while
``to_static`` records the Program) it emits the ``cond`` / ``while`` ops of
`static/control_flow.py`, so a data-dependent branch or loop is captured as control flow
instead of being frozen by the trace. Statements the converter does not model — a branch or loop
body containing ``return`` / ``break`` / ``continue``, ``for`` over anything but ``range`` — are
left as Python (traced as executed).
"""
from __future__ import annotations

import ast
import inspect
import itertools
import textwrap
import types
import warnings

import torch

from . import ProgramTranslator, not_to_static  # noqa: F401


class _Undefined:
    """A variable assigned by only one branch / only inside a loop (reference UndefinedVar)."""

    def __repr__(self):
        return "UNDEFINED"


UNDEFINED = _Undefined()


def _is_var(x):
    from ..static.framework import Variable
    return isinstance(x, Variable)


def _truth(x):
    if isinstance(x, torch.Tensor):
        return bool(x.reshape(-1)[0])
    return bool(x)


# --------------------------------------------------------------------------- run-time helpers
def convert_ifelse(pred, true_fn, false_fn, args=(), *rest, **kw):
    if _is_var(pred):
        from ..static.nn import cond
        return cond(pred, lambda: true_fn(*args), lambda: false_fn(*args))
    return true_fn(*args) if _truth(pred) else false_fn(*args)


def convert_while_loop(cond_fn, body_fn, args=()):
    args = tuple(args)
    c = cond_fn(*args)
    if _is_var(c):
        from ..static.nn import while_loop
        keep = [i for i, a in enumerate(args) if a is not UNDEFINED]
        full = list(args)

        def cf(*xs):
            for i, x in zip(keep, xs):
                full[i] = x
            return cond_fn(*full)

        def bf(*xs):
            for i, x in zip(keep, xs):
                full[i] = x
            out = body_fn(*full)
            return [out[i] for i in keep]
        res = while_loop(cf, bf, [args[i] for i in keep])
        out = list(args)
        for i, r in zip(keep, res):
            out[i] = r
        return tuple(out)
    while _truth(c):
        args = tuple(body_fn(*args))
        c = cond_fn(*args)
    return args


def convert_logical_and(a_fn, b_fn):
    a = a_fn()
    if _is_var(a) or isinstance(a, torch.Tensor):
        return torch.logical_and(a, b_fn())
    return a and b_fn()


def convert_logical_or(a_fn, b_fn):
    a = a_fn()
    if _is_var(a) or isinstance(a, torch.Tensor):
        return torch.logical_or(a, b_fn())
    return a or b_fn()


def convert_logical_not(a):
    if _is_var(a) or isinstance(a, torch.Tensor):
        return torch.logical_not(a)
    return not a


def range_cond(i, stop, step):
    return i < stop if step > 0 else i > stop


def convert_call(func):
    return func


# --------------------------------------------------------------------------- AST transformer
def _stores(nodes):
    """Names assigned (Store context) in ``nodes``, not descending into nested defs / lambdas."""
    out = []

    def visit(n):
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda, ast.ClassDef)):
            return
        if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Store) and n.id not in out \
                and not n.id.startswith("__jst"):
            out.append(n.id)
        for c in ast.iter_child_nodes(n):
            visit(c)
    for n in nodes:
        visit(n)
    return out


def _has_jump(nodes, loops_ok=False):
    """return / break / continue inside ``nodes`` (break/continue of loops nested inside are fine
    when ``loops_ok``)."""
    def visit(n, in_loop):
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda, ast.ClassDef)):
            return False
        if isinstance(n, (ast.Return, ast.Yield, ast.YieldFrom)):
            return True
        if isinstance(n, (ast.Break, ast.Continue)) and not in_loop:
            return True
        nested = in_loop or isinstance(n, (ast.For, ast.While))
        return any(visit(c, nested) for c in ast.iter_child_nodes(n))
    return any(visit(n, False) for n in nodes)


class _Transformer(ast.NodeTransformer):
    def __init__(self):
        self.n = itertools.count()

    # logical operators inside conditions
    def _test(self, node):
        class L(ast.NodeTransformer):
            def visit_BoolOp(s, n):
                s.generic_visit(n)
                fn = "convert_logical_and" if isinstance(n.op, ast.And) else "convert_logical_or"
                expr = n.values[0]
                for v in n.values[1:]:
                    expr = ast.Call(func=ast.Attribute(value=ast.Name("__jst", ast.Load()), attr=fn, ctx=ast.Load()),
                                    args=[ast.Lambda(args=_noargs(), body=expr), ast.Lambda(args=_noargs(), body=v)],
                                    keywords=[])
                return expr

            def visit_UnaryOp(s, n):
                s.generic_visit(n)
                if isinstance(n.op, ast.Not):
                    return _call("convert_logical_not", [n.operand])
                return n
        return L().visit(node)

    def _ensure_defined(self, names):
        out = []
        for nm in names:
            out.append(ast.Try(body=[ast.Expr(ast.Name(nm, ast.Load()))],
                               handlers=[ast.ExceptHandler(type=ast.Name("NameError", ast.Load()), name=None,
                                                           body=[ast.Assign(targets=[ast.Name(nm, ast.Store())],
                                                                            value=_attr("UNDEFINED"))])],
                               orelse=[], finalbody=[]))
        return out

    def visit_If(self, node):
        self.generic_visit(node)
        if _has_jump(node.body) or _has_jump(node.orelse):
            return node
        names = _stores(node.body + node.orelse)
        k = next(self.n)
        tf, ff = f"__jst_true_{k}", f"__jst_false_{k}"
        ret = ast.Return(ast.Tuple([ast.Name(n, ast.Load()) for n in names], ast.Load()))
        defs = [_fdef(tf, names, list(node.body) + [ret]),
                _fdef(ff, names, (list(node.orelse) or [ast.Pass()]) + [ret])]
        call = _call("convert_ifelse", [self._test(node.test), ast.Name(tf, ast.Load()), ast.Name(ff, ast.Load()),
                                         ast.Tuple([ast.Name(n, ast.Load()) for n in names], ast.Load())])
        if names:
            stmt = ast.Assign(targets=[ast.Tuple([ast.Name(n, ast.Store()) for n in names], ast.Store())], value=call)
        else:
            stmt = ast.Expr(call)
        return defs + self._ensure_defined(names) + [stmt]

    def visit_While(self, node):
        self.generic_visit(node)
        if node.orelse or _has_jump(node.body):
            return node
        names = _stores(node.body)
        k = next(self.n)
        cf, bf = f"__jst_cond_{k}", f"__jst_body_{k}"
        ret = ast.Return(ast.Tuple([ast.Name(n, ast.Load()) for n in names], ast.Load()))
        defs = [_fdef(cf, names, [ast.Return(self._test(node.test))]), _fdef(bf, names, list(node.body) + [ret])]
        call = _call("convert_while_loop", [ast.Name(cf, ast.Load()), ast.Name(bf, ast.Load()),
                                             ast.Tuple([ast.Name(n, ast.Load()) for n in names], ast.Load())])
        if not names:
            return node
        stmt = ast.Assign(targets=[ast.Tuple([ast.Name(n, ast.Store()) for n in names], ast.Store())], value=call)
        return defs + self._ensure_defined(names) + [stmt]

    def visit_For(self, node):
        it = node.iter
        if (node.orelse or not isinstance(node.target, ast.Name) or not isinstance(it, ast.Call)
                or not isinstance(it.func, ast.Name) or it.func.id != "range" or it.keywords
                or not 1 <= len(it.args) <= 3 or _has_jump(node.body)):
            self.generic_visit(node)
            return node
        k = next(self.n)
        i, stop, step = f"__jst_i_{k}", f"__jst_stop_{k}", f"__jst_step_{k}"
        a = it.args
        start_e = a[0] if len(a) > 1 else ast.Constant(0)
        stop_e = a[1] if len(a) > 1 else a[0]
        step_e = a[2] if len(a) > 2 else ast.Constant(1)
        pre = [ast.Assign(targets=[ast.Name(i, ast.Store())], value=start_e),
               ast.Assign(targets=[ast.Name(stop, ast.Store())], value=stop_e),
               ast.Assign(targets=[ast.Name(step, ast.Store())], value=step_e)]
        body = [ast.Assign(targets=[ast.Name(node.target.id, ast.Store())], value=ast.Name(i, ast.Load()))] \
            + list(node.body) + \
            [ast.Assign(targets=[ast.Name(i, ast.Store())],
                        value=ast.BinOp(ast.Name(i, ast.Load()), ast.Add(), ast.Name(step, ast.Load())))]
        # the counter is a loop variable too (named without the __jst prefix filter)
        loop = ast.While(test=_call("range_cond", [ast.Name(i, ast.Load()), ast.Name(stop, ast.Load()),
                                                   ast.Name(step, ast.Load())]),
                         body=body, orelse=[])
        out = self.visit_While_counter(loop, i)
        return pre + (out if isinstance(out, list) else [out])

    def visit_While_counter(self, node, counter):
        self.generic_visit(node)
        names = [counter] + _stores(node.body)
        k = next(self.n)
        cf, bf = f"__jst_cond_{k}", f"__jst_body_{k}"
        ret = ast.Return(ast.Tuple([ast.Name(n, ast.Load()) for n in names], ast.Load()))
        defs = [_fdef(cf, names, [ast.Return(node.test)]), _fdef(bf, names, list(node.body) + [ret])]
        call = _call("convert_while_loop", [ast.Name(cf, ast.Load()), ast.Name(bf, ast.Load()),
                                             ast.Tuple([ast.Name(n, ast.Load()) for n in names], ast.Load())])
        stmt = ast.Assign(targets=[ast.Tuple([ast.Name(n, ast.Store()) for n in names], ast.Store())], value=call)
        return defs + self._ensure_defined(names[1:]) + [stmt]


def _noargs():
    return ast.arguments(posonlyargs=[], args=[], vararg=None, kwonlyargs=[], kw_defaults=[], kwarg=None,
                         defaults=[])


def _attr(name):
    return ast.Attribute(value=ast.Name("__jst", ast.Load()), attr=name, ctx=ast.Load())


def _call(name, args):
    return ast.Call(func=_attr(name), args=args, keywords=[])


def _fdef(name, params, body):
    return ast.FunctionDef(name=name, args=ast.arguments(posonlyargs=[], args=[ast.arg(p) for p in params],
                                                         vararg=None, kwonlyargs=[], kw_defaults=[],
                                                         kwarg=None, defaults=[]),
                           body=body, decorator_list=[], returns=None, type_comment=None)


_CACHE = {}


def convert_to_static(fn):
    """Source-to-source conversion of ``fn`` (function or bound method); returns ``fn`` unchanged
    when its source is unavailable or conversion fails (with a warning)."""
    if getattr(fn, "_not_to_static", False):
        return fn
    bound = getattr(fn, "__self__", None) if isinstance(fn, types.MethodType) else None
    raw = fn.__func__ if bound is not None else fn
    if not isinstance(raw, types.FunctionType):
        return fn
    conv = _CACHE.get(raw)
    if conv is None:
        try:
            conv = _convert_function(raw)
        except (OSError, TypeError, SyntaxError, ValueError) as e:
            warnings.warn(f"dy2static: {raw.__qualname__} kept as Python ({e})")
            conv = raw
        _CACHE[raw] = conv
    return types.MethodType(conv, bound) if bound is not None else conv


def _convert_function(raw):
    src = textwrap.dedent(inspect.getsource(raw))
    tree = ast.parse(src)
    fdef = tree.body[0]
    if not isinstance(fdef, ast.FunctionDef):
        raise ValueError("not a plain function definition")
    fdef.decorator_list = []
    fdef = _Transformer().visit(fdef)
    free = list(raw.__code__.co_freevars)
    factory = _fdef("__jst_factory", free, [fdef, ast.Return(ast.Name(fdef.name, ast.Load()))])
    mod = ast.Module(body=[factory], type_ignores=[])
    ast.fix_missing_locations(mod)
    code = compile(mod, filename=f"<dy2static {raw.__qualname__}>", mode="exec")
    import sys
    ns = dict(raw.__globals__)
    ns["__jst"] = sys.modules[__name__]
    exec(code, ns)  # noqa: S102 - compiling the user's own function source, not loaded data
    cells = [c.cell_contents for c in (raw.__closure__ or ())]
    new = ns["__jst_factory"](*cells)
    new.__defaults__ = raw.__defaults__
    new.__kwdefaults__ = raw.__kwdefaults__
    new.__qualname__ = raw.__qualname__
    new._dy2static_source = ast.unparse(fdef)
    return new
