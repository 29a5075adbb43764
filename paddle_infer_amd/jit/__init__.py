"""``paddle.jit`` — to_static / save / load / TracedLayer.

Parity: reference `python/paddle/fluid/dygraph/jit.py` (declarative:164, save:690, load:1127,
TracedLayer:1388) and `fluid/dygraph/io.py` (TranslatedLayer).

MI355X design: ``to_static`` keeps dygraph execution (the same HIP kernels, autograd intact) and
adds the two things a static program is used for:
* ``concrete_program`` / ``jit.save``: the forward is *recorded* into a static Program by running
  it on meta-backed Variables (`static/framework.py`) after the AST conversion of its Python
  control flow (`dy2static.py`: tensor-dependent ``if`` / ``while`` / ``for range`` become
  ``cond`` / ``while`` ops with sub-blocks); dynamic dims of the InputSpec stay symbolic;
  the Program is written as a Paddle-wire ``.pdmodel`` + ``.pdiparams`` that ``jit.load`` and
  ``inference.create_predictor`` read back.
* ``to_static(..., capture=True)``: the call is captured into a hipGraph per input signature
  (``torch.cuda.CUDAGraph``) and replayed — the launch-overhead removal the reference gets from
  running a compiled program.
"""
from __future__ import annotations

import functools
import json
import os

import numpy as np
import torch

from .. import static as _static
from ..static import io as _sio
from ..static.framework import InputSpec

_TO_STATIC = {"enabled": True}


def enable_to_static(enable=True):
    _TO_STATIC["enabled"] = bool(enable)


class ProgramTranslator:
    _inst = None

    def __new__(cls):
        if cls._inst is None:
            cls._inst = super().__new__(cls)
        return cls._inst

    def enable(self, flag):
        enable_to_static(flag)


def set_code_level(level=100, also_to_stdout=False):
    pass


def set_verbosity(level=0, also_to_stdout=False):
    pass


def not_to_static(func=None):
    if func is None:
        return not_to_static
    func._not_to_static = True
    return func


def ignore_module(modules):
    pass


def _spec_of(x, i):
    if isinstance(x, InputSpec):
        return x
    if isinstance(x, torch.Tensor):
        return InputSpec(list(x.shape), str(x.dtype).replace("torch.", ""), f"x{i}")
    raise TypeError(f"cannot build an InputSpec from {type(x)}")


def trace_program(fn, input_spec, layer=None):
    """Record ``fn(*inputs)`` into a static Program. Returns (program, feed_vars, fetch_vars)."""
    specs = [_spec_of(s, i) for i, s in enumerate(input_spec)]
    from .dy2static import convert_to_static
    fn = convert_to_static(fn)
    main, startup = _static.Program(), _static.Program()
    was_training = layer.training if layer is not None else None
    if layer is not None:
        layer.eval()
    try:
        with _static.program_guard(main, startup):
            feeds = [_static.data(s.name or f"x{i}", s.shape, s.dtype) for i, s in enumerate(specs)]
            with torch.no_grad():
                out = fn(*feeds)
    finally:
        if layer is not None and was_training:
            layer.train()
    outs = list(out) if isinstance(out, (list, tuple)) else [out]
    fetch = [o for o in outs if isinstance(o, _static.Variable)]
    main.fetch_names = [v.var_name for v in fetch]
    return main, feeds, fetch


class StaticFunction:
    """Result of ``to_static``: callable with dygraph semantics + program access."""

    def __init__(self, fn, layer=None, input_spec=None, capture=False):
        self._fn = fn
        self._layer = layer
        self._input_spec = input_spec
        self._capture = capture
        self._programs = {}
        self._graphs = {}
        functools.update_wrapper(self, fn)

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self
        bound = StaticFunction(self._fn.__get__(obj, objtype), obj, self._input_spec, self._capture)
        bound._programs, bound._graphs = self._programs, self._graphs
        return bound

    def __call__(self, *args, **kwargs):
        if not _TO_STATIC["enabled"] or getattr(self._fn, "_not_to_static", False):
            return self._fn(*args, **kwargs)
        if self._capture and args and all(isinstance(a, torch.Tensor) and a.is_cuda for a in args) \
                and not kwargs and not torch.is_grad_enabled():
            return self._replay(args)
        return self._fn(*args, **kwargs)

    def _replay(self, args):
        key = tuple((tuple(a.shape), a.dtype) for a in args)
        ent = self._graphs.get(key)
        if ent is None:
            static_in = [a.clone() for a in args]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._fn(*static_in)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                static_out = self._fn(*static_in)
            ent = self._graphs[key] = (g, static_in, static_out)
        g, static_in, static_out = ent
        for d, a in zip(static_in, args):
            d.copy_(a, non_blocking=True)
        g.replay()
        return static_out

    def get_concrete_program(self, *input_spec):
        spec = list(input_spec) or list(self._input_spec or [])
        key = tuple((tuple(s.shape), str(s.dtype)) for s in map(_spec_of, spec, range(len(spec))))
        if key not in self._programs:
            self._programs[key] = trace_program(self._fn, spec, self._layer)
        return self._programs[key]

    @property
    def concrete_program(self):
        return self.get_concrete_program()

    @property
    def main_program(self):
        return self.concrete_program[0]

    def rollback(self):
        return self._fn

    @property
    def dygraph_function(self):
        return self._fn


def to_static(function=None, input_spec=None, build_strategy=None, capture=False, **kw):
    def deco(fn):
        if isinstance(fn, torch.nn.Module):
            layer = fn
            sf = StaticFunction(layer.forward, layer, input_spec, capture)
            layer.forward = sf
            layer._static_function = sf
            return layer
        return StaticFunction(fn, None, input_spec, capture)
    return deco if function is None else deco(function)


declarative = to_static


# ------------------------------------------------------------------------------------ save / load
def save(layer, path, input_spec=None, **configs):
    """Write ``path.pdmodel`` + ``path.pdiparams`` (+ ``path.pdiparams.info``)."""
    if isinstance(layer, StaticFunction):
        fn, lay, spec0 = layer._fn, layer._layer, layer._input_spec
    else:
        sf = getattr(layer, "_static_function", None)
        fn = sf._fn if sf is not None else layer.forward
        lay, spec0 = layer, (sf._input_spec if sf is not None else None)
    spec = input_spec or spec0
    if spec is None:
        raise ValueError("jit.save needs input_spec (or a to_static layer with input_spec)")
    prog, feeds, fetch = trace_program(fn, spec, lay)
    out_spec = configs.get("output_spec")
    if out_spec:
        fetch = [f for f in fetch if f.var_name in {getattr(o, "var_name", o) for o in out_spec}]
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    scope = _static.Scope()
    for n, t in prog.params.items():
        scope.set(n, t.detach())
    with _static.scope_guard(scope):
        _sio.save_inference_model(path, feeds, fetch, None, program=prog,
                                  allow_custom_ops=configs.get("allow_custom_ops", False))
    info = {n: {"shape": list(t.shape), "dtype": str(t.dtype).replace("torch.", ""),
                "structured_name": n, "trainable": bool(t.requires_grad)} for n, t in prog.params.items()}
    with open(path + ".pdiparams.info", "w") as f:
        json.dump(info, f)


class TranslatedLayer(torch.nn.Module):
    """A loaded inference program as a callable layer (reference `fluid/dygraph/io.py`)."""

    def __init__(self, program, feed_names, fetch_names, scope, device=None):
        super().__init__()
        self._program, self._feed_names, self._fetch_names = program, feed_names, fetch_names
        self._scope = scope
        self._exe = _static.Executor(device)
        for i, (n, t) in enumerate(sorted(program.params.items())):
            p = torch.nn.Parameter(scope.get(n) if scope.get(n) is not None else t, requires_grad=False)
            self.register_parameter(f"p{i}", p)
            scope.set(n, p)

    def forward(self, *inputs):
        feed = {n: (x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x)))
                for n, x in zip(self._feed_names, inputs)}
        with _static.scope_guard(self._scope), torch.no_grad():
            outs = self._exe.run(self._program, feed=feed, fetch_list=self._fetch_names,
                                 return_numpy=False)
        return outs[0] if len(outs) == 1 else outs

    def program(self, method_name="forward"):
        return self._program

    def to(self, *a, **k):
        super().to(*a, **k)
        dev = next(iter(self.parameters())).device if len(list(self.parameters())) else None
        for i, (n, _) in enumerate(sorted(self._program.params.items())):
            self._scope.set(n, getattr(self, f"p{i}"))
        if dev is not None:
            self._exe = _static.Executor(dev)
        return self


def load(path, **configs):
    scope = _static.Scope()
    with _static.scope_guard(scope):
        prog, feeds, fetch = _sio.load_inference_model(path, None)
    for n, t in prog.params.items():
        if scope.get(n) is None:
            scope.set(n, t)
    return TranslatedLayer(prog, feeds, [v.var_name for v in fetch], scope)


class TracedLayer:
    """Reference `jit.py:1388`: trace a layer once, run / save the static program."""

    def __init__(self, program, feed_vars, fetch_vars, layer):
        self._program, self._feeds, self._fetch, self._layer = program, feed_vars, fetch_vars, layer
        self._exe = _static.Executor()
        self._scope = _static.Scope()
        for n, t in program.params.items():
            self._scope.set(n, t.detach())

    @staticmethod
    def trace(layer, inputs):
        inputs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        prog, feeds, fetch = trace_program(layer.forward, inputs, layer)
        out = layer(*inputs)
        return out, TracedLayer(prog, feeds, fetch, layer)

    def set_strategy(self, build_strategy=None, exec_strategy=None):
        pass

    def __call__(self, inputs):
        inputs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        feed = {v.var_name: x for v, x in zip(self._feeds, inputs)}
        with _static.scope_guard(self._scope), torch.no_grad():
            return self._exe.run(self._program, feed=feed, fetch_list=[v.var_name for v in self._fetch],
                                 return_numpy=False)

    def save_inference_model(self, path, feed=None, fetch=None, **kwargs):
        feeds = [self._feeds[i] for i in feed] if feed is not None else self._feeds
        fetches = [self._fetch[i] for i in fetch] if fetch is not None else self._fetch
        with _static.scope_guard(self._scope):
            _sio.save_inference_model(path, feeds, fetches, None, program=self._program)


from . import dy2static  # noqa: E402,F401
