"""``paddle.nn.Layer`` on top of ``torch.nn.Module``.

Parity: reference `python/paddle/fluid/dygraph/layers.py` (Layer: create_parameter, parameters,
named_parameters, sublayers, named_sublayers, state_dict/set_state_dict, train/eval, add_sublayer,
add_parameter, register_forward_pre_hook / post hook, full_name, to / astype).

The dygraph engine underneath is torch autograd; a ``Layer`` is a ``torch.nn.Module`` so the
framework's Layers compose with any torch module, and hooks / state dicts work the same way.
Parameter names in ``state_dict`` use Paddle's structured names (``linear_0.w_0`` style is
available through ``param.name``), keys are the attribute paths exactly like Paddle's.
"""
from __future__ import annotations

import itertools
from collections import OrderedDict

import numpy as np
import torch

from ...framework import dtype as _dt
from .. import initializer as _init

_name_counters: dict = {}


def _unique(prefix: str) -> str:
    c = _name_counters.get(prefix, 0)
    _name_counters[prefix] = c + 1
    return f"{prefix}_{c}"


class ParamAttr:
    """``paddle.ParamAttr`` (reference `python/paddle/fluid/param_attr.py`)."""

    def __init__(self, name=None, initializer=None, learning_rate=1.0, regularizer=None,
                 trainable=True, do_model_average=False, need_clip=True):
        self.name = name
        self.initializer = initializer
        self.learning_rate = learning_rate
        self.regularizer = regularizer
        self.trainable = trainable
        self.need_clip = need_clip

    @staticmethod
    def _to_attr(arg):
        if arg is None:
            return ParamAttr()
        if isinstance(arg, ParamAttr):
            return arg
        if isinstance(arg, str):
            return ParamAttr(name=arg)
        if isinstance(arg, bool):
            return ParamAttr() if arg else False
        if isinstance(arg, _init.Initializer):
            return ParamAttr(initializer=arg)
        raise TypeError(f"bad ParamAttr {arg!r}")


def _as_param(t: torch.Tensor, name: str, trainable=True, need_clip=True) -> torch.nn.Parameter:
    # integer parameters (quantized weights) cannot carry gradients
    p = torch.nn.Parameter(t, requires_grad=trainable and (t.is_floating_point() or t.is_complex()))
    p.pd_name = name  # torch reserves Tensor.name
    p.need_clip = need_clip
    p.optimize_attr = {"learning_rate": 1.0}
    return p


class Layer(torch.nn.Module):
    def __init__(self, name_scope=None, dtype="float32"):
        super().__init__()
        self._full_name = _unique(name_scope or self.__class__.__name__.lower())
        self._dtype = _dt.to_torch_dtype(dtype)
        self._helper_counter = itertools.count()

    # ---- naming -------------------------------------------------------------------------
    def full_name(self) -> str:
        return self._full_name

    # ---- parameter creation --------------------------------------------------------------
    def create_parameter(self, shape, attr=None, dtype=None, is_bias=False,
                         default_initializer=None):
        attr = ParamAttr._to_attr(attr)
        if attr is False:
            return None
        dtype = _dt.to_torch_dtype(dtype) if dtype is not None else self._dtype
        init = attr.initializer or default_initializer or (
            _init.Constant(0.0) if is_bias else _init.XavierUniform())
        t = torch.empty([int(s) for s in shape], dtype=dtype)
        init(t)
        name = attr.name or f"{self._full_name}.{'b' if is_bias else 'w'}_{next(self._helper_counter)}"
        p = _as_param(t, name, attr.trainable, attr.need_clip)
        p.optimize_attr = {"learning_rate": attr.learning_rate}
        p.regularizer = attr.regularizer
        return p

    def create_variable(self, name=None, persistable=None, dtype=None):
        return torch.zeros([], dtype=_dt.to_torch_dtype(dtype or "float32"))

    def create_tensor(self, name=None, persistable=None, dtype=None):
        return self.create_variable(name, persistable, dtype)

    def add_parameter(self, name, parameter):
        self.register_parameter(name, parameter)
        return parameter

    def add_sublayer(self, name, sublayer):
        self.add_module(name, sublayer)
        return sublayer

    def register_buffer(self, name, tensor=None, persistable=True):  # noqa: D401
        return super().register_buffer(name, tensor, persistent=persistable)

    # ---- traversal ----------------------------------------------------------------------
    def parameters(self, include_sublayers=True, recurse=None):
        rec = include_sublayers if recurse is None else recurse
        return list(super().parameters(recurse=rec))

    def named_parameters(self, prefix="", include_sublayers=True, remove_duplicate=True, recurse=None):
        rec = include_sublayers if recurse is None else recurse
        return super().named_parameters(prefix=prefix, recurse=rec,
                                        remove_duplicate=remove_duplicate)

    def sublayers(self, include_self=False):
        mods = list(self.modules())
        return mods if include_self else mods[1:]

    def named_sublayers(self, prefix="", include_self=False, layers_set=None):
        for n, m in self.named_modules(prefix=prefix):
            if m is self and not include_self:
                continue
            yield n, m

    def children(self):
        return super().children()

    # ---- state --------------------------------------------------------------------------
    def set_state_dict(self, state_dict, use_structured_name=True):
        sd = {}
        own = dict(self.state_dict())
        for k, v in state_dict.items():
            if k not in own:
                continue
            t = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
            sd[k] = t.to(own[k].dtype)
        missing = [k for k in own if k not in sd]
        with torch.no_grad():
            for k, t in sd.items():
                own[k].copy_(t.reshape(own[k].shape))
        return missing, [k for k in state_dict if k not in own]

    set_dict = set_state_dict
    load_dict = set_state_dict

    # ---- modes / dtype ------------------------------------------------------------------
    def eval(self):
        return super().eval()

    def train(self, mode=True):
        return super().train(mode)

    def astype(self, dtype):
        return self.to(_dt.to_torch_dtype(dtype))

    def to(self, device=None, dtype=None, blocking=None, *args, **kwargs):
        if isinstance(device, str) and device.startswith("gpu"):
            device = device.replace("gpu", "cuda")
        if dtype is not None:
            dtype = _dt.to_torch_dtype(dtype)
        if device is None:
            return super().to(dtype=dtype) if dtype is not None else self
        return super().to(device=device, dtype=dtype) if dtype is not None else super().to(device)

    def register_forward_post_hook(self, hook):
        return self.register_forward_hook(lambda m, i, o: hook(m, i, o))

    def register_forward_pre_hook(self, hook, *args, **kwargs):
        return super().register_forward_pre_hook(hook, *args, **kwargs)

    def clear_gradients(self, set_to_zero=True):
        for p in self.parameters():
            if p.grad is not None:
                if set_to_zero:
                    p.grad.zero_()
                else:
                    p.grad = None

    def extra_repr(self):
        return ""


class LayerList(Layer, torch.nn.ModuleList):
    def __init__(self, sublayers=None):
        Layer.__init__(self)
        torch.nn.ModuleList.__init__(self, sublayers)


class Sequential(Layer):
    def __init__(self, *layers):
        super().__init__()
        if len(layers) == 1 and isinstance(layers[0], (list, tuple)) and layers[0] and \
                isinstance(layers[0][0], (list, tuple)):
            for n, l in layers[0]:
                self.add_module(str(n), l)
        else:
            for i, l in enumerate(layers):
                if isinstance(l, (list, tuple)):
                    self.add_module(str(l[0]), l[1])
                else:
                    self.add_module(str(i), l)

    def forward(self, x):
        for m in self._modules.values():
            x = m(x)
        return x

    def __getitem__(self, i):
        return list(self._modules.values())[i]

    def __len__(self):
        return len(self._modules)


class LayerDict(Layer, torch.nn.ModuleDict):
    def __init__(self, sublayers=None):
        Layer.__init__(self)
        torch.nn.ModuleDict.__init__(self, sublayers)


class ParameterList(Layer):
    def __init__(self, parameters=None):
        super().__init__()
        for i, p in enumerate(parameters or []):
            self.add_parameter(str(i), p)

    def __getitem__(self, i):
        return list(self._parameters.values())[i]

    def __len__(self):
        return len(self._parameters)

    def __iter__(self):
        return iter(self._parameters.values())

    def append(self, p):
        self.add_parameter(str(len(self._parameters)), p)


OrderedDict  # re-export convenience
