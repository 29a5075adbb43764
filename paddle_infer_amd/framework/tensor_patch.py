"""Paddle-only ``Tensor`` methods added to ``torch.Tensor`` (names torch does not define).

Reference: `python/paddle/fluid/dygraph/varbase_patch_methods.py` and `tensor/__init__.py`
(tensor_method_func). Existing torch methods are never overridden.
"""
from __future__ import annotations

import torch

from .dtype import to_torch_dtype as _dt


def _stop_gradient_get(self):
    return not self.requires_grad


def _stop_gradient_set(self, v):
    if self.is_leaf:
        self.requires_grad_(not v)


def _place(self):
    from ..device import Place
    return Place("cpu") if self.device.type == "cpu" else Place("gpu", self.device.index or 0)


def _gradient(self):
    return None if self.grad is None else self.grad.detach().cpu().numpy()


def _clear_gradient(self, set_to_zero=True):
    if self.grad is not None:
        if set_to_zero:
            self.grad.zero_()
        else:
            self.grad = None


def _set_value(self, value):
    with torch.no_grad():
        self.copy_(torch.as_tensor(value, dtype=self.dtype).reshape(self.shape))


_METHODS = {
    "astype": lambda self, dtype: self.to(_dt(dtype)),
    "cast": lambda self, dtype: self.to(_dt(dtype)),
    "place": property(_place),
    "stop_gradient": property(_stop_gradient_get, _stop_gradient_set),
    "gradient": _gradient,
    "clear_gradient": _clear_gradient,
    "clear_grad": _clear_gradient,
    "set_value": _set_value,
    "numel_": lambda self: self.numel(),
    "cpu_": lambda self: self.cpu(),
    "is_tensor": lambda self: True,
    "persistable": False,
}


def patch():
    for name, fn in _METHODS.items():
        if not hasattr(torch.Tensor, name):
            setattr(torch.Tensor, name, fn)


patch()
