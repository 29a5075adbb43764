"""``paddle.incubate.autograd`` (reference `incubate/autograd/functional.py`, `primapi.py`):
vjp / jvp / Jacobian / Hessian and forward-mode gradients on the torch autograd engine. The
reference's "prim" mode (lowering to primitive ops for its static compiler) has no counterpart
here — dygraph autograd already differentiates every op — so enable/disable_prim only toggle the
flag that ``prim_enabled()`` reports."""
from __future__ import annotations

import torch
import torch.autograd.functional as AF

__all__ = ["vjp", "jvp", "Jacobian", "Hessian", "enable_prim", "disable_prim", "prim_enabled",
           "forward_grad", "grad"]

_PRIM = {"on": False}


def _tup(x):
    return tuple(x) if isinstance(x, (list, tuple)) else (x,)


def _untup(x, like):
    return x if isinstance(like, (list, tuple)) else x[0]


def vjp(func, xs, v=None):
    """(func(xs), vᵀ·J); v defaults to ones like the output (reference semantics)."""
    if v is None:
        with torch.no_grad():
            o = func(*_tup(xs))
        v = tuple(torch.ones_like(t) for t in _tup(o)) if isinstance(o, (list, tuple)) else torch.ones_like(o)
    out, g = AF.vjp(lambda *a: func(*a), _tup(xs), v)
    return out, _untup(g, xs)


def jvp(func, xs, v=None):
    """(func(xs), J·v); v defaults to ones like the inputs."""
    if v is None:
        v = tuple(torch.ones_like(t) for t in _tup(xs))
    out, g = AF.jvp(lambda *a: func(*a), _tup(xs), v)
    return out, g


class Jacobian:
    """Lazily evaluated Jacobian, indexable like a matrix (``J[:]``, ``J[i, j]``); ``is_batched``
    treats the leading dimension as batch."""

    def __init__(self, func, xs, is_batched=False):
        self._func, self._xs, self._batched = func, _tup(xs), is_batched
        self._mat = None

    def _full(self):
        if self._mat is None:
            xs = self._xs
            if self._batched:
                B = xs[0].shape[0]
                f = lambda *a: self._func(*a).reshape(B, -1)  # noqa: E731
                jac = AF.jacobian(f, xs, vectorize=True)
                jac = jac if isinstance(jac, tuple) else (jac,)
                cols = [j.reshape(B, -1, B, x[0].numel()).diagonal(dim1=0, dim2=2).permute(2, 0, 1)
                        for j, x in zip(jac, xs)]
                self._mat = torch.cat(cols, -1)
            else:
                f = lambda *a: self._func(*a).reshape(-1)  # noqa: E731
                jac = AF.jacobian(f, xs, vectorize=True)
                jac = jac if isinstance(jac, tuple) else (jac,)
                self._mat = torch.cat([j.reshape(j.shape[0], -1) for j in jac], -1)
        return self._mat

    @property
    def shape(self):
        return tuple(self._full().shape)

    def __getitem__(self, idx):
        return self._full()[idx]


class Hessian(Jacobian):
    def __init__(self, func, xs, is_batched=False):
        def g(*a):
            with torch.enable_grad():
                a = [t if t.requires_grad else t.detach().requires_grad_(True) for t in a]
                y = func(*a)
                gr = torch.autograd.grad(y.sum() if is_batched else y, a, create_graph=True)
            return torch.cat([t.reshape(t.shape[0], -1) if is_batched else t.reshape(-1) for t in gr], -1)
        super().__init__(g, xs, is_batched)


def enable_prim():
    _PRIM["on"] = True


def disable_prim():
    _PRIM["on"] = False


def prim_enabled():
    return _PRIM["on"]


def forward_grad(outputs, inputs, grad_inputs=None):
    """Forward-mode directional derivative of ``outputs`` w.r.t. ``inputs`` (double-vjp trick)."""
    outs, ins = _tup(outputs), _tup(inputs)
    gin = _tup(grad_inputs) if grad_inputs is not None else tuple(torch.ones_like(x) for x in ins)
    us = [torch.zeros_like(o, requires_grad=True) for o in outs]
    g = torch.autograd.grad(outs, ins, us, create_graph=True)
    r = torch.autograd.grad(g, us, gin, allow_unused=True)
    return _untup(tuple(r), outputs)


def grad(outputs, inputs, grad_outputs=None):
    r = torch.autograd.grad(_tup(outputs), _tup(inputs), grad_outputs, allow_unused=True)
    return _untup(r, inputs)
