"""``paddle.autograd`` — backward, grad, PyLayer, functional jacobian/hessian
(reference `python/paddle/autograd/`, `paddle/fluid/eager/backward.cc`).

The dygraph autograd engine is torch's (eager GradNode graph, topological backward on the device
streams); this module exposes Paddle's API on top of it.
"""
from __future__ import annotations

import torch

no_grad = torch.no_grad
enable_grad = torch.enable_grad
set_grad_enabled = torch.set_grad_enabled
is_grad_enabled = torch.is_grad_enabled


def backward(tensors, grad_tensors=None, retain_graph=False):
    if isinstance(tensors, torch.Tensor):
        tensors = [tensors]
    if grad_tensors is not None and isinstance(grad_tensors, torch.Tensor):
        grad_tensors = [grad_tensors]
    torch.autograd.backward(tensors, grad_tensors, retain_graph=retain_graph)


def grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False,
         only_inputs=True, allow_unused=False, no_grad_vars=None):
    single = isinstance(inputs, torch.Tensor)
    outs = [outputs] if isinstance(outputs, torch.Tensor) else list(outputs)
    ins = [inputs] if single else list(inputs)
    go = None
    if grad_outputs is not None:
        go = [grad_outputs] if isinstance(grad_outputs, torch.Tensor) else list(grad_outputs)
    res = torch.autograd.grad(outs, ins, go, retain_graph=retain_graph, create_graph=create_graph,
                              allow_unused=allow_unused)
    return list(res)


class PyLayerContext:
    def __init__(self, tctx):
        self._t = tctx

    def save_for_backward(self, *tensors):
        self._t.save_for_backward(*tensors)

    def saved_tensor(self):
        return self._t.saved_tensors

    def mark_not_inplace(self, *args):
        pass

    def mark_non_differentiable(self, *args):
        self._t.mark_non_differentiable(*args)

    def set_materialize_grads(self, value):
        self._t.set_materialize_grads(value)

    def __setattr__(self, k, v):
        if k == "_t":
            object.__setattr__(self, k, v)
        else:
            setattr(self._t, k, v)

    def __getattr__(self, k):
        return getattr(self._t, k)


class _PyLayerMeta(type):
    def __init__(cls, name, bases, attrs):
        super().__init__(name, bases, attrs)
        if name == "PyLayer":
            return
        user_fwd, user_bwd = attrs.get("forward"), attrs.get("backward")

        def fwd(tctx, *args, **kw):
            return user_fwd(PyLayerContext(tctx), *args, **kw)

        def bwd(tctx, *grads):
            r = user_bwd(PyLayerContext(tctx), *grads)
            return r if isinstance(r, tuple) else (r,)
        cls._fn = type(name + "_Fn", (torch.autograd.Function,),
                       {"forward": staticmethod(fwd), "backward": staticmethod(bwd)})


class PyLayer(metaclass=_PyLayerMeta):
    """Custom differentiable op: subclass with static ``forward(ctx, ...)``/``backward(ctx, ...)``."""

    @classmethod
    def apply(cls, *args, **kwargs):
        if kwargs:
            raise TypeError("PyLayer.apply takes positional arguments only")
        return cls._fn.apply(*args)


def jacobian(ys, xs, batch_axis=None):
    from torch.autograd.functional import jacobian as _j
    if callable(ys):
        return _j(ys, xs)
    return torch.stack([torch.autograd.grad(y, xs, retain_graph=True)[0].reshape(-1) for y in ys.reshape(-1)])


def hessian(func, xs, batch_axis=None):
    from torch.autograd.functional import hessian as _h
    return _h(func, xs)


def saved_tensors_hooks(pack_hook, unpack_hook):
    return torch.autograd.graph.saved_tensors_hooks(pack_hook, unpack_hook)
