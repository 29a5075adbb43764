"""``paddle.nn.utils`` — parameter reparameterisations and flat-vector transforms.

Parity: reference `python/paddle/nn/utils/weight_norm_hook.py` (``weight_norm`` /
``remove_weight_norm``: w = g · v / ‖v‖ with the norm taken over every dim except ``dim``, ``dim``
None → the whole tensor; parameters ``<name>_g`` / ``<name>_v`` recomputed into ``<name>`` by a
forward-pre hook), `spectral_norm_hook.py` (``spectral_norm``: w / σ(W) with σ from power iteration
on persistent buffers ``<name>_u`` / ``<name>_v``, iterated only in training; the original weight
kept as ``<name>_orig``) and `transform_parameters.py` (``parameters_to_vector`` /
``vector_to_parameters``). The normalisations are autograd compositions on the framework's
tensors; gradients flow to g / v / the original weight.
"""
from __future__ import annotations

import torch

from ..clip import clip_grad_norm_, clip_grad_value_  # noqa: F401

__all__ = ["weight_norm", "remove_weight_norm", "spectral_norm", "parameters_to_vector",
           "vector_to_parameters"]

_EPS = 1e-12


def _norm_except_dim(p, dim):
    """‖p‖ over every axis except ``dim`` (-1: over all), eps inside the sqrt like the reference
    ``norm`` op."""
    if dim == -1:
        return torch.sqrt(torch.sum(p * p) + _EPS)
    pt = p.transpose(0, dim) if dim != 0 else p
    m = pt.reshape(pt.shape[0], -1)
    return torch.sqrt(torch.sum(m * m, dim=1) + _EPS)


def _weight_norm(v, g, dim):
    if dim == -1:
        return v * (g / (torch.sqrt(torch.sum(v * v)) + _EPS))
    n = _norm_except_dim(v, dim)
    shape = [1] * v.dim()
    shape[dim] = v.shape[dim]
    return v * (g / n).reshape(shape)


class WeightNorm:
    def __init__(self, name, dim):
        self.name = name
        self.dim = -1 if dim is None else dim

    def compute_weight(self, layer):
        return _weight_norm(getattr(layer, self.name + "_v"), getattr(layer, self.name + "_g"), self.dim)

    @staticmethod
    def apply(layer, name, dim):
        for hook in layer._forward_pre_hooks.values():
            if isinstance(hook, WeightNorm) and hook.name == name:
                raise RuntimeError(f"Cannot register two weight_norm hooks on the same parameter {name}")
        if dim is None:
            dim = -1
        w = layer._parameters[name]
        nd = w.dim()
        assert -nd <= dim < nd, "dim must set between [-R, R), R means the dimension of weight."
        if dim != -1:
            dim = (dim + nd) % nd
        fn = WeightNorm(name, dim)
        with torch.no_grad():
            g0 = _norm_except_dim(w.detach(), dim).reshape(-1 if dim != -1 else 1)
        del layer._parameters[name]
        layer.add_parameter(name + "_v", torch.nn.Parameter(w.detach().clone()))
        layer.add_parameter(name + "_g", torch.nn.Parameter(g0.clone()))
        object.__setattr__(layer, name, fn.compute_weight(layer))
        layer.register_forward_pre_hook(fn)
        return fn

    def remove(self, layer):
        w = self.compute_weight(layer).detach().clone()
        if self.name in layer.__dict__:
            del layer.__dict__[self.name]
        del layer._parameters[self.name + "_g"]
        del layer._parameters[self.name + "_v"]
        layer.add_parameter(self.name, torch.nn.Parameter(w))

    def __call__(self, layer, inputs):
        object.__setattr__(layer, self.name, self.compute_weight(layer))


def weight_norm(layer, name="weight", dim=0):
    """w = g · v / ‖v‖ (reference `weight_norm_hook.py:165`). Returns ``layer``."""
    WeightNorm.apply(layer, name, dim)
    return layer


def remove_weight_norm(layer, name="weight"):
    """Fold g and v back into a plain ``name`` parameter (reference `weight_norm_hook.py:213`)."""
    for k, hook in list(layer._forward_pre_hooks.items()):
        if isinstance(hook, WeightNorm) and hook.name == name:
            hook.remove(layer)
            del layer._forward_pre_hooks[k]
            return layer
    raise ValueError(f"weight_norm of '{name}' not found in {layer}")


def _normalize(x, eps):
    return x / torch.clamp(torch.linalg.vector_norm(x), min=eps)


class SpectralNorm:
    def __init__(self, name="weight", n_power_iterations=1, dim=0, eps=1e-12):
        if n_power_iterations <= 0:
            raise ValueError(f"Expected n_power_iterations to be positive, but got "
                             f"n_power_iterations={n_power_iterations}")
        self.name, self.dim, self.n_power_iterations, self.eps = name, dim, n_power_iterations, eps

    def reshape_weight_to_matrix(self, w):
        if self.dim != 0:
            w = w.permute([self.dim] + [d for d in range(w.dim()) if d != self.dim])
        return w.reshape(w.shape[0], -1)

    def compute_weight(self, layer, do_power_iteration):
        w = getattr(layer, self.name + "_orig")
        u = getattr(layer, self.name + "_u")
        v = getattr(layer, self.name + "_v")
        wm = self.reshape_weight_to_matrix(w)
        if do_power_iteration:
            with torch.no_grad():
                for _ in range(self.n_power_iterations):
                    v.copy_(_normalize(wm.detach().t() @ u, self.eps))
                    u.copy_(_normalize(wm.detach() @ v, self.eps))
            u, v = u.clone(), v.clone()
        sigma = torch.dot(u, wm @ v)
        return w / sigma

    def __call__(self, layer, inputs):
        object.__setattr__(layer, self.name, self.compute_weight(layer, layer.training))

    @staticmethod
    def apply(layer, name, n_power_iterations, dim, eps):
        for hook in layer._forward_pre_hooks.values():
            if isinstance(hook, SpectralNorm) and hook.name == name:
                raise RuntimeError(f"Cannot register two spectral_norm hooks on the same parameter {name}")
        fn = SpectralNorm(name, n_power_iterations, dim, eps)
        w = layer._parameters[name]
        with torch.no_grad():
            h, wd = fn.reshape_weight_to_matrix(w).shape
            u = _normalize(torch.randn(h, dtype=w.dtype, device=w.device), eps)
            v = _normalize(torch.randn(wd, dtype=w.dtype, device=w.device), eps)
        del layer._parameters[name]
        layer.add_parameter(name + "_orig", w)
        object.__setattr__(layer, name, w * 1.0)
        layer.register_buffer(name + "_u", u)
        layer.register_buffer(name + "_v", v)
        layer.register_forward_pre_hook(fn)
        return fn


def spectral_norm(layer, name="weight", n_power_iterations=1, eps=1e-12, dim=None):
    """w / σ(w) (reference `spectral_norm_hook.py:140`). ``dim`` None → 1 for Linear and the
    transposed convolutions (their output axis), else 0."""
    if dim is None:
        from ..layer import layers as L
        tr = tuple(getattr(L, n) for n in ("Conv1DTranspose", "Conv2DTranspose", "Conv3DTranspose",
                                            "Linear") if hasattr(L, n))
        dim = 1 if isinstance(layer, tr) else 0
    SpectralNorm.apply(layer, name, n_power_iterations, dim, eps)
    return layer


def parameters_to_vector(parameters, name=None):
    """Concatenate the flattened parameters into one 1-D tensor (a copy)."""
    ps = list(parameters)
    with torch.no_grad():
        return torch.cat([p.detach().reshape(-1) for p in ps])


def vector_to_parameters(vec, parameters, name=None):
    """Copy consecutive slices of ``vec`` into ``parameters`` (in place)."""
    off = 0
    with torch.no_grad():
        for p in parameters:
            n = p.numel()
            p.copy_(vec[off:off + n].reshape(p.shape).to(p.dtype))
            off += n
    assert off == vec.numel(), f"vector has {vec.numel()} elements, parameters {off}"
