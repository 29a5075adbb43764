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


# ---- Paddle-signature adapters over torch methods of the same name ------------------------------
# Paddle's Tensor methods share names with torch's but take `axis=` (torch: `dim=`), a permutation
# list for transpose, an index TENSOR first for gather / index_select, `num_or_sections` for split,
# transpose flags for matmul. Each adapter recognises the Paddle form (keyword `axis`, a list where
# torch takes ints, a tensor where torch takes an int) and otherwise forwards the call unchanged to
# the original torch method, so torch-style calls inside the framework keep their meaning.
_ORIG = {}
ADAPTER_OF = {}  # original torch method -> its adapter (static tracing records the adapter)


def _orig(name):
    return _ORIG[name]


def _axis_kw(kw):
    if "axis" in kw:
        kw["dim"] = kw.pop("axis")
        if isinstance(kw["dim"], list):
            kw["dim"] = tuple(kw["dim"])
        return True
    return False


def _reduce_adapter(name, values_only=False):
    def fn(self, *args, **kw):
        paddle_form = _axis_kw(kw)
        if paddle_form and kw.get("dim") is None:
            kw.pop("dim")
        if "keepdim" in kw and "dim" not in kw and not args:
            kw.pop("keepdim")  # paddle: keepdim with axis=None is a no-op on a full reduction
        if values_only and paddle_form and "dim" in kw:
            return getattr(torch, "amax" if name == "max" else "amin")(self, **kw)
        return _orig(name)(self, *args, **kw)
    return fn


def _transpose(self, *args, **kw):
    if len(args) == 1 and isinstance(args[0], (list, tuple)) or "perm" in kw:
        return self.permute(*(args[0] if args else kw["perm"]))
    return _orig("transpose")(self, *args, **kw)


def _flatten(self, *args, **kw):
    if "start_axis" in kw or "stop_axis" in kw:
        return _orig("flatten")(self, kw.pop("start_axis", 0), kw.pop("stop_axis", -1))
    return _orig("flatten")(self, *args, **kw)


def _unsqueeze(self, *args, **kw):
    ax = args[0] if args else kw.get("axis", kw.get("dim"))
    if isinstance(ax, (list, tuple)):
        out = self
        for a in sorted(int(v) % (self.dim() + len(ax)) for v in ax):
            out = _orig("unsqueeze")(out, a)
        return out
    return _orig("unsqueeze")(self, ax)


def _squeeze(self, *args, **kw):
    if "axis" in kw:
        ax = kw.pop("axis")
        if ax is None:
            return _orig("squeeze")(self)
        return _orig("squeeze")(self, tuple(ax) if isinstance(ax, (list, tuple)) else ax)
    if args and isinstance(args[0], list):
        return _orig("squeeze")(self, tuple(args[0]))
    return _orig("squeeze")(self, *args, **kw)


def _split(self, *args, **kw):
    if "num_or_sections" in kw or "axis" in kw:
        nos = kw.pop("num_or_sections", args[0] if args else None)
        ax = kw.pop("axis", 0)
        n = self.shape[ax]
        if isinstance(nos, int):
            return list(_orig("split")(self, n // nos, dim=ax))
        secs = list(nos)
        if -1 in secs:
            secs[secs.index(-1)] = n - (sum(secs) + 1)
        return list(_orig("split")(self, secs, dim=ax))
    return _orig("split")(self, *args, **kw)


def _dim_kw_adapter(name, kwname="dim"):
    def fn(self, *args, **kw):
        if _axis_kw(kw) and kwname != "dim":
            d = kw.pop("dim")
            kw[kwname] = tuple(d) if isinstance(d, (list, tuple)) else (d,)
        return _orig(name)(self, *args, **kw)
    return fn


def _sort(self, *args, **kw):
    if _axis_kw(kw):  # paddle: values only
        return torch.sort(self, *args, **kw).values
    return _orig("sort")(self, *args, **kw)


def _paddle_index_form(args, kw):
    """True only when the call cannot be torch's ``(dim, index)`` signature: no ``dim`` keyword
    and either a Tensor first positional argument (Paddle's ``(index, axis)`` order) or an
    ``axis`` keyword. Torch keyword calls (``x.gather(dim=1, index=i)``) are forwarded unchanged."""
    if "dim" in kw:
        return False
    if args:
        return isinstance(args[0], torch.Tensor)
    return "axis" in kw and isinstance(kw.get("index"), torch.Tensor)


def _gather(self, *args, **kw):
    if _paddle_index_form(args, kw):  # paddle.gather(x, index, axis=0): rows along `axis`
        idx = args[0] if args else kw["index"]
        ax = kw.get("axis", args[1] if len(args) > 1 else 0)
        return torch.index_select(self, int(ax or 0), idx.reshape(-1).long())
    return _orig("gather")(self, *args, **kw)


def _index_select(self, *args, **kw):
    if _paddle_index_form(args, kw):  # paddle order: (index, axis)
        idx = args[0] if args else kw["index"]
        ax = kw.get("axis", args[1] if len(args) > 1 else 0)
        return _orig("index_select")(self, int(ax), idx.long())
    return _orig("index_select")(self, *args, **kw)


def _matmul(self, other, *args, **kw):
    tx, ty = kw.pop("transpose_x", False), kw.pop("transpose_y", False)
    if not args and not kw and isinstance(other, torch.Tensor):
        from ..ops.gemm import own_dtype, matmul as _mm
        if own_dtype(self, other):
            return _mm(self, other, tx, ty)
    a = self.transpose(-1, -2) if tx else self
    b = other.transpose(-1, -2) if ty else other
    return _orig("matmul")(a, b, *args, **kw)


def _scale(self, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    out = self * scale + bias if bias_after_scale else (self + bias) * scale
    return torch.relu(out) if act == "relu" else out


_ADAPTERS = {
    "transpose": _transpose, "flatten": _flatten, "unsqueeze": _unsqueeze, "squeeze": _squeeze,
    "split": _split, "sort": _sort, "gather": _gather, "index_select": _index_select,
    "matmul": _matmul,
    **{n: _reduce_adapter(n) for n in ("sum", "mean", "prod", "amax", "amin", "all", "any", "std",
                                        "var", "logsumexp", "nansum", "nanmean", "median")},
    "max": _reduce_adapter("max", values_only=True), "min": _reduce_adapter("min", values_only=True),
    **{n: _dim_kw_adapter(n) for n in ("argmax", "argmin", "cumsum", "cumprod", "topk", "argsort",
                                        "unbind", "chunk", "softmax", "log_softmax", "norm",
                                        "count_nonzero")},
    "flip": _dim_kw_adapter("flip", "dims"), "roll": _dim_kw_adapter("roll", "dims"),
}


def patch():
    for name, fn in _METHODS.items():
        if not hasattr(torch.Tensor, name):
            setattr(torch.Tensor, name, fn)
    if not hasattr(torch.Tensor, "scale"):
        torch.Tensor.scale = _scale
    for name, fn in _ADAPTERS.items():
        if name in _ORIG:
            continue
        _ORIG[name] = getattr(torch.Tensor, name)
        ADAPTER_OF[_ORIG[name]] = fn
        fn.__name__ = name
        fn.__doc__ = f"Paddle-compatible {name} (torch form forwarded unchanged)."
        setattr(torch.Tensor, name, fn)


patch()
