"""NaN/Inf checker — ``FLAGS_check_nan_inf`` (reference
`paddle/fluid/framework/details/nan_inf_utils_detail.{cc,cu}` and `eager/nan_inf_utils.cc`).

When enabled, a ``TorchDispatchMode`` sees every op output. GPU floating tensors get one
``piamd_nan_inf_check`` launch that records the FIRST offending op id into a device int (no host
sync per op); :func:`check` (called by the optimizer step / Executor / user) reads it once and
raises ``FloatingPointError`` naming the op. CPU tensors are checked immediately.
"""
from __future__ import annotations

import torch
from torch.utils._python_dispatch import TorchDispatchMode
from torch.utils._pytree import tree_flatten

_STATE = {"mode": None, "names": [], "flag": {}, "skip": set()}
_BIG = 2 ** 31 - 1


class _NanInfMode(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__) if hasattr(func, "overloadpacket") else str(func)
        if name in _STATE["skip"]:
            return out
        leaves, _ = tree_flatten(out)
        for t in leaves:
            if isinstance(t, torch.Tensor) and t.is_floating_point() and t.numel():
                _check_tensor(t, name)
        return out


def _flag(device):
    f = _STATE["flag"].get(device)
    if f is None:
        f = _STATE["flag"][device] = torch.full((1,), _BIG, dtype=torch.int32, device=device)
    return f


def _check_tensor(t, name):
    if t.is_cuda and t.dtype in (torch.float32, torch.bfloat16, torch.float16):
        from ..ops import _lib
        op_id = len(_STATE["names"])
        _STATE["names"].append(name)
        code = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}[t.dtype]
        tc = t if t.is_contiguous() else t.contiguous()
        _lib.call("piamd_nan_inf_check", code, tc.data_ptr(), tc.numel(), _flag(t.device).data_ptr(),
                  op_id, _lib.stream())
    elif not t.is_cuda:
        if not bool(torch.isfinite(t).all()):
            raise FloatingPointError(f"NaN/Inf detected in output of op '{name}' "
                                     f"(shape {list(t.shape)}, dtype {t.dtype})")


def check_tensor(t, name="tensor"):
    """Explicit check of one tensor (sync-free on GPU; raised by the next :func:`check`)."""
    _check_tensor(t, name)


def enable(on=True, skip_ops=()):
    if on and _STATE["mode"] is None:
        _STATE["skip"] = set(skip_ops)
        _STATE["mode"] = _NanInfMode()
        _STATE["mode"].__enter__()
    elif not on and _STATE["mode"] is not None:
        _STATE["mode"].__exit__(None, None, None)
        _STATE["mode"] = None


def enabled():
    return _STATE["mode"] is not None


def check(reset=True):
    """Raise FloatingPointError if any checked op produced NaN/Inf since the last check."""
    for dev, f in _STATE["flag"].items():
        v = int(f.item())
        if v != _BIG:
            name = _STATE["names"][v] if v < len(_STATE["names"]) else f"op#{v}"
            if reset:
                f.fill_(_BIG)
                _STATE["names"].clear()
            raise FloatingPointError(f"NaN/Inf detected in output of op '{name}' (op #{v}) on {dev}")
    if reset:
        _STATE["names"].clear()
