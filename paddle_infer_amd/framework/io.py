"""``paddle.save`` / ``paddle.load`` (reference `python/paddle/framework/io.py`).

Format: like the reference, a state dict is written as a pickle of ``{name: numpy.ndarray}``
(``.pdparams`` / ``.pdopt``); bf16 tensors are stored as uint16 arrays with a dtype tag, nested
dicts / lists / scalars are kept. Loading uses a RESTRICTED unpickler that can only rebuild numpy
arrays, dtypes and plain containers — nothing in the file can execute code. ``.safetensors``
paths use the safetensors format.
"""
from __future__ import annotations

import collections
import io
import os
import pickle

import numpy as np
import torch

_BF16_TAG = "__bf16__"


def _to_numpy(obj):
    if isinstance(obj, torch.Tensor):
        t = obj.detach().cpu()
        if t.dtype == torch.bfloat16:
            return {_BF16_TAG: t.view(torch.int16).numpy().view(np.uint16)}
        return t.numpy()
    if isinstance(obj, dict):
        return type(obj)((k, _to_numpy(v)) for k, v in obj.items()) if isinstance(obj, collections.OrderedDict) \
            else {k: _to_numpy(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_numpy(v) for v in obj)
    return obj


def _from_numpy(obj, return_numpy=False):
    if isinstance(obj, dict) and set(obj.keys()) == {_BF16_TAG}:
        a = obj[_BF16_TAG]
        return a if return_numpy else torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
    if isinstance(obj, np.ndarray):
        return obj if return_numpy else torch.from_numpy(np.array(obj))
    if isinstance(obj, dict):
        return {k: _from_numpy(v, return_numpy) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_from_numpy(v, return_numpy) for v in obj)
    return obj


class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("collections", "OrderedDict"),
        ("builtins", "set"), ("builtins", "frozenset"), ("builtins", "slice"), ("builtins", "complex"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} (restricted loader)")


def save(obj, path, protocol=4, **configs):
    if hasattr(obj, "state_dict") and not isinstance(obj, dict):
        obj = obj.state_dict()
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    if str(path).endswith(".safetensors"):
        from safetensors.torch import save_file
        save_file({k: v.detach().cpu().contiguous() for k, v in obj.items()}, path)
        return
    with open(path, "wb") as f:
        pickle.dump(_to_numpy(obj), f, protocol=protocol)


def load(path, return_numpy=False, **configs):
    if str(path).endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(path)
        return {k: v.numpy() for k, v in sd.items()} if return_numpy else sd
    with open(path, "rb") as f:
        data = f.read()
    obj = _SafeUnpickler(io.BytesIO(data)).load()
    return _from_numpy(obj, return_numpy)
