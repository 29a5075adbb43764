"""``paddle.set_flags`` / ``get_flags`` (reference `paddle/fluid/platform/flags.cc`).

Flags honoured by this framework: FLAGS_check_nan_inf (NaN/Inf checker on every op output through
``utils.nan_inf``), FLAGS_cudnn_deterministic (torch deterministic algorithms),
FLAGS_use_hipgraph (inference predictor graph capture), FLAGS_allocator_strategy ("auto_growth"
in the environment or set before the first device allocation installs the framework's own
auto-growth best-fit HIP allocator, ``framework/allocator.py``; the in-process default stays
PyTorch's caching allocator), FLAGS_fraction_of_gpu_memory_to_use (accepted).
"""
from __future__ import annotations

import os

import torch

_FLAGS = {
    "FLAGS_check_nan_inf": False,
    "FLAGS_cudnn_deterministic": False,
    "FLAGS_use_hipgraph": True,
    "FLAGS_fraction_of_gpu_memory_to_use": 0.92,
    "FLAGS_allocator_strategy": "auto_growth",
    "FLAGS_eager_delete_tensor_gb": 0.0,
    "FLAGS_benchmark": False,
    "FLAGS_embedding_deterministic": 0,
}
for k in list(_FLAGS):
    if k in os.environ:
        v = os.environ[k]
        d = _FLAGS[k]
        _FLAGS[k] = (v.lower() in ("1", "true")) if isinstance(d, bool) else type(d)(v)


def set_flags(flags: dict):
    for k, v in flags.items():
        _FLAGS[k] = v
        if k == "FLAGS_cudnn_deterministic":
            torch.use_deterministic_algorithms(bool(v), warn_only=True)
        if k == "FLAGS_check_nan_inf":
            from ..utils import nan_inf
            nan_inf.enable(bool(v))
        if k == "FLAGS_allocator_strategy" and v == "auto_growth":
            from . import allocator
            try:
                allocator.enable("auto_growth")
            except RuntimeError as e:  # device memory already in use by the caching allocator
                import warnings
                warnings.warn(f"FLAGS_allocator_strategy=auto_growth not applied: {e}", RuntimeWarning)


def get_flags(flags):
    names = [flags] if isinstance(flags, str) else list(flags)
    return {k: _FLAGS.get(k) for k in names}


def flag(name, default=None):
    return _FLAGS.get(name, default)
