"""Paddle dtype names ↔ torch dtypes (reference `python/paddle/framework/dtype.py`)."""
from __future__ import annotations

import numpy as np
import torch

_MAP = {
    "float32": torch.float32, "fp32": torch.float32, "float": torch.float32,
    "float64": torch.float64, "fp64": torch.float64, "double": torch.float64,
    "float16": torch.float16, "fp16": torch.float16, "half": torch.float16,
    "bfloat16": torch.bfloat16, "bf16": torch.bfloat16,
    "int8": torch.int8, "uint8": torch.uint8, "int16": torch.int16, "int32": torch.int32,
    "int64": torch.int64, "bool": torch.bool, "complex64": torch.complex64,
    "complex128": torch.complex128,
}

float32, float64, float16, bfloat16 = torch.float32, torch.float64, torch.float16, torch.bfloat16
int8, uint8, int16, int32, int64 = torch.int8, torch.uint8, torch.int16, torch.int32, torch.int64
bool_ = torch.bool

_default = [torch.float32]


def to_torch_dtype(d):
    if d is None:
        return _default[0]
    if isinstance(d, torch.dtype):
        return d
    if isinstance(d, str):
        k = d.lower().replace("paddle.", "")
        if k not in _MAP:
            raise TypeError(f"unknown dtype {d}")
        return _MAP[k]
    if isinstance(d, np.dtype) or (isinstance(d, type) and issubclass(d, np.generic)):
        return torch.from_numpy(np.zeros(1, dtype=d)).dtype
    raise TypeError(f"unknown dtype {d!r}")


def dtype_name(d: torch.dtype) -> str:
    for k, v in _MAP.items():
        if v == d and k in ("float32", "float64", "float16", "bfloat16", "int8", "uint8", "int16",
                            "int32", "int64", "bool", "complex64", "complex128"):
            return k
    return str(d).replace("torch.", "")


def set_default_dtype(d):
    _default[0] = to_torch_dtype(d)
    torch.set_default_dtype(_default[0]) if _default[0].is_floating_point else None


def get_default_dtype() -> str:
    return dtype_name(_default[0])


complex64, complex128 = torch.complex64, torch.complex128
dtype = torch.dtype


def iinfo(d):
    return torch.iinfo(to_torch_dtype(d))


def finfo(d):
    return torch.finfo(to_torch_dtype(d))
