"""Python side of the C inference API (``csrc/capi/pd_capi.cc`` → ``libpiamd_capi.so``).

The C library keeps ``Config`` / ``Predictor`` / ``Tensor`` objects of this package and calls the
helpers below for everything that moves data or needs a dtype / shape convention of the C API
(reference `paddle/fluid/inference/capi_exp/pd_tensor.cc`, `pd_predictor.cc`).
"""
from __future__ import annotations

import numpy as np

from .config import Config, PrecisionType
from .predictor import create_predictor, get_version

# PD_DataType codes (pd_common.h)
PD_DT = {np.dtype("float32"): 0, np.dtype("int32"): 1, np.dtype("int64"): 2, np.dtype("uint8"): 3,
         np.dtype("int8"): 4}
NP_DT = {v: k for k, v in PD_DT.items()}
PRECISION = {0: PrecisionType.Float32, 1: PrecisionType.Int8, 2: PrecisionType.Half}


def new_config():
    return Config()


def enable_use_gpu(cfg, pool_mb, device_id, precision):
    cfg.enable_use_gpu(int(pool_mb), int(device_id), PRECISION.get(int(precision), PrecisionType.Float32))


def new_predictor(cfg):
    return create_predictor(cfg)


def copy_from(t, buf, code):
    """Input handle ← host buffer of PD_DataType ``code`` in the handle's reshaped shape."""
    shape = t._shape
    if shape is None:
        raise ValueError(f"PD_TensorReshape must precede the copy into input '{t.name()}'")
    arr = np.frombuffer(buf, dtype=NP_DT[int(code)]).reshape(shape)
    t.copy_from_cpu(arr.copy())


def copy_to(t, code):
    """Output handle → bytes of PD_DataType ``code`` (converted when the tensor's dtype differs)."""
    arr = np.ascontiguousarray(t.copy_to_cpu())
    want = NP_DT[int(code)]
    if arr.dtype != want:
        arr = arr.astype(want)
    return arr.tobytes()


def shape(t):
    s = t.shape()
    return [int(v) for v in (s if s is not None else [])]


def nbytes(t, code):
    n = 1
    for v in shape(t):
        n *= v
    return n * NP_DT[int(code)].itemsize


def dtype(t):
    """PD_DataType of a handle (16-bit floats are read back as float32: PD_DATA_FLOAT32)."""
    try:
        name = str(t.type()).lower()
    except RuntimeError:  # an input not fed yet
        return -1
    for k, v in (("bfloat16", 0), ("float16", 0), ("float32", 0), ("int32", 1), ("int64", 2),
                 ("uint8", 3), ("int8", 4)):
        if k in name:
            return v
    return -1


def set_lod(t, lod):
    t.set_lod([list(level) for level in lod])


def get_lod(t):
    return [list(level) for level in (t.lod() or [])]


def version():
    return get_version()


def all_passes(cfg):
    return list(cfg.pass_builder().all_passes())


def summary(cfg):
    return str(cfg.summary())
