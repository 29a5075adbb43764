"""``paddle.onnx.export`` — reference `python/paddle/onnx/export.py` (which saves the layer as a
Paddle inference program and hands it to paddle2onnx).

Same pipeline here, with no ``onnx`` / ``paddle2onnx`` package: ``jit.save`` writes the
``.pdmodel`` (every recorded op lowered to a reference Paddle op type), ``converter.py`` maps that
ProgramDesc onto ONNX opset-13 operators, and ``proto.py`` serialises the ModelProto with the
framework's own protobuf codec. ``reference.run`` executes a written ``.onnx`` file with a numpy
interpreter of the emitted operator set (used by the tests to check exported graphs numerically).
"""
from __future__ import annotations

import os
import tempfile

import numpy as np

from . import proto
from .converter import ONNXConvertError, program_to_onnx  # noqa: F401
from .reference import run  # noqa: F401

__all__ = ["export", "program_to_onnx", "load_paddle_model", "run", "ONNXConvertError"]


def load_paddle_model(path_prefix: str):
    """(ProgramDesc dict, {persistable name: ndarray}) of a ``.pdmodel`` / ``.pdiparams`` pair."""
    from ..static import proto as sp
    with open(path_prefix + ".pdmodel", "rb") as f:
        desc = sp.decode("ProgramDesc", f.read())
    names = sorted(v["name"] for v in desc["blocks"][0].get("vars", [])
                   if v.get("persistable") and v.get("type", {}).get("type") == sp.VT_LOD_TENSOR)
    params = {}
    pf = path_prefix + ".pdiparams"
    if os.path.exists(pf) and names:
        with open(pf, "rb") as f:
            buf = f.read()
        pos = 0
        for n in names:
            if pos >= len(buf):
                break
            res = sp.tensor_from_stream(buf, pos)
            arr, pos = res[0], res[-1]
            params[n] = arr
    return desc, params


def export(layer, path, input_spec=None, opset_version=13, **configs):
    """Export ``layer`` (dygraph Layer or ``to_static`` function) to ``path`` (``.onnx`` appended
    when missing); returns the written file name. ``input_spec``: list of ``InputSpec`` (``None``
    dims stay symbolic in the ONNX graph inputs)."""
    from .. import jit
    out = path if path.endswith(".onnx") else path + ".onnx"
    with tempfile.TemporaryDirectory() as td:
        prefix = os.path.join(td, "model")
        jit.save(layer, prefix, input_spec=input_spec)
        desc, params = load_paddle_model(prefix)
    model = program_to_onnx(desc, params, opset_version=opset_version)
    d = os.path.dirname(out)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(out, "wb") as f:
        f.write(proto.encode_model(model))
    return out


def load(path: str) -> dict:
    """Decoded ModelProto (dict) of an ``.onnx`` file."""
    with open(path, "rb") as f:
        return proto.decode_model(f.read())


def _np(x):
    return np.asarray(x)
