"""``paddle.onnx.export`` (reference `python/paddle/onnx/export.py`, which delegates to
paddle2onnx). Here the layer is exported through ``torch.onnx.export``; the ``onnx`` package is
not installed in this image, so the call fails loudly with that reason instead of writing a file."""
from __future__ import annotations

import torch

__all__ = ["export"]


def export(layer, path, input_spec=None, opset_version=9, **configs):
    try:
        import onnx  # noqa: F401
    except ImportError as e:
        raise RuntimeError("paddle.onnx.export needs the 'onnx' package, which is not installed") from e
    from ..static import InputSpec
    args = []
    for s in input_spec or []:
        if isinstance(s, InputSpec):
            shape = [d if d is not None and d > 0 else 1 for d in s.shape]
            args.append(torch.zeros(shape, dtype=s.dtype))
        else:
            args.append(s)
    out = path if path.endswith(".onnx") else path + ".onnx"
    torch.onnx.export(layer, tuple(args), out, opset_version=opset_version)
    return out
