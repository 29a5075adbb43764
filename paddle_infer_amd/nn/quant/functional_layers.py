"""Functional ops as layers (reference `nn/quant/functional_layers.py`), so QAT passes can attach
out-scale observers to them."""
import torch

from ..layer.base import Layer


class FloatFunctionalLayer(Layer):
    def __init__(self):
        super().__init__()


def _mk(name, fn):
    return type(name, (FloatFunctionalLayer,), {"forward": lambda self, *a, **k: fn(*a, **k)})


add = _mk("add", lambda x, y, name=None: torch.add(x, y))
subtract = _mk("subtract", lambda x, y, name=None: torch.sub(x, y))
multiply = _mk("multiply", lambda x, y, name=None: torch.mul(x, y))
divide = _mk("divide", lambda x, y, name=None: torch.div(x, y))
reshape = _mk("reshape", lambda x, shape, name=None: torch.reshape(x, shape))
transpose = _mk("transpose", lambda x, perm, name=None: x.permute(*perm))
concat = _mk("concat", lambda x, axis=0, name=None: torch.cat(list(x), axis))
flatten = _mk("flatten", lambda x, start_axis=0, stop_axis=-1, name=None: torch.flatten(x, start_axis, stop_axis))
matmul = _mk("matmul", lambda x, y, transpose_x=False, transpose_y=False, name=None: torch.matmul(
    x.transpose(-1, -2) if transpose_x else x, y.transpose(-1, -2) if transpose_y else y))
