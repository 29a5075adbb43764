"""Quantised-model export format (reference `nn/quant/format.py`): linear quanter / dequanter
pairs and the ConvertibleQuantedLayer protocol used by ``quantization`` to freeze QAT layers."""
from __future__ import annotations

import abc

import torch

from ..layer.base import Layer


class LinearQuanter(Layer):
    def __init__(self, scales, zero_point=None, quant_axis=None, bit_length=8):
        super().__init__()
        self.register_buffer("scales", torch.as_tensor(scales, dtype=torch.float32))
        self.register_buffer("zero_point", torch.as_tensor(0.0 if zero_point is None else zero_point))
        self.quant_axis, self.bit_length = quant_axis, bit_length

    def _bshape(self, x):
        if self.quant_axis is None or self.scales.numel() == 1:
            return self.scales.to(x.device)
        shape = [1] * x.dim()
        shape[self.quant_axis] = -1
        return self.scales.to(x.device).reshape(shape)

    def forward(self, x):
        qmax = 2 ** (self.bit_length - 1) - 1
        s = self._bshape(x).clamp_min(1e-12)
        return torch.clamp(torch.round(x / s * qmax + self.zero_point.to(x.device)), -qmax - 1, qmax)

    @staticmethod
    def from_quanter(quanter):
        return LinearQuanter(quanter.scales(), quanter.zero_points(), quanter.quant_axis(),
                             quanter.bit_length())


class LinearDequanter(LinearQuanter):
    def forward(self, x):
        qmax = 2 ** (self.bit_length - 1) - 1
        return (x - self.zero_point.to(x.device)) * self._bshape(x) / qmax

    @staticmethod
    def from_quanter(quanter):
        return LinearDequanter(quanter.scales(), quanter.zero_points(), quanter.quant_axis(),
                               quanter.bit_length())


class LinearQuanterDequanter(Layer):
    def __init__(self, quanter, dequanter):
        super().__init__()
        self._quanter, self._dequanter = quanter, dequanter

    def forward(self, x):
        out = x
        if self._quanter is not None:
            out = self._quanter(out)
        if self._dequanter is not None:
            out = self._dequanter(out)
        return out

    @staticmethod
    def from_quanter(quanter):
        return LinearQuanterDequanter(LinearQuanter.from_quanter(quanter),
                                      LinearDequanter.from_quanter(quanter))


class ConvertibleQuantedLayer(Layer, metaclass=abc.ABCMeta):
    """A QAT layer that can be frozen: its weight quanter folds into the weight, its activation
    quanters become quanter/dequanter pairs."""

    def __init__(self):
        super().__init__()
        self.converted = False

    @abc.abstractmethod
    def weights_to_quanters(self):
        ...

    @abc.abstractmethod
    def activation_quanters(self):
        ...

    @torch.no_grad()
    def _convert(self):
        for wname, qname in self.weights_to_quanters():
            q = getattr(self, qname)
            if q is not None:
                w = getattr(self, wname)
                w.copy_(q(w))
                setattr(self, qname, None)
        for qname in self.activation_quanters():
            q = getattr(self, qname)
            if q is not None and hasattr(q, "scales"):
                setattr(self, qname, LinearQuanterDequanter.from_quanter(q))
        self.converted = True
