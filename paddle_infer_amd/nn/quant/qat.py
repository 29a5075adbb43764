"""New-style QAT layers (reference `nn/quant/qat/{linear,conv}.py`): quanters come from a
q_config (factories with ``_instance(layer)``) or default to fake abs-max quantisation."""
import torch
import torch.nn.functional as F

from .format import ConvertibleQuantedLayer
from .quant_layers import FakeQuantAbsMax, FakeQuantMovingAverageAbsMax


def _make(factory, layer, default):
    if factory is None:
        return default()
    return factory._instance(layer) if hasattr(factory, "_instance") else factory


class QuantedLinear(ConvertibleQuantedLayer):
    def __init__(self, layer, q_config=None):
        super().__init__()
        self.weight, self.bias = layer.weight, layer.bias
        wq = getattr(q_config, "weight", None) if q_config is not None else None
        aq = getattr(q_config, "activation", None) if q_config is not None else None
        self.weight_quanter = _make(wq, layer, FakeQuantAbsMax)
        self.activation_quanter = _make(aq, layer, FakeQuantMovingAverageAbsMax)

    def forward(self, x):
        w = self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight
        x = self.activation_quanter(x) if self.activation_quanter is not None else x
        y = torch.matmul(x, w.to(x.dtype))
        return y + self.bias if self.bias is not None else y

    def weights_to_quanters(self):
        return [("weight", "weight_quanter")]

    def activation_quanters(self):
        return ["activation_quanter"]


class QuantedConv2D(ConvertibleQuantedLayer):
    def __init__(self, layer, q_config=None):
        super().__init__()
        self._l = layer
        self.weight, self.bias = layer.weight, layer.bias
        wq = getattr(q_config, "weight", None) if q_config is not None else None
        aq = getattr(q_config, "activation", None) if q_config is not None else None
        self.weight_quanter = _make(wq, layer, FakeQuantAbsMax)
        self.activation_quanter = _make(aq, layer, FakeQuantMovingAverageAbsMax)

    def forward(self, x):
        w = self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight
        x = self.activation_quanter(x) if self.activation_quanter is not None else x
        L = self._l
        conv = getattr(L, "_conv", None) or L
        st = getattr(conv, "stride", getattr(L, "_stride", 1))
        pd = getattr(conv, "padding", getattr(L, "_padding", 0))
        dl = getattr(conv, "dilation", getattr(L, "_dilation", 1))
        gr = getattr(conv, "groups", getattr(L, "_groups", 1))
        return F.conv2d(x, w, self.bias, st, pd, dl, gr)

    def weights_to_quanters(self):
        return [("weight", "weight_quanter")]

    def activation_quanters(self):
        return ["activation_quanter"]
