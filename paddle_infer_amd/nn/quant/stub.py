"""Quanter stubs (reference `nn/quant/stub.py`): placeholders replaced by observers / quanters
when a model is prepared for QAT or PTQ."""
from ..layer.base import Layer


class Stub(Layer):
    def __init__(self, observer=None):
        super().__init__()
        self._observer = observer

    def forward(self, x):
        return x


class QuanterStub(Layer):
    def __init__(self, layer: Stub, q_config=None):
        super().__init__()
        self._observer = None
        if layer._observer is not None:
            self._observer = layer._observer._instance(layer) if hasattr(layer._observer, "_instance") \
                else layer._observer

    def forward(self, x):
        return self._observer(x) if self._observer is not None else x
