"""QAT layers (reference `nn/quant/quant_layers.py`). Fake quantisation:
``out = round(x / scale · R) · scale / R`` with ``R = 2^(bits-1) - 1`` and a straight-through
gradient (the reference `fake_quantize_dequantize_*` ops' backward is the identity)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..layer.base import Layer


class _STE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale, qmax):
        s = torch.clamp(scale, min=1e-12)
        return torch.round(torch.clamp(x / s, -1.0, 1.0) * qmax) * s / qmax

    @staticmethod
    def backward(ctx, g):
        return g, None, None


def fake_quant_dequant(x, scale, bits=8):
    return _STE.apply(x, scale.to(x.dtype) if isinstance(scale, torch.Tensor) else
                      torch.tensor(float(scale), dtype=x.dtype, device=x.device), float(2 ** (bits - 1) - 1))


class FakeQuantAbsMax(Layer):
    def __init__(self, name=None, quant_bits=8, dtype="float32", quant_on_weight=False,
                 reduce_type=None):
        super().__init__()
        self._quant_bits, self._reduce_type = quant_bits, reduce_type
        self.register_buffer("_scale", torch.zeros(1))

    def forward(self, x):
        scale = x.detach().abs().max().reshape(1)
        if self._reduce_type == "max" and torch.distributed.is_initialized():
            torch.distributed.all_reduce(scale, op=torch.distributed.ReduceOp.MAX)
        self._scale.copy_(scale.to(self._scale.device, self._scale.dtype))
        return fake_quant_dequant(x, scale, self._quant_bits)


class FakeQuantMovingAverageAbsMax(Layer):
    """scale = accum / state with accum = rate·accum + max|x|, state = rate·state + 1 (training);
    the frozen scale in eval."""

    def __init__(self, name=None, moving_rate=0.9, quant_bits=8, dtype="float32", reduce_type=None):
        super().__init__()
        self._moving_rate, self._quant_bits, self._reduce_type = moving_rate, quant_bits, reduce_type
        self.register_buffer("_scale", torch.full((1,), 0.001))
        self.register_buffer("_state", torch.ones(1))
        self.register_buffer("_accum", torch.ones(1))

    def forward(self, x):
        if self.training:
            cur = x.detach().abs().max().reshape(1).float()
            if self._reduce_type == "max" and torch.distributed.is_initialized():
                torch.distributed.all_reduce(cur, op=torch.distributed.ReduceOp.MAX)
            cur = cur.to(self._accum.device)
            self._state.mul_(self._moving_rate).add_(1.0)
            self._accum.mul_(self._moving_rate).add_(cur)
            self._scale.copy_(self._accum / self._state)
        return fake_quant_dequant(x, self._scale.to(x.device), self._quant_bits)


class FakeQuantChannelWiseAbsMax(Layer):
    def __init__(self, name=None, channel_num=None, quant_bits=8, quant_axis=0, dtype="float32",
                 quant_on_weight=False, reduce_type=None):
        super().__init__()
        self._quant_bits, self._quant_axis = quant_bits, quant_axis
        self.register_buffer("_scale", torch.zeros(channel_num or 1))

    def forward(self, x):
        dims = [d for d in range(x.dim()) if d != self._quant_axis]
        scale = x.detach().abs().amax(dim=dims)
        if self._scale.numel() == scale.numel():
            self._scale.copy_(scale.to(self._scale.device, self._scale.dtype))
        shape = [1] * x.dim()
        shape[self._quant_axis] = -1
        return fake_quant_dequant(x, scale.reshape(shape), self._quant_bits)


class MovingAverageAbsMaxScale(Layer):
    """Records the moving-average abs-max of its input (the out-scale of the previous layer);
    forward is the identity."""

    def __init__(self, name=None, moving_rate=0.9, dtype="float32", reduce_type=None):
        super().__init__()
        self._moving_rate = moving_rate
        self.register_buffer("_scale", torch.zeros(1))
        self.register_buffer("_state", torch.zeros(1))
        self.register_buffer("_accum", torch.zeros(1))

    def forward(self, x):
        if self.training:
            cur = x.detach().abs().max().reshape(1).float().to(self._accum.device)
            self._state.mul_(self._moving_rate).add_(1.0)
            self._accum.mul_(self._moving_rate).add_(cur)
            self._scale.copy_(self._accum / self._state)
        return x


def _quanter(kind, moving_rate, bits, channel_num=None, quant_axis=0, on_weight=False):
    if kind in ("abs_max",):
        return FakeQuantAbsMax(quant_bits=bits, quant_on_weight=on_weight)
    if kind in ("moving_average_abs_max",):
        return FakeQuantMovingAverageAbsMax(moving_rate=moving_rate, quant_bits=bits)
    if kind in ("channel_wise_abs_max",):
        return FakeQuantChannelWiseAbsMax(channel_num=channel_num, quant_bits=bits,
                                          quant_axis=quant_axis, quant_on_weight=on_weight)
    raise ValueError(f"unsupported quantize type {kind}")


class _QuantWrap(Layer):
    WEIGHT_AXIS = 0

    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9,
                 weight_quantize_type="abs_max", activation_quantize_type="abs_max",
                 weight_pre_layer=None, act_pre_layer=None, weight_quant_layer=None,
                 act_quant_layer=None):
        super().__init__()
        self._layer = layer
        self.weight = getattr(layer, "weight", None)
        self.bias = getattr(layer, "bias", None)
        ch = self.weight.shape[self.WEIGHT_AXIS] if self.weight is not None else None
        self._fake_quant_weight = weight_quant_layer() if weight_quant_layer else \
            _quanter(weight_quantize_type, moving_rate, weight_bits, ch, self.WEIGHT_AXIS, True)
        self._fake_quant_input = act_quant_layer() if act_quant_layer else \
            _quanter(activation_quantize_type, moving_rate, activation_bits)
        self._act_preprocess = act_pre_layer() if act_pre_layer else None
        self._weight_preprocess = weight_pre_layer() if weight_pre_layer else None

    def _qw(self):
        w = self.weight
        if self._weight_preprocess is not None:
            w = self._weight_preprocess(w)
        return self._fake_quant_weight(w)

    def _qx(self, x):
        if self._act_preprocess is not None:
            x = self._act_preprocess(x)
        return self._fake_quant_input(x)


class QuantizedLinear(_QuantWrap):
    WEIGHT_AXIS = 1  # Paddle Linear weight [in, out]: per output channel

    def forward(self, x):
        y = torch.matmul(self._qx(x), self._qw().to(x.dtype))
        return y + self.bias if self.bias is not None else y


class QuantizedConv2D(_QuantWrap):
    def forward(self, x):
        L = self._layer
        return F.conv2d(self._qx(x), self._qw(), self.bias, L._stride, L._padding, L._dilation,
                        L._groups) if hasattr(L, "_stride") else \
            L.__class__.forward(_Swap(L, self._qw()), self._qx(x))


class QuantizedConv2DTranspose(_QuantWrap):
    WEIGHT_AXIS = 1

    def forward(self, x, output_size=None):
        return _Swap(self._layer, self._qw()).forward(self._qx(x))


class _Swap:
    """Call ``layer.forward`` with a substituted weight (fake-quantised) without mutating it."""

    def __init__(self, layer, w):
        self._l, self._w = layer, w

    def forward(self, x):
        l = self._l
        saved = l.weight
        try:
            object.__setattr__(l, "weight", self._w) if not isinstance(saved, torch.nn.Parameter) \
                else l._parameters.__setitem__("weight", None)
            if isinstance(saved, torch.nn.Parameter):
                l.weight = self._w
            return l.forward(x)
        finally:
            if isinstance(saved, torch.nn.Parameter):
                del l.weight
                l._parameters["weight"] = saved


class QuantizedColumnParallelLinear(QuantizedLinear):
    def forward(self, x):
        from ...distributed.fleet.mp_layers import c_identity, c_concat
        L = self._layer
        x = c_identity(x, L.group)
        y = torch.matmul(self._qx(x), self._qw().to(x.dtype))
        if self.bias is not None:
            y = y + self.bias
        return c_concat(y, L.group) if L.gather_output else y


class QuantizedRowParallelLinear(QuantizedLinear):
    WEIGHT_AXIS = 1

    def forward(self, x):
        from ...distributed.fleet.mp_layers import c_split, mp_allreduce
        L = self._layer
        if not L.input_is_parallel:
            x = c_split(x, L.group)
        y = mp_allreduce(torch.matmul(self._qx(x), self._qw().to(x.dtype)), L.group)
        return y + self.bias if self.bias is not None else y


class QuantizedMatmul(Layer):
    def __init__(self, layer=None, weight_bits=8, activation_bits=8, moving_rate=0.9,
                 activation_quantize_type="abs_max", **kw):
        super().__init__()
        self._fake_quant_x = _quanter(activation_quantize_type, moving_rate, activation_bits)
        self._fake_quant_y = _quanter(activation_quantize_type, moving_rate, activation_bits)

    def forward(self, x, y, transpose_x=False, transpose_y=False, name=None):
        x, y = self._fake_quant_x(x), self._fake_quant_y(y)
        if transpose_x:
            x = x.transpose(-1, -2)
        if transpose_y:
            y = y.transpose(-1, -2)
        return torch.matmul(x, y)


class MAOutputScaleLayer(Layer):
    """Wraps a layer and records the moving-average abs-max of its output."""

    def __init__(self, layer=None, moving_rate=0.9, name=None, dtype="float32", reduce_type=None):
        super().__init__()
        self._layer = layer
        self._ma_output_scale = MovingAverageAbsMaxScale(moving_rate=moving_rate)

    def forward(self, *args, **kwargs):
        out = self._layer(*args, **kwargs)
        if isinstance(out, (list, tuple)):
            return out
        return self._ma_output_scale(out)


class FakeQuantMAOutputScaleLayer(Layer):
    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9, name=None,
                 reduce_type=None, *args, **kwargs):
        super().__init__()
        self._layer = layer
        self._fake_quant_output = FakeQuantMovingAverageAbsMax(moving_rate=moving_rate,
                                                               quant_bits=activation_bits)

    def forward(self, *args, **kwargs):
        out = self._layer(*args, **kwargs)
        if isinstance(out, (list, tuple)):
            return out
        return self._fake_quant_output(out)


class QuantStub(Layer):
    """Marks where activations enter the quantised region (fake-quantises its input)."""

    def __init__(self, quant_bits=8, moving_rate=0.9):
        super().__init__()
        self._fake_quant = FakeQuantMovingAverageAbsMax(moving_rate=moving_rate, quant_bits=quant_bits)

    def forward(self, x):
        return self._fake_quant(x)
