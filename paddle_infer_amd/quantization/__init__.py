"""``paddle.quantization`` (reference `python/paddle/quantization/__init__.py` → slim imperative
QAT / PTQ): ImperativeQuantAware (swap Linear / Conv2D for fake-quant wrappers, train, save),
ImperativePTQ (observe activation ranges with abs-max / per-channel / KL / histogram quantizers
and write the scales), PTQConfig and the quantizer registry."""
from __future__ import annotations

import math

import torch

from ..nn.quant import quant_layers as QL

__all__ = ["ImperativeQuantAware", "ImperativePTQ", "PTQConfig", "default_ptq_config",
           "BaseQuantizer", "AbsmaxQuantizer", "PerChannelAbsmaxQuantizer", "KLQuantizer",
           "HistQuantizer", "SUPPORT_ACT_QUANTIZERS", "SUPPORT_WT_QUANTIZERS", "PTQRegistry"]

_WRAP = {"Linear": QL.QuantizedLinear, "Conv2D": QL.QuantizedConv2D,
         "Conv2DTranspose": QL.QuantizedConv2DTranspose,
         "ColumnParallelLinear": QL.QuantizedColumnParallelLinear,
         "RowParallelLinear": QL.QuantizedRowParallelLinear}


class ImperativeQuantAware:
    def __init__(self, quantizable_layer_type=("Conv2D", "Linear", "Conv2DTranspose"),
                 weight_quantize_type="abs_max", activation_quantize_type="moving_average_abs_max",
                 weight_bits=8, activation_bits=8, moving_rate=0.9, fuse_conv_bn=False,
                 weight_preprocess_layer=None, act_preprocess_layer=None,
                 weight_quantize_layer=None, act_quantize_layer=None, onnx_format=False):
        self.types = set(quantizable_layer_type)
        self.kw = dict(weight_bits=weight_bits, activation_bits=activation_bits,
                       moving_rate=moving_rate, weight_quantize_type=weight_quantize_type,
                       activation_quantize_type=activation_quantize_type,
                       weight_pre_layer=weight_preprocess_layer, act_pre_layer=act_preprocess_layer,
                       weight_quant_layer=weight_quantize_layer, act_quant_layer=act_quantize_layer)

    def quantize(self, model):
        for name, child in list(model.named_children()):
            t = type(child).__name__
            if t in self.types and t in _WRAP:
                setattr(model, name, _WRAP[t](child, **self.kw))
            else:
                self.quantize(child)
        return model

    def save_quantized_model(self, layer, path, input_spec=None, **config):
        from .. import jit
        layer.eval()
        return jit.save(layer, path, input_spec=input_spec)


class BaseQuantizer:
    def __init__(self, quant_bits=8):
        self.quant_bits = quant_bits
        self.abs_max_vals = []
        self.thresholds = []

    def sample_data(self, layer, tensors):
        raise NotImplementedError

    def cal_thresholds(self):
        self.thresholds = list(self.abs_max_vals)


class AbsmaxQuantizer(BaseQuantizer):
    def sample_data(self, layer, tensors):
        vals = [float(t.detach().abs().max()) for t in tensors]
        if not self.abs_max_vals:
            self.abs_max_vals = vals
        else:
            self.abs_max_vals = [max(a, b) for a, b in zip(self.abs_max_vals, vals)]


class PerChannelAbsmaxQuantizer(BaseQuantizer):
    def sample_data(self, layer, tensors):
        vals = []
        for t in tensors:
            axis = 1 if type(layer).__name__ in ("Linear",) else 0
            dims = [d for d in range(t.dim()) if d != axis]
            vals.append(t.detach().abs().amax(dim=dims).cpu())
        self.abs_max_vals = vals if not self.abs_max_vals else \
            [torch.maximum(a, b) for a, b in zip(self.abs_max_vals, vals)]


class HistQuantizer(BaseQuantizer):
    """Threshold = the ``hist_percent`` quantile of |x| (histogram over ``bins``)."""

    def __init__(self, quant_bits=8, bins=1024, upsample_bins=64, hist_percent=0.99999):
        super().__init__(quant_bits)
        self.bins, self.hist_percent = bins, hist_percent
        self.hists = []

    def sample_data(self, layer, tensors):
        for i, t in enumerate(tensors):
            a = t.detach().abs().float().flatten().cpu()
            mx = float(a.max()) if a.numel() else 0.0
            if len(self.abs_max_vals) <= i:
                self.abs_max_vals.append(mx)
                self.hists.append(None)
            self.abs_max_vals[i] = max(self.abs_max_vals[i], mx)
            h = torch.histc(a, self.bins, 0.0, max(self.abs_max_vals[i], 1e-12))
            self.hists[i] = h if self.hists[i] is None else self.hists[i] + h

    def cal_thresholds(self):
        self.thresholds = []
        for h, mx in zip(self.hists, self.abs_max_vals):
            c = torch.cumsum(h, 0) / h.sum().clamp_min(1)
            idx = int(torch.searchsorted(c, torch.tensor(self.hist_percent)))
            self.thresholds.append((idx + 0.5) / self.bins * mx)


class KLQuantizer(HistQuantizer):
    """TensorRT-style entropy calibration: the threshold minimising KL(P‖Q) between the clipped
    reference histogram and its quantised version."""

    def __init__(self, quant_bits=8, bins=1024, upsample_bins=64):
        super().__init__(quant_bits, bins, upsample_bins)

    def cal_thresholds(self):
        self.thresholds = []
        nq = 2 ** (self.quant_bits - 1)
        for h, mx in zip(self.hists, self.abs_max_vals):
            h = h.double()
            best, best_i = math.inf, self.bins
            for i in range(nq, self.bins + 1, max(1, self.bins // 128)):
                p = h[:i].clone()
                p[-1] += h[i:].sum()
                q = torch.zeros_like(p)
                chunks = torch.tensor_split(torch.arange(i), nq)
                for ch in chunks:
                    if len(ch):
                        seg = h[ch]
                        nz = (seg > 0).sum()
                        if nz:
                            q[ch] = torch.where(seg > 0, seg.sum() / nz, torch.zeros_like(seg))
                ps, qs = p / p.sum().clamp_min(1e-12), q / q.sum().clamp_min(1e-12)
                m = (ps > 0) & (qs > 0)
                kl = float((ps[m] * torch.log(ps[m] / qs[m])).sum())
                if kl < best:
                    best, best_i = kl, i
            self.thresholds.append((best_i + 0.5) / self.bins * mx)


SUPPORT_ACT_QUANTIZERS = [AbsmaxQuantizer, HistQuantizer, KLQuantizer]
SUPPORT_WT_QUANTIZERS = [AbsmaxQuantizer, PerChannelAbsmaxQuantizer]


class PTQConfig:
    def __init__(self, activation_quantizer, weight_quantizer):
        self.in_act_quantizer = activation_quantizer
        self.out_act_quantizer = type(activation_quantizer)()
        self.wt_quantizer = weight_quantizer
        self.quant_hook_handle = None


default_ptq_config = PTQConfig(KLQuantizer(), PerChannelAbsmaxQuantizer())


class PTQRegistry:
    _SUPPORTED = {"Linear", "Conv2D", "Conv2DTranspose", "ReLU", "ReLU6", "Sigmoid", "Tanh",
                  "Softmax", "LeakyReLU", "Hardswish", "BatchNorm2D", "AvgPool2D", "MaxPool2D"}

    @classmethod
    def is_supported_layer(cls, layer):
        return type(layer).__name__ in cls._SUPPORTED

    @classmethod
    def is_simulated_quant_layer(cls, layer):
        return type(layer).__name__ in ("Linear", "Conv2D", "Conv2DTranspose")


class ImperativePTQ:
    """Post-training quantisation: ``quantize`` attaches forward hooks that feed the configured
    quantizers; run calibration batches; ``convert`` computes thresholds and stores them on each
    layer as ``_quant_in_threshold`` / ``_quant_out_threshold`` / ``_quant_weight_threshold``."""

    def __init__(self, quant_config=default_ptq_config):
        self._cfg = quant_config
        self._layers = []

    def quantize(self, model, inplace=False, fuse=False, fuse_list=None):
        import copy
        m = model if inplace else copy.deepcopy(model)
        for layer in m.modules():
            if not PTQRegistry.is_supported_layer(layer):
                continue
            cfg = PTQConfig(type(self._cfg.in_act_quantizer)(), type(self._cfg.wt_quantizer)())

            def hook(mod, inp, out, cfg=cfg):
                cfg.in_act_quantizer.sample_data(mod, [t for t in inp if isinstance(t, torch.Tensor)])
                cfg.out_act_quantizer.sample_data(mod, [out] if isinstance(out, torch.Tensor) else list(out))
            cfg.quant_hook_handle = layer.register_forward_hook(hook)
            layer._ptq_config = cfg
            self._layers.append(layer)
        return m

    def convert(self, model):
        for layer in self._layers:
            cfg = layer._ptq_config
            cfg.quant_hook_handle.remove()
            cfg.in_act_quantizer.cal_thresholds()
            cfg.out_act_quantizer.cal_thresholds()
            layer._quant_in_threshold = cfg.in_act_quantizer.thresholds
            layer._quant_out_threshold = cfg.out_act_quantizer.thresholds
            if PTQRegistry.is_simulated_quant_layer(layer) and getattr(layer, "weight", None) is not None:
                cfg.wt_quantizer.sample_data(layer, [layer.weight])
                cfg.wt_quantizer.cal_thresholds()
                layer._quant_weight_threshold = cfg.wt_quantizer.thresholds
        return model

    def save_quantized_model(self, model, path, input_spec=None, **config):
        from .. import jit
        model.eval()
        return jit.save(model, path, input_spec=input_spec)
