"""``paddle.nn.functional`` (reference `python/paddle/nn/functional/*.py`).

Hot ops route to the framework's HIP kernels on GPU (layer_norm, gelu/silu/relu with bias,
dropout, softmax-with-mask, flash attention, softmax cross entropy); library ops (conv, pooling,
batch norm, interpolation) go through PyTorch-ROCm (MIOpen / rocBLAS).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as TF

from ... import ops as _ops
from ...framework.dtype import to_torch_dtype as _dt

# ------------------------------------------------------------------------------- activations
relu = lambda x, name=None: TF.relu(x)  # noqa: E731
relu_ = lambda x, name=None: TF.relu_(x)  # noqa: E731
relu6 = lambda x, name=None: TF.relu6(x)  # noqa: E731
elu = lambda x, alpha=1.0, name=None: TF.elu(x, alpha)  # noqa: E731
selu = lambda x, scale=1.0507009873554804934193349852946, alpha=1.6732632423543772848170429916717, name=None: scale * TF.elu(x, alpha)  # noqa: E731
celu = lambda x, alpha=1.0, name=None: TF.celu(x, alpha)  # noqa: E731
leaky_relu = lambda x, negative_slope=0.01, name=None: TF.leaky_relu(x, negative_slope)  # noqa: E731
prelu = lambda x, weight, data_format="NCHW", name=None: TF.prelu(x, weight)  # noqa: E731
sigmoid = lambda x, name=None: torch.sigmoid(x)  # noqa: E731
hardsigmoid = lambda x, slope=0.1666667, offset=0.5, name=None: torch.clamp(x * slope + offset, 0, 1)  # noqa: E731
hardswish = lambda x, name=None: TF.hardswish(x)  # noqa: E731
hardtanh = lambda x, min=-1.0, max=1.0, name=None: TF.hardtanh(x, min, max)  # noqa: E731
hardshrink = lambda x, threshold=0.5, name=None: TF.hardshrink(x, threshold)  # noqa: E731
softshrink = lambda x, threshold=0.5, name=None: TF.softshrink(x, threshold)  # noqa: E731
tanhshrink = lambda x, name=None: TF.tanhshrink(x)  # noqa: E731
tanh = lambda x, name=None: torch.tanh(x)  # noqa: E731
softplus = lambda x, beta=1, threshold=20, name=None: TF.softplus(x, beta, threshold)  # noqa: E731
softsign = lambda x, name=None: TF.softsign(x)  # noqa: E731
mish = lambda x, name=None: TF.mish(x)  # noqa: E731
log_sigmoid = lambda x, name=None: TF.logsigmoid(x)  # noqa: E731
thresholded_relu = lambda x, threshold=1.0, name=None: torch.where(x > threshold, x, torch.zeros_like(x))  # noqa: E731
glu = lambda x, axis=-1, name=None: TF.glu(x, axis)  # noqa: E731
maxout = lambda x, groups, axis=1, name=None: x.reshape(*x.shape[:axis], groups, x.shape[axis] // groups, *x.shape[axis + 1:]).max(axis + 1).values  # noqa: E731


def gelu(x, approximate=False, name=None):
    return _ops.gelu(x, approximate)


def silu(x, name=None):
    return _ops.bias_act(x, None, "silu")


swish = silu


def softmax(x, axis=-1, dtype=None, name=None):
    if dtype is not None:
        x = x.to(_dt(dtype))
    if axis in (-1, x.dim() - 1) and x.is_cuda:
        if x.dtype in (torch.bfloat16, torch.float16) or (
                x.dtype == torch.float32 and x.shape[-1] % 8 == 0 and x.shape[-1] <= 4096):
            return _ops.fused_softmax_mask(x)
    return torch.softmax(x, axis)


def log_softmax(x, axis=-1, dtype=None, name=None):
    if dtype is not None:
        x = x.to(_dt(dtype))
    return torch.log_softmax(x, axis)


def gumbel_softmax(x, temperature=1.0, hard=False, axis=-1, name=None):
    return TF.gumbel_softmax(x, temperature, hard, dim=axis)


# ------------------------------------------------------------------------------- common
def linear(x, weight, bias=None, name=None):
    """Paddle layout: weight ``[in_features, out_features]``."""
    from ...ops.linear import linear as _lin
    return _lin(x, weight, bias)


def dropout(x, p=0.5, axis=None, training=True, mode="upscale_in_train", name=None):
    if not training or p == 0.0:
        return x if mode == "upscale_in_train" else x * (1.0 - p)
    if axis is not None:
        shape = [x.shape[i] if i in ([axis] if isinstance(axis, int) else axis) else 1 for i in range(x.dim())]
        mask = (torch.rand(shape, device=x.device) >= p).to(x.dtype)
        return x * mask / (1 - p) if mode == "upscale_in_train" else x * mask
    if mode == "upscale_in_train":
        return _ops.dropout(x, p, training=True)
    return x * (torch.rand_like(x, dtype=torch.float32) >= p).to(x.dtype)


def dropout2d(x, p=0.5, training=True, data_format="NCHW", name=None):
    return TF.dropout2d(x, p, training)


def dropout3d(x, p=0.5, training=True, data_format="NCDHW", name=None):
    return TF.dropout3d(x, p, training)


def alpha_dropout(x, p=0.5, training=True, name=None):
    return TF.alpha_dropout(x, p, training)


def embedding(x, weight, padding_idx=None, sparse=False, name=None):
    """Reference `phi/kernels/gpu/embedding_kernel.cu`: padding_idx rows are zero in the output and
    get no gradient; the own HIP gather / sort-based gradient kernels (`ops/embedding.py lookup`)."""
    if weight.is_cuda:
        from ...ops.embedding import lookup
        return lookup(x, weight, padding_idx)
    if padding_idx is None:
        return TF.embedding(x, weight)
    pad = padding_idx + weight.shape[0] if padding_idx < 0 else padding_idx
    return TF.embedding(x, weight, pad) * (x != pad).unsqueeze(-1).to(weight.dtype)


def one_hot(x, num_classes, name=None):
    return TF.one_hot(x.long(), num_classes).float()


def pad(x, pad, mode="constant", value=0.0, data_format="NCHW", name=None):
    if isinstance(pad, torch.Tensor):
        pad = pad.tolist()
    pad = list(pad)
    nd = x.dim()
    if len(pad) == 2 * nd:  # Paddle full-rank form: [d0_lo, d0_hi, d1_lo, ...] (first dim first)
        tp = []
        for i in reversed(range(nd)):
            tp += [pad[2 * i], pad[2 * i + 1]]
        pad = tp
    elif data_format in ("NHWC", "NLC", "NDHWC"):
        x = x.movedim(-1, 1)
        out = TF.pad(x, pad, mode if mode != "edge" else "replicate", value)
        return out.movedim(1, -1)
    return TF.pad(x, pad, {"edge": "replicate"}.get(mode, mode), value)


def interpolate(x, size=None, scale_factor=None, mode="nearest", align_corners=False,
                align_mode=0, data_format="NCHW", name=None):
    """Reference `nn/functional/common.py:interpolate`; GPU float tensors resample on the own
    kernels (ops/pool_nd.py: nearest / linear / bilinear / trilinear, 'area' = adaptive average
    pooling); bicubic stays on ATen."""
    mode = {"bilinear": "bilinear", "nearest": "nearest", "bicubic": "bicubic", "linear": "linear",
            "trilinear": "trilinear", "area": "area"}[mode.lower()]
    ac = align_corners if mode in ("bilinear", "bicubic", "linear", "trilinear") else None
    xf = _fmt_in(x, data_format) if data_format in ("NHWC", "NLC", "NDHWC") else x
    if x.is_cuda and mode != "bicubic":
        from ...ops import pool_nd
        if pool_nd.supported(x):
            if mode == "area":
                osz = size if size is not None else None
                if osz is None:
                    sf = scale_factor if isinstance(scale_factor, (list, tuple)) else [scale_factor] * (xf.dim() - 2)
                    osz = [int(i * f) for i, f in zip(xf.shape[2:], sf)]
                return _fmt_out(pool_nd.adaptive_pool(xf, xf.dim() - 2, 1, osz), data_format)
            return _fmt_out(pool_nd.interpolate(xf, size, scale_factor, mode, bool(align_corners)), data_format)
    _lib_fallback(x, "interpolate", "bicubic / non-float dtype (ATen)")
    return _fmt_out(TF.interpolate(xf, size, scale_factor, mode, align_corners=ac), data_format)


upsample = interpolate


def pixel_shuffle(x, upscale_factor, data_format="NCHW", name=None):
    return TF.pixel_shuffle(x, upscale_factor)


def unfold(x, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return TF.unfold(x, kernel_sizes, dilations, paddings, strides)


def cosine_similarity(x1, x2, axis=1, eps=1e-8):
    return TF.cosine_similarity(x1, x2, axis, eps)


def normalize(x, p=2, axis=1, epsilon=1e-12, name=None):
    return TF.normalize(x, p, axis, epsilon)


def label_smooth(label, prior_dist=None, epsilon=0.1, name=None):
    k = label.shape[-1]
    prior = prior_dist if prior_dist is not None else torch.full_like(label, 1.0 / k)
    return (1 - epsilon) * label + epsilon * prior


# ------------------------------------------------------------------------------- conv / pool
def _fmt_in(x, data_format):
    return x.movedim(-1, 1) if data_format in ("NHWC", "NLC", "NDHWC") else x


def _fmt_out(y, data_format):
    return y.movedim(1, -1) if data_format in ("NHWC", "NLC", "NDHWC") else y


def _padding(padding, nd):
    if isinstance(padding, str):
        return padding.lower()
    if isinstance(padding, int):
        return padding
    padding = list(padding)
    if len(padding) == nd:
        return tuple(padding)
    if len(padding) == 2 * nd:
        if all(padding[2 * i] == padding[2 * i + 1] for i in range(nd)):
            return tuple(padding[0::2])
    raise ValueError(f"unsupported asymmetric padding {padding}")


def conv1d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCL", name=None):
    pad = _padding(padding, 1)
    if x.is_cuda and x.dim() == 3 and not isinstance(pad, str):
        # a 1 × L image on the 2-D kernels (ops/conv.py)
        from ...ops import conv as _conv
        p = pad[0] if isinstance(pad, (tuple, list)) else pad
        s = stride[0] if isinstance(stride, (tuple, list)) else stride
        d = dilation[0] if isinstance(dilation, (tuple, list)) else dilation
        nlc = data_format == "NLC"
        y = _conv.conv2d_any(x.unsqueeze(1 if nlc else 2), weight.unsqueeze(2), bias, (1, s), (0, p),
                             (1, d), groups, nhwc=nlc)
        if y is not None:
            return y.squeeze(1 if nlc else 2)
    return _fmt_out(TF.conv1d(_fmt_in(x, data_format), weight, bias, stride, pad, dilation, groups), data_format)


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCHW", name=None):
    """Reference `nn/functional/conv.py:conv2d`; GPU tensors run on the framework's own kernels
    (``ops.conv.conv2d_any``: MFMA implicit GEMM for dense bf16/fp16, direct NHWC kernels for
    grouped / depthwise in any float dtype; NCHW via the channels_last view)."""
    nhwc = data_format == "NHWC"
    pad = _padding(padding, 2)
    if pad == "valid":
        pad = 0
    elif pad == "same" and stride in (1, (1, 1), [1, 1]):
        dl = (dilation, dilation) if isinstance(dilation, int) else tuple(dilation)
        tot = [dl[i] * (weight.shape[2 + i] - 1) for i in range(2)]
        if all(t % 2 == 0 for t in tot):
            pad = (tot[0] // 2, tot[1] // 2)
    if x.is_cuda:
        from ...ops import conv as _conv
        y = _conv.conv2d_any(x, weight, bias, stride, pad, dilation, groups, nhwc)
        if y is not None:
            return y
    return _fmt_out(TF.conv2d(_fmt_in(x, data_format), weight, bias, stride, pad, dilation, groups), data_format)


def _lib_fallback(x, op, why="ATen / MIOpen (no own kernel for this op)"):
    """Record (warn once) a GPU call that leaves the framework's HIP kernels (`ops/_lib.py`)."""
    if x.is_cuda:
        from ...ops import _lib
        _lib.fallback(op, why)


def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCDHW", name=None):
    """Reference `nn/functional/conv.py:conv3d`; GPU tensors: kd 2-D convs on the own kernels
    (`ops.conv.conv3d_any`)."""
    pad = _padding(padding, 3)
    if x.is_cuda:
        from ...ops import conv as _conv
        y = _conv.conv3d_any(x, weight, bias, stride, pad, dilation, groups, data_format == "NDHWC")
        if y is not None:
            return y
        _lib_fallback(x, "conv3d", "string padding (MIOpen)")
    return _fmt_out(TF.conv3d(_fmt_in(x, data_format), weight, bias, stride, pad, dilation, groups), data_format)


def conv3d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     data_format="NCDHW", output_size=None, name=None):
    if x.is_cuda:
        from ...ops import conv as _conv
        y = _conv.conv3d_transpose_any(x, weight, bias, stride, _padding(padding, 3), output_padding,
                                       groups, dilation, data_format == "NDHWC", output_size)
        if y is not None:
            return y
        _lib_fallback(x, "conv3d_transpose", "string padding (MIOpen)")
    return _fmt_out(TF.conv_transpose3d(_fmt_in(x, data_format), weight, bias, stride, _padding(padding, 3),
                                        output_padding, groups, dilation), data_format)


def conv2d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                     dilation=1, data_format="NCHW", output_size=None, name=None):
    if x.is_cuda:
        from ...ops import conv as _conv
        y = _conv.conv2d_transpose_any(x, weight, bias, stride, _padding(padding, 2), output_padding,
                                       groups, dilation, data_format == "NHWC", output_size)
        if y is not None:
            return y
    return _fmt_out(TF.conv_transpose2d(_fmt_in(x, data_format), weight, bias, stride, _padding(padding, 2), output_padding, groups, dilation), data_format)


def conv1d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                     dilation=1, output_size=None, data_format="NCL", name=None):
    if x.is_cuda:
        from ...ops import conv as _conv
        y = _conv.conv1d_transpose_any(x, weight, bias, stride, _padding(padding, 1), output_padding,
                                       groups, dilation, data_format == "NLC", output_size)
        if y is not None:
            return y
        _lib_fallback(x, "conv1d_transpose", "string padding (MIOpen)")
    return _fmt_out(TF.conv_transpose1d(_fmt_in(x, data_format), weight, bias, stride, _padding(padding, 1), output_padding, groups, dilation), data_format)


def _own_pool(x, pad):
    """GPU float tensors with numeric padding pool on the own kernels (ops/pool_nd.py)."""
    if not x.is_cuda:
        return False
    from ...ops import pool_nd
    if pool_nd.supported(x) and not isinstance(pad, str):
        return True
    _lib_fallback(x, "pool", "string padding / non-float dtype (ATen)")
    return False


def _pool(x, nd, mode, kernel_size, stride, padding, ceil_mode, exclusive, divisor, return_mask,
          data_format):
    from ...ops import pool_nd
    r = pool_nd.pool(_fmt_in(x, data_format), nd, mode, kernel_size, stride, padding, ceil_mode, exclusive,
                     divisor, return_mask)
    if return_mask:
        return _fmt_out(r[0], data_format), _fmt_out(r[1], data_format)
    return _fmt_out(r, data_format)


def _apool(x, nd, mode, output_size, return_mask, data_format):
    from ...ops import pool_nd
    r = pool_nd.adaptive_pool(_fmt_in(x, data_format), nd, mode, output_size, return_mask)
    if return_mask:
        return _fmt_out(r[0], data_format), _fmt_out(r[1], data_format)
    return _fmt_out(r, data_format)


def max_pool1d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, name=None):
    pad = _padding(padding, 1)
    if _own_pool(x, pad):
        return _pool(x, 1, 0, kernel_size, stride, pad, ceil_mode, True, None, return_mask, "NCL")
    return TF.max_pool1d(x, kernel_size, stride, pad, 1, ceil_mode, return_mask)


def max_pool2d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
               data_format="NCHW", name=None):
    pad = _padding(padding, 2)
    if data_format == "NCHW":
        from ...ops.pool import max_pool2d_nhwc, max_pool2d_supported
        if max_pool2d_supported(x, kernel_size, stride, pad, ceil_mode, return_mask):
            return max_pool2d_nhwc(x, kernel_size, stride, pad)  # own NHWC kernels (channels-last)
    if _own_pool(x, pad):
        return _pool(x, 2, 0, kernel_size, stride, pad, ceil_mode, True, None, return_mask, data_format)
    y = TF.max_pool2d(_fmt_in(x, data_format), kernel_size, stride, pad, 1, ceil_mode, return_mask)
    return y if return_mask else _fmt_out(y, data_format)


def max_pool3d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
               data_format="NCDHW", name=None):
    pad = _padding(padding, 3)
    if _own_pool(x, pad):
        return _pool(x, 3, 0, kernel_size, stride, pad, ceil_mode, True, None, return_mask, data_format)
    y = TF.max_pool3d(_fmt_in(x, data_format), kernel_size, stride, pad, 1, ceil_mode, return_mask)
    return y if return_mask else _fmt_out(y, data_format)


def avg_pool1d(x, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
    pad = _padding(padding, 1)
    if _own_pool(x, pad):
        return _pool(x, 1, 1, kernel_size, stride, pad, ceil_mode, exclusive, None, False, "NCL")
    return TF.avg_pool1d(x, kernel_size, stride, pad, ceil_mode, not exclusive)


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True,
               divisor_override=None, data_format="NCHW", name=None):
    pad = _padding(padding, 2)
    if _own_pool(x, pad):
        return _pool(x, 2, 1, kernel_size, stride, pad, ceil_mode, exclusive, divisor_override, False, data_format)
    return _fmt_out(TF.avg_pool2d(_fmt_in(x, data_format), kernel_size, stride, pad, ceil_mode, not exclusive,
                                  divisor_override), data_format)


def avg_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True,
               divisor_override=None, data_format="NCDHW", name=None):
    pad = _padding(padding, 3)
    if _own_pool(x, pad):
        return _pool(x, 3, 1, kernel_size, stride, pad, ceil_mode, exclusive, divisor_override, False, data_format)
    return _fmt_out(TF.avg_pool3d(_fmt_in(x, data_format), kernel_size, stride, pad, ceil_mode, not exclusive,
                                  divisor_override), data_format)


def adaptive_avg_pool1d(x, output_size, name=None):
    if _own_pool(x, 0):
        return _apool(x, 1, 1, output_size, False, "NCL")
    return TF.adaptive_avg_pool1d(x, output_size)


def adaptive_avg_pool2d(x, output_size, data_format="NCHW", name=None):
    if _own_pool(x, 0):
        return _apool(x, 2, 1, output_size, False, data_format)
    return _fmt_out(TF.adaptive_avg_pool2d(_fmt_in(x, data_format), output_size), data_format)


def adaptive_avg_pool3d(x, output_size, data_format="NCDHW", name=None):
    if _own_pool(x, 0):
        return _apool(x, 3, 1, output_size, False, data_format)
    return _fmt_out(TF.adaptive_avg_pool3d(_fmt_in(x, data_format), output_size), data_format)


def adaptive_max_pool1d(x, output_size, return_mask=False, name=None):
    if _own_pool(x, 0):
        return _apool(x, 1, 0, output_size, return_mask, "NCL")
    return TF.adaptive_max_pool1d(x, output_size, return_mask)


def adaptive_max_pool2d(x, output_size, return_mask=False, name=None):
    if _own_pool(x, 0):
        return _apool(x, 2, 0, output_size, return_mask, "NCHW")
    return TF.adaptive_max_pool2d(x, output_size, return_mask)


def adaptive_max_pool3d(x, output_size, return_mask=False, name=None):
    if _own_pool(x, 0):
        return _apool(x, 3, 0, output_size, return_mask, "NCDHW")
    return TF.adaptive_max_pool3d(x, output_size, return_mask)


# ------------------------------------------------------------------------------- normalization
def layer_norm(x, normalized_shape, weight=None, bias=None, epsilon=1e-5, name=None):
    ns = [normalized_shape] if isinstance(normalized_shape, int) else list(normalized_shape)
    if len(ns) == 1:
        return _ops.layer_norm(x, weight, bias, epsilon)
    return TF.layer_norm(x, ns, weight, bias, epsilon)


def rms_norm(x, weight=None, epsilon=1e-6, name=None):
    return _ops.rms_norm(x, weight, epsilon)


def batch_norm(x, running_mean, running_var, weight=None, bias=None, training=False,
               momentum=0.9, epsilon=1e-5, data_format="NCHW", use_global_stats=None, name=None,
               act=None, residual=None):
    """Reference `nn/functional/norm.py:batch_norm`; on the GPU the fused HIP kernel
    (``ops.batchnorm``: statistics + normalise (+ residual) (+ relu/relu6) in two passes)."""
    if use_global_stats:
        training = False
    if x.is_cuda and act in (None, "relu", "relu6") and x.dim() >= 2:
        from ...ops.batchnorm import batch_norm_act
        return batch_norm_act(x, running_mean, running_var, weight, bias, training, momentum,
                              epsilon, act or "none", residual, data_format)
    y = TF.batch_norm(_fmt_in(x, data_format), running_mean, running_var, weight, bias, training,
                      1.0 - momentum, epsilon)
    y = _fmt_out(y, data_format)
    if residual is not None:
        y = y + residual
    if act == "relu":
        y = torch.relu(y)
    elif act == "relu6":
        y = torch.clamp(y, 0.0, 6.0)
    return y


def instance_norm(x, running_mean=None, running_var=None, weight=None, bias=None,
                  use_input_stats=True, momentum=0.9, eps=1e-5, data_format="NCHW", name=None):
    """Own GroupNorm kernels with one channel per group (`ops/groupnorm.py`); the running-statistics
    update of a training call with running buffers stays on ATen (recorded)."""
    if x.is_cuda:
        from ...ops import groupnorm as _gn
        C = x.shape[1] if x.dim() >= 2 else 0
        if use_input_stats and running_mean is None and running_var is None and _gn.supported(x, max(C, 1)):
            return _gn.group_norm(x, C, weight, bias, eps)
        if (not use_input_stats and running_mean is not None and running_var is not None
                and _gn.supported(x, max(C, 1)) and not (torch.is_grad_enabled() and (
                    x.requires_grad or any(t is not None and t.requires_grad for t in (weight, bias))))):
            return _gn.instance_norm_eval(x, running_mean, running_var, weight, bias, eps)
        _lib_fallback(x, "instance_norm", "running-statistics update / eval under autograd (ATen)")
    return TF.instance_norm(x, running_mean, running_var, weight, bias, use_input_stats, 1 - momentum, eps)


def group_norm(x, num_groups, epsilon=1e-5, weight=None, bias=None, data_format="NCHW", name=None):
    """Own HIP kernels (`ops/groupnorm.py`, plane reductions + Chan merge, deterministic backward)."""
    xin = _fmt_in(x, data_format)
    if x.is_cuda:
        from ...ops import groupnorm as _gn
        if _gn.supported(xin, num_groups):
            return _fmt_out(_gn.group_norm(xin, num_groups, weight, bias, epsilon), data_format)
        _lib_fallback(x, "group_norm", "non-float dtype / channels not divisible by groups (ATen)")
    return _fmt_out(TF.group_norm(xin, num_groups, weight, bias, epsilon), data_format)


def local_response_norm(x, size, alpha=1e-4, beta=0.75, k=1.0, data_format="NCHW", name=None):
    return TF.local_response_norm(x, size, alpha, beta, k)


# ------------------------------------------------------------------------------- losses
def _reduce(loss, reduction):
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss


def _up(t):
    """Loss math in fp32 for 16-bit inputs; fp32 / fp64 keep their precision."""
    return t.float() if t.is_floating_point() and t.element_size() < 4 else t


def cross_entropy(input, label, weight=None, ignore_index=-100, reduction="mean", soft_label=False,  # noqa: A002
                  axis=-1, use_softmax=True, label_smoothing=0.0, name=None):
    if axis not in (-1, input.dim() - 1):
        input = input.movedim(axis, -1)
        label = label.movedim(axis, -1) if soft_label else label
    V = input.shape[-1]
    if soft_label:
        logp = torch.log_softmax(_up(input), -1) if use_softmax else torch.log(_up(input))
        loss = -(_up(label) * logp).sum(-1)
        if weight is not None:
            loss = loss * (_up(label) * weight).sum(-1)
        return _reduce(loss, reduction)
    lab = label.squeeze(-1) if label.dim() == input.dim() else label
    if not use_softmax:
        loss = TF.nll_loss(torch.log(_up(input)).reshape(-1, V), lab.reshape(-1).long(),
                           weight, ignore_index=ignore_index, reduction="none").view(lab.shape)
    elif weight is None and label_smoothing == 0.0:
        loss = _up(_ops.softmax_cross_entropy(input, lab, ignore_index))
    else:
        loss = TF.cross_entropy(_up(input).reshape(-1, V), lab.reshape(-1).long(), weight,
                                ignore_index=ignore_index, reduction="none",
                                label_smoothing=label_smoothing).view(lab.shape)
    if reduction == "mean":
        if weight is not None:
            w = weight[lab.clamp(min=0).long()] * (lab != ignore_index)
            return loss.sum() / w.sum()
        valid = (lab != ignore_index).sum().clamp(min=1)
        return loss.sum() / valid
    out = _reduce(loss, reduction)
    return out.unsqueeze(-1) if reduction == "none" and label.dim() == input.dim() else out


def softmax_with_cross_entropy(logits, label, soft_label=False, ignore_index=-100,
                               numeric_stable_mode=True, return_softmax=False, axis=-1):
    loss = cross_entropy(logits, label, ignore_index=ignore_index, reduction="none",
                         soft_label=soft_label, axis=axis)
    if loss.dim() < logits.dim():
        loss = loss.unsqueeze(axis)
    if return_softmax:
        return loss, torch.softmax(logits, axis)
    return loss


def nll_loss(input, label, weight=None, ignore_index=-100, reduction="mean", name=None):  # noqa: A002
    return TF.nll_loss(input, label.long(), weight, ignore_index=ignore_index, reduction=reduction)


def mse_loss(input, label, reduction="mean", name=None):  # noqa: A002
    return TF.mse_loss(input, label, reduction=reduction)


def l1_loss(input, label, reduction="mean", name=None):  # noqa: A002
    return TF.l1_loss(input, label, reduction=reduction)


def smooth_l1_loss(input, label, reduction="mean", delta=1.0, name=None):  # noqa: A002
    return TF.smooth_l1_loss(input, label, reduction=reduction, beta=delta) * delta


def binary_cross_entropy(input, label, weight=None, reduction="mean", name=None):  # noqa: A002
    return TF.binary_cross_entropy(input, label, weight, reduction=reduction)


def binary_cross_entropy_with_logits(logit, label, weight=None, reduction="mean", pos_weight=None, name=None):
    return TF.binary_cross_entropy_with_logits(logit, label, weight, reduction=reduction, pos_weight=pos_weight)


def kl_div(input, label, reduction="mean", name=None):  # noqa: A002
    return TF.kl_div(input, label, reduction=reduction)


def margin_ranking_loss(input, other, label, margin=0.0, reduction="mean", name=None):  # noqa: A002
    return TF.margin_ranking_loss(input, other, label, margin, reduction=reduction)


def hinge_embedding_loss(input, label, margin=1.0, reduction="mean", name=None):  # noqa: A002
    return TF.hinge_embedding_loss(input, label, margin, reduction=reduction)


def cosine_embedding_loss(input1, input2, label, margin=0, reduction="mean", name=None):
    return TF.cosine_embedding_loss(input1, input2, label, margin, reduction=reduction)


def ctc_loss(log_probs, labels, input_lengths, label_lengths, blank=0, reduction="mean", norm_by_times=False):
    return TF.ctc_loss(log_probs, labels, input_lengths, label_lengths, blank, reduction)


def sigmoid_focal_loss(logit, label, normalizer=None, alpha=0.25, gamma=2.0, reduction="sum", name=None):
    p = torch.sigmoid(logit)
    ce = TF.binary_cross_entropy_with_logits(logit, label, reduction="none")
    pt = p * label + (1 - p) * (1 - label)
    loss = ce * (1 - pt) ** gamma
    loss = (alpha * label + (1 - alpha) * (1 - label)) * loss
    if normalizer is not None:
        loss = loss / normalizer
    return _reduce(loss, reduction)


def triplet_margin_loss(input, positive, negative, margin=1.0, p=2, epsilon=1e-6, swap=False, reduction="mean", name=None):  # noqa: A002
    return TF.triplet_margin_loss(input, positive, negative, margin=margin, p=p, eps=epsilon, swap=swap, reduction=reduction)


def square_error_cost(input, label):  # noqa: A002
    return (input - label) ** 2


# ------------------------------------------------------------------------------- attention
def flash_attention(query, key, value, dropout=0.0, causal=False, return_softmax=False,
                    fixed_seed_offset=None, rng_name="", training=True, name=None):
    """Reference `nn/functional/flash_attention.py:142` — [B, S, H, D] layout. Returns
    ``(out, softmax)`` (softmax is None: never materialised). Attention dropout runs inside the
    MFMA kernel (counter-RNG mask regenerated in backward)."""
    return _ops.flash_attention(query, key, value, causal=causal, dropout_p=dropout,
                                training=training), None


def flash_attn_unpadded(query, key, value, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                        scale, dropout=0.0, causal=False, return_softmax=False, training=True, name=None):
    """Reference `flash_attention.py:flash_attn_unpadded`: packed [total_tokens, H, D] q/k/v with
    cumulative sequence offsets — one variable-length MFMA launch per pass (``flash_attn.hip``)."""
    return _ops.flash_attention_varlen(query, key, value, cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
                                       max_seqlen_k, causal=causal, scale=scale, dropout_p=dropout,
                                       training=training), None


def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0,
                                 is_causal=False, training=True, name=None):
    """Reference `flash_attention.py:440`: [B, S, H, D] layout; additive / bool ``attn_mask`` and
    attention dropout both run inside the MFMA flash kernel."""
    return _ops.flash_attention(query, key, value, causal=is_causal, attn_mask=attn_mask,
                                dropout_p=dropout_p, training=training)


def memory_efficient_attention(query, key, value, attn_bias=None, p=0.0, scale=None, training=True):
    """The fork's `memory_efficient_attention` (cutlass) API: [B, S, H, D]."""
    return _ops.flash_attention(query, key, value, scale=scale, attn_mask=attn_bias, dropout_p=p,
                                training=training)


def sequence_mask(x, maxlen=None, dtype="int64", name=None):
    maxlen = int(maxlen if maxlen is not None else x.max().item())
    return (torch.arange(maxlen, device=x.device) < x.unsqueeze(-1)).to(_dt(dtype))


def temporal_shift(x, seg_num, shift_ratio=0.25, name=None, data_format="NCHW"):
    nt, c, h, w = x.shape
    x = x.reshape(nt // seg_num, seg_num, c, h, w)
    fold = int(c * shift_ratio)
    out = torch.zeros_like(x)
    out[:, :-1, :fold] = x[:, 1:, :fold]
    out[:, 1:, fold:2 * fold] = x[:, :-1, fold:2 * fold]
    out[:, :, 2 * fold:] = x[:, :, 2 * fold:]
    return out.reshape(nt, c, h, w)


def affine_grid(theta, out_shape, align_corners=True, name=None):
    return TF.affine_grid(theta, list(out_shape), align_corners)


def grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=True, name=None):
    """Reference `nn/functional/vision.py:grid_sample`; 4-D GPU float inputs sample on the own
    kernels (ops/pool_nd.py: bilinear / nearest × zeros / border / reflection)."""
    if x.is_cuda:
        from ...ops import pool_nd
        if pool_nd.grid_sample_supported(x, grid, mode, padding_mode):
            return pool_nd.grid_sample(x, grid, mode, padding_mode, align_corners)
    _lib_fallback(x, "grid_sample", "5-D / bicubic (ATen)")
    return TF.grid_sample(x, grid, mode, padding_mode, align_corners)


math  # noqa


def _import_extra():
    from . import extra as _extra
    g = globals()
    for k, v in vars(_extra).items():
        if not k.startswith("_") and callable(v) and getattr(v, "__module__", "") == _extra.__name__ \
                and k not in g:
            g[k] = v


_import_extra()
