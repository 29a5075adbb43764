"""``paddle.nn`` layers (reference `python/paddle/nn/layer/{common,conv,norm,pooling,activation,
loss,transformer,rnn,container,distance,vision}.py`).

State-dict keys and parameter layouts follow Paddle (Linear weight ``[in, out]``; BatchNorm
``weight/bias/_mean/_variance``; MultiHeadAttention ``q_proj/k_proj/v_proj/out_proj``), so
``.pdparams`` produced by the reference load with ``set_state_dict``.
"""
from __future__ import annotations

import math

import torch

from .base import Layer, LayerList, Sequential, LayerDict, ParameterList, ParamAttr  # noqa: F401
from .. import functional as F
from .. import initializer as I


def _ntuple(v, n):
    return tuple(v) if isinstance(v, (list, tuple)) else (v,) * n


# ------------------------------------------------------------------------------- common
class Identity(Layer):
    def __init__(self, *args, **kwargs):
        super().__init__()

    def forward(self, x):
        return x


class Linear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = self.create_parameter([in_features, out_features], attr=weight_attr,
                                            default_initializer=I.XavierUniform())
        self.bias = self.create_parameter([out_features], attr=bias_attr, is_bias=True)

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}"


class Bilinear(Layer):
    def __init__(self, in1_features, in2_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self.weight = self.create_parameter([out_features, in1_features, in2_features], attr=weight_attr)
        self.bias = self.create_parameter([1, out_features], attr=bias_attr, is_bias=True)

    def forward(self, x1, x2):
        return torch.nn.functional.bilinear(x1, x2, self.weight, self.bias.reshape(-1) if self.bias is not None else None)


class Embedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, padding_idx=None, sparse=False,
                 weight_attr=None, name=None):
        super().__init__()
        self.padding_idx = None if padding_idx is None else (padding_idx if padding_idx >= 0 else num_embeddings + padding_idx)
        self.weight = self.create_parameter([num_embeddings, embedding_dim], attr=weight_attr,
                                            default_initializer=I.XavierNormal())
        if self.padding_idx is not None:
            with torch.no_grad():
                self.weight[self.padding_idx].zero_()

    def forward(self, x):
        return F.embedding(x, self.weight, self.padding_idx)


class Dropout(Layer):
    def __init__(self, p=0.5, axis=None, mode="upscale_in_train", name=None):
        super().__init__()
        self.p, self.axis, self.mode = p, axis, mode

    def forward(self, x):
        return F.dropout(x, self.p, self.axis, self.training, self.mode)


class Dropout2D(Layer):
    def __init__(self, p=0.5, data_format="NCHW", name=None):
        super().__init__()
        self.p = p

    def forward(self, x):
        return F.dropout2d(x, self.p, self.training)


class Dropout3D(Dropout2D):
    def forward(self, x):
        return F.dropout3d(x, self.p, self.training)


class AlphaDropout(Dropout2D):
    def forward(self, x):
        return F.alpha_dropout(x, self.p, self.training)


class Flatten(Layer):
    def __init__(self, start_axis=1, stop_axis=-1):
        super().__init__()
        self.start_axis, self.stop_axis = start_axis, stop_axis

    def forward(self, x):
        return torch.flatten(x, self.start_axis, self.stop_axis)


class Unflatten(Layer):
    def __init__(self, axis, shape, name=None):
        super().__init__()
        self.axis, self.shape = axis, shape

    def forward(self, x):
        return x.unflatten(self.axis, self.shape)


class Pad1D(Layer):
    def __init__(self, padding, mode="constant", value=0.0, data_format="NCL", name=None):
        super().__init__()
        self.padding = list(_ntuple(padding, 2))
        self.mode, self.value, self.data_format = mode, value, data_format

    def forward(self, x):
        return F.pad(x, self.padding, self.mode, self.value, self.data_format)


class Pad2D(Pad1D):
    def __init__(self, padding, mode="constant", value=0.0, data_format="NCHW", name=None):
        super().__init__(0, mode, value, data_format)
        self.padding = list(_ntuple(padding, 4))


class Pad3D(Pad1D):
    def __init__(self, padding, mode="constant", value=0.0, data_format="NCDHW", name=None):
        super().__init__(0, mode, value, data_format)
        self.padding = list(_ntuple(padding, 6))


class Upsample(Layer):
    def __init__(self, size=None, scale_factor=None, mode="nearest", align_corners=False,
                 align_mode=0, data_format="NCHW", name=None):
        super().__init__()
        self.size, self.scale_factor, self.mode, self.align_corners = size, scale_factor, mode, align_corners
        self.align_mode, self.data_format = align_mode, data_format

    def forward(self, x):
        return F.interpolate(x, self.size, self.scale_factor, self.mode, self.align_corners, self.align_mode,
                             self.data_format)


class UpsamplingBilinear2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format="NCHW", name=None):
        super().__init__(size, scale_factor, "bilinear", True, data_format=data_format)


class UpsamplingNearest2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format="NCHW", name=None):
        super().__init__(size, scale_factor, "nearest", data_format=data_format)


class PixelShuffle(Layer):
    def __init__(self, upscale_factor, data_format="NCHW", name=None):
        super().__init__()
        self.r = upscale_factor

    def forward(self, x):
        return F.pixel_shuffle(x, self.r)


class CosineSimilarity(Layer):
    def __init__(self, axis=1, eps=1e-8):
        super().__init__()
        self.axis, self.eps = axis, eps

    def forward(self, x1, x2):
        return F.cosine_similarity(x1, x2, self.axis, self.eps)


class PairwiseDistance(Layer):
    def __init__(self, p=2.0, epsilon=1e-6, keepdim=False, name=None):
        super().__init__()
        self.p, self.eps, self.keepdim = p, epsilon, keepdim

    def forward(self, x, y):
        return torch.nn.functional.pairwise_distance(x, y, self.p, self.eps, self.keepdim)


# ------------------------------------------------------------------------------- activations
def _act_layer(name, fn, **defaults):
    def __init__(self, *args, name=None, **kw):
        Layer.__init__(self)
        params = dict(defaults)
        for k, v in zip(list(defaults), args):
            params[k] = v
        params.update({k: v for k, v in kw.items() if k in defaults})
        self._kw = params

    def forward(self, x):
        return fn(x, **self._kw)
    return type(name, (Layer,), {"__init__": __init__, "forward": forward})


ReLU = _act_layer("ReLU", F.relu)
ReLU6 = _act_layer("ReLU6", F.relu6)
GELU = _act_layer("GELU", F.gelu, approximate=False)
Silu = _act_layer("Silu", F.silu)
Swish = _act_layer("Swish", F.swish)
Sigmoid = _act_layer("Sigmoid", F.sigmoid)
Tanh = _act_layer("Tanh", F.tanh)
ELU = _act_layer("ELU", F.elu, alpha=1.0)
SELU = _act_layer("SELU", F.selu)
CELU = _act_layer("CELU", F.celu, alpha=1.0)
LeakyReLU = _act_layer("LeakyReLU", F.leaky_relu, negative_slope=0.01)
Hardswish = _act_layer("Hardswish", F.hardswish)
Hardsigmoid = _act_layer("Hardsigmoid", F.hardsigmoid)
Hardtanh = _act_layer("Hardtanh", F.hardtanh, min=-1.0, max=1.0)
Hardshrink = _act_layer("Hardshrink", F.hardshrink, threshold=0.5)
Softshrink = _act_layer("Softshrink", F.softshrink, threshold=0.5)
Tanhshrink = _act_layer("Tanhshrink", F.tanhshrink)
Softplus = _act_layer("Softplus", F.softplus, beta=1, threshold=20)
Softsign = _act_layer("Softsign", F.softsign)
Mish = _act_layer("Mish", F.mish)
LogSigmoid = _act_layer("LogSigmoid", F.log_sigmoid)
ThresholdedReLU = _act_layer("ThresholdedReLU", F.thresholded_relu, threshold=1.0)
Softmax = _act_layer("Softmax", F.softmax, axis=-1)
LogSoftmax = _act_layer("LogSoftmax", F.log_softmax, axis=-1)
GLU = _act_layer("GLU", F.glu, axis=-1)


class PReLU(Layer):
    def __init__(self, num_parameters=1, init=0.25, weight_attr=None, data_format="NCHW", name=None):
        super().__init__()
        self.weight = self.create_parameter([num_parameters], attr=weight_attr,
                                            default_initializer=I.Constant(init))

    def forward(self, x):
        return torch.nn.functional.prelu(x, self.weight)


class Maxout(Layer):
    def __init__(self, groups, axis=1, name=None):
        super().__init__()
        self.groups, self.axis = groups, axis

    def forward(self, x):
        return F.maxout(x, self.groups, self.axis)


# ------------------------------------------------------------------------------- conv
class _ConvNd(Layer):
    _nd = 2
    _transpose = False

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, padding_mode="zeros", weight_attr=None, bias_attr=None,
                 data_format=None, output_padding=0):
        super().__init__()
        nd = self._nd
        self.kernel_size = _ntuple(kernel_size, nd)
        self.stride, self.padding, self.dilation, self.groups = stride, padding, dilation, groups
        self.output_padding = output_padding
        self.data_format = data_format or {1: "NCL", 2: "NCHW", 3: "NCDHW"}[nd]
        self.padding_mode = padding_mode
        if self._transpose:
            shape = [in_channels, out_channels // groups, *self.kernel_size]
        else:
            shape = [out_channels, in_channels // groups, *self.kernel_size]
        fan_in = (in_channels // groups) * int(math.prod(self.kernel_size))
        self.weight = self.create_parameter(shape, attr=weight_attr,
                                            default_initializer=I.Normal(0.0, (2.0 / fan_in) ** 0.5))
        self.bias = self.create_parameter([out_channels], attr=bias_attr, is_bias=True)

    def _pad_input(self, x):
        if self.padding_mode == "zeros" or isinstance(self.padding, str):
            return x, self.padding
        p = _ntuple(self.padding, self._nd)
        pads = []
        for v in reversed(p):
            pads += [v, v]
        mode = {"reflect": "reflect", "replicate": "replicate", "circular": "circular"}[self.padding_mode]
        return torch.nn.functional.pad(x, pads, mode), 0


class Conv1D(_ConvNd):
    _nd = 1

    def forward(self, x):
        x, pad = self._pad_input(x)
        return F.conv1d(x, self.weight, self.bias, self.stride, pad, self.dilation, self.groups, self.data_format)


class Conv2D(_ConvNd):
    _nd = 2

    def forward(self, x):
        x, pad = self._pad_input(x)
        return F.conv2d(x, self.weight, self.bias, self.stride, pad, self.dilation, self.groups, self.data_format)


class Conv3D(_ConvNd):
    _nd = 3

    def forward(self, x):
        x, pad = self._pad_input(x)
        return F.conv3d(x, self.weight, self.bias, self.stride, pad, self.dilation, self.groups, self.data_format)


class Conv2DTranspose(_ConvNd):
    _nd = 2
    _transpose = True

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0,
                 groups=1, dilation=1, weight_attr=None, bias_attr=None, data_format="NCHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups,
                         "zeros", weight_attr, bias_attr, data_format, output_padding)

    def forward(self, x, output_size=None):
        return F.conv2d_transpose(x, self.weight, self.bias, self.stride, self.padding,
                                  self.output_padding, self.groups, self.dilation, self.data_format)


class Conv1DTranspose(Conv2DTranspose):
    _nd = 1

    def forward(self, x, output_size=None):
        return F.conv1d_transpose(x, self.weight, self.bias, self.stride, self.padding,
                                  self.output_padding, self.groups, self.dilation)


# ------------------------------------------------------------------------------- pooling
class _Pool(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, **kw):
        super().__init__()
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding
        self.kw = kw


class MaxPool1D(_Pool):
    def forward(self, x):
        return F.max_pool1d(x, self.kernel_size, self.stride, self.padding, **self.kw)


class MaxPool2D(_Pool):
    def forward(self, x):
        return F.max_pool2d(x, self.kernel_size, self.stride, self.padding, **self.kw)


class MaxPool3D(_Pool):
    def forward(self, x):
        return F.max_pool3d(x, self.kernel_size, self.stride, self.padding, **self.kw)


class AvgPool1D(_Pool):
    def forward(self, x):
        return F.avg_pool1d(x, self.kernel_size, self.stride, self.padding, **self.kw)


class AvgPool2D(_Pool):
    def forward(self, x):
        return F.avg_pool2d(x, self.kernel_size, self.stride, self.padding, **self.kw)


class AvgPool3D(_Pool):
    def forward(self, x):
        return F.avg_pool3d(x, self.kernel_size, self.stride, self.padding, **self.kw)


class AdaptiveAvgPool1D(Layer):
    def __init__(self, output_size, name=None):
        super().__init__()
        self.output_size = output_size

    def forward(self, x):
        return F.adaptive_avg_pool1d(x, self.output_size)


class AdaptiveAvgPool2D(AdaptiveAvgPool1D):
    def __init__(self, output_size, data_format="NCHW", name=None):
        super().__init__(output_size)
        self.data_format = data_format

    def forward(self, x):
        return F.adaptive_avg_pool2d(x, self.output_size, self.data_format)


class AdaptiveAvgPool3D(AdaptiveAvgPool1D):
    def forward(self, x):
        return F.adaptive_avg_pool3d(x, self.output_size)


class AdaptiveMaxPool1D(AdaptiveAvgPool1D):
    def forward(self, x):
        return F.adaptive_max_pool1d(x, self.output_size)


class AdaptiveMaxPool2D(AdaptiveAvgPool1D):
    def forward(self, x):
        return F.adaptive_max_pool2d(x, self.output_size)


# ------------------------------------------------------------------------------- normalization
class LayerNorm(Layer):
    def __init__(self, normalized_shape, epsilon=1e-5, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self.normalized_shape = [normalized_shape] if isinstance(normalized_shape, int) else list(normalized_shape)
        self.epsilon = epsilon
        self.weight = self.create_parameter(self.normalized_shape, attr=weight_attr,
                                            default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter(self.normalized_shape, attr=bias_attr, is_bias=True)

    def forward(self, x):
        return F.layer_norm(x, self.normalized_shape, self.weight, self.bias, self.epsilon)


class RMSNorm(Layer):
    def __init__(self, hidden_size, epsilon=1e-6, weight_attr=None, name=None):
        super().__init__()
        self.epsilon = epsilon
        self.weight = self.create_parameter([hidden_size], attr=weight_attr, default_initializer=I.Constant(1.0))

    def forward(self, x):
        return F.rms_norm(x, self.weight, self.epsilon)


class _BatchNormBase(Layer):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCHW", use_global_stats=None, name=None):
        super().__init__()
        self.momentum, self.epsilon = momentum, epsilon
        self.data_format = data_format
        self.use_global_stats = use_global_stats
        self.weight = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)
        self.register_buffer("_mean", torch.zeros(num_features))
        self.register_buffer("_variance", torch.ones(num_features))

    def forward(self, x, residual=None, act=None):
        """``act(BN(x) + residual)``; ``residual`` / ``act`` (relu, relu6) fuse the ResNet-style
        tail into the normalisation pass on the GPU."""
        train = self.training and not self.use_global_stats
        return F.batch_norm(x, self._mean, self._variance, self.weight, self.bias, train,
                            self.momentum, self.epsilon, self.data_format, act=act,
                            residual=residual)


class BatchNorm1D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCL", use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr,
                         "NLC" if data_format == "NLC" else "NCHW", use_global_stats)


class BatchNorm2D(_BatchNormBase):
    pass


class BatchNorm3D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCDHW", use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr,
                         "NDHWC" if data_format == "NDHWC" else "NCHW", use_global_stats)


class BatchNorm(_BatchNormBase):
    def __init__(self, num_channels, act=None, is_test=False, momentum=0.9, epsilon=1e-5,
                 param_attr=None, bias_attr=None, dtype="float32", data_layout="NCHW", **kw):
        super().__init__(num_channels, momentum, epsilon, param_attr, bias_attr, data_layout)
        self.act = act

    def forward(self, x):
        if self.act in (None, "relu", "relu6"):
            return super().forward(x, act=self.act)
        return getattr(F, self.act)(super().forward(x))


class SyncBatchNorm(_BatchNormBase):
    """Batch norm whose batch statistics cover every rank of the data-parallel group (reference
    `nn/layer/norm.py` SyncBatchNorm → `phi/kernels/gpu/sync_batch_norm_kernel.cu`): the
    framework's Welford statistics kernels (`batchnorm.hip` piamd_bn_local_stats), an all-gather of
    the per-rank (count, mean, M2) triples over RCCL, the cross-rank Welford merge inside the
    normalise launch, and an all-reduce of the backward sums (`ops.batchnorm.sync_batch_norm`)."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None, group=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format)
        self.group = group

    def forward(self, x):
        import torch.distributed as dist
        if not (self.training and dist.is_initialized() and dist.get_world_size(self.group) > 1):
            return super().forward(x)
        from ...ops.batchnorm import sync_batch_norm
        return sync_batch_norm(x, self._mean, self._variance, self.weight, self.bias, True,
                               self.momentum, self.epsilon, self.group, self.data_format)

    @classmethod
    def convert_sync_batchnorm(cls, layer):
        for name, m in list(layer.named_children()):
            if isinstance(m, _BatchNormBase) and not isinstance(m, SyncBatchNorm):
                new = cls(m.weight.shape[0], m.momentum, m.epsilon,
                          data_format=getattr(m, "data_format", "NCHW"))
                new.load_state_dict(m.state_dict())
                setattr(layer, name, new)
            else:
                cls.convert_sync_batchnorm(m)
        return layer


class _AllReduceSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        import torch.distributed as dist
        y = x.clone()
        dist.all_reduce(y)
        return y

    @staticmethod
    def backward(ctx, g):
        import torch.distributed as dist
        g = g.clone()
        dist.all_reduce(g)
        return g


class GroupNorm(Layer):
    def __init__(self, num_groups, num_channels, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None):
        super().__init__()
        self.num_groups, self.epsilon, self.data_format = num_groups, epsilon, data_format
        self.weight = self.create_parameter([num_channels], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([num_channels], attr=bias_attr, is_bias=True)

    def forward(self, x):
        return F.group_norm(x, self.num_groups, self.epsilon, self.weight, self.bias, self.data_format)


class InstanceNorm2D(Layer):
    def __init__(self, num_features, epsilon=1e-5, momentum=0.9, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None):
        super().__init__()
        self.epsilon = epsilon
        self.scale = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)

    def forward(self, x):
        return F.instance_norm(x, weight=self.scale, bias=self.bias, eps=self.epsilon)


InstanceNorm1D = InstanceNorm3D = InstanceNorm2D


class LocalResponseNorm(Layer):
    def __init__(self, size, alpha=1e-4, beta=0.75, k=1.0, data_format="NCHW", name=None):
        super().__init__()
        self.args = (size, alpha, beta, k)

    def forward(self, x):
        return F.local_response_norm(x, *self.args)


# ------------------------------------------------------------------------------- losses
class CrossEntropyLoss(Layer):
    def __init__(self, weight=None, ignore_index=-100, reduction="mean", soft_label=False,
                 axis=-1, use_softmax=True, label_smoothing=0.0, name=None):
        super().__init__()
        self.kw = dict(weight=weight, ignore_index=ignore_index, reduction=reduction,
                       soft_label=soft_label, axis=axis, use_softmax=use_softmax,
                       label_smoothing=label_smoothing)

    def forward(self, input, label):  # noqa: A002
        return F.cross_entropy(input, label, **self.kw)


def _loss_layer(name, fn, *names, **defaults):
    def __init__(self, *args, name=None, **kw):
        Layer.__init__(self)
        p = dict(defaults)
        for k, v in zip(list(defaults), args):
            p[k] = v
        p.update({k: v for k, v in kw.items() if k in defaults})
        self._kw = p

    def forward(self, *inputs):
        return fn(*inputs, **self._kw)
    return type(name, (Layer,), {"__init__": __init__, "forward": forward})


MSELoss = _loss_layer("MSELoss", F.mse_loss, reduction="mean")
L1Loss = _loss_layer("L1Loss", F.l1_loss, reduction="mean")
SmoothL1Loss = _loss_layer("SmoothL1Loss", F.smooth_l1_loss, reduction="mean", delta=1.0)
BCELoss = _loss_layer("BCELoss", F.binary_cross_entropy, weight=None, reduction="mean")
BCEWithLogitsLoss = _loss_layer("BCEWithLogitsLoss", F.binary_cross_entropy_with_logits, weight=None,
                                reduction="mean", pos_weight=None)
NLLLoss = _loss_layer("NLLLoss", F.nll_loss, weight=None, ignore_index=-100, reduction="mean")
KLDivLoss = _loss_layer("KLDivLoss", F.kl_div, reduction="mean")
MarginRankingLoss = _loss_layer("MarginRankingLoss", F.margin_ranking_loss, margin=0.0, reduction="mean")
HingeEmbeddingLoss = _loss_layer("HingeEmbeddingLoss", F.hinge_embedding_loss, margin=1.0, reduction="mean")
CosineEmbeddingLoss = _loss_layer("CosineEmbeddingLoss", F.cosine_embedding_loss, margin=0, reduction="mean")
TripletMarginLoss = _loss_layer("TripletMarginLoss", F.triplet_margin_loss, margin=1.0, p=2, epsilon=1e-6,
                                swap=False, reduction="mean")
CTCLoss = _loss_layer("CTCLoss", F.ctc_loss, blank=0, reduction="mean")


# ------------------------------------------------------------------------------- transformer
class MultiHeadAttention(Layer):
    """Reference `nn/layer/transformer.py:MultiHeadAttention` ([B, S, E] inputs)."""

    def __init__(self, embed_dim, num_heads, dropout=0.0, kdim=None, vdim=None, need_weights=False,
                 weight_attr=None, bias_attr=None):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.dropout = dropout
        self.need_weights = need_weights
        self.q_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)
        self.k_proj = Linear(kdim or embed_dim, embed_dim, weight_attr, bias_attr)
        self.v_proj = Linear(vdim or embed_dim, embed_dim, weight_attr, bias_attr)
        self.out_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        key = query if key is None else key
        value = query if value is None else value
        B, Sq, _ = query.shape
        q = self.q_proj(query).reshape(B, Sq, self.num_heads, self.head_dim)
        k = self.k_proj(key).reshape(B, key.shape[1], self.num_heads, self.head_dim)
        v = self.v_proj(value).reshape(B, value.shape[1], self.num_heads, self.head_dim)
        if cache is not None and isinstance(cache, tuple) and len(cache) == 2:
            k = torch.cat([cache[0], k], 1)
            v = torch.cat([cache[1], v], 1)
            cache = (k, v)
        if attn_mask is not None and attn_mask.dtype == torch.bool:
            attn_mask = torch.zeros(attn_mask.shape, dtype=q.dtype, device=q.device).masked_fill(~attn_mask, float("-inf"))
        if self.need_weights:
            qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
            s = qt @ kt.transpose(-1, -2) / math.sqrt(self.head_dim)
            if attn_mask is not None:
                s = s + attn_mask
            w = torch.softmax(s.float(), -1).to(q.dtype)
            w = F.dropout(w, self.dropout, training=self.training)
            o = (w @ vt).transpose(1, 2)
        else:
            o = F.scaled_dot_product_attention(q, k, v, attn_mask, self.dropout, training=self.training)
            w = None
        out = self.out_proj(o.reshape(B, Sq, self.embed_dim))
        outs = [out]
        if self.need_weights:
            outs.append(w)
        if cache is not None:
            outs.append(cache)
        return out if len(outs) == 1 else tuple(outs)


class TransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu",
                 attn_dropout=None, act_dropout=None, normalize_before=False, weight_attr=None,
                 bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        self.normalize_before = normalize_before
        self.self_attn = MultiHeadAttention(d_model, nhead, dropout if attn_dropout is None else attn_dropout)
        self.linear1 = Linear(d_model, dim_feedforward, weight_attr, bias_attr)
        self.dropout = Dropout(dropout if act_dropout is None else act_dropout)
        self.linear2 = Linear(dim_feedforward, d_model, weight_attr, bias_attr)
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout)
        self.dropout2 = Dropout(dropout)
        self.activation = getattr(F, activation)

    def forward(self, src, src_mask=None, cache=None):
        residual = src
        if self.normalize_before:
            src = self.norm1(src)
        src = residual + self.dropout1(self.self_attn(src, src, src, src_mask))
        if not self.normalize_before:
            src = self.norm1(src)
        residual = src
        if self.normalize_before:
            src = self.norm2(src)
        src = self.linear2(self.dropout(self.activation(self.linear1(src))))
        src = residual + self.dropout2(src)
        if not self.normalize_before:
            src = self.norm2(src)
        return src


class TransformerEncoder(Layer):
    def __init__(self, encoder_layer, num_layers, norm=None):
        super().__init__()
        import copy
        self.layers = LayerList([encoder_layer if i == 0 else copy.deepcopy(encoder_layer) for i in range(num_layers)])
        self.norm = norm

    def forward(self, src, src_mask=None, cache=None):
        for layer in self.layers:
            src = layer(src, src_mask)
        return self.norm(src) if self.norm is not None else src


class TransformerDecoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu",
                 attn_dropout=None, act_dropout=None, normalize_before=False, weight_attr=None,
                 bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        self.normalize_before = normalize_before
        ad = dropout if attn_dropout is None else attn_dropout
        self.self_attn = MultiHeadAttention(d_model, nhead, ad)
        self.cross_attn = MultiHeadAttention(d_model, nhead, ad)
        self.linear1 = Linear(d_model, dim_feedforward, weight_attr, bias_attr)
        self.dropout = Dropout(dropout if act_dropout is None else act_dropout)
        self.linear2 = Linear(dim_feedforward, d_model, weight_attr, bias_attr)
        self.norm1, self.norm2, self.norm3 = (LayerNorm(d_model, layer_norm_eps) for _ in range(3))
        self.dropout1, self.dropout2, self.dropout3 = (Dropout(dropout) for _ in range(3))
        self.activation = getattr(F, activation)

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        r = tgt
        if self.normalize_before:
            tgt = self.norm1(tgt)
        tgt = r + self.dropout1(self.self_attn(tgt, tgt, tgt, tgt_mask))
        if not self.normalize_before:
            tgt = self.norm1(tgt)
        r = tgt
        if self.normalize_before:
            tgt = self.norm2(tgt)
        tgt = r + self.dropout2(self.cross_attn(tgt, memory, memory, memory_mask))
        if not self.normalize_before:
            tgt = self.norm2(tgt)
        r = tgt
        if self.normalize_before:
            tgt = self.norm3(tgt)
        tgt = r + self.dropout3(self.linear2(self.dropout(self.activation(self.linear1(tgt)))))
        if not self.normalize_before:
            tgt = self.norm3(tgt)
        return tgt


class TransformerDecoder(Layer):
    def __init__(self, decoder_layer, num_layers, norm=None):
        super().__init__()
        import copy
        self.layers = LayerList([decoder_layer if i == 0 else copy.deepcopy(decoder_layer) for i in range(num_layers)])
        self.norm = norm

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        for layer in self.layers:
            tgt = layer(tgt, memory, tgt_mask, memory_mask)
        return self.norm(tgt) if self.norm is not None else tgt


class Transformer(Layer):
    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6,
                 dim_feedforward=2048, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None,
                 custom_encoder=None, custom_decoder=None):
        super().__init__()
        self.encoder = custom_encoder or TransformerEncoder(
            TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout,
                                    act_dropout, normalize_before), num_encoder_layers,
            LayerNorm(d_model) if normalize_before else None)
        self.decoder = custom_decoder or TransformerDecoder(
            TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout,
                                    act_dropout, normalize_before), num_decoder_layers,
            LayerNorm(d_model) if normalize_before else None)

    def forward(self, src, tgt, src_mask=None, tgt_mask=None, memory_mask=None):
        mem = self.encoder(src, src_mask)
        return self.decoder(tgt, mem, tgt_mask, memory_mask)

    @staticmethod
    def generate_square_subsequent_mask(length):
        return torch.triu(torch.full((length, length), float("-inf")), 1)


# ------------------------------------------------------------------------------- RNN
# ------------------------------------------------------------------------------- misc layers
class Conv3DTranspose(_ConvNd):
    _nd = 3
    _transpose = True

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0,
                 groups=1, dilation=1, weight_attr=None, bias_attr=None, data_format="NCDHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups,
                         "zeros", weight_attr, bias_attr, data_format, output_padding)

    def forward(self, x, output_size=None):
        return F.conv3d_transpose(x, self.weight, self.bias, self.stride, self.padding,
                                  self.output_padding, self.groups, self.dilation, self.data_format)


class AdaptiveMaxPool3D(AdaptiveAvgPool1D):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(output_size)
        self.return_mask = return_mask

    def forward(self, x):
        return F.adaptive_max_pool3d(x, self.output_size, self.return_mask)


class _MaxUnPool(Layer):
    _fn = None

    def __init__(self, kernel_size, stride=None, padding=0, data_format=None, output_size=None, name=None):
        super().__init__()
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding
        self.output_size = output_size

    def forward(self, x, indices):
        return type(self)._fn(x, indices, self.kernel_size, self.stride, self.padding,
                              output_size=self.output_size)


class MaxUnPool1D(_MaxUnPool):
    _fn = staticmethod(F.max_unpool1d)


class MaxUnPool2D(_MaxUnPool):
    _fn = staticmethod(F.max_unpool2d)


class MaxUnPool3D(_MaxUnPool):
    _fn = staticmethod(F.max_unpool3d)


class Unfold(Layer):
    def __init__(self, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.args = (kernel_sizes, strides, paddings, dilations)

    def forward(self, x):
        k, s, p, d = self.args
        return F.unfold(x, k, s, p, d)


class Fold(Layer):
    def __init__(self, output_sizes, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.args = (output_sizes, kernel_sizes, strides, paddings, dilations)

    def forward(self, x):
        return F.fold(x, *self.args)


class Softmax2D(Layer):
    """Softmax over the channel axis of [N, C, H, W] / [C, H, W] input."""

    def forward(self, x):
        if x.dim() not in (3, 4):
            raise ValueError(f"Softmax2D expects 3-D or 4-D input, got {x.dim()}-D")
        return torch.softmax(x, -3)


class PixelUnshuffle(Layer):
    def __init__(self, downscale_factor, data_format="NCHW", name=None):
        super().__init__()
        self.r, self.data_format = downscale_factor, data_format

    def forward(self, x):
        return F.pixel_unshuffle(x, self.r, self.data_format)


class ChannelShuffle(Layer):
    def __init__(self, groups, data_format="NCHW", name=None):
        super().__init__()
        self.groups, self.data_format = groups, data_format

    def forward(self, x):
        return F.channel_shuffle(x, self.groups, self.data_format)


class ZeroPad2D(Layer):
    def __init__(self, padding, data_format="NCHW", name=None):
        super().__init__()
        self.padding, self.data_format = padding, data_format

    def forward(self, x):
        return F.zeropad2d(x, self.padding, self.data_format)


class RReLU(Layer):
    def __init__(self, lower=1.0 / 8.0, upper=1.0 / 3.0, name=None):
        super().__init__()
        self.lower, self.upper = lower, upper

    def forward(self, x):
        return F.rrelu(x, self.lower, self.upper, self.training)


class SpectralNorm(Layer):
    """Reference `nn/layer/norm.py:SpectralNorm`: returns weight / σ(weight), σ estimated with
    ``power_iters`` power-iteration steps on persistent u, v buffers (weight reshaped to
    [shape[dim], -1])."""

    def __init__(self, weight_shape, dim=0, power_iters=1, epsilon=1e-12, dtype="float32"):
        super().__init__()
        self.dim, self.power_iters, self.eps = dim, power_iters, epsilon
        h = weight_shape[dim]
        w = int(math.prod(weight_shape)) // h
        self.register_buffer("weight_u", torch.nn.functional.normalize(torch.randn(h), dim=0, eps=epsilon))
        self.register_buffer("weight_v", torch.nn.functional.normalize(torch.randn(w), dim=0, eps=epsilon))

    def forward(self, weight):
        perm = [self.dim] + [i for i in range(weight.dim()) if i != self.dim]
        mat = weight.permute(perm).reshape(weight.shape[self.dim], -1)
        u, v = self.weight_u, self.weight_v
        with torch.no_grad():
            for _ in range(self.power_iters):
                v = torch.nn.functional.normalize(mat.t() @ u, dim=0, eps=self.eps)
                u = torch.nn.functional.normalize(mat @ v, dim=0, eps=self.eps)
            self.weight_u.copy_(u)
            self.weight_v.copy_(v)
        sigma = torch.dot(u, mat @ v)
        return weight / sigma


class HSigmoidLoss(Layer):
    """Hierarchical sigmoid head (reference `nn/layer/loss.py:HSigmoidLoss`): weight
    [num_classes - 1, feature_size], bias [num_classes - 1, 1]."""

    def __init__(self, feature_size, num_classes, weight_attr=None, bias_attr=None, is_custom=False,
                 is_sparse=False, name=None):
        super().__init__()
        if num_classes < 2 and not is_custom:
            raise ValueError("num_classes must be >= 2 with the default tree")
        self.num_classes = num_classes
        self.weight = self.create_parameter([num_classes - 1, feature_size], attr=weight_attr)
        self.bias = self.create_parameter([num_classes - 1, 1], attr=bias_attr, is_bias=True)

    def forward(self, input, label, path_table=None, path_code=None):  # noqa: A002
        return F.hsigmoid_loss(input, label, self.num_classes, self.weight, self.bias,
                               path_table, path_code)


SoftMarginLoss = _loss_layer("SoftMarginLoss", F.soft_margin_loss, reduction="mean")
MultiLabelSoftMarginLoss = _loss_layer("MultiLabelSoftMarginLoss", F.multi_label_soft_margin_loss,
                                       weight=None, reduction="mean")
TripletMarginWithDistanceLoss = _loss_layer(
    "TripletMarginWithDistanceLoss", F.triplet_margin_with_distance_loss, distance_function=None,
    margin=1.0, swap=False, reduction="mean")


from .rnn import (RNNCellBase, SimpleRNNCell, LSTMCell, GRUCell, RNN, BiRNN, SimpleRNN, LSTM,  # noqa: E402,F401
                  GRU, BeamSearchDecoder, dynamic_decode)
