"""``paddle.sparse.nn`` (reference `python/paddle/sparse/nn/`): activations over stored values,
sparse softmax (per row over the stored entries), BatchNorm over the values of a sparse
``[N, D, H, W, C]`` tensor, and 3-D (submanifold) convolution / max pooling / mask attention on
the active sites only (`conv.py`: rulebook + gather → grouped MFMA GEMM → scatter)."""
from __future__ import annotations

import torch

from ...nn.layer.base import Layer


class functional:  # noqa: N801
    @staticmethod
    def relu(x, name=None):
        from .. import relu
        return relu(x)

    @staticmethod
    def relu6(x, name=None):
        from .. import _unary
        return _unary(lambda v: v.clamp(0, 6))(x)

    @staticmethod
    def leaky_relu(x, negative_slope=0.01, name=None):
        from .. import _unary
        return _unary(lambda v: torch.nn.functional.leaky_relu(v, negative_slope))(x)

    @staticmethod
    def softmax(x, axis=-1, name=None):
        return torch.sparse.softmax(x.to_sparse_coo() if x.layout == torch.sparse_csr else x, axis) \
            if x.layout == torch.sparse_csr else torch.sparse.softmax(x.coalesce(), axis)

    @staticmethod
    def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC",
               name=None, subm=False):
        """Sparse conv on the active sites: rulebook + gather → grouped MFMA GEMM → scatter
        (`sparse/nn/conv.py`)."""
        from .conv import conv3d
        return conv3d(x, weight, bias, stride, padding, dilation, groups, data_format, subm=subm)

    @staticmethod
    def subm_conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
                    data_format="NDHWC", key=None, name=None):
        return functional.conv3d(x, weight, bias, stride, padding, dilation, groups, data_format,
                                 subm=True)

    @staticmethod
    def max_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NDHWC",
                   name=None):
        from .conv import max_pool3d
        return max_pool3d(x, kernel_size, stride, padding, ceil_mode, data_format)

    @staticmethod
    def attention(query, key, value, sparse_mask, key_padding_mask=None, attn_mask=None, name=None):
        """Scores only at ``sparse_mask`` (CSR [B*H, S, S]) entries: SDDMM → segment softmax → SpMM."""
        from .conv import mask_attention
        return mask_attention(query, key, value, sparse_mask, key_padding_mask, attn_mask)


class ReLU(Layer):
    def forward(self, x):
        return functional.relu(x)


class ReLU6(Layer):
    def forward(self, x):
        return functional.relu6(x)


class LeakyReLU(Layer):
    def __init__(self, negative_slope=0.01, name=None):
        super().__init__()
        self.negative_slope = negative_slope

    def forward(self, x):
        return functional.leaky_relu(x, self.negative_slope)


class Softmax(Layer):
    def __init__(self, axis=-1, name=None):
        super().__init__()
        self.axis = axis

    def forward(self, x):
        return functional.softmax(x, self.axis)


class BatchNorm(Layer):
    """BatchNorm over the channel (last) dim of the stored values of a sparse NDHWC tensor
    (reference `phi/kernels/sparse/gpu/batch_norm_kernel.cu`: dense batch norm on the non-zero
    feature rows): the values [nnz, C] run the framework's channels-last BN kernels
    (`ops.batchnorm.batch_norm_act`, Paddle momentum convention)."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NDHWC", use_global_stats=None, name=None):
        super().__init__()
        from ...nn import initializer as I
        self.momentum, self.epsilon = momentum, epsilon
        self.use_global_stats = use_global_stats
        self.weight = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)
        self.register_buffer("_mean", torch.zeros(num_features))
        self.register_buffer("_variance", torch.ones(num_features))

    def _values_bn(self, v):
        from ...ops.batchnorm import batch_norm_act
        train = self.training and not self.use_global_stats
        return batch_norm_act(v, self._mean, self._variance, self.weight, self.bias, train, self.momentum,
                              self.epsilon, data_format="NHWC")

    def forward(self, x):
        x = x.coalesce()
        v = self._values_bn(x.values())
        return torch.sparse_coo_tensor(x.indices(), v, x.shape).coalesce()


class SyncBatchNorm(BatchNorm):
    """Sparse BatchNorm with statistics over every rank (reference
    `phi/kernels/sparse/gpu/sync_batch_norm_kernel.cu`): the values' Welford triples all-gathered
    and merged, backward sums all-reduced (`ops.batchnorm.sync_batch_norm`)."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NDHWC", name=None, group=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format)
        self.group = group

    def _values_bn(self, v):
        import torch.distributed as dist
        if not (self.training and dist.is_initialized() and dist.get_world_size(self.group) > 1):
            return super()._values_bn(v)
        from ...ops.batchnorm import sync_batch_norm
        return sync_batch_norm(v, self._mean, self._variance, self.weight, self.bias, True, self.momentum,
                               self.epsilon, self.group, data_format="NHWC")

    @classmethod
    def convert_sync_batchnorm(cls, layer):
        for name, m in list(layer.named_children()):
            if type(m) is BatchNorm:
                new = cls(m.weight.shape[0], m.momentum, m.epsilon)
                new.load_state_dict(m.state_dict())
                setattr(layer, name, new)
            else:
                cls.convert_sync_batchnorm(m)
        return layer


class Conv3D(Layer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, padding_mode="zeros", weight_attr=None, bias_attr=None,
                 data_format="NDHWC", subm=False):
        super().__init__()
        k = (kernel_size,) * 3 if isinstance(kernel_size, int) else tuple(kernel_size)
        self.weight = self.create_parameter(list(k) + [in_channels // groups, out_channels])
        self.bias = self.create_parameter([out_channels], is_bias=True) if bias_attr is not False else None
        self.stride, self.padding, self.dilation, self.groups, self.subm = stride, padding, dilation, groups, subm

    def forward(self, x):
        return functional.conv3d(x, self.weight, self.bias, self.stride, self.padding, self.dilation,
                                 self.groups, subm=self.subm)


class SubmConv3D(Conv3D):
    def __init__(self, *a, **kw):
        kw.pop("key", None)
        super().__init__(*a, subm=True, **kw)


class MaxPool3D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False, return_mask=False,
                 data_format="NDHWC", name=None):
        super().__init__()
        self.k, self.s, self.p, self.c = kernel_size, stride, padding, ceil_mode

    def forward(self, x):
        return functional.max_pool3d(x, self.k, self.s, self.p, self.c)
