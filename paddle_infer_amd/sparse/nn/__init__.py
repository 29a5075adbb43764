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
    """BatchNorm over the channel (last) dim of the stored values of a sparse NDHWC tensor."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NDHWC", use_global_stats=None, name=None):
        super().__init__()
        self.bn = torch.nn.BatchNorm1d(num_features, eps=epsilon, momentum=1 - momentum)

    def forward(self, x):
        x = x.coalesce()
        self.bn.train(self.training)
        v = self.bn(x.values())
        return torch.sparse_coo_tensor(x.indices(), v, x.shape).coalesce()


SyncBatchNorm = BatchNorm


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
