"""Max pooling over channels-last 16-bit activations on the own HIP kernels (``csrc/kernels/pool.hip``):
forward stores the winning tap per element, backward gathers dY through it (no atomics,
deterministic). Parity: reference `phi/kernels/funcs/pooling.cu` (MaxPool2dWithIndex and its
gradient). Other layouts / dtypes / modes stay on ``torch.nn.functional.max_pool2d``."""
from __future__ import annotations

import torch

from . import _lib


def _pair(v):
    return (int(v), int(v)) if isinstance(v, int) else (int(v[0]), int(v[1]))


def max_pool2d_supported(x, kernel_size, stride, padding, ceil_mode=False, return_mask=False):
    if not (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16) and not ceil_mode
            and not return_mask and not isinstance(padding, str) and _lib.available()):
        return False
    if x.shape[1] % 8 or not x.is_contiguous(memory_format=torch.channels_last):
        return False
    kh, kw = _pair(kernel_size)
    ph, pw = _pair(padding)
    return kh * kw <= 255 and 2 * ph <= kh and 2 * pw <= kw


class _MaxPool2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        N, C, H, W = x.shape
        OH = (H + 2 * p[0] - k[0]) // s[0] + 1
        OW = (W + 2 * p[1] - k[1]) // s[1] + 1
        xh = x.permute(0, 2, 3, 1)  # NHWC storage of the channels-last tensor
        y = torch.empty(N, OH, OW, C, dtype=x.dtype, device=x.device)
        idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=x.device)
        _lib.call("piamd_maxpool_fwd_nhwc", xh.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, OH, OW,
                  k[0], k[1], s[0], s[1], p[0], p[1], int(x.dtype == torch.float16), _lib.stream())
        ctx.save_for_backward(idx)
        ctx.geo = (N, C, H, W, OH, OW, k, s, p, x.dtype)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W, OH, OW, k, s, p, dt = ctx.geo
        dyh = dy.permute(0, 2, 3, 1).contiguous().to(dt)
        dx = torch.empty(N, H, W, C, dtype=dt, device=dy.device)
        _lib.call("piamd_maxpool_bwd_nhwc", dyh.data_ptr(), idx.data_ptr(), dx.data_ptr(), N, H, W, C, OH, OW,
                  k[0], k[1], s[0], s[1], p[0], p[1], int(dt == torch.float16), _lib.stream())
        return dx.permute(0, 3, 1, 2), None, None, None


def max_pool2d_nhwc(x, kernel_size, stride=None, padding=0):
    """Max pool of a channels-last NCHW 16-bit tensor (see ``max_pool2d_supported``); returns a
    channels-last NCHW tensor."""
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    return _MaxPool2dNHWC.apply(x, k, s, _pair(padding))
