"""Pooling (max / avg, fixed or adaptive windows, 1-D/2-D/3-D) and linear / nearest resampling on
the own HIP kernels (``csrc/kernels/pool_nd.hip``), forward and backward, f32 / bf16 / fp16 on
contiguous NC[D]H[W] tensors.

Parity: reference `phi/kernels/funcs/pooling.cu` (pooling functors, adaptive windows, exclusive
averaging, MaxPoolWithIndex masks = flat index within the input plane) and
`phi/kernels/gpu/interpolate_kernel.cu` (nearest / linear / bilinear / trilinear, align_corners).
Geometry (output sizes, ceil_mode, the f32 source scales) is computed here on the host; the
kernels take it as plain integers. Max-pool backward gathers dY through the saved argmax
(deterministic); resampling backward scatters its linear weights into an f32 buffer.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
_I3 = ctypes.c_int * 3
_F3 = ctypes.c_float * 3


def supported(x) -> bool:
    return x.is_cuda and x.dtype in _DT


def _tup(v, nd):
    if isinstance(v, int):
        return (int(v),) * nd
    v = tuple(int(t) for t in v)
    return v if len(v) == nd else (v[0],) * nd


def _pad3(v, fill=1):
    return (fill,) * (3 - len(v)) + tuple(v)


def pool_out_size(i, k, s, p, ceil_mode):
    """Output length of one axis (reference `pooling.h` PoolOutputSize, ceil_mode semantics)."""
    num = i + 2 * p - k
    o = (-(-num // s) if ceil_mode else num // s) + 1
    if ceil_mode and (o - 1) * s >= i + p:  # the last window must start inside the input
        o -= 1
    return o


def _plane(x, nd):
    N, C = x.shape[0], x.shape[1]
    return N, C, _pad3(tuple(x.shape[2:2 + nd]))


class _PoolNd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, nd, mode, K, S, P, O, adaptive, exclusive, divisor, want_idx):
        x = x.contiguous()
        N, C, I = _plane(x, nd)
        O3 = _pad3(O)
        y = torch.empty((N, C) + tuple(O), dtype=x.dtype, device=x.device)
        idx = torch.empty((N, C) + tuple(O), dtype=torch.int32, device=x.device) if mode == 0 else None
        g = (_I3(*I), _I3(*O3), _I3(*_pad3(K)), _I3(*_pad3(S)), _I3(*_pad3(P, 0)))
        _lib.call("piamd_pool_nd_fwd", _DT[x.dtype], x.data_ptr(), y.data_ptr(),
                  idx.data_ptr() if idx is not None else None, N, C, *g, mode, int(adaptive),
                  int(exclusive), int(divisor or 0), _lib.stream())
        ctx.geo = (nd, mode, K, S, P, O, adaptive, exclusive, divisor, tuple(x.shape), x.dtype)
        if idx is not None:
            ctx.save_for_backward(idx)
            ctx.mark_non_differentiable(idx)
        return (y, idx) if want_idx else y

    @staticmethod
    def backward(ctx, dy, *_):
        nd, mode, K, S, P, O, adaptive, exclusive, divisor, shape, dt = ctx.geo
        idx = ctx.saved_tensors[0] if mode == 0 else None
        dy = dy.to(dt).contiguous()
        dx = torch.empty(shape, dtype=dt, device=dy.device)
        N, C, I = shape[0], shape[1], _pad3(shape[2:])
        g = (_I3(*I), _I3(*_pad3(O)), _I3(*_pad3(K)), _I3(*_pad3(S)), _I3(*_pad3(P, 0)))
        _lib.call("piamd_pool_nd_bwd", _DT[dt], dy.data_ptr(), idx.data_ptr() if idx is not None else None,
                  dx.data_ptr(), N, C, *g, mode, int(adaptive), int(exclusive), int(divisor or 0),
                  _lib.stream())
        return (dx,) + (None,) * 10


def pool(x, nd, mode, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True,
         divisor_override=None, return_mask=False):
    """Fixed-window max (mode 0) / avg (mode 1) pooling of an NC + nd-spatial tensor."""
    K = _tup(kernel_size, nd)
    S = _tup(stride if stride is not None else kernel_size, nd)
    P = _tup(padding, nd)
    I = tuple(x.shape[2:])
    if any(2 * p > k for p, k in zip(P, K)):
        raise ValueError(f"pad should be at most half of the kernel size, got pad={P}, kernel={K}")
    O = tuple(pool_out_size(i, k, s, p, ceil_mode) for i, k, s, p in zip(I, K, S, P))
    r = _PoolNd.apply(x, nd, mode, K, S, P, O, False, exclusive, divisor_override, bool(return_mask))
    if return_mask:
        return r[0], r[1].long()
    return r


def adaptive_pool(x, nd, mode, output_size, return_mask=False):
    I = tuple(x.shape[2:])
    osz = _tup(output_size, nd) if not isinstance(output_size, (list, tuple)) else tuple(output_size)
    O = tuple(int(o) if o is not None else i for o, i in zip(osz, I))
    r = _PoolNd.apply(x, nd, mode, (1,) * nd, (1,) * nd, (0,) * nd, O, True, True, None, bool(return_mask))
    if return_mask:
        return r[0], r[1].long()
    return r


# ---------------------------------------------------------------------------------- resampling
def _scales(I, O, scale_factor, align_corners, linear):
    out = []
    for a, (i, o) in enumerate(zip(I, O)):
        if linear and align_corners:
            out.append(np.float32(i - 1) / np.float32(o - 1) if o > 1 else np.float32(0))
        elif scale_factor is not None:
            sf = scale_factor[a]
            out.append(np.float32(1.0 / sf))
        else:
            out.append(np.float32(i) / np.float32(o))
    return tuple(float(v) for v in out)


class _Interp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, O, scales, mode, align_corners):
        x = x.contiguous()
        N, C, I = _plane(x, len(O))
        y = torch.empty((N, C) + tuple(O), dtype=x.dtype, device=x.device)
        sc = _F3(*((1.0,) * (3 - len(scales)) + tuple(scales)))
        _lib.call("piamd_interp_fwd", _DT[x.dtype], x.data_ptr(), y.data_ptr(), N, C, _I3(*I), _I3(*_pad3(O)),
                  sc, mode, int(align_corners), _lib.stream())
        ctx.geo = (O, scales, mode, align_corners, tuple(x.shape), x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        O, scales, mode, align_corners, shape, dt = ctx.geo
        dy = dy.to(dt).contiguous()
        dx = torch.zeros(shape, dtype=torch.float32, device=dy.device)
        sc = _F3(*((1.0,) * (3 - len(scales)) + tuple(scales)))
        _lib.call("piamd_interp_bwd", _DT[dt], dy.data_ptr(), dx.data_ptr(), shape[0], shape[1],
                  _I3(*_pad3(shape[2:])), _I3(*_pad3(O)), sc, mode, int(align_corners), _lib.stream())
        return dx.to(dt), None, None, None, None


def interpolate(x, size=None, scale_factor=None, mode="nearest", align_corners=False):
    """nearest / linear / bilinear / trilinear resampling of an NC + (1..3)-spatial tensor."""
    nd = x.dim() - 2
    I = tuple(x.shape[2:])
    sf = None
    if size is not None:
        O = _tup(size, nd) if not isinstance(size, (list, tuple)) else tuple(int(s) for s in size)
    else:
        sf = tuple(float(v) for v in (scale_factor if isinstance(scale_factor, (list, tuple))
                                      else (scale_factor,) * nd))
        O = tuple(int(np.floor(i * f)) for i, f in zip(I, sf))
    linear = mode != "nearest"
    return _Interp.apply(x, O, _scales(I, O, sf, align_corners, linear), int(linear),
                         bool(align_corners and linear))


# --------------------------------------------------------------------------------- grid_sample
_GS_MODE = {"bilinear": 0, "nearest": 1}
_GS_PAD = {"zeros": 0, "border": 1, "reflection": 2}


def grid_sample_supported(x, grid, mode, padding_mode):
    return (supported(x) and x.dim() == 4 and grid.dim() == 4 and grid.shape[-1] == 2 and grid.dtype == x.dtype
            and mode in _GS_MODE and padding_mode in _GS_PAD)


class _GridSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, grid, mode, pad, align_corners):
        x, grid = x.contiguous(), grid.contiguous()
        N, C, IH, IW = x.shape
        OH, OW = grid.shape[1], grid.shape[2]
        y = torch.empty(N, C, OH, OW, dtype=x.dtype, device=x.device)
        _lib.call("piamd_grid_sample_fwd", _DT[x.dtype], x.data_ptr(), grid.data_ptr(), y.data_ptr(), N, C, IH, IW,
                  OH, OW, mode, pad, int(align_corners), _lib.stream())
        ctx.save_for_backward(x, grid)
        ctx.cfg = (mode, pad, align_corners)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, grid = ctx.saved_tensors
        mode, pad, align_corners = ctx.cfg
        N, C, IH, IW = x.shape
        OH, OW = grid.shape[1], grid.shape[2]
        dy = dy.to(x.dtype).contiguous()
        dx = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
        dg = torch.empty(grid.shape, dtype=torch.float32, device=x.device)
        _lib.call("piamd_grid_sample_bwd", _DT[x.dtype], dy.data_ptr(), x.data_ptr(), grid.data_ptr(), dx.data_ptr(),
                  dg.data_ptr(), N, C, IH, IW, OH, OW, mode, pad, int(align_corners), _lib.stream())
        return dx.to(x.dtype), dg.to(grid.dtype), None, None, None


def grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=True):
    """2-D bilinear / nearest sampling (see ``grid_sample_supported``)."""
    return _GridSample.apply(x, grid, _GS_MODE[mode], _GS_PAD[padding_mode], bool(align_corners))
