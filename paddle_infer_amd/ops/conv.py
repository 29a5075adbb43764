"""NHWC bf16 convolution on the MFMA implicit-GEMM kernel (``csrc/kernels/gemm.hip`` conv_fwd).

Parity: reference `phi/kernels/gpudnn/conv_kernel.cu` + `conv_grad_kernel.cu` (cuDNN forward /
backward-data / backward-filter) and the fused conv+bias+act of `fused_conv2d_add_act_kernel.cu`.

* forward: one kernel, bias + activation in the epilogue, activation gathered straight from the
  NHWC tensor by the LDS DMA (no im2col buffer);
* backward-data: for stride 1 the data gradient is itself a stride-1 convolution of dY with the
  spatially flipped, in/out-transposed filter (padding ``dil·(R−1) − pad``) and runs on the same
  kernel; other strides use the library (MIOpen) backward-data;
* backward-filter: library (MIOpen) on the channels-last views, bias gradient a column sum.

Eligible: groups 1, C % 64 == 0, K_out % 4 == 0, symmetric zero padding, bf16 on the GPU.
``conv2d_nhwc`` raises on an ineligible call; ``eligible`` tells the dispatcher.
"""
from __future__ import annotations

import torch

from . import _lib

HIP_CONV = True  # route eligible nn.functional.conv2d calls here
_ACT = {None: 0, "none": 0, "identity": 0, "relu": 3}
_ZERO: dict = {}


def _zero(dev):
    z = _ZERO.get(dev)
    if z is None:
        z = _ZERO[dev] = torch.zeros(128, dtype=torch.bfloat16, device=dev)
    return z


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def eligible(x_nhwc_shape, w_shape, groups=1, padding=0) -> bool:
    if groups != 1 or isinstance(padding, str) or len(w_shape) != 4:
        return False
    if len(_pair(padding)) != 2:
        return False
    C, K = x_nhwc_shape[-1], w_shape[0]
    return C % 64 == 0 and K % 4 == 0 and w_shape[1] == C


def _out_hw(H, W, R, S, st, pad, dil):
    return ((H + 2 * pad[0] - dil[0] * (R - 1) - 1) // st[0] + 1,
            (W + 2 * pad[1] - dil[1] * (S - 1) - 1) // st[1] + 1)


def _plan(M, K, nk):
    """(tile_n, ksplit) from the sweep in ``profiles/conv_nhwc_r1.txt`` (ResNet-50 layers, batch 64;
    the rule picks the measured-best plan on every one of them):
    * very short reductions (≤ 2 k-steps) → 256 × 64 tiles, 4 waves/SIMD hide the epilogue;
    * wide outputs (K_out ≥ 512) with ≥ 192 full tiles → 256 × 256;
    * K_out ≥ 128 with ≥ 128 tiles or a long reduction → 256 × 128; else 256 × 64;
    * split the reduction while the grid is under 128 workgroups and each part keeps ≥ 8 k-steps
      (split-K pays only where the f32 partial planes are cheap against the reduction)."""
    def tiles(tn):
        return -(-M // 256) * -(-K // tn)
    if nk <= 2:
        tn = 64
    elif K >= 512 and tiles(256) >= 192:
        tn = 256
    elif K >= 128 and (tiles(128) >= 128 or nk >= 32):
        tn = 128
    else:
        tn = 64
    ks = 1
    while tiles(tn) * ks < 128 and nk // (ks * 2) >= 8:
        ks *= 2
    return tn, ks


PLAN_OVERRIDE = None  # (tile_n, ksplit) for tuning sweeps


def _launch(x, w_ohwi, bias, st, pad, dil, act):
    """x [N,H,W,C] bf16 contiguous, w_ohwi [K,R,S,C] bf16 contiguous → y [N,OH,OW,K]."""
    N, H, W, C = x.shape
    K, R, S, _ = w_ohwi.shape
    OH, OW = _out_hw(H, W, R, S, st, pad, dil)
    if OH < 1 or OW < 1:
        raise ValueError("convolution output is empty")
    M = N * OH * OW
    tn, ks = PLAN_OVERRIDE or _plan(M, K, R * S * (C // 64))
    y = torch.empty(N, OH, OW, K, dtype=torch.bfloat16, device=x.device)
    ws = torch.empty(ks * M * K, dtype=torch.float32, device=x.device) if ks > 1 else None
    b = bias.to(torch.bfloat16).contiguous() if bias is not None else None
    _lib.call("piamd_conv2d_fwd", x.data_ptr(), w_ohwi.data_ptr(), _zero(x.device).data_ptr(),
              y.data_ptr(), N, H, W, C, OH, OW, R, S, st[0], st[1], pad[0], pad[1], dil[0], dil[1],
              K, act, _lib.ptr(b), tn, ks, _lib.ptr(ws), _lib.stream())
    return y


class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, st, pad, dil, act):
        xc = x.contiguous()
        w_ohwi = weight.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        y = _launch(xc, w_ohwi, bias, st, pad, dil, act)
        ctx.save_for_backward(xc, weight, y if act else None)
        ctx.cfg = (st, pad, dil, act, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        st, pad, dil, act, has_bias = ctx.cfg
        dy = dy.to(torch.bfloat16)
        if act == 3:
            dy = dy * (y > 0)
        dy = dy.contiguous()
        K, C, R, S = weight.shape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            pad_t = (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1])
            if st == (1, 1) and K % 64 == 0 and C % 4 == 0 and min(pad_t) >= 0:
                # dX = conv(dY, flip(W)ᵀ): filter [C][R][S][K] = W[k][c][R-1-r][S-1-s]
                w_t = weight.to(torch.bfloat16).flip(2, 3).permute(1, 2, 3, 0).contiguous()
                dx = _launch(dy, w_t, None, (1, 1), pad_t, dil, 0)
            else:
                dx = torch.ops.aten.convolution_backward(
                    dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), weight.to(torch.bfloat16),
                    None, list(st), list(pad), list(dil), False, [0, 0], 1,
                    [True, False, False])[0].permute(0, 2, 3, 1)
        if ctx.needs_input_grad[1]:
            dw = torch.ops.aten.convolution_backward(
                dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), weight.to(torch.bfloat16), None,
                list(st), list(pad), list(dil), False, [0, 0], 1, [False, True, False])[1]
            dw = dw.to(weight.dtype)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum((0, 1, 2))
        return dx, dw, db, None, None, None, None


def conv2d_nhwc(x, weight, bias=None, stride=1, padding=0, dilation=1, act=None):
    """y[N,OH,OW,K] = act(conv(x[N,H,W,C], weight[K,C,R,S]) + bias) in bf16 on the HIP kernel."""
    if not (x.is_cuda and x.dim() == 4):
        raise ValueError("conv2d_nhwc needs a 4-D GPU tensor")
    if not eligible(x.shape, weight.shape, 1, padding):
        raise ValueError(f"conv2d_nhwc: unsupported shapes x{tuple(x.shape)} w{tuple(weight.shape)}")
    if act not in _ACT:
        raise ValueError(f"conv2d_nhwc: unsupported activation {act}")
    st, pad, dil = _pair(stride), _pair(padding), _pair(dilation)
    return _Conv2dNHWC.apply(x.to(torch.bfloat16), weight, bias, st, pad, dil, _ACT[act])


def conv2d_nchw(x, weight, bias=None, stride=1, padding=0, dilation=1, act=None):
    """Same kernel for an NCHW-indexed tensor: channels_last storage is used as is (a view)."""
    y = conv2d_nhwc(x.permute(0, 2, 3, 1), weight, bias, stride, padding, dilation, act)
    return y.permute(0, 3, 1, 2)
