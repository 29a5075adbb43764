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
    # C ≤ 8: stem mode (channels zero-padded to 8, eight taps per 64-deep k-step)
    return (C % 64 == 0 or C <= 8) and K % 4 == 0 and w_shape[1] == C


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


def _launch(x, w_ohwi, bias, st, pad, dil, act, rs=None):
    """x [N,H,W,C] bf16 contiguous, w_ohwi [K,R,S,C] bf16 contiguous → y [N,OH,OW,K]. ``rs``:
    the true filter size in stem mode (C == 8, w_ohwi = [K][ceil(R·S/8)·64] packed taps)."""
    N, H, W, C = x.shape
    K = w_ohwi.shape[0]
    R, S = rs if rs is not None else w_ohwi.shape[1:3]
    OH, OW = _out_hw(H, W, R, S, st, pad, dil)
    if OH < 1 or OW < 1:
        raise ValueError("convolution output is empty")
    M = N * OH * OW
    nk = -(-(R * S) // 8) if rs is not None else R * S * (C // 64)
    y = torch.empty(N, OH, OW, K, dtype=torch.bfloat16, device=x.device)
    b = bias.to(torch.bfloat16).contiguous() if bias is not None else None

    def run(plan):
        tn, ks = plan
        ws = torch.empty(ks * M * K, dtype=torch.float32, device=x.device) if ks > 1 else None
        _lib.call("piamd_conv2d_fwd", x.data_ptr(), w_ohwi.data_ptr(), _zero(x.device).data_ptr(),
                  y.data_ptr(), N, H, W, C, OH, OW, R, S, st[0], st[1], pad[0], pad[1], dil[0],
                  dil[1], K, act, _lib.ptr(b), tn, ks, _lib.ptr(ws), _lib.stream())
    plan = PLAN_OVERRIDE or _autotuned("conv2d_fwd", (N, H, W, C, K, R, S, st, pad, dil, act),
                                       _plan(M, K, nk), _fwd_candidates(M, K, nk), run)
    run(plan)
    return y


def _fwd_candidates(M, K, nk):
    return [(tn, ks) for tn in (64, 128, 256) if tn <= max(64, K)
            for ks in (1, 2, 4, 8) if ks <= nk and (ks == 1 or nk // ks >= 2)]


def _autotuned(op, shape, default, candidates, run):
    """Plan via the runtime autotune cache (ops/autotune.py) — the heuristic when tuning is off."""
    from . import autotune
    return autotune.choose(autotune.key_of(op, *shape), candidates, default, run)


def _wgrad_plan(M, RSC, K):
    """(tile_n, ksplit) for the weight-gradient kernel: the widest tile dividing K_out, then split
    the N·OH·OW reduction until the grid holds ~256 workgroups (each part ≥ 8 pixel steps of 64)
    while the f32 partial planes stay under 64 MiB (their fixed-order sum was 8% of the ResNet-50
    step at a 512-workgroup / 256 MiB plan)."""
    tn = 256 if K % 256 == 0 else 128 if K % 128 == 0 else 64
    tiles = -(-RSC // 256) * (K // tn)
    nk = -(-M // 64)
    ks = 1
    while tiles * ks < 256 and nk // (ks * 2) >= 8 and 2 * ks * RSC * K * 4 <= (64 << 20):
        ks *= 2
    return tn, ks


WGRAD_PLAN_OVERRIDE = None


def wgrad_eligible(C, K, M) -> bool:
    return C % 8 == 0 and K % 64 == 0 and M < (1 << 24)


def conv2d_wgrad(x, dy, R, S, st, pad, dil):
    """dW [K][C][R][S] f32 of conv(x [N,H,W,C], ·) given dy [N,OH,OW,K] (both bf16 NHWC
    contiguous) on the HIP implicit-GEMM weight-gradient kernel."""
    N, H, W, C = x.shape
    _, OH, OW, K = dy.shape
    M, RSC = N * OH * OW, R * S * C
    if not wgrad_eligible(C, K, M):
        raise ValueError(f"conv2d_wgrad: unsupported C={C} K={K} M={M}")
    d = torch.empty(R, S, C, K, dtype=torch.float32, device=x.device)
    nk = -(-M // 64)

    def run(plan):
        tn, ks = plan
        ks = max(1, min(ks, nk))
        ws = torch.empty(ks * RSC * K, dtype=torch.float32, device=x.device) if ks > 1 else None
        _lib.call("piamd_conv2d_wgrad", x.data_ptr(), dy.data_ptr(), _zero(x.device).data_ptr(),
                  d.data_ptr(), N, H, W, C, OH, OW, R, S, st[0], st[1], pad[0], pad[1], dil[0],
                  dil[1], K, tn, ks, _lib.ptr(ws), 0, _lib.stream())
    default = _wgrad_plan(M, RSC, K)
    cands = [(tn, ks) for tn in (64, 128, 256) if K % tn == 0
             for ks in (1, 4, 16, 64, 256) if ks <= nk and ks * RSC * K * 4 <= (256 << 20)]
    plan = WGRAD_PLAN_OVERRIDE or _autotuned("conv2d_wgrad", (N, H, W, C, K, R, S, st, pad, dil),
                                             default, cands, run)
    run(plan)
    return d.permute(3, 2, 0, 1)


def _phase_taps(R, st, pad, dil, ph):
    """Taps r of a strided conv that reach input rows ih ≡ ph (mod st), as a stride-1 sub-conv over
    dY: returns (taps in sub-filter order, pad', dil') with dX[ph + st·i] = Σ_t dY[i − pad' + t·dil']
    · W[taps[t]], or None when no tap reaches that phase."""
    rs = [r for r in range(R) if (ph + pad - r * dil) % st == 0]
    if not rs:
        return None
    d = [(ph + pad - r * dil) // st for r in rs]  # dY row offset of each tap (decreasing)
    taps = rs[::-1]
    dd = d[::-1]
    dil2 = dd[1] - dd[0] if len(dd) > 1 else 1
    return taps, -dd[0], dil2


def conv2d_dgrad_strided(dy, weight, H, W, st, pad, dil):
    """dX [N,H,W,C] bf16 of a strided conv: one stride-1 HIP convolution per output phase
    (ih mod st_h, iw mod st_w) over dY with the sub-filter of the taps that reach that phase,
    scattered into dX (phases with no tap are zero)."""
    N, OH, OW, K = dy.shape
    Kw, C, R, S = weight.shape
    dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=dy.device)
    wb = weight.to(torch.bfloat16)
    for ph in range(st[0]):
        for pw in range(st[1]):
            Hp, Wp = -(-(H - ph) // st[0]), -(-(W - pw) // st[1])
            if Hp <= 0 or Wp <= 0:
                continue
            th, tw = _phase_taps(R, st[0], pad[0], dil[0], ph), _phase_taps(S, st[1], pad[1], dil[1], pw)
            if th is None or tw is None:
                dx[:, ph::st[0], pw::st[1], :] = 0
                continue
            (rt, ph2, dh2), (stp, pw2, dw2) = th, tw
            # sub-filter [C][R'][S'][K]: W[k][c][rt[i]][stp[j]]
            wsub = wb[:, :, rt][:, :, :, stp].permute(1, 2, 3, 0).contiguous()
            y = _launch_geom(dy, wsub, (1, 1), (ph2, pw2), (dh2, dw2), Hp, Wp)
            dx[:, ph::st[0], pw::st[1], :] = y
    return dx


def _launch_geom(x, w_ohwi, st, pad, dil, OH, OW):
    """conv_fwd with an explicit output size (pads may be negative: taps outside are skipped)."""
    N, H, W, C = x.shape
    K, R, S, _ = w_ohwi.shape
    M = N * OH * OW
    nk = R * S * (C // 64)
    y = torch.empty(N, OH, OW, K, dtype=torch.bfloat16, device=x.device)

    def run(plan):
        tn, ks = plan
        ws = torch.empty(ks * M * K, dtype=torch.float32, device=x.device) if ks > 1 else None
        _lib.call("piamd_conv2d_fwd", x.data_ptr(), w_ohwi.data_ptr(), _zero(x.device).data_ptr(),
                  y.data_ptr(), N, H, W, C, OH, OW, R, S, st[0], st[1], pad[0], pad[1], dil[0],
                  dil[1], K, 0, 0, tn, ks, _lib.ptr(ws), _lib.stream())
    run(_autotuned("conv2d_dgrad", (N, H, W, C, K, R, S, st, pad, dil, OH, OW), _plan(M, K, nk),
                   _fwd_candidates(M, K, nk), run))
    return y


class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, st, pad, dil, act):
        C0 = x.shape[-1]
        if C0 % 64:  # stem mode: zero-pad the image channels to 8
            xc = torch.nn.functional.pad(x, (0, 8 - C0)).contiguous() if C0 < 8 else x.contiguous()
            K, _, R, S = weight.shape
            nk = -(-(R * S) // 8)
            w8 = torch.zeros(K, nk * 64, dtype=torch.bfloat16, device=x.device)
            w8[:, :R * S * 8].view(K, R, S, 8)[..., :C0] = weight.to(torch.bfloat16).permute(0, 2, 3, 1)
            y = _launch(xc, w8.view(K, 1, nk * 8, 8), bias, st, pad, dil, act, rs=(R, S))
        else:
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
        K, C0, R, S = weight.shape
        C = x.shape[-1]  # == C0, or 8 in stem mode (zero-padded channels)
        if C != C0:
            weight = torch.nn.functional.pad(weight, (0, 0, 0, 0, 0, C - C0))
        dx = dw = db = None
        N, H, W, _ = x.shape
        if ctx.needs_input_grad[0]:
            pad_t = (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1])
            if K % 64 == 0 and C % 4 == 0 and st == (1, 1) and dy.shape[1:3] == (H, W):
                # dX = conv(dY, flip(W)ᵀ): filter [C][R][S][K] = W[k][c][R-1-r][S-1-s]
                w_t = weight.to(torch.bfloat16).flip(2, 3).permute(1, 2, 3, 0).contiguous()
                dx = _launch_geom(dy, w_t, (1, 1), pad_t, dil, H, W)
            elif K % 64 == 0 and C % 4 == 0:
                dx = conv2d_dgrad_strided(dy, weight, H, W, st, pad, dil)
            else:
                _lib.fallback("conv2d_dgrad", f"K_out={K} C={C} (needs K%64, C%4)")
                dx = torch.ops.aten.convolution_backward(
                    dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), weight.to(torch.bfloat16),
                    None, list(st), list(pad), list(dil), False, [0, 0], 1,
                    [True, False, False])[0].permute(0, 2, 3, 1)
        if ctx.needs_input_grad[1]:
            if wgrad_eligible(C, K, dy.shape[0] * dy.shape[1] * dy.shape[2]):
                dw = conv2d_wgrad(x, dy, R, S, st, pad, dil)
            else:
                _lib.fallback("conv2d_wgrad", f"K_out={K} C={C} (needs K%64, C%8)")
                dw = torch.ops.aten.convolution_backward(
                    dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), weight.to(torch.bfloat16), None,
                    list(st), list(pad), list(dil), False, [0, 0], 1, [False, True, False])[1]
            dw = dw.to(weight.dtype)
        if C != C0:
            dx = dx[..., :C0] if dx is not None else None
            dw = dw[:, :C0].contiguous() if dw is not None else None
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
