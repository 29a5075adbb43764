"""NHWC convolution on the framework's own kernels — every 2-D conv of a bf16/fp16/fp32 (or
autocast) model, dense, grouped or depthwise, runs without the library (MIOpen).

Parity: reference `phi/kernels/gpudnn/conv_kernel.cu` + `conv_grad_kernel.cu` (cuDNN forward /
backward-data / backward-filter), `phi/kernels/gpu/depthwise_conv_kernel.cu` (depthwise) and the
fused conv+bias+act of `fused_conv2d_add_act_kernel.cu`.

Routes (``conv2d_any``, called by ``nn.functional.conv2d`` for GPU tensors):

* dense (groups 1), bf16 / fp16 → MFMA implicit GEMM (``csrc/kernels/gemm.hip`` conv_fwd, bf16 or
  f16 MFMA): bias + activation in the epilogue, the activation gathered straight from the NHWC
  tensor by the LDS DMA (no im2col buffer). Channel counts that are not a multiple of 64 are
  zero-padded to one (≤ 8 input channels: stem mode, eight taps per k-step);
  - data gradient: stride 1 → the same kernel on dY with the flipped, in/out-transposed filter;
    other strides → one stride-1 sub-convolution per output phase;
  - weight gradient: the implicit-GEMM wgrad kernel (reduction over N·OH·OW output pixels);
* dense 1×1 with unaligned channels → a plain GEMM over the pixel rows (``ops.linear.mm_nt``);
* grouped / depthwise, any float dtype → the direct NHWC kernels of ``csrc/kernels/conv_dw.hip``
  (forward, transposed-geometry data gradient, deterministic split weight gradient);
* NCHW inputs are used through their channels_last view when they have one; a plain NCHW tensor
  is re-laid-out once (the output is channels_last, so every later layer takes the view);
* dense fp32 without autocast → the same MFMA implicit GEMM as three bf16 products accumulated in
  f32 (``_Conv2dF32``: ≈2^-16 relative per product; ``FP32_SPLIT = False`` keeps the library).
"""
from __future__ import annotations

import math
import os
import threading

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


_HALF = (torch.bfloat16, torch.float16)


def _f16(t) -> int:
    return int(t.dtype == torch.float16)


def _pad64(n: int) -> int:
    return -(-n // 64) * 64


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def eligible(x_nhwc_shape, w_shape, groups=1, padding=0) -> bool:
    """Dense conv the MFMA kernels take: groups 1, symmetric padding, matching channels (channel
    counts off the 64-grid are zero-padded; ≤ 8 input channels run in stem mode)."""
    if groups != 1 or isinstance(padding, str) or len(w_shape) != 4:
        return False
    if len(_pair(padding)) != 2:
        return False
    return w_shape[1] == x_nhwc_shape[-1]


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


def _launch(x, w_ohwi, bias, st, pad, dil, act, rs=None, out_f32=False, stats_out=None):
    """x [N,H,W,C] bf16 contiguous, w_ohwi [K,R,S,C] bf16 contiguous → y [N,OH,OW,K]. ``rs``:
    the true filter size in stem mode (C == 8, w_ohwi = [K][ceil(R·S/8)·64] packed taps).
    ``out_f32``: y in f32 (no bias / activation). ``stats_out`` (a list): when the chosen plan
    runs unsplit and y takes no bias / activation, the kernel also writes per-tile BatchNorm
    statistics of y and ``(stats [3, K, P], P)`` is appended (see conv_tile_stats)."""
    N, H, W, C = x.shape
    K = w_ohwi.shape[0]
    R, S = rs if rs is not None else w_ohwi.shape[1:3]
    OH, OW = _out_hw(H, W, R, S, st, pad, dil)
    if OH < 1 or OW < 1:
        raise ValueError("convolution output is empty")
    M = N * OH * OW
    nk = -(-(R * S) // 8) if rs is not None else R * S * (C // 64)
    y = torch.empty(N, OH, OW, K, dtype=torch.float32 if out_f32 else x.dtype, device=x.device)
    b = bias.to(x.dtype).contiguous() if bias is not None else None
    assert not (out_f32 and (b is not None or act))
    flags = _f16(x) | (2 if out_f32 else 0)

    def run(plan, stats=None):
        tn, ks = plan
        ws = torch.empty(ks * M * K, dtype=torch.float32, device=x.device) if ks > 1 else None
        _lib.call("piamd_conv2d_fwd2", x.data_ptr(), w_ohwi.data_ptr(), _zero(x.device).data_ptr(),
                  y.data_ptr(), N, H, W, C, OH, OW, R, S, st[0], st[1], pad[0], pad[1], dil[0],
                  dil[1], K, act, _lib.ptr(b), tn, ks, _lib.ptr(ws), flags, _lib.ptr(stats),
                  _lib.stream())
    plan = PLAN_OVERRIDE or _autotuned("conv2d_fwd", (N, H, W, C, K, R, S, st, pad, dil, act)
                                       + (("f32",) if out_f32 else ()),
                                       _plan(M, K, nk), _fwd_candidates(M, K, nk), run)
    stats = None
    if stats_out is not None and plan[1] == 1 and b is None and not act and not out_f32:
        P = -(-M // 256)
        stats = torch.empty(3, K, P, dtype=torch.float32, device=x.device)
        stats_out.append((stats, P))
    run(plan, stats)
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


def conv2d_wgrad(x, dy, R, S, st, pad, dil, layout=None):
    """dW [K][C][R][S] f32 of conv(x [N,H,W,C], ·) given dy [N,OH,OW,K] (both bf16 or both fp16,
    NHWC contiguous) on the HIP implicit-GEMM weight-gradient kernel. ``layout`` "kcrs" / "ohwi":
    the gradient is stored in the filter parameter's own memory layout (contiguous / channels_last),
    so autograd adopts it as ``.grad`` without a relayout copy (the split-K finish writes it
    permuted; only split plans then); None: HWIO storage."""
    N, H, W, C = x.shape
    _, OH, OW, K = dy.shape
    M, RSC = N * OH * OW, R * S * C
    if not wgrad_eligible(C, K, M):
        raise ValueError(f"conv2d_wgrad: unsupported C={C} K={K} M={M}")
    nk = -(-M // 64)
    if nk < 4:
        layout = None
    ohwi = layout is not None
    shape = {"ohwi": (K, R, S, C), "kcrs": (K, C, R, S)}.get(layout, (R, S, C, K))
    d = torch.empty(shape, dtype=torch.float32, device=x.device)
    mode = {"ohwi": 2, "kcrs": 4}.get(layout, 0)

    def run(plan):
        tn, ks = plan
        ks = max(4 if ohwi else 1, min(ks, nk))
        ws = torch.empty(ks * RSC * K, dtype=torch.float32, device=x.device) if ks > 1 else None
        _lib.call("piamd_conv2d_wgrad", x.data_ptr(), dy.data_ptr(), _zero(x.device).data_ptr(),
                  d.data_ptr(), N, H, W, C, OH, OW, R, S, st[0], st[1], pad[0], pad[1], dil[0],
                  dil[1], K, tn, ks, _lib.ptr(ws), mode, _f16(x), _lib.stream())
    default = _wgrad_plan(M, RSC, K)
    if ohwi:
        default = (default[0], max(4, default[1]))
    cands = [(tn, ks) for tn in (64, 128, 256) if K % tn == 0
             for ks in ((4, 16, 64, 256) if ohwi else (1, 4, 16, 64, 256))
             if ks <= nk and ks * RSC * K * 4 <= (256 << 20)]
    plan = WGRAD_PLAN_OVERRIDE or _autotuned("conv2d_wgrad", (N, H, W, C, K, R, S, st, pad, dil)
                                             + (("perm",) if ohwi else ()), default, cands, run)
    run(plan)
    if layout == "kcrs":
        return d
    return d.permute(0, 3, 1, 2) if layout == "ohwi" else d.permute(3, 2, 0, 1)


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


def _take_ap(t, dim, idx):
    """t.index_select(dim, idx) for an arithmetic progression idx, as a strided slice (+ flip when
    descending): no host-built index tensor, so it is legal inside hipGraph capture."""
    if len(idx) == 1:
        return t.narrow(dim, idx[0], 1)
    step = idx[1] - idx[0]
    assert all(b - a == step for a, b in zip(idx, idx[1:])), idx
    lo = min(idx[0], idx[-1])
    sl = [slice(None)] * t.dim()
    sl[dim] = slice(lo, lo + abs(step) * (len(idx) - 1) + 1, abs(step))
    out = t[tuple(sl)]
    return out.flip(dim) if step < 0 else out


_PHASE_IDX = {}


def _phase_filters(wb, st, pad, dil):
    """Every phase sub-filter of a strided conv's data gradient, {(ph, pw): [C][R'][S'][K]
    contiguous view}, gathered from the [K][C][R][S] filter ``wb`` by ONE ``torch.take`` with a
    cached device index (instead of slice + flip + copy per phase). None when the index is not
    cached yet and a graph capture is running (its host-built index cannot be uploaded there)."""
    K, C, R, S = wb.shape
    key = (tuple(wb.shape), tuple(st), tuple(pad), tuple(dil), wb.device)
    ent = _PHASE_IDX.get(key)
    if ent is None:
        if wb.is_cuda and torch.cuda.is_current_stream_capturing():
            return None
        parts, views, off = [], {}, 0
        k, c = torch.arange(K), torch.arange(C)
        for ph in range(st[0]):
            for pw in range(st[1]):
                th, tw = _phase_taps(R, st[0], pad[0], dil[0], ph), _phase_taps(S, st[1], pad[1], dil[1], pw)
                if th is None or tw is None:
                    continue
                r, s_ = torch.tensor(th[0]), torch.tensor(tw[0])
                flat = (((k[None, None, None, :] * C + c[:, None, None, None]) * R + r[None, :, None, None]) * S
                        + s_[None, None, :, None])  # [C][R'][S'][K] → W[k][c][r][s]
                parts.append(flat.reshape(-1))
                views[(ph, pw)] = (off, (C, len(th[0]), len(tw[0]), K))
                off += flat.numel()
        ent = _PHASE_IDX[key] = (torch.cat(parts).to(wb.device), views)
    idx, views = ent
    buf = torch.take(wb, idx)
    return {p: buf[o:o + math.prod(shape)].view(shape) for p, (o, shape) in views.items()}


def conv2d_dgrad_strided(dy, weight, H, W, st, pad, dil, out_f32=False):
    """dX [N,H,W,C] (dtype of dy, or f32) of a strided conv: one stride-1 HIP convolution per output
    phase (ih mod st_h, iw mod st_w) over dY with the sub-filter of the taps that reach that phase,
    scattered into dX (phases with no tap are zero)."""
    N, OH, OW, K = dy.shape
    Kw, C, R, S = weight.shape
    # phases no tap reaches stay zero: one fill of dX up front instead of a strided fill per phase
    tapless = any(_phase_taps(R, st[0], pad[0], dil[0], ph) is None or _phase_taps(S, st[1], pad[1], dil[1], pw) is None
                  for ph in range(st[0]) for pw in range(st[1]))
    dx = (torch.zeros if tapless else torch.empty)(N, H, W, C, dtype=torch.float32 if out_f32 else dy.dtype,
                                                  device=dy.device)
    wb = weight.to(dy.dtype)
    subs = _phase_filters(wb.contiguous(), st, pad, dil)
    for ph in range(st[0]):
        for pw in range(st[1]):
            Hp, Wp = -(-(H - ph) // st[0]), -(-(W - pw) // st[1])
            if Hp <= 0 or Wp <= 0:
                continue
            th, tw = _phase_taps(R, st[0], pad[0], dil[0], ph), _phase_taps(S, st[1], pad[1], dil[1], pw)
            if th is None or tw is None:
                continue
            (rt, ph2, dh2), (stp, pw2, dw2) = th, tw
            # sub-filter [C][R'][S'][K]: W[k][c][rt[i]][stp[j]] — from the one-gather buffer, or
            # (uncached index inside a capture) strided slices + flips of the filter
            wsub = (subs[(ph, pw)] if subs is not None
                    else _take_ap(_take_ap(wb, 2, rt), 3, stp).permute(1, 2, 3, 0).contiguous())
            # the phase convolution writes its outputs straight into dX's phase pixels
            _launch_geom(dy, wsub, (1, 1), (ph2, pw2), (dh2, dw2), Hp, Wp, out_f32,
                         out=dx, phase=(st[0], st[1], ph, pw))
    return dx


def _launch_geom(x, w_ohwi, st, pad, dil, OH, OW, out_f32=False, out=None, phase=None, acc=None):
    """conv_fwd with an explicit output size (pads may be negative: taps outside are skipped).
    ``out`` [N, H', W', K] + ``phase`` (rs_h, rs_w, ph, pw): the OH × OW outputs are written to
    pixels (oh·rs_h + ph, ow·rs_w + pw) of ``out`` (unsplit plans in the kernel epilogue, split-K
    plans through a copy). ``acc`` [N, OH, OW, K] (16-bit): the result is added to it (in the
    epilogue for unsplit plans) and it is returned."""
    N, H, W, C = x.shape
    K, R, S, _ = w_ohwi.shape
    M = N * OH * OW
    nk = R * S * (C // 64)
    dt = torch.float32 if out_f32 else x.dtype
    flags = _f16(x) | (2 if out_f32 else 0)
    if out is not None:
        assert out.dtype == dt and out.is_contiguous() and out.shape[0] == N and out.shape[3] == K
    y = None

    if acc is not None:
        assert out is None and not out_f32 and acc.shape == (N, OH, OW, K) and acc.dtype == x.dtype
        # tuning runs would add into acc repeatedly: the plan is tuned (same cache key as the plain
        # data gradient) on a scratch output, then the chosen plan accumulates once
        scratch = []

        def run_plain(plan):
            tn_, ks_ = plan
            if not scratch:
                scratch.append(torch.empty(N, OH, OW, K, dtype=dt, device=x.device))
            ws = torch.empty(ks_ * M * K, dtype=torch.float32, device=x.device) if ks_ > 1 else None
            _lib.call("piamd_conv2d_fwd3", x.data_ptr(), w_ohwi.data_ptr(), _zero(x.device).data_ptr(),
                      scratch[0].data_ptr(), N, H, W, C, OH, OW, R, S, st[0], st[1], pad[0], pad[1],
                      dil[0], dil[1], K, 0, 0, tn_, ks_, _lib.ptr(ws), flags, None, 0, 0, 0, 0, 0, 0,
                      _lib.stream())
        tn, ks = _autotuned("conv2d_dgrad", (N, H, W, C, K, R, S, st, pad, dil, OH, OW),
                            _plan(M, K, nk), _fwd_candidates(M, K, nk), run_plain)
        if ks != 1:
            acc += _launch_geom(x, w_ohwi, st, pad, dil, OH, OW)
            return acc
        _lib.call("piamd_conv2d_fwd3", x.data_ptr(), w_ohwi.data_ptr(), _zero(x.device).data_ptr(),
                  acc.data_ptr(), N, H, W, C, OH, OW, R, S, st[0], st[1], pad[0], pad[1], dil[0],
                  dil[1], K, 0, 0, tn, 1, None, flags | 4, None, 0, 0, 0, 0, 0, 0, _lib.stream())
        return acc

    def run(plan):
        nonlocal y
        tn, ks = plan
        ws = torch.empty(ks * M * K, dtype=torch.float32, device=x.device) if ks > 1 else None
        direct = out is not None and ks == 1
        if not direct and y is None:
            y = torch.empty(N, OH, OW, K, dtype=dt, device=x.device)
        dst = out if direct else y
        geo = (out.shape[1], out.shape[2]) + tuple(phase) if direct else (0, 0, 0, 0, 0, 0)
        _lib.call("piamd_conv2d_fwd3", x.data_ptr(), w_ohwi.data_ptr(), _zero(x.device).data_ptr(),
                  dst.data_ptr(), N, H, W, C, OH, OW, R, S, st[0], st[1], pad[0], pad[1], dil[0],
                  dil[1], K, 0, 0, tn, ks, _lib.ptr(ws), flags, None, *geo, _lib.stream())
        if out is not None and not direct:
            rs_h, rs_w, ph, pw = phase
            out[:, ph::rs_h, pw::rs_w, :] = y
    run(_autotuned("conv2d_dgrad", (N, H, W, C, K, R, S, st, pad, dil, OH, OW)
                   + (("f32",) if out_f32 else ()) + (("phase",) if out is not None else ()),
                   _plan(M, K, nk), _fwd_candidates(M, K, nk), run))
    return out if out is not None else y


def _padc(t, n):
    """zero-pad the last dim of t to n."""
    return t if t.shape[-1] == n else torch.nn.functional.pad(t, (0, n - t.shape[-1]))


# Per-tile BatchNorm statistics from the conv forward epilogue (PIAMD_CONV_BN_STATS=0: off): a
# training conv without bias / activation attaches them to its output, and a BatchNorm applied
# to that output finalizes them instead of reading the output once more (ops/batchnorm.py).
BN_STATS = os.environ.get("PIAMD_CONV_BN_STATS", "1") != "0"
_STATS = threading.local()


def _take_stats():
    v = getattr(_STATS, "v", None)
    _STATS.v = None
    return v


# Residual-gradient join (PIAMD_RES_JOIN=0: off). A residual block feeds its input x to a conv and,
# as the residual, to the BatchNorm closing the block; autograd then sums the two gradients of x
# with an ATen add. With a join, the BN's backward (which runs first) hands its residual gradient
# to the join instead of returning it, and the conv's backward adds it in its data-gradient
# epilogue (the kernel accumulates into it): one gradient, no add pass.
RES_JOIN = os.environ.get("PIAMD_RES_JOIN", "1") != "0"
_JOIN = threading.local()


class ResidualGradJoin:
    """Token shared by the conv that consumes a block input (``join_source``) and the BatchNorm that
    adds it as the residual (``ops.batchnorm.join_sink``). ``armed``: the conv will take the
    gradient; ``dres``: the BN's residual gradient (NHWC contiguous) until the conv consumes it."""

    def __init__(self):
        self.armed = False
        self.dres = None


class join_source:
    """``with join_source(j):`` the next dense HIP conv consumes the residual gradient of ``j``."""

    def __init__(self, j):
        self.j = j

    def __enter__(self):
        _JOIN.src = self.j
        return self.j

    def __exit__(self, *exc):
        _JOIN.src = None
        return False


def _take_join():
    j = getattr(_JOIN, "src", None)
    _JOIN.src = None
    return j


class join_give:
    """``with join_give(j):`` the next dense HIP conv GIVES its data gradient to the join ``j``
    (stored in ``j.dres``, None returned to autograd) when the join's source conv — another conv
    of the same input — has not run its backward yet; that source then adds it in its
    data-gradient epilogue. A downsampling residual block: the shortcut conv gives, the main
    path's first conv takes (no ATen add of the two block-input gradients). If the source ran
    first (it closes the join), the giver returns its gradient normally."""

    def __init__(self, j):
        self.j = j

    def __enter__(self):
        _JOIN.give = self.j
        return self.j

    def __exit__(self, *exc):
        _JOIN.give = None
        return False


def _take_give():
    j = getattr(_JOIN, "give", None)
    _JOIN.give = None
    return j


def _give(ctx, x, dx):
    """The giver's side of a conv→conv join: hand dX (same NHWC shape / dtype as the shared
    input) to a still-open join instead of returning it."""
    g = getattr(ctx, "give", None)
    if (g is None or dx is None or not g.armed or g.dres is not None or dx.shape != x.shape
            or dx.dtype != x.dtype):
        return dx
    g.dres = dx.contiguous()
    return None


class _Conv2dNHWC(torch.autograd.Function):
    """Dense conv on the MFMA kernels: x [N,H,W,C0] bf16/fp16 (contiguous), weight [K0,C0,R,S].
    ``want_stats``: leave the output's per-tile BN statistics in the thread-local slot."""

    @staticmethod
    def forward(ctx, x, weight, bias, st, pad, dil, act, want_stats=False, join=None, give=None):
        dt = x.dtype
        K0, C0, R, S = weight.shape
        K = -(-K0 // 4) * 4  # the epilogue stores 4 output channels per lane
        prep = (C0 > 8 and st == (1, 1) and _wprep_ok(x, weight)
                and _out_hw(x.shape[1], x.shape[2], R, S, st, pad, dil) == tuple(x.shape[1:3]))
        # the filter gradient is produced in the parameter's own layout (no AccumulateGrad copy)
        ctx.w_layout = ("kcrs" if weight.is_contiguous() else
                        "ohwi" if weight.is_contiguous(memory_format=torch.channels_last) else None)
        wq0 = weight if prep else weight.to(dt)  # the prep path casts inside its own kernel
        wq = wq0 if (K == K0 or prep) else torch.nn.functional.pad(wq0, (0, 0, 0, 0, 0, 0, 0, K - K0))
        b = None if bias is None else _padc(bias.to(dt), K)
        so = [] if (want_stats and K == K0) else None
        _STATS.v = None
        ctx.join = join
        ctx.give = give
        if C0 <= 8:  # stem mode: zero-pad the image channels to 8
            xc = _padc(x, 8).contiguous()
            nk = -(-(R * S) // 8)
            w8 = torch.zeros(K, nk * 64, dtype=dt, device=x.device)
            w8[:, :R * S * 8].view(K, R, S, 8)[..., :C0] = wq.permute(0, 2, 3, 1)
            y = _launch(xc, w8.view(K, 1, nk * 8, 8), b, st, pad, dil, act, rs=(R, S), stats_out=so)
        else:  # channels zero-padded to a multiple of 64 (one k-step never straddles two taps)
            C = _pad64(C0)
            xc = _padc(x, C).contiguous()
            w_t = None
            if prep:
                # ONE launch: master filter → forward OHWI operand + the stride-1 data gradient's
                # flipped [C][R][S][Kp] operand (no cast / permute / flip kernels in either pass)
                Kp = _pad64(K0)
                w_ohwi = torch.empty(K, R, S, C, dtype=dt, device=x.device)
                w_t = torch.empty(C, R, S, Kp, dtype=dt, device=x.device) if ctx.needs_input_grad[0] else None
                wc = weight.detach().contiguous()
                _lib.call("piamd_conv_wprep", _WSRC[wc.dtype], _f16(x), wc.data_ptr(), w_ohwi.data_ptr(),
                          _lib.ptr(w_t), K0, C0, R, S, K, C, Kp, _lib.stream())
            else:
                w_ohwi = _padc(wq.permute(0, 2, 3, 1), C).contiguous()
            y = _launch(xc, w_ohwi, b, st, pad, dil, act, stats_out=so)
            if so:
                _STATS.v = so[0]
            if prep:
                if K != K0:
                    y = y[..., :K0].contiguous()
                ctx.save_for_backward(xc, w_t, y if act else None)
                ctx.cfg = (st, pad, dil, act, bias is not None, weight.dtype)
                ctx.wshape = (K0, C0, R, S)
                return y
        if K != K0:
            y = y[..., :K0].contiguous()
        if so:
            _STATS.v = so[0]
        # the half-precision weight is kept for the backward (no second cast of the master weight)
        ctx.save_for_backward(xc, wq0, y if act else None)
        ctx.cfg = (st, pad, dil, act, bias is not None, weight.dtype)
        ctx.wshape = None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wq, y = ctx.saved_tensors
        st, pad, dil, act, has_bias, wdt = ctx.cfg
        dt = x.dtype
        dy = dy.to(dt)
        if act == 3:
            dy = dy * (y > 0)
        dy = dy.contiguous()
        if ctx.wshape is not None:  # filter prepared in forward (stride 1, same size)
            return _Conv2dNHWC._backward_prepped(ctx, x, wq, dy)
        K0, C0, R, S = wq.shape
        C = x.shape[-1]  # == C0, or C0 zero-padded (to 8 in stem mode, else to a multiple of 64)
        N, H, W, _ = x.shape
        M = dy.shape[0] * dy.shape[1] * dy.shape[2]
        Kp = _pad64(K0)  # dY channels padded: the dgrad reduction / wgrad tile runs over 64s
        if C != C0 or Kp != K0:
            wq = torch.nn.functional.pad(wq, (0, 0, 0, 0, 0, C - C0, 0, Kp - K0))
        dyp = _padc(dy, Kp)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if st == (1, 1) and dy.shape[1:3] == (H, W):
                # dX = conv(dY, flip(W)ᵀ): filter [C][R][S][K] = W[k][c][R-1-r][S-1-s]
                pad_t = (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1])
                w_t = wq.flip(2, 3).permute(1, 2, 3, 0).contiguous()
                dx = _launch_geom(dyp, w_t, (1, 1), pad_t, dil, H, W, acc=_join_acc(ctx, x, C0))
            else:
                dx = conv2d_dgrad_strided(dyp, wq, H, W, st, pad, dil)
            dx = _give(ctx, x, _join_finish(ctx, dx[..., :C0] if C != C0 else dx))
        if ctx.needs_input_grad[1]:
            if wgrad_eligible(C, Kp, M):
                dw = conv2d_wgrad(x, dyp, R, S, st, pad, dil, layout=ctx.w_layout)[:K0, :C0]
            else:  # > 2^24 output pixels: the direct kernel's pixel-chunked reduction
                dw = _direct_wgrad(x[..., :C0].contiguous(), dy, R, S, st, pad, dil, C0, K0)
            dw = dw.to(wdt)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum((0, 1, 2)).to(wdt)
        return dx, dw, db, None, None, None, None, None, None, None

    @staticmethod
    def _backward_prepped(ctx, x, w_t, dy):
        st, pad, dil, act, has_bias, wdt = ctx.cfg
        K0, C0, R, S = ctx.wshape
        C = x.shape[-1]
        N, H, W, _ = x.shape
        M = dy.shape[0] * dy.shape[1] * dy.shape[2]
        Kp = _pad64(K0)
        dyp = _padc(dy, Kp)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            pad_t = (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1])
            dx = _launch_geom(dyp, w_t, (1, 1), pad_t, dil, H, W, acc=_join_acc(ctx, x, C0))
            dx = _give(ctx, x, _join_finish(ctx, dx[..., :C0] if C != C0 else dx))
        if ctx.needs_input_grad[1]:
            if wgrad_eligible(C, Kp, M):
                dw = conv2d_wgrad(x, dyp, R, S, st, pad, dil, layout=ctx.w_layout)[:K0, :C0]
            else:
                dw = _direct_wgrad(x[..., :C0].contiguous(), dy, R, S, st, pad, dil, C0, K0)
            dw = dw.to(wdt)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum((0, 1, 2)).to(wdt)
        return dx, dw, db, None, None, None, None, None, None, None


def _join_acc(ctx, x, C0):
    """The joined residual gradient when the data-gradient kernel can accumulate into it (same
    NHWC shape and dtype as dX, no channel padding); it is then consumed."""
    j = ctx.join
    d = j.dres if j is not None else None
    if d is None or x.shape[-1] != C0 or d.shape != x.shape or d.dtype != x.dtype or not d.is_contiguous():
        return None
    j.dres = None
    return d


def _join_finish(ctx, dx):
    """dX plus a joined residual gradient the kernel did not take; the join is closed (a giver
    whose backward comes later returns its gradient itself)."""
    j = ctx.join
    if j is not None:
        if j.dres is not None:
            dx = dx + j.dres.to(dx.dtype)
            j.dres = None
        j.armed = False
    return dx


_WSRC = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
WPREP = os.environ.get("PIAMD_CONV_WPREP", "1") != "0"


def _wprep_ok(x, weight):
    """One-launch filter preparation (``conv_wprep.hip``) for this conv's weight."""
    return (WPREP and x.is_cuda and weight.is_cuda and weight.dim() == 4 and weight.dtype in _WSRC
            and x.dtype in (torch.bfloat16, torch.float16) and _lib.has("piamd_conv_wprep"))


# ------------------------------------------------------------------------- dense fp32 (split bf16)
FP32_SPLIT = True  # dense fp32 convs on the split-bf16 MFMA path (False: the library, exact fp32)


def _split2(t):
    """t (f32) → (hi, lo) bf16 with t ≈ hi + lo to ≈2^-17 relative."""
    hi = t.to(torch.bfloat16)
    return hi, (t - hi.float()).to(torch.bfloat16)


def _cat_c(parts, n):
    """Concatenate NHWC (or OHWI) tensors along the last dim, each zero-padded to n."""
    return torch.cat([_padc(p, n) for p in parts], -1).contiguous()


def _stem_f32(x, w, st, pad, dil):
    """Stem-mode (≤ 8 input channels) convolution with f32 output: x [N,H,W,Cs] bf16, w [K,Cs,R,S]."""
    K, Cs, R, S = w.shape
    nk = -(-(R * S) // 8)
    w8 = torch.zeros(K, nk * 64, dtype=w.dtype, device=w.device)
    w8[:, :R * S * 8].view(K, R, S, 8)[..., :Cs] = w.permute(0, 2, 3, 1)
    return _launch(_padc(x, 8).contiguous(), w8.view(K, 1, nk * 8, 8), None, st, pad, dil, 0,
                   rs=(R, S), out_f32=True)


class _Conv2dF32(torch.autograd.Function):
    """Dense fp32 conv on the bf16 MFMA implicit GEMM, as three bf16 products accumulated in f32 by
    the MFMA itself: x·w ≈ x_hi·w_hi + x_lo·w_hi + x_hi·w_lo (x = x_hi + x_lo, both bf16). The
    three products are ONE convolution over channel-concatenated operands ([x_hi, x_lo, x_hi] ·
    [w_hi, w_hi, w_lo]) written in f32, so the error is ≈2^-16 relative per product (fp32 storage,
    well inside TF32-class accuracy) at three bf16 MACs per fp32 MAC — a third of the bf16 rate, ~2.7×
    the chip's fp32-MFMA peak. Data gradient: the same concatenation over dY and the flipped filter
    (stride 1) or the per-phase sub-convolutions (strided); weight gradient: the implicit-GEMM
    wgrad kernel over batch-stacked [x_hi; x_lo; x_hi] and [dy_hi; dy_hi; dy_lo].
    x [N,H,W,C0] f32 contiguous, weight [K0,C0,R,S]."""

    @staticmethod
    def forward(ctx, x, weight, bias, st, pad, dil):
        K0, C0, R, S = weight.shape
        K = -(-K0 // 4) * 4
        wf = weight.float()
        if K != K0:
            wf = torch.nn.functional.pad(wf, (0, 0, 0, 0, 0, 0, 0, K - K0))
        xh, xl = _split2(x)
        wh, wl = _split2(wf)
        if 2 * C0 <= 8:  # stem mode: [x_hi, x_lo]·[w_hi, w_hi] + x_hi·w_lo
            y = _stem_f32(torch.cat([xh, xl], -1), torch.cat([wh, wh], 1), st, pad, dil)
            y += _stem_f32(xh, wl, st, pad, dil)
        else:
            C = _pad64(C0)
            whp, wlp = wh.permute(0, 2, 3, 1), wl.permute(0, 2, 3, 1)
            y = _launch(_cat_c((xh, xl, xh), C), _cat_c((whp, whp, wlp), C), None, st, pad, dil, 0,
                        out_f32=True)
        if K != K0:
            y = y[..., :K0].contiguous()
        if bias is not None:
            y += bias.float()
        ctx.save_for_backward(xh, xl, wh[:K0], wl[:K0])
        ctx.cfg = (st, pad, dil, bias is not None, weight.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        xh, xl, wh, wl = ctx.saved_tensors
        st, pad, dil, has_bias, wdt = ctx.cfg
        dy = dy.float().contiguous()
        K0, C0, R, S = wh.shape
        N, H, W, _ = xh.shape
        M = dy.shape[0] * dy.shape[1] * dy.shape[2]
        dyh, dyl = _split2(dy)
        Kp = _pad64(K0)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            C4 = -(-C0 // 4) * 4  # data-gradient output channels: 4 per epilogue lane
            pw = (0, 0, 0, 0, 0, C4 - C0, 0, Kp - K0)
            whp, wlp = torch.nn.functional.pad(wh, pw), torch.nn.functional.pad(wl, pw)
            d3 = _cat_c((dyh, dyl, dyh), Kp)
            if st == (1, 1) and dy.shape[1:3] == (H, W):
                pad_t = (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1])
                fh, fl = (t.flip(2, 3).permute(1, 2, 3, 0) for t in (whp, wlp))
                dx = _launch_geom(d3, _cat_c((fh, fh, fl), Kp), (1, 1), pad_t, dil, H, W, out_f32=True)
            else:
                dx = conv2d_dgrad_strided(d3, torch.cat([whp, whp, wlp], 0), H, W, st, pad, dil,
                                          out_f32=True)
            dx = dx[..., :C0]
        if ctx.needs_input_grad[1]:
            C8 = -(-C0 // 8) * 8
            if wgrad_eligible(C8, Kp, 3 * M):
                x3 = torch.cat([_padc(xh, C8), _padc(xl, C8), _padc(xh, C8)], 0).contiguous()
                d3w = torch.cat([_padc(dyh, Kp), _padc(dyh, Kp), _padc(dyl, Kp)], 0).contiguous()
                dw = conv2d_wgrad(x3, d3w, R, S, st, pad, dil)[:K0, :C0]
            else:  # ≥ 2^24 stacked pixels: the direct kernel's exact f32 reduction
                xf = xh.float() + xl.float()
                dw = _direct_wgrad(xf.contiguous(), dy, R, S, st, pad, dil, C0, K0)
            dw = dw.to(wdt)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.sum((0, 1, 2)).to(wdt)
        return dx, dw, db, None, None, None


# ---------------------------------------------------------------- direct grouped / depthwise conv
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _direct_v(dt, K, kg, dw):
    vmax = 4 if dt == torch.float32 else 8
    return vmax if K % vmax == 0 and (dw or kg % vmax == 0) else 1


def _direct_wgrad(x, dy, R, S, st, pad, dil, C, K, groups=1):
    """dW [K][C/groups][R][S] f32 on the direct kernel's deterministic split reduction."""
    N, H, W, _ = x.shape
    _, OH, OW, _ = dy.shape
    cg, kg = C // groups, K // groups
    M = N * OH * OW
    v = _direct_v(x.dtype, K, kg, cg == 1 and kg == 1)
    ncol = (K // v) * cg
    cb = 1
    while cb < ncol and cb < 64:
        cb *= 2
    gy, gz, pl = -(-ncol // cb), -(-(R * S) // 9), 256 // cb
    plane = R * S * cg * K
    parts = max(1, min(-(-2048 // (gy * gz)), M // (pl * 8), (16 << 20) // plane))
    # depthwise 3x3 (pad 1, stride 1/2, 16-bit): the sliding-window kernel fixes its own split
    fast = _lib.lib().piamd_dconv2d_wgrad_parts(N, H, W, C, OH, OW, K, R, S, st[0], st[1], pad[0], pad[1],
                                               dil[0], dil[1], cg, kg, _DT[x.dtype])
    if fast > 0:
        parts = int(fast)
    d = torch.empty(plane, dtype=torch.float32, device=x.device)
    ws = torch.empty((parts + 64) * plane, dtype=torch.float32, device=x.device)  # + slice sums
    _lib.call("piamd_dconv2d_wgrad", x.data_ptr(), dy.data_ptr(), d.data_ptr(), ws.data_ptr(), parts,
              N, H, W, C, OH, OW, K, R, S, st[0], st[1], pad[0], pad[1], dil[0], dil[1], cg, kg,
              _DT[x.dtype], _lib.stream())
    return d.view(R, S, cg, K).permute(3, 2, 0, 1)


def _direct(inp, w_rsck, bias, OH, OW, Cout, R, S, st, pad, dil, cin_g, cout_g, transposed):
    N, H, W, Cin = inp.shape
    out = torch.empty(N, OH, OW, Cout, dtype=inp.dtype, device=inp.device)
    _lib.call("piamd_dconv2d", inp.data_ptr(), w_rsck.data_ptr(), _lib.ptr(bias), out.data_ptr(),
              N, H, W, Cin, OH, OW, Cout, R, S, st[0], st[1], pad[0], pad[1], dil[0], dil[1],
              cin_g, cout_g, int(transposed), _DT[inp.dtype], _lib.stream())
    return out


class _ConvDirect(torch.autograd.Function):
    """Grouped / depthwise conv, x [N,H,W,C] (f32, bf16 or fp16), weight [K, C/groups, R, S]."""

    @staticmethod
    def forward(ctx, x, weight, bias, st, pad, dil, groups):
        dt = x.dtype
        N, H, W, C = x.shape
        K, cg, R, S = weight.shape
        kg = K // groups
        OH, OW = _out_hw(H, W, R, S, st, pad, dil)
        if OH < 1 or OW < 1:
            raise ValueError("convolution output is empty")
        w_rsck = weight.to(dt).permute(2, 3, 1, 0).contiguous()  # W'[r][s][c][k]
        b = bias.to(dt).contiguous() if bias is not None else None
        y = _direct(x, w_rsck, b, OH, OW, K, R, S, st, pad, dil, cg, kg, False)
        ctx.save_for_backward(x, weight)
        ctx.cfg = (st, pad, dil, groups, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        st, pad, dil, groups, has_bias = ctx.cfg
        dt = x.dtype
        dy = dy.to(dt).contiguous()
        N, H, W, C = x.shape
        K, cg, R, S = weight.shape
        kg = K // groups
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            # transposed geometry: in = dY (K channels, groups of kg), out = dX (C, groups of cg),
            # W''[r][s][k_local][c] = W[g·kg + k_local][c − g·cg][r][s]
            w_t = (weight.to(dt).view(groups, kg, cg, R, S).permute(3, 4, 1, 0, 2)
                   .reshape(R, S, kg, C).contiguous())
            dx = _direct(dy, w_t, None, H, W, C, R, S, st, pad, dil, kg, cg, True)
        if ctx.needs_input_grad[1]:
            dw = _direct_wgrad(x, dy, R, S, st, pad, dil, C, K, groups).to(weight.dtype)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum((0, 1, 2)).to(weight.dtype)
        return dx, dw, db, None, None, None, None


def _tall_wgrad(dy2, x2):
    """dyᵀ·x [K, C] (f32) of a 1×1 conv over M ≫ K, C pixel rows: the own assembly GEMM (split-K
    over the pixel rows into f32 planes, reduced in a fixed order — `ops.linear.wgrad_into`). A
    library GEMM with a K×C output had only a handful of output tiles (hipBLASLt: 10-19
    workgroups, ~1 ms at MobileNetV2's 112×112 layers, profiles/conv_nets_r3.txt)."""
    from .gemm import own_dtype
    if own_dtype(dy2, x2):
        from .linear import wgrad_into
        out = torch.zeros((dy2.shape[1], x2.shape[1]), dtype=torch.float32, device=dy2.device)
        return wgrad_into(out, dy2.contiguous(), x2.contiguous())
    M, K = dy2.shape
    C = x2.shape[1]
    S = 1
    while S < 256 and M % (2 * S) == 0 and M // (2 * S) >= 2048:
        S *= 2
    if S == 1:
        return torch.mm(dy2.t(), x2).float()
    a3 = dy2.view(S, M // S, K).transpose(1, 2)
    b3 = x2.contiguous().view(S, M // S, C)
    try:
        part = torch.bmm(a3, b3, out_dtype=torch.float32)
    except (RuntimeError, TypeError, NotImplementedError):
        part = torch.bmm(a3, b3).float()
    return part.sum(0)


class _Conv1x1(torch.autograd.Function):
    """Dense 1×1 conv with channels off the 64-grid as a GEMM over pixel rows on the framework's
    GEMMs (forward ops.linear.mm_nt, data gradient ops.gemm.matmul, weight gradient wgrad_into)."""

    @staticmethod
    def forward(ctx, x, weight, bias, st):
        from .linear import mm_nt
        dt = x.dtype
        xs = x[:, ::st[0], ::st[1]] if st != (1, 1) else x
        N, OH, OW, C = xs.shape
        K = weight.shape[0]
        x2 = xs.reshape(-1, C)
        w_kc = weight.to(dt).reshape(K, C)
        y2 = mm_nt(x2, w_kc, bias.to(dt) if bias is not None else None)
        ctx.save_for_backward(x2, w_kc)
        ctx.cfg = (tuple(x.shape), st, bias is not None, weight.dtype)
        return y2.view(N, OH, OW, K)

    @staticmethod
    def backward(ctx, dy):
        x2, w_kc = ctx.saved_tensors
        xshape, st, has_bias, wdt = ctx.cfg
        K, C = w_kc.shape
        dy2 = dy.to(x2.dtype).reshape(-1, K)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            from .gemm import matmul as _mm
            dx2 = _mm(dy2, w_kc)
            if st != (1, 1):
                dx = torch.zeros(xshape, dtype=x2.dtype, device=x2.device)
                dx[:, ::st[0], ::st[1]] = dx2.view(dy.shape[:3] + (C,))
            else:
                dx = dx2.view(xshape)
        if ctx.needs_input_grad[1]:
            dw = _tall_wgrad(dy2, x2).view(K, C, 1, 1).to(wdt)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy2.float().sum(0).to(wdt)
        return dx, dw, db, None


def conv2d_any(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, nhwc=False):
    """Own-kernel route for a 2-D conv of a GPU tensor (NCHW or NHWC by ``nhwc``); ``None`` when
    the call stays on the library (string padding, or dense fp32 with ``FP32_SPLIT`` off)."""
    if not (HIP_CONV and x.is_cuda and x.dim() == 4 and weight.dim() == 4) or isinstance(padding, str):
        return None
    pad, st, dil = _pair(padding), _pair(stride), _pair(dilation)
    if len(pad) != 2 or len(st) != 2 or len(dil) != 2:
        return None
    dt = x.dtype
    if torch.is_autocast_enabled("cuda") and dt in _DT:
        dt = torch.get_autocast_dtype("cuda")
    if dt not in _DT:
        return None
    C = x.shape[-1] if nhwc else x.shape[1]
    K, cg, R, S = weight.shape
    if cg * groups != C or K % groups:
        raise ValueError(f"conv2d: weight {tuple(weight.shape)} does not match {C} input channels "
                         f"in {groups} groups")
    if groups == 1 and dt == torch.float32:
        if not FP32_SPLIT:
            _lib.fallback("conv2d", "dense fp32 conv with FP32_SPLIT off (library)")
            return None
        with torch.autocast("cuda", enabled=False):
            xf = (x if nhwc else x.permute(0, 2, 3, 1)).float().contiguous()
            y = _Conv2dF32.apply(xf, weight, bias, st, pad, dil)
        return y if nhwc else y.permute(0, 3, 1, 2)
    with torch.autocast("cuda", enabled=False):
        xh = (x if nhwc else x.permute(0, 2, 3, 1)).to(dt)
        xh = xh.contiguous()  # a view for NHWC / channels_last storage; one re-layout otherwise
        if groups > 1:
            y = _ConvDirect.apply(xh, weight, bias, st, pad, dil, groups)
        elif R == S == 1 and pad == (0, 0) and C % 64 and C > 8:
            y = _Conv1x1.apply(xh, weight, bias, st)
        else:
            want = BN_STATS and bias is None and torch.is_grad_enabled()
            join = _take_join()
            if join is not None:
                join.armed = True
            y = _Conv2dNHWC.apply(xh, weight, bias, st, pad, dil, 0, want, join, _take_give())
            part = _take_stats() if want else None
            out = y if nhwc else y.permute(0, 3, 1, 2)
            if part is not None:  # consumed by a BatchNorm of this very tensor (same version)
                out._piamd_bn_part = (part[0], part[1], out._version)
            return out
    return y if nhwc else y.permute(0, 3, 1, 2)


class _ConvTranspose(torch.autograd.Function):
    """Transposed conv, x [N,H,W,Cin], weight [Cin, Cout/groups, R, S]: the forward is the data
    gradient of the conv it transposes (dense half → the MFMA phase decomposition, else the direct
    kernel's transposed geometry); its data gradient is that conv's forward and its weight gradient
    that conv's weight gradient with the roles of input and output swapped."""

    @staticmethod
    def forward(ctx, x, weight, bias, st, pad, out_pad, dil, groups):
        dt = x.dtype
        N, H, W, Cin = x.shape
        _, og, R, S = weight.shape
        Cout = og * groups
        Ho = (H - 1) * st[0] - 2 * pad[0] + dil[0] * (R - 1) + out_pad[0] + 1
        Wo = (W - 1) * st[1] - 2 * pad[1] + dil[1] * (S - 1) + out_pad[1] + 1
        if groups == 1 and dt in _HALF:
            Kp, Cp = _pad64(Cin), -(-Cout // 4) * 4
            wq = torch.nn.functional.pad(weight.to(dt), (0, 0, 0, 0, 0, Cp - Cout, 0, Kp - Cin))
            y = conv2d_dgrad_strided(_padc(x, Kp).contiguous(), wq, Ho, Wo, st, pad, dil)
            y = y[..., :Cout]
            if bias is not None:
                y = y + bias.to(dt)
            y = y.contiguous()
        elif groups == 1 and dt == torch.float32:  # split-bf16 products (see _Conv2dF32)
            Kp, Cp = _pad64(Cin), -(-Cout // 4) * 4
            pw = (0, 0, 0, 0, 0, Cp - Cout, 0, Kp - Cin)
            xh, xl = _split2(x)
            wh, wl = (torch.nn.functional.pad(t, pw) for t in _split2(weight.float()))
            y = conv2d_dgrad_strided(_cat_c((xh, xl, xh), Kp), torch.cat([wh, wh, wl], 0), Ho, Wo,
                                     st, pad, dil, out_f32=True)[..., :Cout]
            if bias is not None:
                y = y + bias.float()
            y = y.contiguous()
        else:
            w_t = (weight.to(dt).view(groups, Cin // groups, og, R, S).permute(3, 4, 1, 0, 2)
                   .reshape(R, S, Cin // groups, Cout).contiguous())
            b = bias.to(dt).contiguous() if bias is not None else None
            y = _direct(x, w_t, b, Ho, Wo, Cout, R, S, st, pad, dil, Cin // groups, og, True)
        ctx.save_for_backward(x, weight)
        ctx.cfg = (st, pad, dil, groups, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        st, pad, dil, groups, has_bias = ctx.cfg
        dt = x.dtype
        dy = dy.to(dt).contiguous()
        N, H, W, Cin = x.shape
        _, og, R, S = weight.shape
        Cout = og * groups
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if groups == 1 and dt in _HALF:
                dx = _Conv2dNHWC.apply(dy, weight, None, st, pad, dil, 0)
            elif groups == 1 and dt == torch.float32:
                dx = _Conv2dF32.apply(dy, weight, None, st, pad, dil)
            else:
                dx = _ConvDirect.apply(dy, weight, None, st, pad, dil, groups)
            dx = dx[:, :H, :W]
        if ctx.needs_input_grad[1]:
            if groups == 1 and dt in _HALF and wgrad_eligible(8, 64, N * H * W):
                Cp, Kp = -(-Cout // 8) * 8, _pad64(Cin)
                dw = conv2d_wgrad(_padc(dy, Cp).contiguous(), _padc(x, Kp).contiguous(), R, S, st,
                                  pad, dil)[:Cin, :Cout]
            elif groups == 1 and dt == torch.float32 and wgrad_eligible(8, 64, 3 * N * H * W):
                Cp, Kp = -(-Cout // 8) * 8, _pad64(Cin)
                dyh, dyl = _split2(dy)
                xh, xl = _split2(x)
                d3 = torch.cat([_padc(dyh, Cp), _padc(dyl, Cp), _padc(dyh, Cp)], 0).contiguous()
                x3 = torch.cat([_padc(xh, Kp), _padc(xh, Kp), _padc(xl, Kp)], 0).contiguous()
                dw = conv2d_wgrad(d3, x3, R, S, st, pad, dil)[:Cin, :Cout]
            else:
                dw = _direct_wgrad(dy, x, R, S, st, pad, dil, Cout, Cin, groups)
            dw = dw.to(weight.dtype)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum((0, 1, 2)).to(weight.dtype)
        return dx, dw, db, None, None, None, None, None, None


def conv2d_transpose_any(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                         dilation=1, nhwc=False, output_size=None):
    """Own-kernel route for ``conv2d_transpose`` of a GPU tensor; ``None`` → library (string
    padding, or dense fp32 with ``FP32_SPLIT`` off)."""
    if not (HIP_CONV and x.is_cuda and x.dim() == 4 and weight.dim() == 4) or isinstance(padding, str):
        return None
    pad, st, dil, op = _pair(padding), _pair(stride), _pair(dilation), _pair(output_padding)
    if len(pad) != 2:
        return None
    dt = x.dtype
    if torch.is_autocast_enabled("cuda") and dt in _DT:
        dt = torch.get_autocast_dtype("cuda")
    if dt not in _DT:
        return None
    Cin = x.shape[-1] if nhwc else x.shape[1]
    if weight.shape[0] != Cin or Cin % groups:
        raise ValueError(f"conv2d_transpose: weight {tuple(weight.shape)} does not match {Cin} "
                         f"input channels in {groups} groups")
    H, W = (x.shape[1:3] if nhwc else x.shape[2:4])
    R, S = weight.shape[2:]
    if output_size is not None:
        osz = list(output_size)[-2:]
        op = tuple(osz[i] - ((H, W)[i] - 1) * st[i] + 2 * pad[i] - dil[i] * ((R, S)[i] - 1) - 1
                   for i in range(2))
        if any(o < 0 or o >= max(st[i], dil[i]) for i, o in enumerate(op)):
            raise ValueError(f"conv2d_transpose: output_size {output_size} is not reachable")
    if groups == 1 and dt == torch.float32 and not FP32_SPLIT:
        _lib.fallback("conv2d_transpose", "dense fp32 transposed conv with FP32_SPLIT off (library)")
        return None
    with torch.autocast("cuda", enabled=False):
        xh = (x if nhwc else x.permute(0, 2, 3, 1)).to(dt).contiguous()
        y = _ConvTranspose.apply(xh, weight, bias, st, pad, op, dil, groups)
    return y if nhwc else y.permute(0, 3, 1, 2)


def conv2d_nhwc(x, weight, bias=None, stride=1, padding=0, dilation=1, act=None):
    """y[N,OH,OW,K] = act(conv(x[N,H,W,C], weight[K,C,R,S]) + bias) on the MFMA kernel, in x's
    dtype when bf16/fp16 (else bf16)."""
    if not (x.is_cuda and x.dim() == 4):
        raise ValueError("conv2d_nhwc needs a 4-D GPU tensor")
    if not eligible(x.shape, weight.shape, 1, padding):
        raise ValueError(f"conv2d_nhwc: unsupported shapes x{tuple(x.shape)} w{tuple(weight.shape)}")
    if act not in _ACT:
        raise ValueError(f"conv2d_nhwc: unsupported activation {act}")
    st, pad, dil = _pair(stride), _pair(padding), _pair(dilation)
    xh = x if x.dtype in _HALF else x.to(torch.bfloat16)
    return _Conv2dNHWC.apply(xh, weight, bias, st, pad, dil, _ACT[act])


def conv2d_nchw(x, weight, bias=None, stride=1, padding=0, dilation=1, act=None):
    """Same kernel for an NCHW-indexed tensor: channels_last storage is used as is (a view)."""
    y = conv2d_nhwc(x.permute(0, 2, 3, 1), weight, bias, stride, padding, dilation, act)
    return y.permute(0, 3, 1, 2)


# ------------------------------------------------------------------------- 3-D / 1-D transposed
def _triple(v):
    v = tuple(v) if isinstance(v, (list, tuple)) else (v, v, v)
    return v if len(v) == 3 else (v[0],) * 3


def conv3d_any(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, ndhwc=False):
    """Own-kernel route for a 3-D conv of a GPU tensor (reference `phi/kernels/gpudnn/
    conv_kernel.cu:456`): the kd depth taps are kd 2-D convs on the framework's kernels
    (`conv2d_any`: MFMA implicit GEMM / direct / split-bf16 fp32), each over the batch of output
    depths (input depth d·s − p + z·dil gathered channels-last), summed in f32 — no MIOpen.
    ``None`` when the call stays on the library (string padding)."""
    if not (HIP_CONV and x.is_cuda and x.dim() == 5 and weight.dim() == 5) or isinstance(padding, str):
        return None
    st, pad, dil = _triple(stride), _triple(padding), _triple(dilation)
    xl = x if ndhwc else x.permute(0, 2, 3, 4, 1)                     # [N, D, H, W, C]
    N, D, H, W, C = xl.shape
    K, cg, kd, kh, kw = weight.shape
    Do = (D + 2 * pad[0] - dil[0] * (kd - 1) - 1) // st[0] + 1
    if Do <= 0:
        return None
    if pad[0]:
        xl = torch.nn.functional.pad(xl, (0, 0, 0, 0, 0, 0, pad[0], pad[0]))
    base = torch.arange(Do, device=x.device) * st[0]
    y = None
    for z in range(kd):
        xs = xl.index_select(1, base + z * dil[0]).reshape(N * Do, H, W, C)
        yz = conv2d_any(xs, weight[:, :, z], None, st[1:], pad[1:], dil[1:], groups, nhwc=True)
        if yz is None:
            return None
        y = yz.float() if y is None else y + yz.float()
    Ho, Wo = y.shape[1], y.shape[2]
    if bias is not None:
        y = y + bias.float()
    y = y.to(yz.dtype).reshape(N, Do, Ho, Wo, K)
    return y if ndhwc else y.permute(0, 4, 1, 2, 3)


def conv3d_transpose_any(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                         dilation=1, ndhwc=False, output_size=None):
    """Own-kernel route for ``conv3d_transpose``: per depth tap z a 2-D transposed conv
    (`conv2d_transpose_any`) over all input depths, scattered (index_add) to output depths
    d·s + z·dil of the uncropped volume, then cropped by the depth padding."""
    if not (HIP_CONV and x.is_cuda and x.dim() == 5 and weight.dim() == 5) or isinstance(padding, str):
        return None
    st, pad, dil, op = _triple(stride), _triple(padding), _triple(dilation), _triple(output_padding)
    xl = x if ndhwc else x.permute(0, 2, 3, 4, 1)                     # [N, D, H, W, Cin]
    N, D, H, W, Cin = xl.shape
    _, og, kd, kh, kw = weight.shape
    if output_size is not None:
        osz = list(output_size)[-3:]
        op = tuple(osz[i] - ((D, H, W)[i] - 1) * st[i] + 2 * pad[i] - dil[i] * ((kd, kh, kw)[i] - 1) - 1
                   for i in range(3))
    Do = (D - 1) * st[0] - 2 * pad[0] + dil[0] * (kd - 1) + op[0] + 1
    full = (D - 1) * st[0] + dil[0] * (kd - 1) + 1
    xs = xl.reshape(N * D, H, W, Cin)
    out = None
    base = torch.arange(D, device=x.device) * st[0]
    for z in range(kd):
        yz = conv2d_transpose_any(xs, weight[:, :, z], None, st[1:], pad[1:], op[1:], groups, dil[1:],
                                  nhwc=True)
        if yz is None:
            return None
        Ho, Wo, Co = yz.shape[1:]
        yz = yz.float().reshape(N, D, Ho, Wo, Co)
        if out is None:
            out = torch.zeros((N, max(full, pad[0] + Do), Ho, Wo, Co), dtype=torch.float32, device=x.device)
        out = out.index_add(1, base + z * dil[0], yz)
    out = out[:, pad[0]:pad[0] + Do]
    if bias is not None:
        out = out + bias.float()
    out = out.to(yz.dtype if yz is not None else x.dtype)
    return out if ndhwc else out.permute(0, 4, 1, 2, 3)


def conv1d_transpose_any(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                         dilation=1, nlc=False, output_size=None):
    """``conv1d_transpose`` as a 1 × L transposed 2-D conv on the own kernels."""
    one = lambda v: v[0] if isinstance(v, (list, tuple)) else v  # noqa: E731
    if not (HIP_CONV and x.is_cuda and x.dim() == 3) or isinstance(padding, str):
        return None
    xi = x.unsqueeze(1) if nlc else x.unsqueeze(2)
    osz = None if output_size is None else [1, list(output_size)[-1]] if isinstance(output_size, (list, tuple)) \
        else [1, output_size]
    y = conv2d_transpose_any(xi, weight.unsqueeze(2), bias, (1, one(stride)), (0, one(padding)),
                             (0, one(output_padding)), groups, (1, one(dilation)), nhwc=nlc, output_size=osz)
    if y is None:
        return None
    return y.squeeze(1) if nlc else y.squeeze(2)
