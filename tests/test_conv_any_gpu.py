"""Every 2-D conv route of ``ops.conv.conv2d_any`` against a PyTorch fp32 reference of the same op:
depthwise / grouped (direct NHWC kernels, f32 / bf16 / fp16), dense fp32 (split-bf16 products on the
MFMA kernel), dense fp16 and channel counts off the
64-grid (MFMA implicit GEMM with zero-padded channels), 1×1 convs as GEMMs, plain NCHW inputs
(re-laid-out once, channels_last output), conv1d; and a MobileNetV2 bf16 training step whose
profile holds no library (MIOpen) convolution or batch-norm op."""
import pytest
import torch

import paddle_infer_amd as paddle
import paddle_infer_amd.nn.functional as F
from paddle_infer_amd.ops import conv as CV

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 2e-5, torch.bfloat16: 1.2e-2, torch.float16: 2e-3}


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _check(dt, N, C, H, W, K, R, st, pad, dil, groups, nchw=False, bias=True):
    g = torch.Generator(device="cuda").manual_seed(C * 131 + K + R)
    x = torch.randn(N, C, H, W, device="cuda", generator=g)
    w = torch.randn(K, C // groups, R, R, device="cuda", generator=g) / (C // groups * R * R) ** 0.5
    b = torch.randn(K, device="cuda", generator=g) if bias else None
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True) if bias else None
    with torch.backends.cudnn.flags(enabled=True, deterministic=True, allow_tf32=False):
        yr = torch.nn.functional.conv2d(xr, wr, br, st, pad, dil, groups)
    dy = torch.randn(yr.shape, device="cuda", generator=g)
    yr.backward(dy)

    xi = x.to(dt)
    xi = xi if nchw else xi.contiguous(memory_format=torch.channels_last)
    xi.requires_grad_(True)
    wi = w.clone().requires_grad_(True)
    bi = b.clone().requires_grad_(True) if bias else None
    y = CV.conv2d_any(xi, wi, bi, st, pad, dil, groups)
    assert y is not None
    assert y.dtype == dt and y.shape == yr.shape
    assert y.is_contiguous(memory_format=torch.channels_last)
    y.backward(dy.to(dt))
    tol = TOL[dt]
    assert _rel(y, yr) < tol, ("y", _rel(y, yr))
    assert _rel(xi.grad, xr.grad) < tol, ("dx", _rel(xi.grad, xr.grad))
    assert _rel(wi.grad, wr.grad) < tol * (2 if dt != torch.float32 else 5), ("dw", _rel(wi.grad, wr.grad))
    if bias:
        assert _rel(bi.grad, br.grad) < tol, ("db", _rel(bi.grad, br.grad))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [
    # N, C, H, W, K, R, st, pad, dil
    (2, 32, 14, 14, 32, 3, 1, 1, 1),      # depthwise 3x3
    (2, 96, 15, 15, 96, 3, 2, 1, 1),      # depthwise stride 2, odd size
    (2, 40, 12, 12, 40, 5, 1, 2, 1),      # 5x5: two tap slices in the weight gradient
    (1, 24, 13, 11, 24, 3, 1, 2, 2),      # dilation 2
    (2, 16, 10, 10, 32, 3, 1, 1, 1),      # channel multiplier 2
    # sliding-window 3x3 weight gradient (dw3_wgrad_kernel): row segments, 1..120 channel vectors
    (2, 8, 9, 37, 8, 3, 1, 1, 1),         # one channel vector, 3 row segments of 13
    (1, 960, 7, 7, 960, 3, 1, 1, 1),      # 120 channel vectors (2 slots per workgroup)
    (2, 144, 34, 34, 144, 3, 2, 1, 1),    # stride 2, even size, 2 segments
    (3, 48, 20, 33, 48, 3, 2, 1, 1),      # stride 2, non-square
])
def test_depthwise(dt, shape):
    N, C, H, W, K, R, st, pad, dil = shape
    _check(dt, N, C, H, W, K, R, st, pad, dil, groups=C)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,groups", [
    ((2, 32, 12, 12, 64, 3, 1, 1, 1), 4),   # grouped, 8 in / 16 out per group
    ((2, 64, 9, 9, 64, 3, 2, 1, 1), 32),    # ResNeXt-style narrow groups (2 in / 2 out)
    ((2, 12, 8, 8, 18, 1, 1, 0, 1), 3),     # grouped 1x1, lanes of width 1
])
def test_grouped(dt, shape, groups):
    N, C, H, W, K, R, st, pad, dil = shape
    _check(dt, N, C, H, W, K, R, st, pad, dil, groups=groups)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [
    (2, 64, 14, 14, 128, 3, 1, 1, 1),     # aligned: the tuned implicit GEMM
    (2, 48, 14, 14, 40, 3, 1, 1, 1),      # C and K off the 64-grid: zero-padded
    (2, 3, 32, 32, 32, 3, 2, 1, 1),       # stem mode (C <= 8)
    (2, 72, 13, 13, 36, 3, 2, 1, 1),      # strided dgrad with padded channels
])
def test_dense_half(dt, shape):
    N, C, H, W, K, R, st, pad, dil = shape
    _check(dt, N, C, H, W, K, R, st, pad, dil, groups=1)


@pytest.mark.parametrize("shape", [
    (2, 64, 14, 14, 128, 3, 1, 1, 1),     # aligned
    (2, 48, 13, 13, 40, 3, 2, 1, 1),      # unaligned channels, strided data gradient
    (2, 3, 32, 32, 32, 7, 2, 3, 1),       # stem (two stem-mode products)
    (2, 24, 14, 14, 144, 1, 1, 0, 1),     # 1x1
    (1, 32, 11, 9, 36, 3, 1, 2, 2),       # dilation 2
])
def test_dense_fp32_split(shape):
    """Dense fp32 convs (Paddle's default dtype) run on the MFMA kernels as three bf16 products
    accumulated in f32 — no library fallback, fp32-class error against the exact reference."""
    from paddle_infer_amd.ops import _lib
    _lib.FALLBACKS.clear()
    N, C, H, W, K, R, st, pad, dil = shape
    _check(torch.float32, N, C, H, W, K, R, st, pad, dil, groups=1)
    _check(torch.float32, N, C, H, W, K, R, st, pad, dil, groups=1, nchw=True, bias=False)
    assert not _lib.FALLBACKS, _lib.FALLBACKS


@pytest.mark.parametrize("st", [1, 2])
def test_pointwise_gemm_route(st):
    _check(torch.bfloat16, 2, 24, 14, 14, 144, 1, st, 0, 1, groups=1)
    _check(torch.float16, 2, 160, 7, 7, 40, 1, st, 0, 1, groups=1, bias=False)


def test_plain_nchw_input():
    """A contiguous NCHW tensor (Paddle's default layout) runs on the own kernels, once re-laid-out;
    the output is channels_last so the next layer takes the view."""
    _check(torch.bfloat16, 2, 64, 12, 12, 64, 3, 1, 1, 1, groups=1, nchw=True)
    _check(torch.float32, 2, 32, 12, 12, 32, 3, 1, 1, 1, groups=32, nchw=True)


def test_functional_conv1d_and_autocast():
    x = torch.randn(2, 32, 50, device="cuda")
    w = torch.randn(32, 1, 5, device="cuda")
    y = F.conv1d(x, w, None, 1, 2, 1, 32)
    ref = torch.nn.functional.conv1d(x, w, None, 1, 2, 1, 32)
    assert _rel(y, ref) < 2e-5
    # autocast: f32 input and weights compute in fp16 on the MFMA kernel
    x2 = torch.randn(2, 64, 10, 10, device="cuda").contiguous(memory_format=torch.channels_last)
    w2 = torch.randn(64, 64, 3, 3, device="cuda") / 24
    with torch.autocast("cuda", dtype=torch.float16):
        y2 = F.conv2d(x2, w2, padding=1)
    assert y2.dtype == torch.float16
    assert _rel(y2, torch.nn.functional.conv2d(x2, w2, padding=1)) < 2e-3


def test_mobilenet_v2_step_without_library_conv():
    """MobileNetV2 (depthwise 3x3, unaligned 1x1, stem) trains under bf16 autocast with every
    convolution and batch norm on the framework's kernels: the profile has no aten convolution or
    MIOpen op, and a few steps on a fixed batch reduce the loss."""
    from paddle_infer_amd.vision.models import mobilenet_v2
    torch.manual_seed(0)
    m = mobilenet_v2(num_classes=10).cuda().to(memory_format=torch.channels_last)
    opt = paddle.optimizer.Momentum(learning_rate=0.05, momentum=0.9, parameters=m.parameters())
    x = torch.randn(8, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        return loss.item()

    first = step()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        step()
    names = {e.key for e in prof.key_averages()}
    bad = sorted(n for n in names if "convolution" in n or "miopen" in n.lower()
                 or n in ("aten::batch_norm", "aten::native_batch_norm"))
    assert not bad, bad
    losses = [step() for _ in range(6)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < first


@pytest.mark.parametrize("dt,Cin,Cout,R,st,pad,op,groups", [
    (torch.bfloat16, 64, 32, 4, 2, 1, 0, 1),    # DCGAN-style upsampling, MFMA phases
    (torch.float16, 40, 24, 3, 2, 1, 1, 1),     # unaligned channels + output_padding
    (torch.bfloat16, 32, 32, 3, 1, 1, 0, 1),    # stride 1
    (torch.float32, 32, 64, 3, 2, 1, 1, 4),     # grouped, direct kernel
    (torch.float32, 40, 24, 3, 2, 1, 1, 1),     # dense fp32: split-bf16 MFMA phases
    (torch.bfloat16, 48, 48, 4, 2, 1, 0, 48),   # depthwise transposed
])
def test_conv2d_transpose(dt, Cin, Cout, R, st, pad, op, groups):
    g = torch.Generator(device="cuda").manual_seed(Cin + Cout)
    x = torch.randn(2, Cin, 9, 7, device="cuda", generator=g)
    w = torch.randn(Cin, Cout // groups, R, R, device="cuda", generator=g) / (Cin * R) ** 0.5
    b = torch.randn(Cout, device="cuda", generator=g)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.conv_transpose2d(xr, wr, br, st, pad, op, groups)
    dy = torch.randn(yr.shape, device="cuda", generator=g)
    yr.backward(dy)
    xi = x.to(dt).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wi, bi = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = F.conv2d_transpose(xi, wi, bi, st, pad, op, groups)
    assert y.dtype == dt and y.shape == yr.shape
    y.backward(dy.to(dt))
    tol = TOL[dt]
    assert _rel(y, yr) < tol, _rel(y, yr)
    assert _rel(xi.grad, xr.grad) < tol, _rel(xi.grad, xr.grad)
    assert _rel(wi.grad, wr.grad) < tol * (2 if dt != torch.float32 else 5), _rel(wi.grad, wr.grad)
    assert _rel(bi.grad, br.grad) < tol
    # output_size picks the output padding
    y2 = F.conv2d_transpose(xi.detach(), w, b, st, pad, 0, groups, output_size=list(yr.shape[2:]))
    assert y2.shape == yr.shape
