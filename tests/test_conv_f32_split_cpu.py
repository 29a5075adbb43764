"""The split-bf16 fp32 convolution (`ops.conv._Conv2dF32`): the operand arrangement it hands the MFMA
kernel — channels [x_hi, x_lo, x_hi] against filter channels [w_hi, w_hi, w_lo], and the batch-
stacked weight-gradient operands — reproduces the fp64 convolution to ~2^-16, emulated here with
PyTorch convolutions over the bf16-valued parts in f64 (what the kernel's f32 MFMA accumulation
computes, up to summation order)."""
import torch

from paddle_infer_amd.ops.conv import _split2


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def test_split2_residual():
    x = torch.randn(4096, dtype=torch.float32) * 10
    hi, lo = _split2(x)
    assert hi.dtype == lo.dtype == torch.bfloat16
    err = (hi.double() + lo.double() - x.double()).abs() / x.double().abs()
    assert err.max().item() < 2 ** -16


def test_split_products_match_fp64_conv():
    torch.manual_seed(0)
    N, C, H, W, K, R = 2, 24, 11, 9, 16, 3
    x = torch.randn(N, C, H, W)
    w = torch.randn(K, C, R, R) / (C * R * R) ** 0.5
    ref = torch.nn.functional.conv2d(x.double(), w.double(), padding=1)
    xh, xl = (t.double() for t in _split2(x))
    wh, wl = (t.double() for t in _split2(w))
    x3 = torch.cat([xh, xl, xh], 1)
    w3 = torch.cat([wh, wh, wl], 1)
    y = torch.nn.functional.conv2d(x3, w3, padding=1)
    assert _rel(y, ref) < 2e-5
    # one bf16 product alone is ~2^-9: the split is what buys the precision
    assert _rel(torch.nn.functional.conv2d(xh, wh, padding=1), ref) > 5e-4
    # weight gradient: batch-stacked [x_hi; x_lo; x_hi] against [dy_hi; dy_hi; dy_lo]
    dy = torch.randn(ref.shape)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    torch.nn.functional.conv2d(xr, wr, padding=1).backward(dy.double())
    dyh, dyl = (t.double() for t in _split2(dy))
    xs = torch.cat([xh, xl, xh], 0)
    dys = torch.cat([dyh, dyh, dyl], 0)
    dw = torch.nn.grad.conv2d_weight(xs, w.shape, dys, padding=1)
    assert _rel(dw, wr.grad) < 2e-5
