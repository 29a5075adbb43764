"""Fused BatchNorm (+ residual) (+ ReLU) HIP kernels (``batchnorm.hip``) against the plain
PyTorch fp32 reference: training / eval, NCHW / channels_last / NHWC, f32 / bf16, gradients of
x, gamma, beta and the residual, running-statistics update."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    assert err <= atol + rtol * b.abs().max().item(), err


def _ref(x, rm, rv, w, b, training, act, res):
    y = F.batch_norm(x.float(), rm, rv, w, b, training, 0.1, 1e-5)
    if res is not None:
        y = y + res.float()
    return torch.relu(y) if act == "relu" else y


@pytest.mark.parametrize("layout", ["nchw", "channels_last", "nhwc"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("C,residual", [(64, True), (96, False), (512, True), (2560, False),
                                        (36, True)])
def test_bn_act(layout, dtype, training, C, residual):
    from paddle_infer_amd.ops.batchnorm import batch_norm_act
    # NHWC / channels_last with C ∤ 256, C % 8 != 0, C < 256 (C = 36) runs the NCHW kernels on
    # channel-major copies: same parity bar
    torch.manual_seed(C)
    N, H, W = 4, 9, 7
    x = (torch.randn(N, C, H, W, device=DEV) * 2 + 0.5).to(dtype)
    res = torch.randn(N, C, H, W, device=DEV).to(dtype) if residual else None
    w = (torch.rand(C, device=DEV) + 0.5).requires_grad_(True)
    b = torch.randn(C, device=DEV).requires_grad_(True)
    rm, rv = torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5
    rm_ref, rv_ref = rm.clone(), rv.clone()
    if layout == "channels_last":
        xin = x.contiguous(memory_format=torch.channels_last)
        rin = res.contiguous(memory_format=torch.channels_last) if res is not None else None
        fmt = "NCHW"
    elif layout == "nhwc":
        xin = x.permute(0, 2, 3, 1).contiguous()
        rin = res.permute(0, 2, 3, 1).contiguous() if res is not None else None
        fmt = "NHWC"
    else:
        xin, rin, fmt = x, res, "NCHW"
    xin = xin.detach().requires_grad_(True)
    if rin is not None:
        rin = rin.detach().requires_grad_(True)
    y = batch_norm_act(xin, rm, rv, w, b, training, 0.9, 1e-5, "relu", rin, fmt)
    xr = x.detach().float().requires_grad_(True)
    rr = res.detach().float().requires_grad_(True) if res is not None else None
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yr = _ref(xr, rm_ref, rv_ref, wr, br, training, "relu", rr)
    yc = y.permute(0, 3, 1, 2) if layout == "nhwc" else y
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    _close(yc, yr, tol)
    if training:
        _close(rm, rm_ref, 1e-5)
        _close(rv, rv_ref, 1e-4)
    g = torch.randn_like(yr)
    gin = g.permute(0, 2, 3, 1).contiguous() if layout == "nhwc" else g
    ins = [xin, w, b] + ([rin] if rin is not None else [])
    got = torch.autograd.grad(y, ins, gin.to(y.dtype))
    exp = torch.autograd.grad(yr, [xr, wr, br] + ([rr] if rr is not None else []), g)
    gtol = 6e-2 if dtype == torch.bfloat16 else 1e-3
    for i, (a, e) in enumerate(zip(got, exp)):
        if layout == "nhwc" and i in (0, 3):
            a = a.permute(0, 3, 1, 2)
        _close(a, e, gtol)


def test_resnet_block_uses_fused_bn():
    from paddle_infer_amd.vision.models import resnet18
    torch.manual_seed(0)
    m = resnet18(num_classes=10).to(DEV)
    x = torch.randn(2, 3, 64, 64, device=DEV)
    y = m(x)
    y.sum().backward()
    assert torch.isfinite(y).all() and m.conv1.weight.grad is not None


@pytest.mark.parametrize("N,H,W,C", [(16, 32, 32, 64), (8, 8, 8, 2048), (4, 16, 16, 24)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_vectorised_multiblock(N, H, W, C, dtype):
    """Shapes that split the vectorised NHWC reductions over many blocks (and NCHW with H·W % 8
    == 0, the 8-wide apply kernels); statistics offset from zero to exercise the shifted sums."""
    from paddle_infer_amd.ops.batchnorm import batch_norm_act
    torch.manual_seed(N + C)
    x = (torch.randn(N, C, H, W, device=DEV) * 3 + 5).to(dtype)
    w = (torch.rand(C, device=DEV) + 0.5).requires_grad_(True)
    b = torch.randn(C, device=DEV).requires_grad_(True)
    for layout in ("channels_last", "nchw"):
        xin = (x.contiguous(memory_format=torch.channels_last) if layout == "channels_last"
               else x).detach().requires_grad_(True)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        # no activation here: an output within rounding of the ReLU kink flips its mask (the
        # ReLU paths are covered by test_bn_act)
        y = batch_norm_act(xin, rm, rv, w, b, True, 0.9, 1e-5, "none", None, "NCHW")
        xr = x.detach().float().requires_grad_(True)
        yr = F.batch_norm(xr, None, None, w, b, True, 0.1, 1e-5)
        tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
        _close(y, yr, tol)
        g = torch.randn_like(yr)
        got = torch.autograd.grad(y, [xin, w, b], g.to(y.dtype))
        exp = torch.autograd.grad(yr, [xr, w, b], g)
        for a, e in zip(got, exp):
            _close(a, e, 6e-2 if dtype == torch.bfloat16 else 1e-3)
