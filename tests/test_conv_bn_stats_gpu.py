"""BatchNorm statistics from the conv forward epilogue (gemm.hip conv_tile_stats →
batchnorm.hip bn_finalize_t): a training conv without bias leaves per-tile (count, mean, M2)
partials on its output and the BatchNorm that consumes it skips its own statistics pass. Checked
against the plain PyTorch fp32 reference of conv → batch_norm (training) → ReLU, and against the
same framework path with the fusion off."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    assert err <= atol + rtol * b.abs().max().item(), err


# (N, C, H, W, K, R, stride, pad): 1x1, 3x3, strided 1x1 (last tile partial), the 7x7 stem
# (small-channel mode) and M not a multiple of the 256-row tile
@pytest.mark.parametrize("shape", [(4, 64, 28, 28, 64, 1, 1, 0), (4, 64, 28, 28, 128, 3, 1, 1),
                                   (3, 256, 14, 14, 128, 1, 2, 0), (2, 3, 64, 64, 64, 7, 2, 3),
                                   (1, 64, 9, 13, 256, 3, 1, 1)])
def test_conv_bn_statistics_fused(shape):
    from paddle_infer_amd import nn
    from paddle_infer_amd.ops import conv as oc
    N, C, H, W, K, R, s, p = shape
    torch.manual_seed(sum(shape))
    x = (torch.randn(N, C, H, W, device=DEV) + 0.3).to(memory_format=torch.channels_last)
    conv = nn.Conv2D(C, K, R, s, p, bias_attr=False).to(DEV)
    bn = nn.BatchNorm2D(K).to(DEV)
    with torch.no_grad():  # a large per-channel offset: the shifted partial sums must not cancel
        conv.weight.add_(0.05)
    ref_conv_w = conv.weight.detach().clone().requires_grad_(True)

    def run(fused):
        oc.BN_STATS = fused
        try:
            bn._mean.fill_(0.0)
            bn._variance.fill_(1.0)
            conv.weight.grad = None
            xi = x.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                h = conv(xi)
                assert hasattr(h, "_piamd_bn_part") == fused
                y = bn(h, act="relu")
            y.float().sum().backward()
            return y.detach(), bn._mean.clone(), bn._variance.clone(), conv.weight.grad.clone(), xi.grad
        finally:
            oc.BN_STATS = True

    yf, mf, vf, gf, xf = run(True)
    yu, mu, vu, gu, xu = run(False)
    # fp32 reference of the same math (bf16 conv output, batch statistics, ReLU)
    xr = x.clone().requires_grad_(True)
    h = F.conv2d(xr.bfloat16().float(), ref_conv_w.bfloat16().float(), None, s, p).bfloat16().float()
    rm, rv = torch.zeros(K, device=DEV), torch.ones(K, device=DEV)
    yr = F.relu(F.batch_norm(h, rm, rv, bn.weight.detach().float(), bn.bias.detach().float(), True,
                             0.1, bn.epsilon))
    yr.sum().backward()
    _close(yf, yr, 3e-2)
    _close(yf, yu, 2e-2)
    _close(mf, rm, 1e-3, 1e-3)
    _close(vf, rv, 1e-3, 1e-3)
    _close(mf, mu, 1e-4, 1e-4)
    _close(vf, vu, 1e-4, 1e-4)
    _close(gf, ref_conv_w.grad, 3e-2, 3e-2)
    _close(gf, gu, 1e-2, 1e-2)
    _close(xf, xu, 1e-2, 1e-2)


@pytest.mark.parametrize("block", ["bottleneck", "basic"])
def test_residual_gradient_join(block):
    """Residual-gradient join (ops/conv.py ResidualGradJoin): the residual BatchNorm hands its
    residual gradient to the block's first conv, whose data-gradient epilogue adds it. Gradients
    of the block input and of every parameter against the same block with the join off (whose
    parts are each checked against fp32 references in test_conv_gpu / test_batchnorm_gpu)."""
    from paddle_infer_amd.ops import conv as oc
    from paddle_infer_amd.vision import models as VM
    torch.manual_seed(3)
    C = 256 if block == "bottleneck" else 64
    blk = (VM.BottleneckBlock(C, C // 4) if block == "bottleneck" else VM.BasicBlock(C, C)).to(DEV)
    x0 = torch.randn(4, C, 14, 14, device=DEV).to(memory_format=torch.channels_last)

    def run(on):
        oc.RES_JOIN = on
        try:
            for p in blk.parameters():
                p.grad = None
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = blk(x)
            (y.float() * torch.linspace(-1, 1, y.numel(), device=DEV).view_as(y)).sum().backward()
            return x.grad.float(), [p.grad.float().clone() for p in blk.parameters() if p.grad is not None]
        finally:
            oc.RES_JOIN = True

    gx_on, gp_on = run(True)
    gx_off, gp_off = run(False)
    _close(gx_on, gx_off, 1e-2, 1e-2)
    assert len(gp_on) == len(gp_off)
    for a, b in zip(gp_on, gp_off):
        _close(a, b, 1e-2, 1e-2)
    assert gx_on.abs().max() > 0
