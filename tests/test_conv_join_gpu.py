"""Conv→conv gradient join in downsampling residual blocks (ops/conv.py join_give): the shortcut
conv hands its block-input gradient to the main path's first conv, whose data-gradient epilogue
adds it — same gradients as the unjoined block (PIAMD_RES_JOIN off), and the hand-over happens."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("stride,block", [(1, "bottleneck"), (2, "bottleneck"), (2, "basic")])
def test_downsample_block_join_matches_unjoined(stride, block, monkeypatch):
    import paddle_infer_amd as paddle
    from paddle_infer_amd import nn
    from paddle_infer_amd.ops import conv as C
    from paddle_infer_amd.vision import models as M
    paddle.seed(3)
    cin, planes = 64, 64
    if block == "bottleneck":
        ds = nn.Sequential(nn.Conv2D(cin, planes * 4, 1, stride, bias_attr=False), nn.BatchNorm2D(planes * 4))
        blk = M.BottleneckBlock(cin, planes, stride, ds)
    else:
        ds = nn.Sequential(nn.Conv2D(cin, planes * 2, 1, stride, bias_attr=False), nn.BatchNorm2D(planes * 2))
        blk = M.BasicBlock(cin, planes * 2, stride, ds)
    blk = blk.to(DEV)
    blk.train()
    x0 = torch.randn(8, cin, 28, 28, device=DEV).to(memory_format=torch.channels_last)

    gave = []
    orig = C._give

    def spy(ctx, x, dx):
        r = orig(ctx, x, dx)
        gave.append(r is None and dx is not None)
        return r
    monkeypatch.setattr(C, "_give", spy)

    def run(join):
        monkeypatch.setattr(C, "RES_JOIN", join)
        gave.clear()
        x = x0.clone().requires_grad_(True)
        for p in blk.parameters():
            p.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = blk(x)
        (y.float() * torch.linspace(-1, 1, y.shape[1], device=DEV).view(1, -1, 1, 1)).sum().backward()
        return x.grad.float().clone(), [p.grad.float().clone() for p in blk.parameters()], list(gave)

    gx1, gp1, g1 = run(True)
    gx0, gp0, g0 = run(False)
    assert any(g1) and not any(g0), (g1, g0)  # the shortcut conv handed its gradient over
    torch.testing.assert_close(gx1, gx0, atol=2e-2, rtol=2e-2)
    for a, b in zip(gp1, gp0):
        torch.testing.assert_close(a, b, atol=2e-2, rtol=2e-2)
