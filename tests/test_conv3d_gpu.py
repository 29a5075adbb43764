"""Dense Conv3D / Conv3DTranspose / Conv1DTranspose on the framework's own conv kernels (depth taps
as 2-D convs / transposed convs, `ops/conv.py` conv3d_any / conv3d_transpose_any /
conv1d_transpose_any) against fp32 PyTorch, forward and backward, with no library fallback."""
import pytest
import torch
import torch.nn.functional as TF

import paddle_infer_amd.nn.functional as F
from paddle_infer_amd.ops import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_fallback():
    _lib.lib()
    _lib.FALLBACKS.clear()
    yield
    assert not _lib.FALLBACKS, f"ops left the HIP path: {_lib.FALLBACKS}"


def _tol(dt):
    return (3e-2, 3e-2) if dt == torch.bfloat16 else (2e-3, 2e-3)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cfg", [dict(C=16, K=32, k=3, s=1, p=1, d=1, g=1), dict(C=8, K=16, k=3, s=2, p=1, d=1, g=1),
                                 dict(C=16, K=16, k=3, s=1, p=2, d=2, g=4)])
def test_conv3d_fwd_bwd(dt, cfg):
    torch.manual_seed(0)
    x = torch.randn(2, cfg["C"], 6, 10, 10, device="cuda").to(dt).requires_grad_(True)
    w = (0.1 * torch.randn(cfg["K"], cfg["C"] // cfg["g"], cfg["k"], cfg["k"], cfg["k"], device="cuda")).to(dt) \
        .requires_grad_(True)
    b = torch.randn(cfg["K"], device="cuda").to(dt).requires_grad_(True)
    y = F.conv3d(x, w, b, cfg["s"], cfg["p"], cfg["d"], cfg["g"])
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = TF.conv3d(xr, wr, br, cfg["s"], cfg["p"], cfg["d"], cfg["g"])
    rt, at = _tol(dt)
    torch.testing.assert_close(y.float(), yr, rtol=rt, atol=at * yr.abs().max().item())
    dy = torch.randn_like(yr)
    y.backward(dy.to(dt))
    yr.backward(dy)
    for g, r in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        torch.testing.assert_close(g.float(), r, rtol=rt, atol=at * r.abs().max().item())


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("s,p,op", [(1, 1, 0), (2, 1, 1)])
def test_conv3d_transpose_fwd_bwd(dt, s, p, op):
    torch.manual_seed(1)
    x = torch.randn(2, 16, 4, 6, 6, device="cuda").to(dt).requires_grad_(True)
    w = (0.1 * torch.randn(16, 8, 3, 3, 3, device="cuda")).to(dt).requires_grad_(True)
    y = F.conv3d_transpose(x, w, None, s, p, op)
    xr, wr = (t.detach().float().requires_grad_(True) for t in (x, w))
    yr = TF.conv_transpose3d(xr, wr, None, s, p, op)
    rt, at = _tol(dt)
    torch.testing.assert_close(y.float(), yr, rtol=rt, atol=at * yr.abs().max().item())
    dy = torch.randn_like(yr)
    y.backward(dy.to(dt))
    yr.backward(dy)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=rt, atol=at * xr.grad.abs().max().item())
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=rt, atol=at * wr.grad.abs().max().item())


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_conv1d_transpose(dt):
    torch.manual_seed(2)
    x = torch.randn(3, 32, 50, device="cuda").to(dt).requires_grad_(True)
    w = (0.1 * torch.randn(32, 16, 5, device="cuda")).to(dt).requires_grad_(True)
    b = torch.randn(16, device="cuda").to(dt)
    y = F.conv1d_transpose(x, w, b, stride=2, padding=2, output_padding=1)
    xr, wr = (t.detach().float().requires_grad_(True) for t in (x, w))
    yr = TF.conv_transpose1d(xr, wr, b.float(), 2, 2, 1)
    rt, at = _tol(dt)
    torch.testing.assert_close(y.float(), yr, rtol=rt, atol=at * yr.abs().max().item())
    dy = torch.randn_like(yr)
    y.backward(dy.to(dt))
    yr.backward(dy)
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=rt, atol=at * wr.grad.abs().max().item())
