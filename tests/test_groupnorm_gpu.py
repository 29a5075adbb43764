"""GroupNorm / InstanceNorm on the own HIP kernels (groupnorm.hip) against the fp32 PyTorch
reference: forward, dx / dγ / dβ, ragged plane sizes (HW % 8 ≠ 0), NHWC input, running-statistics
InstanceNorm, bitwise-deterministic backward; no library fallback on these paths."""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tol(dt):
    return {torch.float32: 2e-4, torch.bfloat16: 3e-2, torch.float16: 5e-3}[dt]


@pytest.fixture(autouse=True)
def _no_fallback(monkeypatch):
    from paddle_infer_amd.ops import _lib
    seen = []
    monkeypatch.setattr(_lib, "fallback", lambda op, why="": seen.append(op))
    yield
    assert not seen, seen


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape,G", [((4, 32, 16, 16), 8), ((2, 64, 7, 7), 32), ((3, 6, 5), 3),
                                     ((2, 8, 4, 6, 10), 2), ((1, 4, 3000), 1)])
def test_group_norm_fwd_bwd(dt, shape, G):
    import paddle_infer_amd.nn.functional as F
    torch.manual_seed(sum(shape))
    x = (torch.randn(shape, device=DEV) * 2 + 0.5).to(dt).requires_grad_(True)
    C = shape[1]
    w = (1 + 0.3 * torch.randn(C, device=DEV)).requires_grad_(True)
    b = (0.2 * torch.randn(C, device=DEV)).requires_grad_(True)
    y = F.group_norm(x, G, 1e-5, w, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yr = TF.group_norm(xr, G, wr, br, 1e-5)
    yr.backward(dy.float())
    t = _tol(dt)
    torch.testing.assert_close(y.float(), yr, atol=t * 4, rtol=t)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=t * 4, rtol=t * 4)
    torch.testing.assert_close(w.grad, wr.grad, atol=t * 20 * shape[0], rtol=t * 4)
    torch.testing.assert_close(b.grad, br.grad, atol=t * 20 * shape[0], rtol=t * 4)


def test_group_norm_nhwc_and_determinism():
    import paddle_infer_amd.nn.functional as F
    torch.manual_seed(3)
    x = torch.randn(2, 9, 11, 32, device=DEV).bfloat16().requires_grad_(True)  # NHWC, C = 32
    w = torch.ones(32, device=DEV, requires_grad=True)
    grads = []
    for _ in range(2):
        x.grad = None
        y = F.group_norm(x, 4, 1e-5, w, None, data_format="NHWC")
        y.float().square().sum().backward()
        grads.append(x.grad.clone())
    ref = TF.group_norm(x.detach().float().permute(0, 3, 1, 2), 4, w.detach(), None, 1e-5).permute(0, 2, 3, 1)
    torch.testing.assert_close(y.float(), ref, atol=0.05, rtol=0.03)
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_instance_norm(dt):
    import paddle_infer_amd.nn.functional as F
    torch.manual_seed(5)
    x = torch.randn(3, 16, 12, 12, device=DEV).to(dt).requires_grad_(True)
    w, b = torch.rand(16, device=DEV) + 0.5, torch.randn(16, device=DEV)
    y = F.instance_norm(x, weight=w, bias=b, eps=1e-5)
    y.float().sum().backward()
    xr = x.detach().float().requires_grad_(True)
    yr = TF.instance_norm(xr, weight=w, bias=b, eps=1e-5)
    yr.sum().backward()
    t = _tol(dt)
    torch.testing.assert_close(y.float(), yr, atol=t * 4, rtol=t)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=t * 4, rtol=t * 4)
    rm, rv = torch.randn(16, device=DEV), torch.rand(16, device=DEV) + 0.5
    with torch.no_grad():
        ye = F.instance_norm(x, rm, rv, w, b, use_input_stats=False, eps=1e-5)
    ref = TF.instance_norm(x.detach().float(), rm, rv, w, b, use_input_stats=False, eps=1e-5)
    torch.testing.assert_close(ye.float(), ref, atol=t * 4, rtol=t)
