"""NHWC max pooling on the own kernels (csrc/kernels/pool.hip) against torch's max_pool2d in fp32
on the same 16-bit inputs: forward values, the tap chosen (gradient routing) and the gradient."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape,k,s,p", [
    ((4, 64, 112, 112), 3, 2, 1),   # ResNet stem pool
    ((2, 32, 15, 17), 3, 2, 1),     # odd sizes
    ((2, 16, 12, 12), 2, 2, 0),     # 2x2 stride 2
    ((1, 8, 9, 9), 3, 1, 1),        # stride 1: windows overlap 3x3
])
def test_maxpool_nhwc_matches_torch(dt, shape, k, s, p):
    import paddle_infer_amd.nn.functional as F
    from paddle_infer_amd.ops.pool import max_pool2d_supported
    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    assert max_pool2d_supported(x, k, s, p)
    xa = x.clone().requires_grad_(True)
    y = F.max_pool2d(xa, k, s, p)
    xr = x.float().clone().requires_grad_(True)
    yr = torch.nn.functional.max_pool2d(xr, k, s, p)
    assert torch.equal(y.float(), yr), (y.float() - yr).abs().max()
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g.to(dt).float())
    # same routing; sums of ≤ 9 16-bit values rounded once
    torch.testing.assert_close(xa.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)
    assert y.is_contiguous(memory_format=torch.channels_last)
