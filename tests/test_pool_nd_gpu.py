"""Own pooling / resampling kernels (csrc/kernels/pool_nd.hip via ops/pool_nd.py, routed from
nn.functional) against the PyTorch fp32 reference of the same op on the CPU: values, max masks and
input (and grid) gradients, with the no-fallback fixture."""
import pytest
import torch
import torch.nn.functional as TF

import paddle_infer_amd as paddle

pytestmark = pytest.mark.gpu
F = paddle.nn.functional


@pytest.fixture(autouse=True)
def _no_fallback():
    from paddle_infer_amd.ops import _lib
    _lib.lib()
    _lib.FALLBACKS.clear()
    yield
    assert not _lib.FALLBACKS, f"ops left the HIP path: {_lib.FALLBACKS}"


def _check(ours, ref, shape, dt=torch.float32, extra=(), seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(shape, generator=g)
    if dt != torch.float32:
        x = x.to(dt).float()
    xr = x.clone().requires_grad_()
    yr = ref(xr)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xg = x.to("cuda", dt).requires_grad_()
    yg = ours(xg)
    yg.backward(dy.to("cuda", dt))
    tol = dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(yg.float().cpu(), yr.detach(), **tol)
    torch.testing.assert_close(xg.grad.float().cpu(), xr.grad, **tol)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ceil", [False, True])
def test_max_pool_nd(dt, ceil):
    _check(lambda x: F.max_pool1d(x, 3, 2, 1, ceil_mode=ceil), lambda x: TF.max_pool1d(x, 3, 2, 1, ceil_mode=ceil),
           (2, 5, 37), dt)
    _check(lambda x: F.max_pool2d(x, 3, 2, 1, ceil_mode=ceil),
           lambda x: TF.max_pool2d(x, 3, 2, 1, ceil_mode=ceil), (2, 6, 17, 19), dt)
    _check(lambda x: F.max_pool3d(x, (2, 3, 3), (2, 2, 1), (1, 1, 0), ceil_mode=ceil),
           lambda x: TF.max_pool3d(x, (2, 3, 3), (2, 2, 1), (1, 1, 0), ceil_mode=ceil), (2, 3, 7, 9, 8), dt)


def test_max_pool_mask_matches():
    x = torch.randn(2, 4, 13, 11)
    y, m = F.max_pool2d(x.cuda(), 3, 2, 1, return_mask=True)
    yr, mr = TF.max_pool2d(x, 3, 2, 1, return_indices=True)
    torch.testing.assert_close(y.cpu(), yr)
    assert torch.equal(m.cpu(), mr)
    y, m = F.adaptive_max_pool2d(x.cuda(), (5, 4), return_mask=True)
    yr, mr = TF.adaptive_max_pool2d(x, (5, 4), return_indices=True)
    torch.testing.assert_close(y.cpu(), yr)
    assert torch.equal(m.cpu(), mr)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("exclusive", [True, False])
@pytest.mark.parametrize("ceil", [False, True])
def test_avg_pool_nd(dt, exclusive, ceil):
    _check(lambda x: F.avg_pool1d(x, 4, 3, 2, exclusive=exclusive, ceil_mode=ceil),
           lambda x: TF.avg_pool1d(x, 4, 3, 2, ceil_mode=ceil, count_include_pad=not exclusive), (2, 3, 29), dt)
    _check(lambda x: F.avg_pool2d(x, 3, 2, 1, ceil_mode=ceil, exclusive=exclusive),
           lambda x: TF.avg_pool2d(x, 3, 2, 1, ceil_mode=ceil, count_include_pad=not exclusive), (2, 5, 15, 18), dt)
    _check(lambda x: F.avg_pool3d(x, 3, 2, 1, ceil_mode=ceil, exclusive=exclusive),
           lambda x: TF.avg_pool3d(x, 3, 2, 1, ceil_mode=ceil, count_include_pad=not exclusive), (1, 3, 7, 8, 9), dt)


def test_avg_pool_divisor_and_nhwc():
    _check(lambda x: F.avg_pool2d(x, 3, 2, 1, divisor_override=5),
           lambda x: TF.avg_pool2d(x, 3, 2, 1, divisor_override=5), (2, 4, 11, 12))
    _check(lambda x: F.avg_pool2d(x, 2, 2, data_format="NHWC"),
           lambda x: TF.avg_pool2d(x.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1), (2, 10, 12, 6))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_adaptive_pools(dt):
    _check(lambda x: F.adaptive_avg_pool1d(x, 7), lambda x: TF.adaptive_avg_pool1d(x, 7), (2, 4, 30), dt)
    _check(lambda x: F.adaptive_avg_pool2d(x, (5, 3)), lambda x: TF.adaptive_avg_pool2d(x, (5, 3)), (2, 4, 17, 13), dt)
    _check(lambda x: F.adaptive_avg_pool2d(x, 1), lambda x: TF.adaptive_avg_pool2d(x, 1), (2, 64, 7, 7), dt)
    _check(lambda x: F.adaptive_avg_pool3d(x, (2, 3, 4)), lambda x: TF.adaptive_avg_pool3d(x, (2, 3, 4)),
           (1, 3, 5, 7, 9), dt)
    _check(lambda x: F.adaptive_max_pool1d(x, 6), lambda x: TF.adaptive_max_pool1d(x, 6), (2, 4, 25), dt)
    _check(lambda x: F.adaptive_max_pool2d(x, (4, 6)), lambda x: TF.adaptive_max_pool2d(x, (4, 6)), (2, 3, 9, 14), dt)
    _check(lambda x: F.adaptive_max_pool3d(x, 3), lambda x: TF.adaptive_max_pool3d(x, 3), (1, 2, 7, 5, 8), dt)
    # adaptive up-sampling windows (O > I overlap)
    _check(lambda x: F.adaptive_avg_pool2d(x, (7, 9)), lambda x: TF.adaptive_avg_pool2d(x, (7, 9)), (1, 2, 3, 4), dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ac", [False, True])
def test_interpolate_linear(dt, ac):
    _check(lambda x: F.interpolate(x, size=[23], mode="linear", align_corners=ac),
           lambda x: TF.interpolate(x, size=[23], mode="linear", align_corners=ac), (2, 3, 10), dt)
    _check(lambda x: F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=ac),
           lambda x: TF.interpolate(x, scale_factor=2, mode="bilinear", align_corners=ac), (2, 4, 9, 11), dt)
    _check(lambda x: F.interpolate(x, size=[5, 7], mode="bilinear", align_corners=ac),
           lambda x: TF.interpolate(x, size=[5, 7], mode="bilinear", align_corners=ac), (2, 4, 12, 13), dt)
    _check(lambda x: F.interpolate(x, size=[6, 7, 9], mode="trilinear", align_corners=ac),
           lambda x: TF.interpolate(x, size=[6, 7, 9], mode="trilinear", align_corners=ac), (1, 2, 4, 5, 6), dt)


def test_interpolate_nearest_and_area():
    _check(lambda x: F.interpolate(x, scale_factor=2, mode="nearest"),
           lambda x: TF.interpolate(x, scale_factor=2, mode="nearest"), (2, 3, 7, 9))
    _check(lambda x: F.interpolate(x, size=[5, 13], mode="nearest"),
           lambda x: TF.interpolate(x, size=[5, 13], mode="nearest"), (2, 3, 11, 6))
    _check(lambda x: F.interpolate(x, scale_factor=1.5, mode="nearest"),
           lambda x: TF.interpolate(x, scale_factor=1.5, mode="nearest"), (1, 2, 5, 6, 7))
    _check(lambda x: F.interpolate(x, size=[4, 5], mode="area"),
           lambda x: TF.interpolate(x, size=[4, 5], mode="area"), (2, 3, 9, 11))
    _check(lambda x: F.interpolate(x, scale_factor=2, mode="bilinear", data_format="NHWC"),
           lambda x: TF.interpolate(x.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear").permute(0, 2, 3, 1),
           (2, 6, 5, 3))


@pytest.mark.parametrize("mode", ["bilinear", "nearest"])
@pytest.mark.parametrize("pad", ["zeros", "border", "reflection"])
@pytest.mark.parametrize("ac", [False, True])
def test_grid_sample(mode, pad, ac):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 3, 9, 11, generator=g)
    grid = 1.3 * (2 * torch.rand(2, 7, 8, 2, generator=g) - 1)  # some samples outside [-1, 1]
    xr, gr = x.clone().requires_grad_(), grid.clone().requires_grad_()
    yr = TF.grid_sample(xr, gr, mode, pad, ac)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xg, gg = x.cuda().requires_grad_(), grid.cuda().requires_grad_()
    yg = F.grid_sample(xg, gg, mode, pad, ac)
    yg.backward(dy.cuda())
    torch.testing.assert_close(yg.cpu(), yr.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(xg.grad.cpu(), xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gg.grad.cpu(), gr.grad, rtol=1e-3, atol=1e-3)


def test_pool_layers_route_to_own_kernels():
    nn = paddle.nn
    x = torch.randn(2, 8, 14, 14, device="cuda", dtype=torch.bfloat16)
    for layer, ref in ((nn.AdaptiveAvgPool2D(1), lambda t: TF.adaptive_avg_pool2d(t, 1)),
                       (nn.AvgPool2D(2, 2), lambda t: TF.avg_pool2d(t, 2, 2)),
                       (nn.Upsample(scale_factor=2, mode="nearest"), lambda t: TF.interpolate(t, scale_factor=2))):
        torch.testing.assert_close(layer(x).float(), ref(x.float()), rtol=2e-2, atol=2e-2)
