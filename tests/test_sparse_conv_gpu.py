"""Sparse conv3d / subm_conv3d on the GPU gather → grouped MFMA GEMM → scatter path
(`sparse/nn/conv.py` _ggs / _wgrad on `ops/moe.py` grouped kernels; fp32 as split-bf16) against
the same ops on the CPU in fp32 — values and both gradients, with the no-fallback fixture."""
import pytest
import torch

import paddle_infer_amd as paddle

pytestmark = pytest.mark.gpu
SF = paddle.sparse.nn.functional


@pytest.fixture(autouse=True)
def _no_fallback():
    from paddle_infer_amd.ops import _lib
    _lib.lib()
    _lib.FALLBACKS.clear()
    yield
    assert not _lib.FALLBACKS, f"ops left the HIP path: {_lib.FALLBACKS}"


def _rand_sparse(B, D, H, W, C, density, seed=0):
    g = torch.Generator().manual_seed(seed)
    n = max(1, int(B * D * H * W * density))
    keys = torch.randperm(B * D * H * W, generator=g)[:n]
    idx = torch.stack([keys // (D * H * W), (keys // (H * W)) % D, (keys // W) % H, keys % W])
    val = torch.randn(n, C, generator=g)
    return idx, val, (B, D, H, W, C)


def _run(idx, val, shape, w, subm, dev, dt):
    xv = val.to(dev, dt).requires_grad_()
    wv = w.to(dev, dt).requires_grad_()
    xs = torch.sparse_coo_tensor(idx.to(dev), xv, shape)
    fn = SF.subm_conv3d if subm else SF.conv3d
    y = fn(xs, wv, None, 1, 1)
    g = torch.Generator().manual_seed(7)
    dy = torch.randn(y.values().shape, generator=g).to(dev, dt)
    gx, gw = torch.autograd.grad(y.values(), (xv, wv), dy)
    return y.indices().cpu(), y.values().float().cpu(), gx.float().cpu(), gw.float().cpu()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("subm", [True, False])
@pytest.mark.parametrize("cin,cout", [(16, 32), (64, 64)])
def test_sparse_conv_gpu_matches_cpu(dt, subm, cin, cout):
    idx, val, shape = _rand_sparse(2, 12, 12, 12, cin, 0.1, seed=cin + cout)
    w = 0.1 * torch.randn(3, 3, 3, cin, cout, generator=torch.Generator().manual_seed(1))
    if dt == torch.bfloat16:  # same rounded inputs on both sides
        val, w = val.bfloat16().float(), w.bfloat16().float()
    ri, rv, rgx, rgw = _run(idx, val, shape, w, subm, "cpu", torch.float32)
    gi, gv, ggx, ggw = _run(idx, val, shape, w, subm, "cuda", dt)
    assert torch.equal(ri, gi)
    # bf16: the outputs themselves are bf16-rounded (2^-8 relative) after an f32 reduction over up
    # to 27·Cin products — compare against the output scale
    tol = dict(rtol=3e-2, atol=1e-2) if dt == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    for got, ref in ((gv, rv), (ggx, rgx), (ggw, rgw)):
        scale = max(ref.abs().max().item(), 1e-6)
        torch.testing.assert_close(got / scale, ref / scale, **tol)
