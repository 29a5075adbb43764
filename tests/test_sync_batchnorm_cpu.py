"""SyncBatchNorm (dense and sparse) over 2 gloo ranks against single-process BatchNorm on the
concatenated batch (reference `phi/kernels/gpu/sync_batch_norm_kernel.cu`): outputs, input
gradients, running statistics, and dγ/dβ (the local sums add up to the full-batch gradient)."""
import pytest
import torch

from dist_utils import run_distributed


def _worker(rank, world, x_full, dy_full, fmt):
    import paddle_infer_amd as paddle
    torch.manual_seed(0)
    C = x_full.shape[-1] if fmt == "NHWC" else x_full.shape[1]
    bn = paddle.nn.SyncBatchNorm(C, data_format=fmt)
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, C))
        bn.bias.copy_(torch.linspace(-1, 1, C))
    bn.train()
    x = x_full.chunk(world)[rank].clone().requires_grad_(True)
    y = bn(x)
    y.backward(dy_full.chunk(world)[rank])
    return y.detach(), x.grad, bn._mean.clone(), bn._variance.clone(), bn.weight.grad, bn.bias.grad


@pytest.mark.parametrize("fmt", ["NCHW", "NHWC"])
def test_sync_batchnorm_matches_full_batch(fmt):
    import paddle_infer_amd as paddle
    torch.manual_seed(1)
    shape = (6, 5, 4, 3) if fmt == "NCHW" else (6, 4, 3, 5)
    x = torch.randn(*shape) * 3 + 7  # large mean: single-pass E[x²]−E[x]² would lose digits
    dy = torch.randn(*shape)
    res = run_distributed(_worker, 2, x, dy, fmt)
    C = 5
    ref = paddle.nn.BatchNorm2D(C, data_format=fmt)
    with torch.no_grad():
        ref.weight.copy_(torch.linspace(0.5, 1.5, C))
        ref.bias.copy_(torch.linspace(-1, 1, C))
    ref.train()
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(dy)
    ys = torch.cat([torch.as_tensor(res[r][0]) for r in range(2)])
    gs = torch.cat([torch.as_tensor(res[r][1]) for r in range(2)])
    torch.testing.assert_close(ys, yr.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gs, xr.grad, rtol=1e-4, atol=1e-4)
    for r in range(2):
        torch.testing.assert_close(torch.as_tensor(res[r][2]), ref._mean, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(torch.as_tensor(res[r][3]), ref._variance, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(torch.as_tensor(res[0][4]) + torch.as_tensor(res[1][4]), ref.weight.grad,
                               rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(torch.as_tensor(res[0][5]) + torch.as_tensor(res[1][5]), ref.bias.grad,
                               rtol=1e-4, atol=1e-4)


def _sparse_worker(rank, world, vals):
    import paddle_infer_amd as paddle
    bn = paddle.sparse.nn.SyncBatchNorm(4)
    bn.train()
    v = vals.chunk(world)[rank]
    n = v.shape[0]
    idx = torch.stack([torch.zeros(n, dtype=torch.long), torch.arange(n), torch.zeros(n, dtype=torch.long),
                       torch.zeros(n, dtype=torch.long)])
    sp = torch.sparse_coo_tensor(idx, v, (1, n, 1, 1, 4)).coalesce()
    out = bn(sp)
    return out.values(), bn._mean.clone()


def test_sparse_sync_batchnorm_uses_global_statistics():
    torch.manual_seed(2)
    vals = torch.randn(10, 4) * 2 + 1
    res = run_distributed(_sparse_worker, 2, vals)
    mean, var = vals.mean(0), vals.var(0, unbiased=False)
    ref = (vals - mean) / torch.sqrt(var + 1e-5)
    got = torch.cat([torch.as_tensor(res[r][0]) for r in range(2)])
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(torch.as_tensor(res[0][1]), 0.1 * mean, rtol=1e-5, atol=1e-5)
