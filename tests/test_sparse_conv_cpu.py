"""Sparse conv3d / subm_conv3d / max_pool3d / mask attention on the active sites
(`sparse/nn/conv.py`, reference `phi/kernels/sparse/gpu/conv_kernel.cu` rulebook +
gather-GEMM-scatter) against dense PyTorch references of the same op on small grids, gradients
included, and a 1 %-dense 128³ grid that runs without materialising the dense volume."""
import pytest
import torch
import torch.nn.functional as F

import paddle_infer_amd as paddle

SF = paddle.sparse.nn.functional


def _rand_sparse(B, D, H, W, C, density, seed=0):
    g = torch.Generator().manual_seed(seed)
    n = max(1, int(B * D * H * W * density))
    keys = torch.randperm(B * D * H * W, generator=g)[:n]
    idx = torch.stack([keys // (D * H * W), (keys // (H * W)) % D, (keys // W) % H, keys % W])
    val = torch.randn(n, C, generator=g)
    return torch.sparse_coo_tensor(idx, val, (B, D, H, W, C)).coalesce()


def _dense_conv(xd, w, b, stride, padding, dilation):
    y = F.conv3d(xd.permute(0, 4, 1, 2, 3), w.permute(4, 3, 0, 1, 2), b, stride, padding, dilation)
    return y.permute(0, 2, 3, 4, 1)


@pytest.mark.parametrize("stride,padding,dilation,k", [(1, 0, 1, 3), (2, 1, 1, 3), (1, 1, 2, 3), (2, 0, 1, 2)])
def test_sparse_conv3d_matches_dense(stride, padding, dilation, k):
    x = _rand_sparse(2, 9, 8, 10, 4, 0.15, seed=stride + k)
    w = 0.3 * torch.randn(k, k, k, 4, 6)
    b = 0.1 * torch.randn(6)
    y = SF.conv3d(x, w, b, stride, padding, dilation)
    ref = _dense_conv(x.to_dense(), w, b, stride, padding, dilation)
    yd = y.to_dense()
    assert yd.shape == ref.shape
    # active outputs = every site some active input reaches; elsewhere the dense conv is the bias
    active = yd.ne(0).any(-1) | torch.zeros_like(yd[..., 0], dtype=torch.bool).index_put_(
        tuple(y.indices()), torch.tensor(True))
    torch.testing.assert_close(yd[active], ref[active], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(ref[~active], b.expand_as(ref[~active]), rtol=1e-5, atol=1e-6)


def test_subm_conv3d_matches_dense_on_input_sites_with_grads():
    x = _rand_sparse(1, 7, 7, 7, 5, 0.2, seed=3)
    w = (0.3 * torch.randn(3, 3, 3, 5, 8)).requires_grad_()
    xv = x.values().clone().requires_grad_()
    xs = torch.sparse_coo_tensor(x.indices(), xv, x.shape)
    y = SF.subm_conv3d(xs, w, None, 1, 1)
    assert torch.equal(y.indices(), x.indices())
    xd = torch.zeros(x.shape).index_put_(tuple(x.indices()), xv.detach()).requires_grad_()
    wr = w.detach().clone().requires_grad_()
    ref = _dense_conv(xd, wr, None, 1, 1, 1)[tuple(x.indices())]
    torch.testing.assert_close(y.values(), ref, rtol=1e-4, atol=1e-5)
    g = torch.randn_like(ref)
    gx, gw = torch.autograd.grad(y.values(), (xv, w), g)
    rx, rw = torch.autograd.grad(ref, (xd, wr), g)
    torch.testing.assert_close(gx, rx[tuple(x.indices())], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gw, rw, rtol=1e-4, atol=1e-5)


def test_sparse_max_pool3d_over_active_sites():
    x = _rand_sparse(2, 8, 8, 8, 3, 0.2, seed=5)
    y = SF.max_pool3d(x, 2, 2)
    xd = x.to_dense()
    act = torch.zeros(xd.shape[:4], dtype=torch.bool).index_put_(tuple(x.indices()), torch.tensor(True))
    masked = torch.where(act[..., None], xd, torch.full_like(xd, float("-inf")))
    ref = F.max_pool3d(masked.permute(0, 4, 1, 2, 3), 2, 2).permute(0, 2, 3, 4, 1)
    yi = tuple(y.indices())
    torch.testing.assert_close(y.values(), ref[yi])
    assert torch.isfinite(ref[yi]).all() and int(torch.isfinite(ref[..., 0]).sum()) == y.values().shape[0]


def test_huge_sparse_grid_never_densified():
    """1 % of a 128³ grid active (and a 4096³ grid: 68 G voxels, impossible to densify)."""
    x = _rand_sparse(1, 128, 128, 128, 16, 0.01, seed=7)
    w = 0.1 * torch.randn(3, 3, 3, 16, 16)
    y = SF.subm_conv3d(x, w, None, 1, 1)
    assert y.values().shape == (x.values().shape[0], 16)
    # spot check 50 sites against a direct neighbourhood sum
    xd_idx = {tuple(v.tolist()): i for i, v in enumerate(x.indices().t())}
    for i in range(50):
        b, z, yy, xx = x.indices()[:, i].tolist()
        acc = torch.zeros(16)
        for dz in range(3):
            for dy in range(3):
                for dx in range(3):
                    j = xd_idx.get((b, z + dz - 1, yy + dy - 1, xx + dx - 1))
                    if j is not None:
                        acc += x.values()[j] @ w[dz, dy, dx]
        torch.testing.assert_close(y.values()[i], acc, rtol=1e-4, atol=1e-5)
    big = torch.sparse_coo_tensor(torch.tensor([[0, 0], [10, 11], [4000, 4000], [7, 7]]), torch.randn(2, 4),
                                  (1, 4096, 4096, 4096, 4)).coalesce()
    out = SF.conv3d(big, torch.randn(3, 3, 3, 4, 2), None, 1, 1)
    assert out.shape == (1, 4096, 4096, 4096, 2) and out.values().shape[0] == 3 * 3 * 3 + 9 * 2 - 9


def test_sparse_mask_attention_matches_masked_dense():
    B, Hh, S, d = 2, 2, 12, 8
    q, k, v = (torch.randn(B, Hh, S, d) for _ in range(3))
    one = (torch.rand(S, S) < 0.3) | torch.eye(S, dtype=torch.bool)
    mask = one.expand(B * Hh, S, S)
    out = SF.attention(q, k, v, mask.float().to_sparse_csr())  # batched CSR: one pattern per batch
    torch.testing.assert_close(SF.attention(q, k, v, mask.float().to_sparse()), out)
    s = (q @ k.transpose(-1, -2)) * d ** -0.5
    s = s.masked_fill(~mask.reshape(B, Hh, S, S), float("-inf"))
    ref = torch.softmax(s, -1) @ v
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
