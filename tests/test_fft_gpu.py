"""fft.hip (LDS Stockham, batched rows) and the GPU compositions over it (four-step for long
power-of-two rows, Bluestein for other lengths, r2c / c2r) against numpy's float64 FFT."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _c(rows, n, seed=0):
    rs = np.random.RandomState(seed)
    return (rs.randn(rows, n) + 1j * rs.randn(rows, n)).astype(np.complex64)


@pytest.mark.parametrize("N", [2, 4, 16, 128, 1024, 2048, 4096])
@pytest.mark.parametrize("inverse", [False, True])
def test_kernel_pow2_rows(N, inverse):
    from paddle_infer_amd.ops import fft as F
    rows = 37 if N <= 1024 else 5
    x = _c(rows, N)
    y = F._pow2(torch.from_numpy(x).cuda(), inverse).cpu().numpy()
    ref = np.fft.ifft(x.astype(np.complex128)) * N if inverse else np.fft.fft(x.astype(np.complex128))
    err = np.abs(y - ref).max() / np.abs(ref).max()
    assert err < 2e-6 * max(1.0, np.log2(N)), err


@pytest.mark.parametrize("N", [16384, 1000, 4097])
def test_four_step_and_bluestein_on_gpu(N):
    from paddle_infer_amd import fft as pfft
    x = _c(3, N, seed=N)
    y = pfft.fft(torch.from_numpy(x).cuda()).cpu().numpy()
    ref = np.fft.fft(x.astype(np.complex128))
    assert np.abs(y - ref).max() / np.abs(ref).max() < 1e-5


def test_real_roundtrip_gpu():
    from paddle_infer_amd import fft as pfft
    x = torch.randn(8, 512, device="cuda")
    X = pfft.rfft(x)
    np.testing.assert_allclose(X.cpu().numpy(), np.fft.rfft(x.cpu().double().numpy()), atol=2e-3, rtol=1e-4)
    back = pfft.irfft(X, n=512)
    torch.testing.assert_close(back, x, atol=2e-5, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [64, 100, 8192])
def test_fft_kernel_gradients_match_cpu(n):
    """fft / rfft / irfft through the HIP kernel (pow2, Bluestein, four-step) are differentiable
    and their gradients equal the CPU Stockham path's (reference fft_c2c_grad / fft_r2c_grad)."""
    import paddle_infer_amd as paddle
    torch.manual_seed(0)
    x = torch.randn(3, n)
    w = torch.randn(3, n)
    outs = []
    for dev in ("cpu", "cuda"):
        xx = x.to(dev).requires_grad_(True)
        y = paddle.fft.fft(xx)
        r = paddle.fft.irfft(paddle.fft.rfft(xx), n=n)
        loss = (y.real * w.to(dev)).sum() + (y.imag ** 2).sum() * 1e-3 + (r * w.to(dev)).sum()
        (g,) = torch.autograd.grad(loss, xx)
        outs.append(g.cpu())
    torch.testing.assert_close(outs[1], outs[0], rtol=2e-3, atol=2e-3 * n ** 0.5)
