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
