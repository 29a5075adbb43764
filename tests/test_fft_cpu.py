"""paddle.fft on the framework's own DFT core (Stockham / four-step / Bluestein, ops/fft.py)
against numpy.fft: every transform family, power-of-two and odd lengths, n padding/truncation,
all three norms, n-d axes."""
import numpy as np
import pytest
import torch

from paddle_infer_amd import fft as pfft

RS = np.random.RandomState(0)


def _c(*shape):
    return (RS.randn(*shape) + 1j * RS.randn(*shape)).astype(np.complex128)


@pytest.mark.parametrize("N", [1, 2, 8, 64, 7, 12, 100, 243])
@pytest.mark.parametrize("norm", ["backward", "forward", "ortho"])
def test_c2c_matches_numpy(N, norm):
    x = _c(3, N)
    np.testing.assert_allclose(pfft.fft(torch.from_numpy(x), norm=norm).numpy(),
                               np.fft.fft(x, norm=norm), rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(pfft.ifft(torch.from_numpy(x), norm=norm).numpy(),
                               np.fft.ifft(x, norm=norm), rtol=1e-9, atol=1e-9)


def test_four_step_long_pow2():
    from paddle_infer_amd.ops import fft as F
    x = torch.from_numpy(_c(2, 8192))
    y = F._four_step(x, False)
    np.testing.assert_allclose(y.numpy(), np.fft.fft(x.numpy()), rtol=1e-8, atol=1e-7)


@pytest.mark.parametrize("n", [None, 10, 20])
def test_real_transforms(n):
    x = RS.randn(4, 15)
    t = torch.from_numpy(x)
    np.testing.assert_allclose(pfft.rfft(t, n=n).numpy(), np.fft.rfft(x, n=n), atol=1e-9)
    X = np.fft.rfft(x)
    np.testing.assert_allclose(pfft.irfft(torch.from_numpy(X), n=n).numpy(), np.fft.irfft(X, n=n), atol=1e-9)
    np.testing.assert_allclose(pfft.hfft(torch.from_numpy(X), n=n).numpy(), np.fft.hfft(X, n=n), atol=1e-9)
    np.testing.assert_allclose(pfft.ihfft(t, n=n).numpy(), np.fft.ihfft(x, n=n), atol=1e-9)


def test_nd_transforms():
    x = _c(3, 6, 8)
    xr = RS.randn(3, 6, 8)
    np.testing.assert_allclose(pfft.fft2(torch.from_numpy(x)).numpy(), np.fft.fft2(x), atol=1e-9)
    np.testing.assert_allclose(pfft.ifftn(torch.from_numpy(x), axes=(0, 2)).numpy(),
                               np.fft.ifftn(x, axes=(0, 2)), atol=1e-9)
    np.testing.assert_allclose(pfft.rfftn(torch.from_numpy(xr)).numpy(), np.fft.rfftn(xr), atol=1e-9)
    X = np.fft.rfft2(xr)
    np.testing.assert_allclose(pfft.irfft2(torch.from_numpy(X), s=(6, 8)).numpy(),
                               np.fft.irfft2(X, s=(6, 8)), atol=1e-9)
    np.testing.assert_allclose(pfft.fftn(torch.from_numpy(x), s=(4, 10), axes=(1, 2)).numpy(),
                               np.fft.fftn(x, s=(4, 10), axes=(1, 2)), atol=1e-9)
