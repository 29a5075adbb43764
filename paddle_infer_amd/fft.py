"""``paddle.fft`` — discrete Fourier transforms (reference `python/paddle/fft.py`).

Paddle's argument names (``n, axis, norm`` / ``s, axes``) and normalisation modes
("backward" | "forward" | "ortho"). Every transform is composed from ONE complex DFT core
(``ops/fft.py``: the ``fft.hip`` LDS Stockham kernel on the GPU for power-of-two rows ≤ 4096,
four-step above that, Bluestein for other lengths): r2c keeps the first N/2 + 1 bins, c2r builds
the Hermitian spectrum, hfft / ihfft are c2r / r2c of the conjugate with the swapped norm, n-d
transforms run the 1-D transform axis by axis. Real inputs of c2c are promoted to complex like
the reference.
"""
from __future__ import annotations

import torch

__all__ = ["fft", "ifft", "rfft", "irfft", "hfft", "ihfft", "fft2", "ifft2", "rfft2", "irfft2",
           "hfft2", "ihfft2", "fftn", "ifftn", "rfftn", "irfftn", "hfftn", "ihfftn", "fftfreq",
           "rfftfreq", "fftshift", "ifftshift"]

_NORMS = ("backward", "forward", "ortho")


def _norm(norm):
    if norm not in _NORMS:
        raise ValueError(f"Unexpected norm: {norm}. Norm should be forward, backward or ortho")
    return norm


def _t(x):
    return x if isinstance(x, torch.Tensor) else torch.as_tensor(x)


def _swap(norm):
    return {"backward": "forward", "forward": "backward", "ortho": "ortho"}[norm]


def _c2c(x, n, axis, inverse, norm):
    from .ops.fft import c2c
    return c2c(_t(x), axis=axis, n=n, inverse=inverse, norm=_norm(norm))


def fft(x, n=None, axis=-1, norm="backward", name=None):
    return _c2c(x, n, axis, False, norm)


def ifft(x, n=None, axis=-1, norm="backward", name=None):
    return _c2c(x, n, axis, True, norm)


def rfft(x, n=None, axis=-1, norm="backward", name=None):
    x = _t(x)
    if x.is_complex():
        raise TypeError("rfft expects a real input")
    y = _c2c(x, n, axis, False, norm)
    ax = axis % y.dim()
    return y.narrow(ax, 0, y.shape[ax] // 2 + 1)


def irfft(x, n=None, axis=-1, norm="backward", name=None):
    """c2r: the Hermitian-symmetric full spectrum of the given half, inverse c2c, real part."""
    x = _t(x)
    if not x.is_complex():
        x = x.to(torch.complex128 if x.dtype == torch.float64 else torch.complex64)
    ax = axis % x.dim()
    n = 2 * (x.shape[ax] - 1) if n is None else n
    m = n // 2 + 1
    h = x.narrow(ax, 0, min(m, x.shape[ax]))
    if h.shape[ax] < m:
        pad = list(h.shape)
        pad[ax] = m - h.shape[ax]
        h = torch.cat([h, torch.zeros(pad, dtype=h.dtype, device=h.device)], dim=ax)
    # X[0] and (even n) X[n/2] contribute their real parts only
    idx = [0] + ([m - 1] if n % 2 == 0 and m > 1 else [])
    h = h.clone()
    for i in idx:
        sl = h.narrow(ax, i, 1)
        sl.copy_(sl.real.to(h.dtype))
    tail = h.narrow(ax, 1, n - m).flip(ax).conj() if n - m > 0 else None
    full = torch.cat([h, tail], dim=ax) if tail is not None else h
    return _c2c(full, None, ax, True, norm).real


def hfft(x, n=None, axis=-1, norm="backward", name=None):
    return irfft(_t(x).conj(), n, axis, _swap(_norm(norm)))


def ihfft(x, n=None, axis=-1, norm="backward", name=None):
    return rfft(x, n, axis, _swap(_norm(norm))).conj().resolve_conj()


def _axes_sizes(x, s, axes):
    nd = x.dim()
    if axes is None:
        axes = list(range(nd)) if s is None else list(range(nd - len(s), nd))
    axes = [a % nd for a in axes]
    s = [None] * len(axes) if s is None else list(s)
    return axes, s


def fftn(x, s=None, axes=None, norm="backward", name=None):
    x = _t(x)
    axes, s = _axes_sizes(x, s, axes)
    for a, n in zip(axes, s):
        x = _c2c(x, n, a, False, norm)
    return x


def ifftn(x, s=None, axes=None, norm="backward", name=None):
    x = _t(x)
    axes, s = _axes_sizes(x, s, axes)
    for a, n in zip(axes, s):
        x = _c2c(x, n, a, True, norm)
    return x


def rfftn(x, s=None, axes=None, norm="backward", name=None):
    x = _t(x)
    axes, s = _axes_sizes(x, s, axes)
    y = rfft(x, s[-1], axes[-1], norm)
    for a, n in zip(axes[:-1], s[:-1]):
        y = _c2c(y, n, a, False, norm)
    return y


def irfftn(x, s=None, axes=None, norm="backward", name=None):
    x = _t(x)
    axes, s = _axes_sizes(x, s, axes)
    for a, n in zip(axes[:-1], s[:-1]):
        x = _c2c(x, n, a, True, norm)
    return irfft(x, s[-1], axes[-1], norm)


def hfftn(x, s=None, axes=None, norm="backward", name=None):
    return irfftn(_t(x).conj(), s, axes, _swap(_norm(norm)))


def ihfftn(x, s=None, axes=None, norm="backward", name=None):
    return rfftn(x, s, axes, _swap(_norm(norm))).conj().resolve_conj()


def fft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return fftn(x, s, axes, norm)


def ifft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return ifftn(x, s, axes, norm)


def rfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return rfftn(x, s, axes, norm)


def irfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return irfftn(x, s, axes, norm)


def hfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return hfftn(x, s, axes, norm)


def ihfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return ihfftn(x, s, axes, norm)


def fftfreq(n, d=1.0, dtype=None, name=None):
    from .framework.dtype import to_torch_dtype
    return torch.fft.fftfreq(n, d=d, dtype=to_torch_dtype(dtype) if dtype else None)


def rfftfreq(n, d=1.0, dtype=None, name=None):
    from .framework.dtype import to_torch_dtype
    return torch.fft.rfftfreq(n, d=d, dtype=to_torch_dtype(dtype) if dtype else None)


def fftshift(x, axes=None, name=None):
    return torch.fft.fftshift(_t(x), dim=axes)


def ifftshift(x, axes=None, name=None):
    return torch.fft.ifftshift(_t(x), dim=axes)
