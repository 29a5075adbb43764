"""``paddle.fft`` — discrete Fourier transforms (reference `python/paddle/fft.py`).

Paddle's argument names (``n, axis, norm`` / ``s, axes``) and normalisation modes
("backward" | "forward" | "ortho") over the rocFFT-backed ``torch.fft`` kernels (hipFFT on
MI355X); real inputs of the c2c transforms are promoted to complex like the reference.
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


def fft(x, n=None, axis=-1, norm="backward", name=None):
    return torch.fft.fft(_t(x), n=n, dim=axis, norm=_norm(norm))


def ifft(x, n=None, axis=-1, norm="backward", name=None):
    return torch.fft.ifft(_t(x), n=n, dim=axis, norm=_norm(norm))


def rfft(x, n=None, axis=-1, norm="backward", name=None):
    return torch.fft.rfft(_t(x), n=n, dim=axis, norm=_norm(norm))


def irfft(x, n=None, axis=-1, norm="backward", name=None):
    return torch.fft.irfft(_t(x), n=n, dim=axis, norm=_norm(norm))


def hfft(x, n=None, axis=-1, norm="backward", name=None):
    return torch.fft.hfft(_t(x), n=n, dim=axis, norm=_norm(norm))


def ihfft(x, n=None, axis=-1, norm="backward", name=None):
    return torch.fft.ihfft(_t(x), n=n, dim=axis, norm=_norm(norm)).resolve_conj()


def fftn(x, s=None, axes=None, norm="backward", name=None):
    return torch.fft.fftn(_t(x), s=s, dim=axes, norm=_norm(norm))


def ifftn(x, s=None, axes=None, norm="backward", name=None):
    return torch.fft.ifftn(_t(x), s=s, dim=axes, norm=_norm(norm))


def rfftn(x, s=None, axes=None, norm="backward", name=None):
    return torch.fft.rfftn(_t(x), s=s, dim=axes, norm=_norm(norm))


def irfftn(x, s=None, axes=None, norm="backward", name=None):
    return torch.fft.irfftn(_t(x), s=s, dim=axes, norm=_norm(norm))


def hfftn(x, s=None, axes=None, norm="backward", name=None):
    return torch.fft.hfftn(_t(x), s=s, dim=axes, norm=_norm(norm))


def ihfftn(x, s=None, axes=None, norm="backward", name=None):
    return torch.fft.ihfftn(_t(x), s=s, dim=axes, norm=_norm(norm)).resolve_conj()


def fft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return torch.fft.fft2(_t(x), s=s, dim=axes, norm=_norm(norm))


def ifft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return torch.fft.ifft2(_t(x), s=s, dim=axes, norm=_norm(norm))


def rfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return torch.fft.rfft2(_t(x), s=s, dim=axes, norm=_norm(norm))


def irfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return torch.fft.irfft2(_t(x), s=s, dim=axes, norm=_norm(norm))


def hfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return torch.fft.hfft2(_t(x), s=s, dim=axes, norm=_norm(norm))


def ihfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return torch.fft.ihfft2(_t(x), s=s, dim=axes, norm=_norm(norm)).resolve_conj()


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
