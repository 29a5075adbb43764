"""Complex FFT core of ``paddle.fft`` on the framework's own kernels.

* power-of-two rows ≤ 4096 (complex64 on the GPU): ``fft.hip`` (LDS Stockham, batched rows);
* longer power-of-two rows: four-step (N = N1·N2: column FFTs, twiddle, row FFTs, transpose);
* any other length: Bluestein / chirp-z (a length-N DFT as a power-of-two circular convolution);
* CPU (and complex128): the same Stockham stages vectorised over rows in PyTorch.

Parity: reference `paddle/phi/kernels/funcs/fft.cu` + `fft_c2c/r2c/c2r` kernels (cuFFT plans).
"""
from __future__ import annotations

import math

import torch

from . import _lib

MAX_KERNEL_N = 4096


def _is_pow2(n):
    return n > 0 and (n & (n - 1)) == 0


def _stockham_torch(x, inverse):
    """Stockham radix-2 over the last dim (power-of-two length) in PyTorch ops."""
    N = x.shape[-1]
    lead = x.shape[:-1]
    x = x.reshape(-1, N)
    half = N // 2
    s = 0
    j = torch.arange(half, device=x.device)
    sgn = 1.0 if inverse else -1.0
    while (1 << s) < N:
        Ls = 1 << s
        k = j & (Ls - 1)
        ang = sgn * math.pi * k.to(torch.float64) / Ls
        w = torch.polar(torch.ones_like(ang), ang).to(x.dtype)
        a, b = x[:, :half], x[:, half:] * w
        y = torch.empty_like(x)
        o = ((j >> s) << (s + 1)) + k
        y[:, o] = a + b
        y[:, o + Ls] = a - b
        x = y
        s += 1
    return x.reshape(*lead, N)


class _KernelDFT(torch.autograd.Function):
    """`fft.hip` rows as an autograd op. y = F·x with F unitary up to scale, so the vector-Jacobian
    product (PyTorch's conjugate-Wirtinger convention) is Fᴴ·g: the unscaled DFT of the opposite
    sign — composes through four-step, Bluestein, r2c and c2r (reference fft_c2c_grad)."""

    @staticmethod
    def forward(ctx, x, inverse):
        ctx.inverse = inverse
        N = x.shape[-1]
        out = torch.empty_like(x)
        xc = x.contiguous()
        _lib.call("piamd_fft_c2c", xc.data_ptr(), out.data_ptr(), xc.numel() // N, N,
                  int(inverse), 1.0, _lib.stream())
        return out

    @staticmethod
    def backward(ctx, g):
        return _pow2(g.contiguous(), not ctx.inverse), None


def _pow2(x, inverse):
    """Unscaled DFT (sign by ``inverse``) of contiguous rows, power-of-two length."""
    N = x.shape[-1]
    if N == 1:
        return x.clone()
    if x.is_cuda and x.dtype == torch.complex64:
        if N <= MAX_KERNEL_N:
            return _KernelDFT.apply(x, inverse)
        return _four_step(x, inverse)
    return _stockham_torch(x, inverse)


def _four_step(x, inverse):
    """N = N1·N2 (N2 = 4096): X[k1 + N1·k2] = Σ_j2 W_N2^{j2·k2} W_N^{j2·k1} Σ_j1 x[j1·N2 + j2] W_N1^{j1·k1}."""
    N = x.shape[-1]
    N2 = MAX_KERNEL_N
    N1 = N // N2
    lead = x.shape[:-1]
    v = x.reshape(-1, N1, N2).transpose(1, 2).contiguous()            # [B, j2, j1]
    v = _pow2(v, inverse)                                               # [B, j2, k1]
    j2 = torch.arange(N2, device=x.device, dtype=torch.float64).unsqueeze(1)
    k1 = torch.arange(N1, device=x.device, dtype=torch.float64).unsqueeze(0)
    ang = (1.0 if inverse else -1.0) * 2.0 * math.pi * torch.remainder(j2 * k1, N) / N
    v = v * torch.polar(torch.ones_like(ang), ang).to(x.dtype)
    v = v.transpose(1, 2).contiguous()                                  # [B, k1, j2]
    v = _pow2(v, inverse)                                               # [B, k1, k2]
    return v.transpose(1, 2).reshape(*lead, N)                          # index k2·N1 + k1


def _bluestein(x, inverse):
    """Arbitrary-length unscaled DFT as a chirp-z circular convolution of power-of-two length."""
    N = x.shape[-1]
    M = 1 << (2 * N - 2).bit_length()
    n = torch.arange(N, device=x.device, dtype=torch.int64)
    sq = torch.remainder(n * n, 2 * N).to(torch.float64)
    sgn = 1.0 if inverse else -1.0
    ang = sgn * math.pi * sq / N
    chirp = torch.polar(torch.ones_like(ang), ang).to(x.dtype)          # exp(∓iπ n²/N)
    a = torch.zeros(*x.shape[:-1], M, dtype=x.dtype, device=x.device)
    a[..., :N] = x * chirp
    b = torch.zeros(M, dtype=x.dtype, device=x.device)
    cb = chirp.conj()
    b[:N] = cb
    b[M - N + 1:] = cb[1:].flip(0)
    conv = _pow2(_pow2(a, False) * _pow2(b, False), True) / M
    return conv[..., :N] * chirp


def dft(x, inverse=False):
    """Unscaled DFT along the LAST dim of a complex tensor (any length)."""
    x = x.contiguous()
    N = x.shape[-1]
    if N == 0:
        return x.clone()
    if _is_pow2(N):
        return _pow2(x, inverse)
    return _bluestein(x, inverse)


def c2c(x, axis=-1, n=None, inverse=False, norm="backward"):
    """Complex transform along ``axis`` with Paddle's ``n`` (zero-pad / truncate) and norm."""
    if not x.is_complex():
        x = x.to(torch.complex128 if x.dtype == torch.float64 else torch.complex64)
    axis = axis % x.dim()
    if n is not None:
        L = x.shape[axis]
        if n < L:
            x = x.narrow(axis, 0, n)
        elif n > L:
            pad = list(x.shape)
            pad[axis] = n - L
            x = torch.cat([x, torch.zeros(pad, dtype=x.dtype, device=x.device)], dim=axis)
    N = x.shape[axis]
    y = dft(x.movedim(axis, -1), inverse).movedim(-1, axis)
    if norm == "ortho":
        y = y / math.sqrt(N)
    elif (norm == "backward") == inverse and N:
        y = y / N
    return y
