"""``paddle.signal`` — frame / overlap_add / stft / istft (reference `python/paddle/signal.py`).

``frame`` and ``overlap_add`` follow Paddle's layout: with ``axis=-1`` the frames are
``[..., frame_length, num_frames]``; with ``axis=0`` ``[num_frames, frame_length, ...]``.
STFT/ISTFT run on hipFFT through ``torch.stft`` with Paddle's argument semantics (``onesided``,
``normalized``, window defaults to a rectangular window of ``win_length``)."""
from __future__ import annotations

import torch

__all__ = ["stft", "istft", "frame", "overlap_add"]


def frame(x, frame_length, hop_length, axis=-1, name=None):
    if axis not in (0, -1):
        raise ValueError("Unexpected axis: it should be 0 or -1")
    if axis == -1:
        f = x.unfold(-1, frame_length, hop_length)  # [..., num_frames, frame_length]
        return f.transpose(-1, -2).contiguous()
    f = x.unfold(0, frame_length, hop_length)  # [num_frames, ..., frame_length]
    return f.movedim(-1, 1).contiguous()


def overlap_add(x, hop_length, axis=-1, name=None):
    if axis not in (0, -1):
        raise ValueError("Unexpected axis: it should be 0 or -1")
    if axis == -1:
        fl, nf = x.shape[-2], x.shape[-1]
        lead = x.shape[:-2]
        xf = x.reshape(-1, fl, nf)
    else:
        nf, fl = x.shape[0], x.shape[1]
        lead = x.shape[2:]
        xf = x.reshape(nf, fl, -1).permute(2, 1, 0)
    L = (nf - 1) * hop_length + fl
    out = torch.nn.functional.fold(xf, (1, L), (1, fl), stride=(1, hop_length)).reshape(-1, L)
    if axis == -1:
        return out.reshape(*lead, L)
    return out.t().reshape(L, *lead)


def stft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, pad_mode="reflect",
         normalized=False, onesided=True, name=None):
    win_length = win_length or n_fft
    hop_length = hop_length or n_fft // 4
    if window is None:
        window = torch.ones(win_length, dtype=x.real.dtype if x.is_complex() else x.dtype,
                            device=x.device)
    return torch.stft(x, n_fft, hop_length, win_length, window, center=center, pad_mode=pad_mode,
                      normalized=normalized, onesided=onesided if not x.is_complex() else False,
                      return_complex=True)


def istft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, normalized=False,
          onesided=True, length=None, return_complex=False, name=None):
    win_length = win_length or n_fft
    hop_length = hop_length or n_fft // 4
    if window is None:
        window = torch.ones(win_length, dtype=x.real.dtype, device=x.device)
    return torch.istft(x, n_fft, hop_length, win_length, window, center=center,
                       normalized=normalized, onesided=onesided, length=length,
                       return_complex=return_complex)
