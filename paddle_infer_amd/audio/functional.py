"""Audio DSP helpers (reference `audio/functional/functional.py`, `window.py`)."""
from __future__ import annotations

import math

import numpy as np
import torch

__all__ = ["compute_fbank_matrix", "create_dct", "fft_frequencies", "hz_to_mel", "mel_frequencies",
           "mel_to_hz", "power_to_db", "get_window"]


def _dt(dtype):
    from ..framework.dtype import to_torch_dtype
    return to_torch_dtype(dtype)


def hz_to_mel(freq, htk=False):
    t = isinstance(freq, torch.Tensor)
    f = freq if t else torch.tensor(float(freq), dtype=torch.float64)
    if htk:
        m = 2595.0 * torch.log10(1.0 + f / 700.0)
    else:
        f_sp = 200.0 / 3
        m = f / f_sp
        min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, math.log(6.4) / 27.0
        m = torch.where(f >= min_log_hz, min_log_mel + torch.log(torch.clamp(f, min=1e-10) / min_log_hz) / logstep, m)
    return m if t else float(m)


def mel_to_hz(mel, htk=False):
    t = isinstance(mel, torch.Tensor)
    m = mel if t else torch.tensor(float(mel), dtype=torch.float64)
    if htk:
        f = 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    else:
        f_sp = 200.0 / 3
        f = f_sp * m
        min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, math.log(6.4) / 27.0
        f = torch.where(m >= min_log_mel, min_log_hz * torch.exp(logstep * (m - min_log_mel)), f)
    return f if t else float(f)


def mel_frequencies(n_mels=64, f_min=0.0, f_max=11025.0, htk=False, dtype="float32"):
    lo, hi = hz_to_mel(float(f_min), htk), hz_to_mel(float(f_max), htk)
    mels = torch.linspace(lo, hi, n_mels, dtype=torch.float64)
    return mel_to_hz(mels, htk).to(_dt(dtype))


def fft_frequencies(sr, n_fft, dtype="float32"):
    return torch.linspace(0, float(sr) / 2, int(1 + n_fft // 2), dtype=_dt(dtype))


def compute_fbank_matrix(sr, n_fft, n_mels=64, f_min=0.0, f_max=None, htk=False, norm="slaney",
                         dtype="float32"):
    f_max = float(sr) / 2 if f_max is None else f_max
    fftfreqs = fft_frequencies(sr, n_fft, "float64")
    mel_f = mel_frequencies(n_mels + 2, f_min, f_max, htk, "float64")
    fdiff = mel_f[1:] - mel_f[:-1]
    ramps = mel_f[:, None] - fftfreqs[None, :]
    lower = -ramps[:n_mels] / fdiff[:n_mels, None]
    upper = ramps[2:n_mels + 2] / fdiff[1:n_mels + 1, None]
    w = torch.clamp(torch.minimum(lower, upper), min=0.0)
    if norm == "slaney":
        enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
        w = w * enorm[:, None]
    elif isinstance(norm, (int, float)):
        w = w / torch.linalg.vector_norm(w, ord=norm, dim=-1, keepdim=True).clamp_min(1e-10)
    return w.to(_dt(dtype))


def power_to_db(spect, ref_value=1.0, amin=1e-10, top_db=80.0):
    if amin <= 0:
        raise ValueError("amin must be strictly positive")
    if ref_value <= 0:
        raise ValueError("ref_value must be strictly positive")
    log_spec = 10.0 * torch.log10(torch.clamp(spect, min=amin))
    log_spec = log_spec - 10.0 * math.log10(max(amin, ref_value))
    if top_db is not None:
        if top_db < 0:
            raise ValueError("top_db must be non-negative")
        log_spec = torch.maximum(log_spec, log_spec.max() - top_db)
    return log_spec


def create_dct(n_mfcc, n_mels, norm="ortho", dtype="float32"):
    n = torch.arange(n_mels, dtype=torch.float64)
    k = torch.arange(n_mfcc, dtype=torch.float64).unsqueeze(1)
    dct = torch.cos(math.pi / float(n_mels) * (n + 0.5) * k)  # [n_mfcc, n_mels]
    if norm is None:
        dct = dct * 2.0
    else:
        assert norm == "ortho"
        dct[0] *= 1.0 / math.sqrt(2.0)
        dct = dct * math.sqrt(2.0 / float(n_mels))
    return dct.t().to(_dt(dtype))


def get_window(window, win_length, fftbins=True, dtype="float64"):
    """Window by name (or ``(name, param)``), scipy.signal conventions (periodic when fftbins)."""
    from scipy.signal import get_window as _gw
    w = _gw(window, win_length, fftbins=fftbins)
    return torch.from_numpy(np.asarray(w, dtype=np.float64)).to(_dt(dtype))
