"""Audio feature layers (reference `audio/features/layers.py`)."""
from __future__ import annotations

import torch

from ..nn.layer.base import Layer
from .. import signal
from . import functional as AF

__all__ = ["LogMelSpectrogram", "MelSpectrogram", "MFCC", "Spectrogram"]


class Spectrogram(Layer):
    def __init__(self, n_fft=512, hop_length=512, win_length=None, window="hann", power=1.0,
                 center=True, pad_mode="reflect", dtype="float32"):
        super().__init__()
        assert power > 0, "Power of spectrogram must be > 0."
        self.power, self.n_fft, self.hop_length = power, n_fft, hop_length
        self.win_length = win_length or n_fft
        self.center, self.pad_mode = center, pad_mode
        self.register_buffer("fft_window", AF.get_window(window, self.win_length, True, dtype))

    def forward(self, x):
        s = signal.stft(x, self.n_fft, self.hop_length, self.win_length,
                        self.fft_window.to(x.device, x.dtype), self.center, self.pad_mode)
        return s.abs() ** self.power


class MelSpectrogram(Layer):
    def __init__(self, sr=22050, n_fft=2048, hop_length=512, win_length=None, window="hann",
                 power=2.0, center=True, pad_mode="reflect", n_mels=64, f_min=50.0, f_max=None,
                 htk=False, norm="slaney", dtype="float32"):
        super().__init__()
        self._spectrogram = Spectrogram(n_fft, hop_length, win_length, window, power, center,
                                        pad_mode, dtype)
        self.register_buffer("fbank_matrix", AF.compute_fbank_matrix(sr, n_fft, n_mels, f_min,
                                                                     f_max, htk, norm, dtype))

    def forward(self, x):
        spect = self._spectrogram(x)
        return torch.matmul(self.fbank_matrix.to(spect.device, spect.dtype), spect)


class LogMelSpectrogram(Layer):
    def __init__(self, sr=22050, n_fft=512, hop_length=None, win_length=None, window="hann",
                 power=2.0, center=True, pad_mode="reflect", n_mels=64, f_min=50.0, f_max=None,
                 htk=False, norm="slaney", ref_value=1.0, amin=1e-10, top_db=None, dtype="float32"):
        super().__init__()
        self._melspectrogram = MelSpectrogram(sr, n_fft, hop_length, win_length, window, power,
                                              center, pad_mode, n_mels, f_min, f_max, htk, norm,
                                              dtype)
        self.ref_value, self.amin, self.top_db = ref_value, amin, top_db

    def forward(self, x):
        return AF.power_to_db(self._melspectrogram(x), self.ref_value, self.amin, self.top_db)


class MFCC(Layer):
    def __init__(self, sr=22050, n_mfcc=40, n_fft=512, hop_length=None, win_length=None,
                 window="hann", power=2.0, center=True, pad_mode="reflect", n_mels=64, f_min=50.0,
                 f_max=None, htk=False, norm="slaney", ref_value=1.0, amin=1e-10, top_db=None,
                 dtype="float32"):
        super().__init__()
        assert n_mfcc <= n_mels, "n_mfcc cannot be larger than n_mels"
        self._log_melspectrogram = LogMelSpectrogram(sr, n_fft, hop_length, win_length, window,
                                                     power, center, pad_mode, n_mels, f_min,
                                                     f_max, htk, norm, ref_value, amin, top_db,
                                                     dtype)
        self.register_buffer("dct_matrix", AF.create_dct(n_mfcc, n_mels, "ortho", dtype))

    def forward(self, x):
        lm = self._log_melspectrogram(x)  # [N, n_mels, frames]
        return torch.matmul(lm.transpose(-1, -2), self.dct_matrix.to(lm.device, lm.dtype)).transpose(-1, -2)
