"""Audio I/O backend (reference `audio/backends/`): 16-bit PCM WAV through the stdlib ``wave``
module (the only backend available without soundfile)."""
from __future__ import annotations

import wave
from dataclasses import dataclass

import numpy as np
import torch

__all__ = ["get_current_backend", "list_available_backends", "set_backend", "load", "save", "info"]

_BACKEND = {"name": "wave_backend"}


def list_available_backends():
    return ["wave_backend"]


def get_current_backend():
    return _BACKEND["name"]


def set_backend(backend_name):
    if backend_name not in list_available_backends():
        raise NotImplementedError(f"backend {backend_name} is not available")
    _BACKEND["name"] = backend_name


@dataclass
class AudioInfo:
    sample_rate: int
    num_frames: int
    num_channels: int
    bits_per_sample: int
    encoding: str


def info(filepath):
    with wave.open(str(filepath), "rb") as f:
        return AudioInfo(f.getframerate(), f.getnframes(), f.getnchannels(), 8 * f.getsampwidth(),
                         "PCM_S")


def load(filepath, frame_offset=0, num_frames=-1, normalize=True, channels_first=True):
    with wave.open(str(filepath), "rb") as f:
        sr, ch, sw = f.getframerate(), f.getnchannels(), f.getsampwidth()
        f.setpos(frame_offset)
        n = f.getnframes() - frame_offset if num_frames < 0 else num_frames
        raw = f.readframes(n)
    assert sw == 2, "wave_backend reads 16-bit PCM"
    a = np.frombuffer(raw, dtype="<i2").reshape(-1, ch)
    t = torch.from_numpy(a.astype(np.float32) / 32768.0 if normalize else a.astype(np.int16).copy())
    return (t.t().contiguous() if channels_first else t), sr


def save(filepath, src, sample_rate, channels_first=True, encoding=None, bits_per_sample=16):
    x = src.detach().cpu()
    x = x if x.dim() == 2 else x.unsqueeze(0 if channels_first else 1)
    if channels_first:
        x = x.t()
    if x.is_floating_point():
        x = (x.clamp(-1, 1) * 32767.0).round()
    a = x.to(torch.int16).numpy()
    with wave.open(str(filepath), "wb") as f:
        f.setnchannels(a.shape[1])
        f.setsampwidth(2)
        f.setframerate(int(sample_rate))
        f.writeframes(a.astype("<i2").tobytes())
