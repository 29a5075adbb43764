"""``paddle.audio`` (reference `python/paddle/audio/`): window functions, mel filter banks,
dB conversion, DCT, and the Spectrogram / MelSpectrogram / LogMelSpectrogram / MFCC layers
(STFT on hipFFT via ``paddle.signal.stft``; the filter-bank / DCT products are plain GEMMs), plus
a WAV backend (``load`` / ``save`` / ``info``, 16-bit PCM via the stdlib ``wave`` module)."""
from . import functional, features, backends, datasets  # noqa: F401
from .backends import info, load, save  # noqa: F401

__all__ = ["functional", "features", "datasets", "backends", "load", "info", "save"]
