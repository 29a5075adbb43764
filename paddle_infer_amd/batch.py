"""``paddle.batch`` (reference `python/paddle/batch.py`)."""
from .reader import batch  # noqa: F401

__all__ = []
