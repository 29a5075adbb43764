"""``paddle.callbacks`` (reference `python/paddle/callbacks.py`)."""
from .hapi.callbacks import (Callback, ProgBarLogger, ModelCheckpoint, EarlyStopping,  # noqa: F401
                             LRScheduler, ReduceLROnPlateau, VisualDL)
