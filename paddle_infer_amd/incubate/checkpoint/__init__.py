"""``paddle.fluid.incubate.checkpoint`` equivalent: auto checkpoint (``auto_checkpoint``)."""
from . import auto_checkpoint  # noqa: F401
from .auto_checkpoint import train_epoch_range  # noqa: F401
