"""``paddle.regularizer`` (reference `python/paddle/regularizer.py`): L1Decay / L2Decay, accepted
by every optimizer's ``weight_decay`` and by ``ParamAttr(regularizer=...)``."""
from .optimizer import L1Decay, L2Decay  # noqa: F401

__all__ = ["L1Decay", "L2Decay"]
