"""paddle_infer_amd — an MI355X-native deep-learning framework with PaddlePaddle's capabilities.

Compute path: PyTorch-ROCm tensors + autograd, hand-written CDNA4 HIP kernels (``ops``) for the
hot fused ops, hipBLASLt for plain GEMMs, RCCL over xGMI for collectives.
"""
__version__ = "0.1.0"

import torch as _torch  # noqa: F401  (must load before the HIP kernel library)

from .framework import random as _random
from .framework.random import seed, get_rng_state, set_rng_state  # noqa: F401
from . import ops  # noqa: F401
