"""``paddle.incubate`` (reference `python/paddle/incubate/`): fused transformer layers and ops,
MoE, fused softmax-mask ops."""
from . import nn  # noqa: F401
from . import distributed  # noqa: F401
from . import moe  # noqa: F401
from . import autotune  # noqa: F401
from .nn.functional import softmax_mask_fuse, softmax_mask_fuse_upper_triangle  # noqa: F401
