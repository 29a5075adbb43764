"""``paddle.incubate`` (reference `python/paddle/incubate/`): fused transformer layers and ops,
MoE, fused softmax-mask ops."""
from . import nn  # noqa: F401
from . import distributed  # noqa: F401
from . import moe  # noqa: F401
from . import autotune  # noqa: F401
from .nn.functional import softmax_mask_fuse, softmax_mask_fuse_upper_triangle  # noqa: F401
from . import optimizer  # noqa: F401,E402
from . import autograd  # noqa: F401,E402
from . import asp  # noqa: F401,E402
from .optimizer import LookAhead, ModelAverage  # noqa: F401,E402
from .tensor import (segment_sum, segment_mean, segment_max, segment_min,  # noqa: F401,E402
                     graph_send_recv, graph_reindex, graph_sample_neighbors, graph_khop_sampler,
                     identity_loss)
