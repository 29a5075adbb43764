"""``paddle.distributed.communication`` (reference `distributed/communication/`): the collective
API plus the ``stream`` variants (``use_calc_stream=True`` runs on the compute stream — on ROCm
RCCL enqueues on the caller's current HIP stream when the op is synchronous, so the calc-stream
form is the synchronous call without the extra event wait)."""
from ..collective import (all_reduce, all_gather, alltoall, alltoall_single, broadcast, reduce,  # noqa: F401
                          reduce_scatter, recv, scatter, send, ReduceOp, Group, new_group,
                          get_group, barrier)
from . import stream  # noqa: F401
