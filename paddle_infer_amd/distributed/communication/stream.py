"""``paddle.distributed.communication.stream`` (reference `communication/stream/*.py`)."""
from .. import collective as _c

__all__ = ["all_gather", "all_reduce", "alltoall", "alltoall_single", "broadcast", "reduce",
           "reduce_scatter", "recv", "scatter", "send"]


def all_reduce(tensor, op=_c.ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
    return _c.all_reduce(tensor, op, group, sync_op, use_calc_stream)


def all_gather(tensor_or_tensor_list, tensor, group=None, sync_op=True, use_calc_stream=False):
    if isinstance(tensor_or_tensor_list, list):
        return _c.all_gather(tensor_or_tensor_list, tensor, group, sync_op, use_calc_stream)
    import torch.distributed as dist
    w = dist.all_gather_into_tensor(tensor_or_tensor_list, tensor.contiguous(), group=_c._pg(group),
                                    async_op=not sync_op)
    return _c._ret(w, sync_op)


def alltoall(out_tensor_or_tensor_list, in_tensor_or_tensor_list, group=None, sync_op=True,
             use_calc_stream=False):
    if isinstance(in_tensor_or_tensor_list, list):
        return _c.alltoall(in_tensor_or_tensor_list, out_tensor_or_tensor_list, group, sync_op,
                           use_calc_stream)
    return _c.alltoall_single(in_tensor_or_tensor_list, out_tensor_or_tensor_list, None, None,
                              group, sync_op, use_calc_stream)


def alltoall_single(out_tensor, in_tensor, out_split_sizes=None, in_split_sizes=None, group=None,
                    sync_op=True, use_calc_stream=False):
    return _c.alltoall_single(in_tensor, out_tensor, in_split_sizes, out_split_sizes, group,
                              sync_op, use_calc_stream)


def broadcast(tensor, src=0, group=None, sync_op=True, use_calc_stream=False):
    return _c.broadcast(tensor, src, group, sync_op, use_calc_stream)


def reduce(tensor, dst=0, op=_c.ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
    return _c.reduce(tensor, dst, op, group, sync_op, use_calc_stream)


def reduce_scatter(tensor, tensor_or_tensor_list, op=_c.ReduceOp.SUM, group=None, sync_op=True,
                   use_calc_stream=False):
    if isinstance(tensor_or_tensor_list, list):
        return _c.reduce_scatter(tensor, tensor_or_tensor_list, op, group, sync_op, use_calc_stream)
    import torch.distributed as dist
    w = dist.reduce_scatter_tensor(tensor, tensor_or_tensor_list.contiguous(), op=op,
                                   group=_c._pg(group), async_op=not sync_op)
    return _c._ret(w, sync_op)


def recv(tensor, src=0, group=None, sync_op=True, use_calc_stream=False):
    return _c.recv(tensor, src, group, sync_op, use_calc_stream)


def scatter(tensor, tensor_or_tensor_list=None, src=0, group=None, sync_op=True,
            use_calc_stream=False):
    return _c.scatter(tensor, tensor_or_tensor_list, src, group, sync_op, use_calc_stream)


def send(tensor, dst=0, group=None, sync_op=True, use_calc_stream=False):
    return _c.send(tensor, dst, group, sync_op, use_calc_stream)
