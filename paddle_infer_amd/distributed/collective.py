"""Collective communication API (reference `python/paddle/distributed/collective.py`,
`communication/`, `paddle/fluid/distributed/collective/ProcessGroupNCCL.cc`).

Backend: ``nccl`` in torch.distributed is RCCL on ROCm — one process per MI355X, collectives over
xGMI; ``gloo`` on CPU. Paddle's list-returning signatures (``all_gather(tensor_list, tensor)``,
``alltoall(in_list, out_list)``) and ``use_calc_stream`` / ``sync_op`` flags are honoured:
``sync_op=False`` returns a task whose ``wait()`` makes the caller's stream wait (no host block).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class ReduceOp:
    SUM = dist.ReduceOp.SUM
    MAX = dist.ReduceOp.MAX
    MIN = dist.ReduceOp.MIN
    PROD = dist.ReduceOp.PRODUCT
    AVG = "avg"


class Group:
    """Paddle-style group handle around a torch ProcessGroup."""

    def __init__(self, pg, ranks, gid=0):
        self.pg, self.ranks, self.id = pg, list(ranks), gid

    @property
    def rank(self):
        g = dist.get_rank()
        return self.ranks.index(g) if g in self.ranks else -1

    @property
    def nranks(self):
        return len(self.ranks)

    world_size = nranks

    def is_member(self):
        return dist.get_rank() in self.ranks

    def get_group_rank(self, rank):
        return self.ranks.index(rank) if rank in self.ranks else -1

    def __repr__(self):
        return f"Group(id={self.id}, ranks={self.ranks})"


_GROUPS = {}


def _pg(group):
    if group is None:
        return None
    return group.pg if isinstance(group, Group) else group


def collectives_forced() -> bool:
    """``PIAMD_FORCE_COLLECTIVES=1``: the data / tensor-parallel engines issue their collectives
    even over a 1-rank group (the RCCL code paths — reduce-scatter hooks, async all-reduces, comm
    streams, ``record_stream`` — exercised on a single GPU; `tests/test_rccl_world1_gpu.py`)."""
    import os
    return os.environ.get("PIAMD_FORCE_COLLECTIVES", "0") == "1" and dist.is_available() and dist.is_initialized()


def multi_rank(group=None) -> bool:
    """True when collectives over ``group`` must run (world > 1, or forced on a 1-rank group)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    pg = _pg(group) if group is not None else None
    return dist.get_world_size(pg) > 1 or collectives_forced()


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def get_rank(group=None):
    if not is_initialized():
        return 0
    return dist.get_rank(_pg(group)) if group is not None else dist.get_rank()


def get_world_size(group=None):
    if not is_initialized():
        return 1
    return dist.get_world_size(_pg(group)) if group is not None else dist.get_world_size()


def new_group(ranks=None, backend=None, timeout=None):
    ranks = list(range(get_world_size())) if ranks is None else sorted(ranks)
    pg = dist.new_group(ranks, backend=backend) if is_initialized() else None
    g = Group(pg, ranks, len(_GROUPS) + 1)
    _GROUPS[g.id] = g
    return g


_RINGS = {}  # ring_id -> Group bound by a program helper (e.g. the mp ring of hybrid inference)


def bind_ring(ring_id, group):
    """Make program ops with ``ring_id`` run on ``group`` (reference c_comm_init of a ring)."""
    _RINGS[int(ring_id)] = group


def get_group(id=0):  # noqa: A002
    if id in _RINGS:
        return _RINGS[id]
    if id == 0:
        return Group(None, list(range(get_world_size())), 0)
    return _GROUPS.get(id)


def destroy_process_group(group=None):
    if group is None:
        if is_initialized():
            dist.destroy_process_group()
        _GROUPS.clear()
    else:
        dist.destroy_process_group(_pg(group))


def _ret(work, sync_op):
    if work is None:
        return None
    if sync_op:
        work.wait()
        return None
    return work


def all_reduce(tensor, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=None):
    if get_world_size(group) == 1:
        return None
    if op == ReduceOp.AVG:
        w = dist.all_reduce(tensor, dist.ReduceOp.SUM, group=_pg(group), async_op=not sync_op)
        if sync_op:
            tensor.div_(get_world_size(group))
        return w
    return _ret(dist.all_reduce(tensor, op, group=_pg(group), async_op=True), sync_op)


def broadcast(tensor, src, group=None, sync_op=True, use_calc_stream=None):
    if get_world_size(group) == 1:
        return None
    return _ret(dist.broadcast(tensor, src, group=_pg(group), async_op=True), sync_op)


def reduce(tensor, dst, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=None):
    if get_world_size(group) == 1:
        return None
    return _ret(dist.reduce(tensor, dst, op, group=_pg(group), async_op=True), sync_op)


def all_gather(tensor_list, tensor, group=None, sync_op=True, use_calc_stream=None):
    n = get_world_size(group)
    if n == 1:
        tensor_list.clear()
        tensor_list.append(tensor.clone())
        return None
    flat = torch.empty(n * tensor.numel(), dtype=tensor.dtype, device=tensor.device)
    dist.all_gather_into_tensor(flat, tensor.contiguous().view(-1), group=_pg(group))
    tensor_list.clear()
    tensor_list.extend(flat.view((n,) + tuple(tensor.shape)).unbind(0))
    return None


def all_gather_object(object_list, obj, group=None):
    n = get_world_size(group)
    out = [None] * n
    if n == 1:
        out = [obj]
    else:
        dist.all_gather_object(out, obj, group=_pg(group))
    object_list.clear()
    object_list.extend(out)


def reduce_scatter(tensor, tensor_list, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=None):
    if get_world_size(group) == 1:
        tensor.copy_(tensor_list[0])
        return None
    inp = torch.cat([t.reshape(-1) for t in tensor_list])
    return _ret(dist.reduce_scatter_tensor(tensor.view(-1), inp, op, group=_pg(group), async_op=True), sync_op)


def scatter(tensor, tensor_list=None, src=0, group=None, sync_op=True, use_calc_stream=None):
    n = get_world_size(group)
    if n == 1:
        tensor.copy_(tensor_list[0])
        return None
    if get_rank() == src:
        tl = [t.contiguous() for t in tensor_list]
    else:
        tl = None
    return _ret(dist.scatter(tensor, tl, src, group=_pg(group), async_op=True), sync_op)


def alltoall(in_tensor_list, out_tensor_list, group=None, sync_op=True, use_calc_stream=None):
    n = get_world_size(group)
    if n == 1:
        out_tensor_list.clear()
        out_tensor_list.extend(t.clone() for t in in_tensor_list)
        return None
    outs = [torch.empty_like(t) for t in in_tensor_list]
    ins = [t.contiguous() for t in in_tensor_list]
    if dist.get_backend(_pg(group)) == "gloo":  # gloo has no all_to_all: paired point-to-point
        me = get_rank(group)
        ranks = group.ranks if isinstance(group, Group) else list(range(n))
        ops = []
        for j in range(n):
            if j == me:
                outs[j].copy_(ins[j])
                continue
            ops.append(dist.P2POp(dist.isend, ins[j], ranks[j], _pg(group)))
            ops.append(dist.P2POp(dist.irecv, outs[j], ranks[j], _pg(group)))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    else:
        dist.all_to_all(outs, ins, group=_pg(group))
    out_tensor_list.clear()
    out_tensor_list.extend(outs)
    return None


def alltoall_single(in_tensor, out_tensor, in_split_sizes=None, out_split_sizes=None, group=None,
                    sync_op=True, use_calc_stream=None):
    if get_world_size(group) == 1:
        out_tensor.copy_(in_tensor)
        return None
    return _ret(dist.all_to_all_single(out_tensor, in_tensor, out_split_sizes, in_split_sizes,
                                       group=_pg(group), async_op=True), sync_op)


def send(tensor, dst=0, group=None, sync_op=True, use_calc_stream=None):
    return _ret(dist.isend(tensor.contiguous(), dst, group=_pg(group)), sync_op)


def recv(tensor, src=0, group=None, sync_op=True, use_calc_stream=None):
    return _ret(dist.irecv(tensor, src, group=_pg(group)), sync_op)


def isend(tensor, dst, group=None):
    return dist.isend(tensor.contiguous(), dst, group=_pg(group))


def irecv(tensor, src=None, group=None):
    return dist.irecv(tensor, src, group=_pg(group))


class P2POp:
    def __init__(self, op, tensor, peer, group=None):
        self.op, self.tensor, self.peer, self.group = op, tensor, peer, group

    def to_torch(self):
        fn = dist.isend if self.op in (isend, dist.isend, "isend") else dist.irecv
        return dist.P2POp(fn, self.tensor, self.peer, _pg(self.group))


def batch_isend_irecv(p2p_op_list):
    return dist.batch_isend_irecv([p.to_torch() for p in p2p_op_list])


def barrier(group=None):
    if get_world_size(group) > 1:
        dist.barrier(group=_pg(group))


def wait(tensor, group=None, use_calc_stream=True):
    if tensor.is_cuda:
        torch.cuda.current_stream().synchronize() if not use_calc_stream else None


def split(x, size, operation="linear", axis=0, num_partitions=1, gather_out=True, weight_attr=None,
          bias_attr=None, name=None):
    """Reference `distributed/collective.py:split` — build a model-parallel linear/embedding."""
    from .fleet.mp_layers import ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding
    from .fleet import get_hybrid_communicate_group
    hcg = get_hybrid_communicate_group()
    grp = hcg.get_model_parallel_group() if hcg else None
    if operation == "embedding":
        layer = VocabParallelEmbedding(size[0], size[1], weight_attr, mp_group=grp)
    elif axis == 1:
        layer = ColumnParallelLinear(size[0], size[1], weight_attr, bias_attr is not False, gather_out, mp_group=grp)
    else:
        layer = RowParallelLinear(size[0], size[1], weight_attr, bias_attr is not False, False, mp_group=grp)
    layer = layer.to(x.device)
    return layer(x)
