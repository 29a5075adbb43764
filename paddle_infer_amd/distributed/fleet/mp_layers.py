"""Tensor-parallel (Megatron-style) layers and their collective ops.

Parity: reference `python/paddle/distributed/fleet/layers/mpu/mp_layers.py`
(VocabParallelEmbedding:39, ColumnParallelLinear:155, RowParallelLinear:293,
ParallelCrossEntropy:438) and `mp_ops.py` (_c_identity, _mp_allreduce, _c_split, _c_concat).

Weights use Paddle's ``[in, out]`` layout: ColumnParallelLinear holds ``[in, out/mp]``,
RowParallelLinear ``[in/mp, out]``. The forward all-reduce of RowParallelLinear runs on RCCL over
the (intra-node, xGMI) model-parallel group.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ...nn.layer.base import Layer
from ...nn import initializer as I
from ...ops.linear import linear as _linear
from ...ops.loss import softmax_cross_entropy


def _ws(group):
    return dist.get_world_size(group) if group is not None else 1


def _rank(group):
    return dist.get_rank(group) if group is not None else 0


class _CIdentity(torch.autograd.Function):
    """fwd identity, bwd all-reduce (input of a column-parallel region)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        if _ws(ctx.group) > 1:
            g = g.contiguous()
            dist.all_reduce(g, group=ctx.group)
        return g, None


class _MPAllReduce(torch.autograd.Function):
    """fwd all-reduce, bwd identity (output of a row-parallel region)."""

    @staticmethod
    def forward(ctx, x, group):
        if _ws(group) > 1:
            x = x.contiguous()
            dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _CSplit(torch.autograd.Function):
    """fwd: keep this rank's slice of the last dim; bwd: all-gather."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        n = _ws(group)
        if n == 1:
            return x
        return x.chunk(n, dim=-1)[_rank(group)].contiguous()

    @staticmethod
    def backward(ctx, g):
        return _gather_last(g, ctx.group), None


class _CConcat(torch.autograd.Function):
    """fwd: all-gather along the last dim; bwd: split."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _gather_last(x, group)

    @staticmethod
    def backward(ctx, g):
        n = _ws(ctx.group)
        if n == 1:
            return g, None
        return g.chunk(n, dim=-1)[_rank(ctx.group)].contiguous(), None


def _gather_last(x, group):
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty(n * x.numel(), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x.view(-1), group=group)
    out = out.view((n,) + tuple(x.shape))
    return torch.cat(list(out.unbind(0)), dim=-1)


def c_identity(x, group=None):
    return _CIdentity.apply(x, group)


def mp_allreduce(x, group=None):
    return _MPAllReduce.apply(x, group)


def c_split(x, group=None):
    return _CSplit.apply(x, group)


def c_concat(x, group=None):
    return _CConcat.apply(x, group)


def _mark(p, distributed: bool, split_axis=None):
    p.is_distributed = distributed
    p.split_axis = split_axis
    return p


class VocabParallelEmbedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, weight_attr=None, mp_group=None, name=None,
                 dtype="float32"):
        super().__init__(dtype=dtype)
        self.group = mp_group
        n, r = _ws(mp_group), _rank(mp_group)
        assert num_embeddings % n == 0, "vocab must divide the mp degree"
        self.per_part = num_embeddings // n
        self.vocab_start = r * self.per_part
        self.embedding_dim = embedding_dim
        self.weight = self.create_parameter([self.per_part, embedding_dim], attr=weight_attr,
                                            default_initializer=I.XavierNormal())
        _mark(self.weight, n > 1, 0)

    def forward(self, x):
        from ...ops.embedding import embedding
        out = embedding(x, self.weight, self.vocab_start)  # zero rows outside this vocab shard
        if _ws(self.group) == 1:
            return out
        return mp_allreduce(out, self.group)


class ColumnParallelLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True,
                 gather_output=True, fuse_matmul_bias=False, mp_group=None, name=None,
                 dtype="float32"):
        super().__init__(dtype=dtype)
        self.group = mp_group
        n = _ws(mp_group)
        assert out_features % n == 0
        self.out_per_part = out_features // n
        self.gather_output = gather_output
        self.weight = self.create_parameter([in_features, self.out_per_part], attr=weight_attr,
                                            default_initializer=I.XavierUniform(in_features, out_features))
        _mark(self.weight, n > 1, 1)
        self.bias = self.create_parameter([self.out_per_part], is_bias=True) if has_bias else None
        if self.bias is not None:
            _mark(self.bias, n > 1, 0)

    def forward(self, x):
        x = c_identity(x, self.group)
        y = _linear(x, self.weight, self.bias)
        if self.gather_output and _ws(self.group) > 1:
            y = c_concat(y, self.group)
        return y


class RowParallelLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True,
                 input_is_parallel=False, fuse_matmul_bias=False, mp_group=None, name=None,
                 dtype="float32"):
        super().__init__(dtype=dtype)
        self.group = mp_group
        n = _ws(mp_group)
        assert in_features % n == 0
        self.in_per_part = in_features // n
        self.input_is_parallel = input_is_parallel
        self.weight = self.create_parameter([self.in_per_part, out_features], attr=weight_attr,
                                            default_initializer=I.XavierUniform(in_features, out_features))
        _mark(self.weight, n > 1, 0)
        self.bias = self.create_parameter([out_features], is_bias=True) if has_bias else None
        if self.bias is not None:
            _mark(self.bias, False)

    def forward(self, x):
        if not self.input_is_parallel:
            x = c_split(x, self.group)
        y = _linear(x, self.weight, None)
        y = mp_allreduce(y, self.group)
        return y + self.bias if self.bias is not None else y


class ParallelCrossEntropy(Layer):
    def __init__(self, mp_group=None, name=None, ignore_index=-100):
        super().__init__()
        self.group = mp_group
        self.ignore_index = ignore_index

    def forward(self, input, label):
        g = self.group if _ws(self.group) > 1 else None
        lab = label.squeeze(-1) if label.dim() == input.dim() else label
        return softmax_cross_entropy(input, lab, self.ignore_index, group=g).unsqueeze(-1)
