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


def _coll(group):
    """Collectives over the mp group run (world > 1, or forced on a 1-rank group for testing)."""
    if group is None:
        return False
    from ..collective import collectives_forced
    return _ws(group) > 1 or collectives_forced()


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
        if _coll(ctx.group):
            g = g.contiguous()
            dist.all_reduce(g, group=ctx.group)
        return g, None


class _MPAllReduce(torch.autograd.Function):
    """fwd all-reduce, bwd identity (output of a row-parallel region)."""

    @staticmethod
    def forward(ctx, x, group):
        if _coll(group):
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


class _ColumnParallelFn(torch.autograd.Function):
    """``c_identity`` + linear of a column-parallel layer in one Function, so the backward
    overlaps the input-gradient all-reduce with the weight-gradient GEMM (reference
    `mp_layers.py:155` runs them back to back; this is the Megatron async-grad-allreduce order):
    dX = dY·Wᵀ → RCCL all-reduce of dX launched asynchronously → dW = Xᵀ·dY (+ dB) on the compute
    stream while the collective runs on RCCL's stream → wait."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, w, b, group):
        wc, bc = w, b
        if x.is_cuda and w.dtype == torch.float32 and torch.is_autocast_enabled("cuda"):
            # compute on an autocast-dtype copy; the weight gradient still goes to the fp32
            # parameter itself (its main_grad / grad-ready hook live there, ops/linear.py:264)
            dt = torch.get_autocast_dtype("cuda")
            x, wc, bc = x.to(dt), w.to(dt), b.to(dt) if b is not None else None
        with torch.no_grad():
            y = _linear(x, wc, bc)
        ctx.save_for_backward(x, w, wc)
        ctx.bias, ctx.group, ctx.shp = b, group, x.shape
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        from ...ops.linear import bias_grad, input_grad, weight_grad
        x, w, wc = ctx.saved_tensors
        x2 = x.reshape(-1, x.shape[-1])
        dy2 = dy.reshape(-1, w.shape[1]).contiguous()
        dx = work = None
        if ctx.needs_input_grad[0]:
            dx = input_grad(dy2, wc).view(ctx.shp).contiguous()
            if _coll(ctx.group):
                work = dist.all_reduce(dx, group=ctx.group, async_op=True)
        dw = None
        if ctx.needs_input_grad[1]:
            dw = weight_grad(x2, dy2, w)
            if dw is not None and dw.dtype != w.dtype:
                dw = dw.to(w.dtype)
        db = None
        if ctx.bias is not None and ctx.needs_input_grad[2]:
            db = bias_grad(dy2, ctx.bias)
            if db is not None and db.dtype != ctx.bias.dtype:
                db = db.to(ctx.bias.dtype)
        if work is not None:
            work.wait()
        return dx, dw, db, None


class _MPAllReduceBias(torch.autograd.Function):
    """Row-parallel output all-reduce whose bias was added by ONE rank's GEMM epilogue (rank 0):
    fwd all-reduce; bwd identity for the activation and, on the ranks that did not add the bias,
    its gradient Σ_rows dY — every rank ends with the same replicated bias gradient."""

    @staticmethod
    def forward(ctx, y, b, group):
        ctx.n = b.shape[-1]
        if _coll(group):
            y = y.contiguous()
            dist.all_reduce(y, group=group)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, g.reshape(-1, ctx.n).sum(0), None


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
        if torch.is_grad_enabled() and (self.weight.requires_grad or getattr(self.weight, "main_grad", None)
                                        is not None):
            y = _ColumnParallelFn.apply(x, self.weight, self.bias, self.group)
        else:
            if torch.is_grad_enabled() and x.requires_grad:
                # frozen weight (LoRA / BitFit): the input gradient still needs the mp all-reduce
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
        if self.bias is None or _ws(self.group) == 1:
            y = _linear(x, self.weight, self.bias)
            return mp_allreduce(y, self.group)
        # the bias rides rank 0's GEMM epilogue (added once before the sum), no separate pass
        if _rank(self.group) == 0:
            return mp_allreduce(_linear(x, self.weight, self.bias), self.group)
        return _MPAllReduceBias.apply(_linear(x, self.weight, None), self.bias, self.group)


class ParallelCrossEntropy(Layer):
    def __init__(self, mp_group=None, name=None, ignore_index=-100):
        super().__init__()
        self.group = mp_group
        self.ignore_index = ignore_index

    def forward(self, input, label):
        g = self.group if _ws(self.group) > 1 else None
        lab = label.squeeze(-1) if label.dim() == input.dim() else label
        return softmax_cross_entropy(input, lab, self.ignore_index, group=g).unsqueeze(-1)
