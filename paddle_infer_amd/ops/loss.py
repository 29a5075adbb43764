"""Softmax cross-entropy (single-device and vocab-parallel) backed by ``csrc/kernels/xent.hip``.

Parity: ``paddle.nn.functional.cross_entropy`` / ``softmax_with_cross_entropy`` (reference
`python/paddle/nn/functional/loss.py`) and ``fleet.meta_parallel.ParallelCrossEntropy``
(`c_softmax_with_cross_entropy_op.cu`).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import _lib


def _stats(logits2, labels, vocab_start, ignore_index):
    rows, V = logits2.shape
    m = torch.empty(rows, device=logits2.device, dtype=torch.float32)
    s = torch.empty_like(m)
    t = torch.empty_like(m)
    _lib.call("piamd_xent_stats", _lib.dtype_code(logits2, fp16=True), logits2.data_ptr(), labels.data_ptr(),
              rows, V, int(vocab_start), int(ignore_index), m.data_ptr(), s.data_ptr(), t.data_ptr(),
              _lib.stream())
    return m, s, t


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, group, inplace_backward):
        V = logits.shape[-1]
        lg = logits.contiguous().view(-1, V)
        lab = labels.contiguous().view(-1).to(torch.int64)
        vocab_start = 0
        if group is not None:
            vocab_start = dist.get_rank(group) * V
        m, s, t = _stats(lg, lab, vocab_start, ignore_index)
        if group is not None:
            M = m.clone()
            dist.all_reduce(M, op=dist.ReduceOp.MAX, group=group)
            s = s * torch.exp(m - M)
            dist.all_reduce(s, group=group)
            dist.all_reduce(t, group=group)
            m = M
        lse = torch.log(s) + m
        valid = lab != ignore_index
        loss = torch.where(valid, lse - t, torch.zeros_like(lse))
        ctx.save_for_backward(lg, lab, lse)
        ctx.meta = (ignore_index, vocab_start, inplace_backward, logits.shape)
        return loss.view(labels.shape)

    @staticmethod
    def backward(ctx, dloss):
        lg, lab, lse = ctx.saved_tensors
        ignore_index, vocab_start, inplace, shp = ctx.meta
        rows, V = lg.shape
        d = dloss.contiguous().view(-1).float()
        grad = lg if inplace else torch.empty_like(lg)
        _lib.call("piamd_xent_bwd", _lib.dtype_code(lg, fp16=True), lg.data_ptr(), lab.data_ptr(), lse.data_ptr(),
                  d.data_ptr(), 0.0, rows, V, int(vocab_start), int(ignore_index), grad.data_ptr(),
                  _lib.stream())
        return grad.view(shp), None, None, None, None


def _reference(logits, labels, ignore_index):
    V = logits.shape[-1]
    x = logits.float() if logits.element_size() < 4 else logits
    return F.cross_entropy(x.reshape(-1, V), labels.reshape(-1).long(),
                           ignore_index=ignore_index, reduction="none").view(labels.shape)


def softmax_cross_entropy(logits, labels, ignore_index: int = -100, group=None,
                          inplace_backward: bool = False):
    """Per-token loss (no reduction). ``group``: model-parallel group for vocab-sharded logits
    (each rank holds a contiguous V/mp slice, rank r owning [r*V_local, (r+1)*V_local))."""
    if logits.is_cuda and logits.dtype in (torch.bfloat16, torch.float16, torch.float32):
        return _XentFn.apply(logits, labels, ignore_index, group, inplace_backward)
    if group is not None and dist.get_world_size(group) > 1:
        return _parallel_reference(logits, labels, ignore_index, group)
    return _reference(logits, labels, ignore_index)


def vocab_parallel_softmax_xent(logits, labels, ignore_index=-100, group=None, rank=None):
    """Forward of the static ``c_softmax_with_cross_entropy`` op (reference
    `c_softmax_with_cross_entropy_op.cu`): this rank's vocab slice of the globally normalised
    softmax and the per-row loss. GPU: the row statistics (max, Σexp, target logit) come from
    ``xent.hip`` in one pass over the logits, all-reduced over ``group``; the softmax slice is one
    elementwise pass exp(x − lse). ``rank`` defaults to the group rank."""
    V = logits.shape[-1]
    lg = logits.reshape(-1, V)
    lab = labels.reshape(-1).to(torch.int64)
    if rank is None:
        rank = dist.get_rank(group) if group is not None else 0
    start = int(rank) * V
    if lg.is_cuda and lg.dtype in (torch.bfloat16, torch.float16, torch.float32):
        lgc = lg.contiguous()
        m, s, t = _stats(lgc, lab, start, ignore_index)
    else:
        x = lg.float()
        m = x.max(dim=-1).values
        s = torch.exp(x - m[:, None]).sum(-1)
        inr = (lab >= start) & (lab < start + V)
        idx = torch.where(inr, lab - start, torch.zeros_like(lab))
        t = torch.gather(x, -1, idx[:, None]).squeeze(-1) * inr
    if group is not None and dist.get_world_size(group) > 1:
        M = m.clone()
        dist.all_reduce(M, op=dist.ReduceOp.MAX, group=group)
        s = s * torch.exp(m - M)
        dist.all_reduce(s, group=group)
        dist.all_reduce(t, group=group)
        m = M
    lse = torch.log(s) + m
    loss = torch.where(lab != ignore_index, lse - t, torch.zeros_like(lse))
    softmax = torch.exp(lg.float() - lse[:, None]).to(logits.dtype)
    return softmax.reshape(logits.shape), loss.reshape(labels.shape)


def _parallel_reference(logits, labels, ignore_index, group):
    """Vocab-parallel CE composed from torch ops (CPU / gloo path)."""
    V = logits.shape[-1]
    rank = dist.get_rank(group)
    start = rank * V
    x = logits.float()
    m = x.max(dim=-1).values.detach()
    M = _AllReduceMax.apply(m, group)
    e = torch.exp(x - M.unsqueeze(-1))
    s = _AllReduceSum.apply(e.sum(-1), group)
    lab = labels.long()
    inr = (lab >= start) & (lab < start + V)
    idx = torch.where(inr, lab - start, torch.zeros_like(lab))
    t = torch.gather(x, -1, idx.unsqueeze(-1)).squeeze(-1) * inr
    t = _AllReduceSum.apply(t, group)
    loss = torch.log(s) + M - t
    return torch.where(lab != ignore_index, loss, torch.zeros_like(loss))


class _AllReduceSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        y = x.clone()
        dist.all_reduce(y, group=group)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None


class _AllReduceMax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        y = x.clone()
        dist.all_reduce(y, op=dist.ReduceOp.MAX, group=group)
        return y

    @staticmethod
    def backward(ctx, g):
        return torch.zeros_like(g), None
