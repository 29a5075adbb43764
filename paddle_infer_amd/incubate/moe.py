"""Mixture-of-Experts dispatch / combine and the fused MoE FFN.

Parity: reference `python/paddle/incubate/distributed/models/moe/moe_layer.py` (MoEScatter /
MoEGather over global_scatter / global_gather), `utils.py` (count_by_gate, limit_by_capacity)
and the fused inference op `fluid/operators/fused/fused_moe_op.cu` / `moe_expert_gemm.h`.

MI355X design: tokens are sorted by expert id once (one argsort), exchanged with a single
variable-split RCCL ``all_to_all_single`` over xGMI (expert parallel), each local expert runs one
contiguous hipBLASLt GEMM pair on its token segment, and the reverse all-to-all + one
``index_add_`` weighted by the gate values combines them. Dropped tokens (capacity) carry
expert id -1 and contribute zero.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .. import ops


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_splits, in_splits, group):
        ctx.splits = (out_splits, in_splits)
        ctx.group = group
        out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
        dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        out_splits, in_splits = ctx.splits
        gi = g.new_empty((sum(in_splits),) + tuple(g.shape[1:]))
        dist.all_to_all_single(gi, g.contiguous(), in_splits, out_splits, group=ctx.group)
        return gi, None, None, None


def _ws(group):
    if group is None:
        return 1
    return group.nranks if hasattr(group, "nranks") else dist.get_world_size(group)


def _pg(group):
    return getattr(group, "process_group", group)


def dispatch(x, expert_idx, num_local_expert, group=None):
    """x [T, E]; expert_idx [T, k] global expert ids (-1 = dropped). Returns
    (x_local [N_local, E] grouped by local expert, local_counts list[int], ctx)."""
    T, k = expert_idx.shape
    ws = _ws(group)
    ne_tot = num_local_expert * ws
    flat = expert_idx.reshape(-1)
    valid = flat >= 0
    key = torch.where(valid, flat, torch.full_like(flat, ne_tot))
    order = torch.argsort(key, stable=True)
    counts = torch.bincount(key, minlength=ne_tot + 1)[:ne_tot]
    nvalid = int(counts.sum())
    order = order[:nvalid]
    tok = order // k
    xs = x.index_select(0, tok)
    ctx = {"order": order, "tok": tok, "T": T, "k": k, "ws": ws, "ne": num_local_expert}
    if ws == 1:
        return xs, counts.tolist(), ctx
    pg = _pg(group)
    c2 = counts.view(ws, num_local_expert)
    recv = torch.empty_like(c2)
    dist.all_to_all_single(recv, c2.contiguous(), group=pg)
    send_splits = c2.sum(1).tolist()
    recv_splits = recv.sum(1).tolist()
    xr = _AllToAll.apply(xs, recv_splits, send_splits, pg)
    # xr is ordered (src rank, local expert); regroup by local expert
    rc = recv.cpu()
    seg_src, off = [], 0
    for r in range(ws):
        for e in range(num_local_expert):
            n = int(rc[r, e])
            seg_src.append((e, r, off, n))
            off += n
    perm = []
    for e in range(num_local_expert):
        for (ee, r, o, n) in seg_src:
            if ee == e and n:
                perm.append(torch.arange(o, o + n))
    perm = torch.cat(perm).to(x.device) if perm else torch.zeros(0, dtype=torch.long, device=x.device)
    ctx.update(perm=perm, send_splits=send_splits, recv_splits=recv_splits, pg=pg)
    local_counts = rc.sum(0).tolist()
    return xr.index_select(0, perm), local_counts, ctx


def combine(y_local, weights, ctx):
    """Inverse of :func:`dispatch`; weights [T, k] gate values. Returns [T, E]."""
    if ctx["ws"] > 1:
        inv = torch.empty_like(ctx["perm"])
        inv[ctx["perm"]] = torch.arange(ctx["perm"].numel(), device=inv.device)
        y = y_local.index_select(0, inv)
        y = _AllToAll.apply(y, ctx["send_splits"], ctx["recv_splits"], ctx["pg"])
    else:
        y = y_local
    w = weights.reshape(-1).index_select(0, ctx["order"]).to(y.dtype)
    out = y.new_zeros((ctx["T"], y.shape[-1]))
    return out.index_add(0, ctx["tok"], y * w[:, None])


def run_experts(x, counts, experts):
    """Apply ``experts[i]`` to its contiguous segment of ``x``."""
    outs, off = [], 0
    for e, n in enumerate(counts):
        if n:
            outs.append(experts[e](x[off:off + n]))
        off += n
    if not outs:
        return x[:0]
    return torch.cat(outs, 0)


def topk_gate(logits, k, renormalize=True):
    probs = torch.softmax(logits.float(), -1)
    val, idx = probs.topk(k, -1)
    if renormalize and k > 1:
        val = val / val.sum(-1, keepdim=True)
    return val, idx


def limit_by_capacity(idx, num_expert_total, capacity):
    """Drop (set -1) assignments beyond ``capacity`` tokens per expert, in token order."""
    flat = idx.reshape(-1)
    onehot = F.one_hot(flat.clamp_min(0), num_expert_total) * (flat >= 0)[:, None]
    rank_in_expert = (onehot.cumsum(0) * onehot).sum(-1) - 1
    keep = (rank_in_expert < capacity) & (flat >= 0)
    return torch.where(keep, flat, torch.full_like(flat, -1)).reshape(idx.shape)


_STACK_CACHE = {}


def stacked(params):
    """[P_0, …, P_{E-1}] → one [E, …] tensor. Under no_grad (serving) the stack is cached until
    any expert parameter changes (keyed by storage + version); with grad it is rebuilt so the
    gradient flows back to every expert."""
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        return torch.stack(list(params))
    key = tuple((p.data_ptr(), p._version) for p in params)
    hit = _STACK_CACHE.get(key)
    if hit is None:
        if len(_STACK_CACHE) > 256:
            _STACK_CACHE.clear()
        hit = _STACK_CACHE[key] = torch.stack([p.detach() for p in params])
    return hit


def _grouped_ok(x, w1s, w2s):
    """The grouped MFMA path: bf16 on the GPU, K multiple of 64, N multiple of 256 for both."""
    if not (x.is_cuda and x.dtype == torch.bfloat16):
        return False
    H, Fd = w1s[0].shape
    return H % 256 == 0 and Fd % 256 == 0


def grouped_moe_ffn(x, idx, val, W1, B1, W2, B2, act="gelu"):
    """Expert FFN on one rank: sorted-row layout + two grouped GEMM launches (ops/moe.py)."""
    from ..ops import moe as gm
    r = gm.permute(idx, W1.shape[0])
    xs = gm.gather(x, r)
    ys = gm.grouped_ffn(xs, W1, B1, W2, B2, r, act)
    return gm.combine(ys, val, r)


def moe_ffn(x, gate_weight, gate_bias, w1s, b1s, w2s, b2s, top_k=2, act="gelu", group=None,
            capacity=None):
    """Fused MoE FFN (inference op ``fused_moe``): x [T, E] → [T, E]."""
    logits = torch.matmul(x, gate_weight)
    if gate_bias is not None:
        logits = logits + gate_bias
    val, idx = topk_gate(logits, top_k)
    if capacity is not None:
        idx = limit_by_capacity(idx, logits.shape[-1], capacity)
    if _ws(group) == 1 and _grouped_ok(x, w1s, w2s):
        nb = lambda bs, n: stacked(bs) if bs[0] is not None else None  # noqa: E731
        return grouped_moe_ffn(x, idx, val, stacked(w1s), nb(b1s, 0), stacked(w2s), nb(b2s, 0), act)
    xl, counts, ctx = dispatch(x, idx, len(w1s), group)

    def expert(e):
        def f(t):
            return torch.matmul(ops.bias_act(torch.matmul(t, w1s[e]), b1s[e], act), w2s[e]) + b2s[e]
        return f
    yl = run_experts(xl, counts, [expert(e) for e in range(len(w1s))])
    return combine(yl, val, ctx)
