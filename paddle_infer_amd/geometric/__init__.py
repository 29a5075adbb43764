"""``paddle.geometric`` (reference `python/paddle/geometric/`): graph message passing, segment
reductions, neighbour sampling and reindexing.

Message passing gathers source rows and reduces them into destination rows with the device
``scatter_reduce`` kernels (sum / mean / max / min); empty destinations get 0 like the reference.
"""
from __future__ import annotations

import torch

__all__ = ["send_u_recv", "send_ue_recv", "send_uv", "segment_sum", "segment_mean", "segment_min",
           "segment_max", "reindex_graph", "reindex_heter_graph", "sample_neighbors",
           "weighted_sample_neighbors"]

_RED = {"sum": "sum", "mean": "mean", "max": "amax", "min": "amin"}


def _reduce(msg, dst, n, reduce_op):
    reduce_op = reduce_op.lower()
    shape = (n,) + tuple(msg.shape[1:])
    out = torch.zeros(shape, dtype=msg.dtype, device=msg.device)
    if msg.shape[0] == 0:
        return out
    idx = dst.long().view(-1, *([1] * (msg.dim() - 1))).expand_as(msg)
    out = out.scatter_reduce(0, idx, msg, _RED[reduce_op], include_self=False)
    return out


def send_u_recv(x, src_index, dst_index, reduce_op="sum", out_size=None, name=None):
    n = x.shape[0] if out_size is None or int(out_size) <= 0 else int(out_size)
    return _reduce(x.index_select(0, src_index.long()), dst_index, n, reduce_op)


def _combine(a, b, op):
    return {"add": a + b, "sub": a - b, "mul": a * b, "div": a / b}[op.lower()]


def send_ue_recv(x, y, src_index, dst_index, message_op="add", reduce_op="sum", out_size=None,
                 name=None):
    n = x.shape[0] if out_size is None or int(out_size) <= 0 else int(out_size)
    msg = _combine(x.index_select(0, src_index.long()), y, message_op)
    return _reduce(msg, dst_index, n, reduce_op)


def send_uv(x, y, src_index, dst_index, message_op="add", name=None):
    return _combine(x.index_select(0, src_index.long()), y.index_select(0, dst_index.long()), message_op)


def _segment(data, segment_ids, op):
    n = int(segment_ids.max().item()) + 1 if segment_ids.numel() else 0
    return _reduce(data, segment_ids, n, op)


def segment_sum(data, segment_ids, name=None):
    return _segment(data, segment_ids, "sum")


def segment_mean(data, segment_ids, name=None):
    return _segment(data, segment_ids, "mean")


def segment_max(data, segment_ids, name=None):
    return _segment(data, segment_ids, "max")


def segment_min(data, segment_ids, name=None):
    return _segment(data, segment_ids, "min")


def reindex_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    """Renumber ``x`` (0..len(x)-1) then the unseen neighbours in first-appearance order.
    Returns (reindex_src, reindex_dst, out_nodes)."""
    xs = x.tolist()
    mapping = {v: i for i, v in enumerate(xs)}
    out_nodes = list(xs)
    src = []
    for v in neighbors.tolist():
        if v not in mapping:
            mapping[v] = len(out_nodes)
            out_nodes.append(v)
        src.append(mapping[v])
    dst = []
    for i, c in enumerate(count.tolist()):
        dst += [i] * int(c)
    dev = x.device
    return (torch.tensor(src, dtype=x.dtype, device=dev), torch.tensor(dst, dtype=x.dtype, device=dev),
            torch.tensor(out_nodes, dtype=x.dtype, device=dev))


def reindex_heter_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    """Heterogeneous variant: ``neighbors`` / ``count`` are lists (one per edge type) sharing one
    node numbering."""
    xs = x.tolist()
    mapping = {v: i for i, v in enumerate(xs)}
    out_nodes = list(xs)
    src, dst = [], []
    for nb, cnt in zip(neighbors, count):
        for v in nb.tolist():
            if v not in mapping:
                mapping[v] = len(out_nodes)
                out_nodes.append(v)
            src.append(mapping[v])
        for i, c in enumerate(cnt.tolist()):
            dst += [i] * int(c)
    dev = x.device
    return (torch.tensor(src, dtype=x.dtype, device=dev), torch.tensor(dst, dtype=x.dtype, device=dev),
            torch.tensor(out_nodes, dtype=x.dtype, device=dev))


def _sample(row, colptr, input_nodes, sample_size, weights, eids, return_eids, perm_buffer, gen):
    rows, counts, out_eids = [], [], []
    for v in input_nodes.tolist():
        a, b = int(colptr[v]), int(colptr[v + 1])
        deg = b - a
        if sample_size < 0 or deg <= sample_size:
            pick = torch.arange(a, b)
        elif weights is None:
            pick = a + torch.randperm(deg, generator=gen)[:sample_size]
        else:
            pick = a + torch.multinomial(weights[a:b].float().cpu(), sample_size, replacement=False,
                                         generator=gen)
        rows.append(row.cpu()[pick])
        counts.append(len(pick))
        if return_eids:
            out_eids.append(eids.cpu()[pick])
    dev = row.device
    nb = torch.cat(rows).to(dev) if rows else row[:0]
    cnt = torch.tensor(counts, dtype=row.dtype if row.dtype in (torch.int32, torch.int64) else torch.int64,
                       device=dev)
    if return_eids:
        return nb, cnt, (torch.cat(out_eids).to(dev) if out_eids else eids[:0])
    return nb, cnt


def sample_neighbors(row, colptr, input_nodes, sample_size=-1, eids=None, return_eids=False,
                     perm_buffer=None, name=None):
    """Uniform neighbour sampling on a CSC graph (``row`` / ``colptr``)."""
    return _sample(row, colptr, input_nodes, sample_size, None, eids, return_eids, perm_buffer, None)


def weighted_sample_neighbors(row, colptr, edge_weight, input_nodes, sample_size=-1, eids=None,
                              return_eids=False, name=None):
    return _sample(row, colptr, input_nodes, sample_size, edge_weight, eids, return_eids, None, None)
