"""``paddle.incubate`` segment / graph ops (reference `incubate/tensor/math.py`,
`incubate/operators/graph_*`): aliases of ``paddle.geometric``."""
from ..geometric import (segment_sum, segment_mean, segment_max, segment_min,  # noqa: F401
                         send_u_recv, reindex_graph, sample_neighbors)


def graph_send_recv(x, src_index, dst_index, pool_type="sum", out_size=None, name=None):
    return send_u_recv(x, src_index, dst_index, pool_type, out_size)


def graph_reindex(x, neighbors, count, value_buffer=None, index_buffer=None, flag_buffer_hashtable=False,
                  name=None):
    return reindex_graph(x, neighbors, count)


def graph_sample_neighbors(row, colptr, input_nodes, eids=None, perm_buffer=None, sample_size=-1,
                           return_eids=False, flag_perm_buffer=False, name=None):
    return sample_neighbors(row, colptr, input_nodes, sample_size, eids, return_eids)


def graph_khop_sampler(row, colptr, input_nodes, sample_sizes, sorted_eids=None, return_eids=False,
                       name=None):
    """Multi-hop sampling: returns (edge_src, edge_dst, sample_index, reindex_nodes[, edge_eids])."""
    import torch
    nodes = input_nodes
    srcs, dsts = [], []
    frontier = input_nodes
    for k in sample_sizes:
        nb, cnt = sample_neighbors(row, colptr, frontier, k)
        srcs.append(nb)
        dsts.append(torch.repeat_interleave(frontier, cnt.long()))
        frontier = torch.unique(nb)
        nodes = torch.cat([nodes, nb])
    src, dst = torch.cat(srcs), torch.cat(dsts)
    uniq = []
    seen = {}
    for v in nodes.tolist():
        if v not in seen:
            seen[v] = len(uniq)
            uniq.append(v)
    remap = lambda t: torch.tensor([seen[v] for v in t.tolist()], dtype=t.dtype, device=t.device)  # noqa: E731
    sample_index = torch.tensor(uniq, dtype=input_nodes.dtype, device=input_nodes.device)
    return remap(src), remap(dst), sample_index, remap(input_nodes)


def identity_loss(x, reduction="none"):
    """Reference `incubate.identity_loss` (IPU): marks ``x`` as the loss; reduction sum/mean/none."""
    r = {0: "sum", 1: "mean", 2: "none"}.get(reduction, reduction)
    return x.sum() if r == "sum" else x.mean() if r == "mean" else x
