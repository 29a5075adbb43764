"""Hybrid-parallel topology: dp × pp × sharding × mp process grid over torch.distributed.

Parity: reference `python/paddle/distributed/fleet/base/topology.py` (CommunicateTopology,
HybridCommunicateGroup, ParallelMode). Axis order is Paddle's — ``[data, pipe, sharding, model]``
with ``model`` fastest-varying — so a tensor-parallel group is a run of adjacent ranks: on an
8×MI355X node those are direct xGMI peers, and the per-layer TP all-reduces never leave the node.
All groups are RCCL (``nccl`` backend) on GPU, gloo on CPU.
"""
from __future__ import annotations

import itertools
from functools import reduce

import numpy as np
import torch.distributed as dist


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3


class CommunicateTopology:
    def __init__(self, hybrid_group_names=("data", "pipe", "sharding", "model"),
                 dims=(1, 1, 1, 1)):
        self._names = list(hybrid_group_names)
        self._dims = list(dims)
        self._world = reduce(lambda a, b: a * b, self._dims, 1)
        self._coords = list(itertools.product(*[range(d) for d in self._dims]))
        self._rank_of = {c: i for i, c in enumerate(self._coords)}

    def get_hybrid_group_names(self):
        return self._names

    def get_dim(self, axis_name):
        return self._dims[self._names.index(axis_name)]

    get_dim_size = get_dim

    def world_size(self):
        return self._world

    def get_rank(self, **kw):
        c = tuple(kw[n] for n in self._names)
        return self._rank_of[c]

    def get_coord(self, rank):
        return dict(zip(self._names, self._coords[rank]))

    def get_axis_list(self, axis_name, index):
        a = self._names.index(axis_name)
        return sorted(r for r, c in enumerate(self._coords) if c[a] == index)

    def get_comm_list(self, axis_name):
        """All rank lists that vary only along ``axis_name``."""
        a = self._names.index(axis_name)
        others = [range(d) for i, d in enumerate(self._dims) if i != a]
        out = []
        for oc in itertools.product(*others):
            ranks = []
            for k in range(self._dims[a]):
                c = list(oc)
                c.insert(a, k)
                ranks.append(self._rank_of[tuple(c)])
            out.append(ranks)
        return out

    def get_rank_from_stage(self, global_rank, **kw):
        c = self.get_coord(global_rank)
        c.update(kw)
        return self.get_rank(**c)


class HybridCommunicateGroup:
    """Builds one process group per axis slice; exposes Paddle's accessor names."""

    def __init__(self, topology: CommunicateTopology):
        self._topo = topology
        self.global_rank = dist.get_rank() if dist.is_initialized() else 0
        self.nranks = topology.world_size()
        self._dp_degree = topology.get_dim("data")
        self._pp_degree = topology.get_dim("pipe")
        self._sharding_degree = topology.get_dim("sharding")
        self._mp_degree = topology.get_dim("model")
        self._groups = {}
        self._ranks = {}
        for axis in self._topo.get_hybrid_group_names():
            for ranks in self._topo.get_comm_list(axis):
                g = None
                if dist.is_initialized() and dist.get_world_size() > 1:
                    g = dist.new_group(ranks) if len(ranks) > 1 else None
                if self.global_rank in ranks:
                    self._groups[axis] = g
                    self._ranks[axis] = ranks
        # data-parallel + sharding fused group for gradient reduction
        self._coord = self._topo.get_coord(self.global_rank)

    # ---- parallel mode -----------------------------------------------------------------
    def get_parallel_mode(self):
        if self._mp_degree == 1 and self._pp_degree == 1 and self._sharding_degree == 1:
            return ParallelMode.DATA_PARALLEL
        if self._pp_degree > 1:
            return ParallelMode.PIPELINE_PARALLEL
        if self._mp_degree > 1:
            return ParallelMode.TENSOR_PARALLEL
        return ParallelMode.SHARDING_PARALLEL

    def topology(self):
        return self._topo

    def get_global_rank(self):
        return self.global_rank

    # ---- data parallel -----------------------------------------------------------------
    def get_data_parallel_rank(self):
        return self._coord["data"]

    def get_data_parallel_world_size(self):
        return self._dp_degree

    def get_data_parallel_group(self):
        return self._groups.get("data")

    def get_data_parallel_group_src_rank(self):
        return self._ranks["data"][0]

    # ---- model parallel ----------------------------------------------------------------
    def get_model_parallel_rank(self):
        return self._coord["model"]

    def get_model_parallel_world_size(self):
        return self._mp_degree

    def get_model_parallel_group(self):
        return self._groups.get("model")

    def get_model_parallel_group_src_rank(self):
        return self._ranks["model"][0]

    # ---- pipeline ----------------------------------------------------------------------
    def get_stage_id(self):
        return self._coord["pipe"]

    def get_pipe_parallel_world_size(self):
        return self._pp_degree

    def get_pipe_parallel_group(self):
        return self._groups.get("pipe")

    def get_pipe_parallel_ranks(self):
        return self._ranks["pipe"]

    def is_first_stage(self):
        return self._coord["pipe"] == 0

    def is_last_stage(self):
        return self._coord["pipe"] == self._pp_degree - 1

    # ---- sharding ----------------------------------------------------------------------
    def get_sharding_parallel_rank(self):
        return self._coord["sharding"]

    def get_sharding_parallel_world_size(self):
        return self._sharding_degree

    def get_sharding_parallel_group(self):
        return self._groups.get("sharding")

    def get_sharding_parallel_group_src_rank(self):
        return self._ranks["sharding"][0]

    def get_sharding_parallel_group_ranks(self):
        return self._ranks["sharding"]

    def get_check_parallel_group(self, sharding=False):
        return self._groups.get("model")

    def ranks_of(self, axis):
        return self._ranks[axis]


def local_topology(dp=1, pp=1, sharding=1, mp=1):
    return CommunicateTopology(("data", "pipe", "sharding", "model"), (dp, pp, sharding, mp))


np  # noqa
