"""``paddle.distributed.fleet`` — collective hybrid parallelism.

Parity: reference `python/paddle/distributed/fleet/fleet.py` (init, distributed_model,
distributed_optimizer, worker_index/num), `base/distributed_strategy.py` (DistributedStrategy:
hybrid_configs, amp, recompute, sharding, pipeline, tensor_parallel, gradient_merge),
`meta_parallel/` and `meta_optimizers/dygraph_optimizer/hybrid_parallel_optimizer.py`.

``distributed_optimizer`` on GPU upgrades an AdamW/Adam to the flat-buffer engine with the
hybrid groups (bucketed reduce-scatter over the dp group when ``sharding`` is on, global-norm
clip across dp/mp/pp) — the same engine ``bench.py`` measures.
"""
from __future__ import annotations

import copy
import os

import torch
import torch.distributed as dist

from .topology import CommunicateTopology, HybridCommunicateGroup, ParallelMode  # noqa: F401
from .mp_layers import (VocabParallelEmbedding, ColumnParallelLinear, RowParallelLinear,  # noqa: F401
                        ParallelCrossEntropy)
from .pipeline import LayerDesc, SharedLayerDesc, PipelineLayer, PipelineParallel  # noqa: F401
from .recompute import recompute  # noqa: F401
from ...framework.random import get_rng_state_tracker, model_parallel_random_seed  # noqa: F401

_STATE = {"hcg": None, "strategy": None, "inited": False}


class DistributedStrategy:
    def __init__(self):
        self._hybrid = {"dp_degree": -1, "mp_degree": 1, "pp_degree": 1, "sharding_degree": 1,
                        "sep_degree": 1, "order": ["dp", "pp", "sharding", "mp"]}
        self.amp = False
        self.amp_configs = {"init_loss_scaling": 32768.0, "use_pure_fp16": False, "use_bf16": True}
        self.recompute = False
        self.recompute_configs = {"checkpoints": []}
        self.sharding = False
        self.sharding_configs = {"sharding_degree": 1, "stage": 1, "segment_broadcast_MB": 32}
        self.pipeline = False
        self.pipeline_configs = {"accumulate_steps": 1, "micro_batch_size": 1}
        self.tensor_parallel = False
        self.tensor_parallel_configs = {"tensor_parallel_degree": 1}
        self.gradient_merge = False
        self.gradient_merge_configs = {"k_steps": 1, "avg": True}
        self.lamb = self.lars = self.dgc = self.localsgd = self.asp = False
        self.fuse_all_reduce_ops = True
        self.fuse_grad_size_in_MB = 256
        self.find_unused_parameters = False
        self.without_graph_optimization = True
        self.a_sync = False
        self.heter_ccl_mode = False

    @property
    def hybrid_configs(self):
        return self._hybrid

    @hybrid_configs.setter
    def hybrid_configs(self, cfg):
        cfg = dict(cfg)
        pp = cfg.pop("pp_configs", None)
        self._hybrid.update(cfg)
        if pp:
            self.pipeline_configs.update(pp)

    def __repr__(self):
        return f"DistributedStrategy(hybrid={self._hybrid}, sharding={self.sharding}, amp={self.amp})"


class UserDefinedRoleMaker:
    def __init__(self, is_collective=True, **kw):
        self.kw = kw


class PaddleCloudRoleMaker(UserDefinedRoleMaker):
    pass


def init(role_maker=None, is_collective=True, strategy=None, log_level="INFO"):
    from ..parallel import init_parallel_env
    strategy = strategy or DistributedStrategy()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 or dist.is_initialized():
        init_parallel_env()
    world = dist.get_world_size() if dist.is_initialized() else 1
    h = strategy.hybrid_configs
    mp, pp = int(h.get("mp_degree", 1)), int(h.get("pp_degree", 1))
    sh = int(h.get("sharding_degree", 1))
    dp = int(h.get("dp_degree", -1))
    if dp in (-1, 0):
        dp = world // (mp * pp * sh)
    assert dp * mp * pp * sh == world, f"dp{dp}*mp{mp}*pp{pp}*sharding{sh} != world {world}"
    topo = CommunicateTopology(("data", "pipe", "sharding", "model"), (dp, pp, sh, mp))
    hcg = HybridCommunicateGroup(topo)
    _STATE.update(hcg=hcg, strategy=strategy, inited=True)
    model_parallel_random_seed(2048 + hcg.get_data_parallel_rank() * 0, hcg.get_model_parallel_rank(),
                               hcg.get_stage_id())
    return None


def get_hybrid_communicate_group():
    return _STATE["hcg"]


def _strategy():
    return _STATE["strategy"] or DistributedStrategy()


def worker_index():
    return dist.get_rank() if dist.is_initialized() else 0


def worker_num():
    return dist.get_world_size() if dist.is_initialized() else 1


def is_first_worker():
    return worker_index() == 0


def barrier_worker():
    if dist.is_initialized():
        dist.barrier()


def is_worker():
    return True


def is_server():
    return False


class _HybridModel(torch.nn.Module):
    """TensorParallel / ShardingParallel wrapper: syncs replicated weights, forwards calls."""

    def __init__(self, layers, hcg):
        super().__init__()
        self._layers = layers
        self.hcg = hcg
        if dist.is_initialized():
            mp_g = hcg.get_model_parallel_group()
            dp_g = hcg.get_data_parallel_group()
            for p in layers.parameters():
                if mp_g is not None and not getattr(p, "is_distributed", False):
                    dist.broadcast(p.data, hcg.get_model_parallel_group_src_rank(), group=mp_g)
                if dp_g is not None:
                    dist.broadcast(p.data, hcg.get_data_parallel_group_src_rank(), group=dp_g)

    def forward(self, *a, **k):
        return self._layers(*a, **k)

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, sd):
        return self._layers.set_state_dict(sd)

    def parameters(self, recurse=True):
        return self._layers.parameters()


TensorParallel = ShardingParallel = _HybridModel


def distributed_model(model):
    hcg = _STATE["hcg"]
    if hcg is None:
        return model
    st = _strategy()
    if isinstance(model, PipelineLayer) and hcg.get_pipe_parallel_world_size() > 1:
        return PipelineParallel(model, hcg, st)
    if hcg.get_model_parallel_world_size() > 1 or hcg.get_sharding_parallel_world_size() > 1 or st.sharding:
        return _HybridModel(model, hcg)
    if hcg.get_data_parallel_world_size() > 1:
        from ..parallel import DataParallel
        return DataParallel(model, group=hcg.get_data_parallel_group(),
                            comm_buffer_size=st.fuse_grad_size_in_MB,
                            find_unused_parameters=st.find_unused_parameters)
    return model


class HybridParallelOptimizer:
    """Wraps a Paddle optimizer for hybrid parallel training: gradient reduction over the dp (and
    sharding) group unless a DataParallel reducer already did it, global-norm clipping that counts
    mp-distributed parameters once per shard and replicated ones once, then the inner step."""

    def __init__(self, optimizer, hcg, strategy):
        self._inner = optimizer
        self.hcg, self.strategy = hcg, strategy
        self._flat = None
        dp_g = hcg.get_data_parallel_group() if hcg else None
        inner_flat = getattr(optimizer, "_flat", None)
        if inner_flat is not None:  # rebuild the fused engine with the hybrid groups
            from ...parallel.flat_engine import FlatTrainer
            old = inner_flat
            named = [(getattr(p, "pd_name", str(i)), p) for i, p in enumerate(optimizer._parameter_list)]
            stage = int(strategy.sharding_configs.get("stage", 1)) if (strategy.sharding or hcg.get_sharding_parallel_world_size() > 1) else 0
            self._flat = FlatTrainer(None, lr=optimizer.get_lr(), betas=(old.beta1, old.beta2),
                                     eps=old.eps, weight_decay=old.groups[0].weight_decay,
                                     grad_clip=old.grad_clip, dp_group=dp_g,
                                     mp_group=hcg.get_model_parallel_group(),
                                     pp_group=hcg.get_pipe_parallel_group(), sharding_stage=stage,
                                     named_params=named, bucket_mb=strategy.fuse_grad_size_in_MB)
            optimizer._flat = self._flat

    def __getattr__(self, k):
        return getattr(self._inner, k)

    @torch.no_grad()
    def _reduce_grads(self):
        dp_g = self.hcg.get_data_parallel_group()
        n = self.hcg.get_data_parallel_world_size()
        if dp_g is None or n == 1:
            return
        for p in self._inner._parameter_list:
            if p.grad is not None and not getattr(p, "_dp_bucket", None) is not None:
                dist.all_reduce(p.grad, group=dp_g)
                p.grad.div_(n)

    @torch.no_grad()
    def _clip(self):
        clip = self._inner._grad_clip
        if clip is None or not hasattr(clip, "clip_norm"):
            return
        dist_sq = torch.zeros((), dtype=torch.float32)
        rep_sq = torch.zeros((), dtype=torch.float32)
        dev = None
        for p in self._inner._parameter_list:
            if p.grad is None:
                continue
            dev = p.grad.device
            s = p.grad.float().pow(2).sum().cpu()
            if getattr(p, "is_distributed", False):
                dist_sq += s
            else:
                rep_sq += s
        mp_g = self.hcg.get_model_parallel_group()
        if mp_g is not None:
            t = dist_sq.to(dev or "cpu")
            dist.all_reduce(t, group=mp_g)
            dist_sq = t.cpu()
        total = dist_sq + rep_sq
        pp_g = self.hcg.get_pipe_parallel_group()
        if pp_g is not None:
            t = total.to(dev or "cpu")
            dist.all_reduce(t, group=pp_g)
            total = t.cpu()
        coef = min(1.0, clip.clip_norm / (float(total.sqrt()) + 1e-6))
        for p in self._inner._parameter_list:
            if p.grad is not None:
                p.grad.mul_(coef)
        self._inner._grad_clip, self._saved_clip = None, clip

    def step(self):
        if self._flat is not None:
            self._inner._step += 1
            self._flat.step(self._inner.get_lr())
            return
        self._reduce_grads()
        self._clip()
        try:
            self._inner.step()
        finally:
            if getattr(self, "_saved_clip", None) is not None:
                self._inner._grad_clip = self._saved_clip
                self._saved_clip = None

    def clear_grad(self, set_to_zero=True):
        if self._flat is not None:
            self._flat.zero_grad()
            return
        self._inner.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()


def distributed_optimizer(optimizer, strategy=None):
    if strategy is not None:
        _STATE["strategy"] = strategy
    hcg = _STATE["hcg"]
    if hcg is None:
        return optimizer
    return HybridParallelOptimizer(optimizer, hcg, _strategy())


def distributed_scaler(scaler):
    return scaler


class _MetaParallel:
    LayerDesc = LayerDesc
    SharedLayerDesc = SharedLayerDesc
    PipelineLayer = PipelineLayer
    PipelineParallel = PipelineParallel
    TensorParallel = TensorParallel
    ShardingParallel = ShardingParallel
    VocabParallelEmbedding = VocabParallelEmbedding
    ColumnParallelLinear = ColumnParallelLinear
    RowParallelLinear = RowParallelLinear
    ParallelCrossEntropy = ParallelCrossEntropy
    get_rng_state_tracker = staticmethod(get_rng_state_tracker)
    model_parallel_random_seed = staticmethod(model_parallel_random_seed)


meta_parallel = _MetaParallel()


class _Utils:
    recompute = staticmethod(recompute)


utils = _Utils()


class _Layers:
    class mpu:
        VocabParallelEmbedding = VocabParallelEmbedding
        ColumnParallelLinear = ColumnParallelLinear
        RowParallelLinear = RowParallelLinear
        ParallelCrossEntropy = ParallelCrossEntropy


layers = _Layers()
copy  # noqa
