"""Group-sharded (ZeRO) data parallelism: ``group_sharded_parallel`` levels ``os`` / ``os_g`` /
``p_g_os`` and ``save_group_sharded_model``.

Parity: reference `python/paddle/distributed/sharding/group_sharded.py` and
`fleet/meta_parallel/sharding/group_sharded_{optimizer_stage2,stage2,stage3,storage}.py`.

* ``os`` / ``os_g`` (stage 1 / 2): the optimizer becomes the flat-buffer engine with
  ``sharding_stage`` 1/2 — gradients are reduce-scattered bucket by bucket during backward into a
  contiguous local shard, ONE fused AdamW launch updates the shard's fp32 master/moments, the bf16
  shard is all-gathered back.
* ``p_g_os`` (stage 3): additionally the *parameters* live only as 1/N flat shards. Every top-level
  sub-layer all-gathers its flat parameter right before its forward (pre-hook) and frees it right
  after; backward re-gathers it (module backward pre-hook) and, once its weight grads exist,
  reduce-scatters them into the shard and frees the full copy again — peak parameter memory is one
  layer, not the model (the 288 GB-per-GPU budget then goes to activations / bigger batches).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..parallel.flat_engine import FlatTrainer, _ceil


def _pg(group):
    return group.pg if hasattr(group, "pg") else group


class _Stage3Unit:
    """One sub-layer's parameters as a flat, rank-sharded buffer."""

    def __init__(self, module, group, world, rank):
        self.module, self.group, self.world, self.rank = module, group, world, rank
        self.params = [p for p in module.parameters() if p.requires_grad]
        dtype = self.params[0].dtype
        dev = self.params[0].device
        self.shapes = [p.shape for p in self.params]
        self.numels = [p.numel() for p in self.params]
        total = _ceil(sum(self.numels), world * 64)
        self.total = total
        full = torch.zeros(total, dtype=dtype, device=dev)
        o = 0
        for p, n in zip(self.params, self.numels):
            full[o:o + n].copy_(p.data.reshape(-1))
            o += n
        L = total // world
        self.shard = full[rank * L:(rank + 1) * L].clone()
        self.shard_grad = torch.zeros(L, dtype=torch.float32, device=dev)
        self.full = None
        self.gathered = False
        self.pending = 0
        self._release()

    def gather(self):
        if self.gathered:
            return
        full = torch.empty(self.total, dtype=self.shard.dtype, device=self.shard.device)
        if self.world > 1:
            dist.all_gather_into_tensor(full, self.shard, group=self.group)
        else:
            full.copy_(self.shard)
        o = 0
        for p, n, s in zip(self.params, self.numels, self.shapes):
            p.data = full[o:o + n].view(s)
            o += n
        self.full = full
        self.gathered = True

    def _release(self):
        for p in self.params:
            p.data = torch.empty(0, dtype=self.shard.dtype, device=self.shard.device)
        self.full = None
        self.gathered = False

    def release(self):
        self._release()

    def reduce_grads(self):
        flat = torch.zeros(self.total, dtype=torch.float32, device=self.shard.device)
        o = 0
        for p, n in zip(self.params, self.numels):
            if p.grad is not None:
                flat[o:o + n].copy_(p.grad.reshape(-1).float())
                p.grad = None
            o += n
        L = self.total // self.world
        out = torch.empty(L, dtype=torch.float32, device=flat.device)
        if self.world > 1:
            dist.reduce_scatter_tensor(out, flat, group=self.group)
            out.div_(self.world)
        else:
            out.copy_(flat)
        self.shard_grad.add_(out)


class GroupShardedStage3(torch.nn.Module):
    def __init__(self, layer, optimizer=None, group=None, sync_buffers=False, segment_size=2 ** 20,
                 offload=False, sync_comm=False):
        super().__init__()
        self._layer = layer
        self.group = _pg(group)
        self.world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(self.group) if dist.is_initialized() else 0
        units = []
        leaf_owner = [m for m in layer.children()] or [layer]
        for m in leaf_owner:
            if any(p.requires_grad for p in m.parameters()):
                units.append(_Stage3Unit(m, self.group, self.world, self.rank))
        self.units = units
        for u in units:
            u.module.register_forward_pre_hook(lambda m, i, _u=u: _u.gather())
            u.module.register_forward_hook(lambda m, i, o, _u=u: self._after_forward(_u))
            u.module.register_full_backward_pre_hook(lambda m, g, _u=u: _u.gather())
            for p in u.params:
                p.register_post_accumulate_grad_hook(lambda t, _u=u: self._grad_hook(_u))
        self._optim = optimizer
        self._training_forward = True

    def _after_forward(self, u):
        if not torch.is_grad_enabled():
            u.release()
            return
        u.pending = len(u.params)
        u.release()

    def _grad_hook(self, u):
        u.pending -= 1
        if u.pending == 0:
            u.reduce_grads()
            u.release()

    def forward(self, *a, **k):
        return self._layer(*a, **k)

    def shard_params_and_grads(self):
        return [(u.shard, u.shard_grad) for u in self.units]

    @torch.no_grad()
    def get_all_parameters(self):
        for u in self.units:
            u.gather()

    def state_dict(self, *a, **k):
        self.get_all_parameters()
        sd = {kk: v.clone() for kk, v in self._layer.state_dict().items()}
        for u in self.units:
            u.release()
        return sd


class _Stage3Optimizer:
    """AdamW over the rank-local fp32 shards of a GroupShardedStage3 model."""

    def __init__(self, model: GroupShardedStage3, inner):
        from ..ops.optim import adamw_flat
        self._adamw = adamw_flat
        self.model, self.inner = model, inner
        self.masters = [u.shard.float().clone() for u in model.units]
        self.m = [torch.zeros_like(t) for t in self.masters]
        self.v = [torch.zeros_like(t) for t in self.masters]
        self.t = 0

    @torch.no_grad()
    def step(self):
        self.t += 1
        lr = self.inner.get_lr()
        b1 = getattr(self.inner, "_beta1", 0.9)
        b2 = getattr(self.inner, "_beta2", 0.999)
        eps = getattr(self.inner, "_epsilon", 1e-8)
        wd = getattr(self.inner, "_wd", 0.0)
        for u, mst, m, v in zip(self.model.units, self.masters, self.m, self.v):
            self._adamw(mst, m, v, u.shard_grad, lr, b1, b2, eps, wd, self.t)
            u.shard.copy_(mst)

    def clear_grad(self, set_to_zero=True):
        for u in self.model.units:
            u.shard_grad.zero_()

    clear_gradients = clear_grad

    def get_lr(self):
        return self.inner.get_lr()


def group_sharded_parallel(model, optimizer, level, scaler=None, group=None, offload=False,
                           sync_buffers=False, buffer_max_size=2 ** 23, segment_size=2 ** 20,
                           sync_comm=False, dp_group=None, exclude_layer=None):
    assert level in ("os", "os_g", "p_g_os"), level
    pg = _pg(group) if group is not None else (dist.group.WORLD if dist.is_initialized() else None)
    if level == "p_g_os":
        m = GroupShardedStage3(model, optimizer, pg)
        return m, _Stage3Optimizer(m, optimizer), scaler
    stage = 1 if level == "os" else 2
    old = getattr(optimizer, "_flat", None)
    named = [(getattr(p, "pd_name", str(i)), p) for i, p in enumerate(optimizer._parameter_list)]
    ft = FlatTrainer(None, lr=optimizer.get_lr(),
                     betas=(getattr(optimizer, "_beta1", 0.9), getattr(optimizer, "_beta2", 0.999)),
                     eps=getattr(optimizer, "_epsilon", 1e-8),
                     weight_decay=getattr(optimizer, "_wd", 0.0),
                     grad_clip=getattr(optimizer._grad_clip, "clip_norm", None), dp_group=pg,
                     sharding_stage=stage, named_params=named,
                     bucket_mb=max(1, buffer_max_size // 2 ** 20))
    del old
    optimizer._flat = ft
    if not hasattr(optimizer, "_update") or type(optimizer).step is not getattr(type(optimizer), "step"):
        pass
    return model, _FlatOptimizer(optimizer, ft), scaler


class _FlatOptimizer:
    def __init__(self, inner, flat):
        self._inner, self._flat = inner, flat

    def step(self):
        self._inner._step += 1
        self._flat.step(self._inner.get_lr())

    def clear_grad(self, set_to_zero=True):
        self._flat.zero_grad()

    clear_gradients = clear_grad

    def __getattr__(self, k):
        return getattr(self._inner, k)

    def state_dict(self):
        return self._flat.state_dict()


def save_group_sharded_model(model, output, optimizer=None):
    import os
    from ..framework.io import save
    os.makedirs(output, exist_ok=True)
    sd = model.state_dict()
    if not dist.is_initialized() or dist.get_rank() == 0:
        save(sd, os.path.join(output, "model.pdmodel"))
    if optimizer is not None:
        r = dist.get_rank() if dist.is_initialized() else 0
        save(optimizer.state_dict(), os.path.join(output, f"model.pdopt.rank{r}"))
