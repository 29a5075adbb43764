"""Group-sharded (ZeRO) data parallelism: ``group_sharded_parallel`` levels ``os`` / ``os_g`` /
``p_g_os`` and ``save_group_sharded_model``.

Parity: reference `python/paddle/distributed/sharding/group_sharded.py` and
`fleet/meta_parallel/sharding/group_sharded_{optimizer_stage2,stage2,stage3,storage}.py`.

* ``os`` / ``os_g`` (stage 1 / 2): the optimizer becomes the flat-buffer engine with
  ``sharding_stage`` 1/2 — gradients are reduce-scattered bucket by bucket during backward into a
  contiguous local shard, ONE fused AdamW launch updates the shard's fp32 master/moments, the bf16
  shard is all-gathered back.
* ``p_g_os`` (stage 3): additionally the *parameters* live only as 1/N flat shards per block
  (decoder layer / embedding table / the root's own weights). A block all-gathers right before its
  forward while the next block's gather is already in flight, frees after; backward re-gathers
  (previous block prefetched), reduce-scatters its grads into an f32 shard once they all exist and
  frees again; global-norm clip + fused AdamW run on the flat shards — peak parameter memory is
  about two blocks, not the model (the 288 GB-per-GPU budget goes to activations / bigger batches).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..parallel.flat_engine import FlatTrainer, _ceil


def _pg(group):
    return group.pg if hasattr(group, "pg") else group


class _Stage3Unit:
    """One block's parameters as a flat buffer sharded 1/N over the group: rank-local bf16/f32 shard
    + f32 master / Adam moments / gradient shard. The full buffer exists only while the block runs
    (or always, for ``persistent`` units whose weights are used outside their own module)."""

    def __init__(self, name, module, named, group, world, rank, persistent, decays):
        self.name, self.module, self.group, self.world, self.rank = name, module, group, world, rank
        self.persistent = persistent
        order = sorted(range(len(named)), key=lambda i: not decays[i])  # decay params first
        self.names = [named[i][0] for i in order]
        self.params = [named[i][1] for i in order]
        self.decay_numel = sum(self.params[i].numel() for i in range(len(order)) if decays[order[i]])
        dtype, dev = self.params[0].dtype, self.params[0].device
        self.shapes = [p.shape for p in self.params]
        self.numels = [p.numel() for p in self.params]
        self.total = _ceil(sum(self.numels), world * 64)
        full = torch.zeros(self.total, dtype=dtype, device=dev)
        o = 0
        for p, n in zip(self.params, self.numels):
            full[o:o + n].copy_(p.data.reshape(-1))
            p._piamd_no_t = True  # no cached transposed copy (it would pin a full weight)
            o += n
        L = self.total // world
        self.L, self.lo = L, rank * L
        self.shard = full[self.lo:self.lo + L].clone()
        self.master = self.shard.float()
        self.m = torch.zeros(L, dtype=torch.float32, device=dev)
        self.v = torch.zeros(L, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(L, dtype=torch.float32, device=dev)
        self.full, self.handle, self.gathered = None, None, False
        self.pending, self.reduced = 0, True
        if persistent:
            self._bind(full)
        else:
            self.release(force=True)

    def _bind(self, full):
        o = 0
        for p, n, s in zip(self.params, self.numels, self.shapes):
            p.data = full[o:o + n].view(s)
            o += n
        self.full, self.gathered = full, True

    def gather_async(self):
        if self.gathered or self.handle is not None:
            return
        full = torch.empty(self.total, dtype=self.shard.dtype, device=self.shard.device)
        if self.world > 1:
            self.handle = dist.all_gather_into_tensor(full, self.shard, group=self.group, async_op=True)
        else:
            full.copy_(self.shard)
        self._incoming = full
        if self.world == 1:
            self._bind(full)

    def gather(self):
        self.gather_async()
        if self.handle is not None:
            self.handle.wait()
            self.handle = None
            self._bind(self._incoming)
        self._incoming = None

    def discard_prefetch(self):
        """Drop an outstanding or bound prefetch (its buffer holds the PRE-step shard): called
        before the shards change so the next forward re-gathers the updated weights."""
        if self.handle is not None:
            self.handle.wait()
            self.handle = None
        self._incoming = None
        if self.gathered and not self.persistent:
            self.release()

    def release(self, force=False):
        if self.persistent and not force:
            return
        for p in self.params:
            p.data = torch.empty(0, dtype=self.shard.dtype, device=self.shard.device)
        self.full, self.gathered = None, False

    def refresh_persistent(self):
        if self.persistent:
            full = self.full
            if self.world > 1:
                dist.all_gather_into_tensor(full, self.shard, group=self.group)
            else:
                full.copy_(self.shard)

    def reduce_grads(self):
        """Reduce-scatter this block's gradients (param dtype on the wire) into the f32 shard."""
        flat = torch.zeros(self.total, dtype=self.shard.dtype, device=self.shard.device)
        o = 0
        for p, n in zip(self.params, self.numels):
            if p.grad is not None:
                flat[o:o + n].copy_(p.grad.reshape(-1))
                p.grad = None
            o += n
        if self.world > 1:
            out = torch.empty(self.L, dtype=flat.dtype, device=flat.device)
            dist.reduce_scatter_tensor(out, flat, group=self.group)
            self.grad.add_(out.float(), alpha=1.0 / self.world)
        else:
            self.grad.add_(flat.float())
        self.reduced = True


_CONTAINERS = (torch.nn.ModuleList, torch.nn.Sequential)


def _has_container(m):
    return any(isinstance(c, _CONTAINERS) for c in m.modules())


def _split_units(root, exclude):
    """Blocks of the module tree. Every element of a layer container (LayerList / Sequential —
    e.g. GPT's decoder layers) is ONE unit, gathered by its own forward hooks. Every module on the
    path from the root to those containers contributes the rest of its parameters (direct ones and
    those of its non-container sub-layers — embeddings, final norm, an untied LM head) as one unit
    gathered for that module's whole forward. ``exclude``: modules whose weights are used outside
    their own forward (a tied LM head) — persistent units, gathered for the whole step."""
    units = []
    seen = set()

    def take(m, skip):
        out = []
        for n, p in m.named_parameters():
            if p.requires_grad and id(p) not in seen and id(p) not in skip:
                seen.add(id(p))
                out.append((n, p))
        return out

    ex_ids = {id(p) for e in exclude for p in e.parameters()}

    def visit(prefix, m):
        if isinstance(m, _CONTAINERS):
            for n, c in m.named_children():
                visit(f"{prefix}{n}.", c)
            return
        if not _has_container(m):
            ps = take(m, ex_ids)
            if ps:
                units.append((prefix.rstrip(".") or "<root>", m, [(prefix + n, p) for n, p in ps], False))
            return
        rest = [(prefix + n, p) for n, p in m.named_parameters(recurse=False)
                if p.requires_grad and id(p) not in ex_ids and id(p) not in seen]
        for p in rest:
            seen.add(id(p[1]))
        for n, c in m.named_children():
            if not _has_container(c) and not isinstance(c, _CONTAINERS):
                rest += [(f"{prefix}{n}.{pn}", p) for pn, p in take(c, ex_ids)]
        if rest:
            units.append((prefix.rstrip(".") or "<root>", m, rest, False))
        for n, c in m.named_children():
            if _has_container(c) or isinstance(c, _CONTAINERS):
                visit(f"{prefix}{n}.", c)

    for e in exclude:
        ps = [(n, p) for n, p in e.named_parameters() if p.requires_grad and id(p) not in seen]
        for _, p in ps:
            seen.add(id(p))
        if ps:
            units.append((f"<persistent:{type(e).__name__}>", e, ps, True))
    visit("", root)
    return units


class GroupShardedStage3(torch.nn.Module):
    """ZeRO-3 (reference `group_sharded_stage3.py:60`): parameters, gradients and optimizer states
    all live as 1/N flat shards per block. A block's parameters are all-gathered right before its
    forward — the NEXT block's gather is issued asynchronously at the same time (prefetch along the
    recorded execution order, reverse order in backward, `group_sharded_stage3.py:399`) — and freed
    right after; backward re-gathers them, and once every weight gradient of the block exists they
    are reduce-scattered into the block's f32 gradient shard and the full copy is freed again.
    Peak parameter memory ≈ two blocks, not the model."""

    def __init__(self, layer, optimizer=None, group=None, sync_buffers=False, segment_size=2 ** 20,
                 offload=False, sync_comm=False, exclude_layer=None, apply_decay_param_fun=None):
        super().__init__()
        self._layer = layer
        self.group = _pg(group)
        self.world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(self.group) if dist.is_initialized() else 0
        excl = list(exclude_layer or [])
        # models that pass one block's weights into the next block's kernels switch that off
        layer.apply(lambda m: setattr(m, "_zero3", True))
        for path in getattr(layer, "_stage3_persistent", []) or []:
            mod = layer
            for part in path.split("."):
                mod = getattr(mod, part)
            if mod not in excl:
                excl.append(mod)
        decay_fn = apply_decay_param_fun or (lambda n: True)
        self.units = []
        for name, mod, named, persistent in _split_units(layer, excl):
            decays = [bool(decay_fn(getattr(p, "pd_name", n))) for n, p in named]
            self.units.append(_Stage3Unit(name, mod, named, self.group, self.world, self.rank,
                                          persistent, decays))
        self._order, self._recording = [], True
        self._root_units = [u for u in self.units if u.module is layer]
        for u in self.units:
            if u.module is layer or u.persistent:
                continue
            u.module.register_forward_pre_hook(lambda m, i, _u=u: self._pre_forward(_u))
            u.module.register_forward_hook(lambda m, i, o, _u=u: self._post_forward(_u))
            u.module.register_full_backward_pre_hook(lambda m, g, _u=u: self._pre_backward(_u))
        for u in self.units:
            for p in u.params:
                p.register_post_accumulate_grad_hook(lambda t, _u=u: self._grad_hook(_u))
        if self._root_units:
            layer.register_full_backward_pre_hook(lambda m, g: self._gather_root())
        self._optim = optimizer

    # ---- forward / backward hooks
    def _neighbour(self, u, step):
        if self._recording or u not in self._order:
            return None
        i = self._order.index(u) + step
        return self._order[i] if 0 <= i < len(self._order) else None

    def _pre_forward(self, u):
        in_backward = torch._C._current_graph_task_id() != -1
        if self._recording and not in_backward and u not in self._order:
            self._order.append(u)
        u.gather()
        # a forward run INSIDE backward is a recompute: the next block's backward already ran,
        # so prefetching it would leave a gather nobody consumes (and a stale buffer after the
        # optimizer step) — backward prefetches the previous block instead (_pre_backward)
        nxt = None if in_backward else self._neighbour(u, 1)
        if nxt is not None:
            nxt.gather_async()

    def _post_forward(self, u):
        if torch.is_grad_enabled():
            u.pending = sum(1 for p in u.params if p.requires_grad)
            u.reduced = False
        u.release()

    def _pre_backward(self, u):
        u.gather()
        prv = self._neighbour(u, -1)
        if prv is not None:
            prv.gather_async()

    def _gather_root(self):
        for u in self._root_units:
            u.gather()  # returns None: a backward pre-hook's return value would replace grad_output

    def _grad_hook(self, u):
        u.pending -= 1
        if u.pending == 0 and not u.reduced:
            u.reduce_grads()
            u.release()

    def forward(self, *a, **k):
        for u in self._root_units:
            u.gather()
        if torch.is_grad_enabled():
            for u in self.units:
                if u.module is self._layer or u.persistent:
                    u.pending = len(u.params)
                    u.reduced = False
        out = self._layer(*a, **k)
        self._recording = False
        for u in self._root_units:
            u.release()
        return out

    def finalize_grads(self):
        """Reduce every block whose gradients were not all produced (unused parameters): the same
        fixed order on every rank keeps the collectives matched."""
        for u in self.units:
            if not u.reduced:
                u.reduce_grads()
                u.release()
            u.pending = 0
            u.discard_prefetch()

    def shard_params_and_grads(self):
        return [(u.shard, u.grad) for u in self.units]

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

    def parameters(self, recurse=True):
        return self._layer.parameters(recurse)


class _Stage3Optimizer:
    """AdamW (Paddle semantics) over the rank-local f32 shards of a GroupShardedStage3 model: ONE
    device-side global grad norm (sum of shard squares, all-reduced over the group) drives the
    clip coefficient, which the fused flat AdamW kernel applies as its grad scale."""

    def __init__(self, model: GroupShardedStage3, inner):
        from ..ops.optim import adamw_flat, sumsq
        self._adamw, self._sumsq = adamw_flat, sumsq
        self.model, self.inner = model, inner
        self.t = 0
        clip = getattr(inner, "_grad_clip", None)
        self.clip_norm = getattr(clip, "clip_norm", None)
        self.wd = inner._decay_coeff() if getattr(inner, "_decoupled", False) else 0.0

    @torch.no_grad()
    def step(self):
        from ..ops.linear import bump_param_epoch
        self.model.finalize_grads()
        self.t += 1
        lr = self.inner.get_lr()
        b1 = getattr(self.inner, "_beta1", 0.9)
        b2 = getattr(self.inner, "_beta2", 0.999)
        eps = getattr(self.inner, "_epsilon", 1e-8)
        units = self.model.units
        coef = None
        if self.clip_norm is not None and units:
            tot = torch.zeros((), dtype=torch.float32, device=units[0].grad.device)
            for u in units:
                self._sumsq(u.grad, out=tot, accumulate=True)
            if self.model.world > 1:
                dist.all_reduce(tot, group=self.model.group)
            coef = torch.clamp(self.clip_norm / (tot.sqrt() + 1e-6), max=1.0).reshape(1)
        for u in units:
            d = min(max(u.decay_numel - u.lo, 0), u.L)  # decay / no-decay split of this shard
            for a, b, wd in ((0, d, self.wd), (d, u.L, 0.0)):
                if b > a:
                    self._adamw(u.master[a:b], u.m[a:b], u.v[a:b], u.grad[a:b], lr, b1, b2, eps, wd,
                                self.t, grad_scale=coef)
            u.shard.copy_(u.master)
            u.refresh_persistent()
        bump_param_epoch()
        if hasattr(self.inner, "_step"):
            self.inner._step += 1

    def clear_grad(self, set_to_zero=True):
        for u in self.model.units:
            u.grad.zero_()
            for p in u.params:
                p.grad = None

    clear_gradients = clear_grad

    def get_lr(self):
        return self.inner.get_lr()

    def state_dict(self):
        return {f"{u.name}.{k}": getattr(u, k) for u in self.model.units for k in ("master", "m", "v")} | {"t": self.t}


def group_sharded_parallel(model, optimizer, level, scaler=None, group=None, offload=False,
                           sync_buffers=False, buffer_max_size=2 ** 23, segment_size=2 ** 20,
                           sync_comm=False, dp_group=None, exclude_layer=None):
    assert level in ("os", "os_g", "p_g_os"), level
    pg = _pg(group) if group is not None else (dist.group.WORLD if dist.is_initialized() else None)
    if level == "p_g_os":
        m = GroupShardedStage3(model, optimizer, pg, segment_size=segment_size, exclude_layer=exclude_layer,
                               apply_decay_param_fun=getattr(optimizer, "_apply_decay_param_fun", None))
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
