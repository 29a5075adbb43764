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
    (or always, for ``persistent`` units whose weights are used outside their own module).

    ``offload`` keeps the f32 master and moments in pinned host memory and runs the update there
    (reference `group_sharded_stage3.py:84-93`): device memory per parameter drops from 14 bytes
    (bf16 shard + f32 grad/master/m/v) to 6. ``replica_group``: a data-parallel axis OVER the
    sharding axis (hybrid dp × sharding) — reduced shards are averaged over it as well."""

    def __init__(self, name, module, named, group, world, rank, persistent, offload=False,
                 replica_group=None, mp_world=1):
        self.name, self.module, self.group, self.world, self.rank = name, module, group, world, rank
        self.persistent, self.offload = persistent, offload
        self.replica_group = replica_group
        self.replica_world = dist.get_world_size(replica_group) if replica_group is not None else 1
        # matrices first: with the usual decay rule (no decay on biases / norms) the shard splits
        # into one decay and one no-decay segment (`set_decay`)
        order = sorted(range(len(named)), key=lambda i: named[i][1].dim() <= 1)
        self.names = [named[i][0] for i in order]
        self.params = [named[i][1] for i in order]
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
        host = offload and dev.type == "cuda"
        self.master = self.shard.float().cpu().pin_memory() if host else self.shard.float()
        sdev = self.master.device
        self.m = torch.zeros(L, dtype=torch.float32, device=sdev)
        self.v = torch.zeros(L, dtype=torch.float32, device=sdev)
        if host:
            self.m, self.v = self.m.pin_memory(), self.v.pin_memory()
            self._host_grad = torch.empty(L, dtype=torch.float32).pin_memory()
        self.grad = torch.zeros(L, dtype=torch.float32, device=dev)
        # grad-norm weight per shard range: a pipeline-shared copy that is not the first counts 0,
        # a parameter replicated over tensor-parallel ranks 1/mp (the norm is summed over mp)
        ws = [0.0 if getattr(p, "is_firstly_shared", True) is False else
              (1.0 if mp_world == 1 or getattr(p, "is_distributed", False) else 1.0 / mp_world)
              for p in self.params]
        self.norm_segs = self._segments(ws)
        self.decay_segs = [(0, L, True)]
        self.full, self.handle, self.gathered = None, None, False
        self.pending, self.reduced = 0, True
        self._rs = None
        if persistent:
            self._bind(full)
        else:
            self.release(force=True)

    def _segments(self, per_param):
        """Runs of equal per-parameter values → [(a, b, value)] in shard-local coordinates."""
        segs, o = [], 0
        for val, n in zip(per_param, self.numels):
            a, b = max(o, self.lo) - self.lo, min(o + n, self.lo + self.L) - self.lo
            if b > a:
                if segs and segs[-1][2] == val and segs[-1][1] == a:
                    segs[-1] = (segs[-1][0], b, val)
                else:
                    segs.append((a, b, val))
            o += n
        return segs

    def set_decay(self, flags):
        """Per-parameter weight-decay flags (in ``self.params`` order) → shard segments."""
        self.decay_segs = self._segments([bool(f) for f in flags])

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
        """Start reducing this block's gradients (param dtype on the wire) into the f32 shard: the
        reduce-scatter runs asynchronously (RCCL's stream) while backward continues into the
        previous block; `complete_reduce` folds it in."""
        self.complete_reduce()  # a previous micro-batch's reduce of this block still in flight
        flat = torch.zeros(self.total, dtype=self.shard.dtype, device=self.shard.device)
        o = 0
        for p, n in zip(self.params, self.numels):
            if p.grad is not None:
                flat[o:o + n].copy_(p.grad.reshape(-1))
                p.grad = None
            o += n
        self.reduced = True
        if self.world > 1:
            out = torch.empty(self.L, dtype=flat.dtype, device=flat.device)
            h = dist.reduce_scatter_tensor(out, flat, group=self.group, async_op=True)
            self._rs = (h, out, flat)
        else:
            self._rs = (None, flat, flat)

    def complete_reduce(self):
        if self._rs is None:
            return
        h, out, _ = self._rs
        self._rs = None
        if h is not None:
            h.wait()
        g = out.float()
        if self.replica_world > 1:
            dist.all_reduce(g, group=self.replica_group)
        self.grad.add_(g, alpha=1.0 / (self.world * self.replica_world))


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
    are reduce-scattered (asynchronously, at most ``max_inflight`` blocks in flight so the full-size
    gradient buffers stay bounded) into the block's f32 gradient shard and the full copy is freed
    again. Peak parameter memory ≈ two blocks, not the model.

    Composes with pipeline / tensor parallelism (reference `sharding_optimizer.py:127-134`: the
    sharding axis inside each pipeline stage): wrap a stage's ``PipelineLayer`` (its micro-batches
    accumulate into the block gradients; each block is reduced once its last micro-batch's backward
    is done) with pipeline-shared layers as persistent units whose gradients are reduced only after
    the pipeline's shared-weight all-reduce (`finalize_grads`); tensor-parallel layers shard their
    local slices. ``replica_group`` is a data-parallel axis over the sharding axis."""

    def __init__(self, layer, optimizer=None, group=None, sync_buffers=False, segment_size=2 ** 20,
                 offload=False, sync_comm=False, exclude_layer=None, apply_decay_param_fun=None,
                 replica_group=None, mp_group=None, pp_group=None, max_inflight=2):
        super().__init__()
        self._layer = layer
        self.group = _pg(group)
        self.world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(self.group) if dist.is_initialized() else 0
        self.replica_group = _pg(replica_group) if replica_group is not None else None
        self.mp_group = _pg(mp_group) if mp_group is not None else None
        self.pp_group = _pg(pp_group) if pp_group is not None else None
        mp_world = dist.get_world_size(self.mp_group) if self.mp_group is not None else 1
        self.offload, self.sync_comm = offload, sync_comm
        self.max_inflight = 0 if sync_comm else max_inflight
        excl = list(exclude_layer or [])
        # models that pass one block's weights into the next block's kernels switch that off
        layer.apply(lambda m: setattr(m, "_zero3", True))
        for path in getattr(layer, "_stage3_persistent", []) or []:
            mod = layer
            for part in path.split("."):
                mod = getattr(mod, part)
            if mod not in excl:
                excl.append(mod)
        self.units = []
        for name, mod, named, persistent in _split_units(layer, excl):
            self.units.append(_Stage3Unit(name, mod, named, self.group, self.world, self.rank,
                                          persistent, offload=offload, replica_group=self.replica_group,
                                          mp_world=mp_world))
        self.set_decay_fn(apply_decay_param_fun)
        self._order, self._recording = [], True
        self._inflight = []
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

    def set_decay_fn(self, fn):
        """Weight-decay rule (Paddle ``apply_decay_param_fun`` on parameter names; default: all)."""
        for u in self.units:
            u.set_decay([fn is None or bool(fn(getattr(p, "pd_name", n))) for n, p in zip(u.names, u.params)])

    # ---- forward / backward hooks
    def _neighbour(self, u, step):
        if self._recording or u not in self._order:
            return None
        i = self._order.index(u) + step
        return self._order[i] if 0 <= i < len(self._order) else None

    def _pre_forward(self, u):
        in_backward = torch._C._current_graph_task_id() != -1
        if self._recording and not in_backward:
            if u in self._order:  # a second micro-batch (pipeline): the order is complete
                self._recording = False
            else:
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
            # one more backward to wait for (micro-batches of a pipeline stage accumulate)
            u.pending += sum(1 for p in u.params if p.requires_grad)
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
        # persistent units (pipeline-shared / tied weights) reduce in finalize_grads, after the
        # cross-stage shared-weight all-reduce
        if u.pending == 0 and not u.reduced and not u.persistent:
            self._reduce(u)

    def _reduce(self, u):
        u.reduce_grads()
        u.release()
        self._inflight.append(u)
        while len(self._inflight) > self.max_inflight:
            self._inflight.pop(0).complete_reduce()

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
        """Reduce every block whose gradients were not all produced (unused parameters) and the
        persistent ones: the same fixed order on every rank keeps the collectives matched."""
        for u in self.units:
            if not u.reduced or u.persistent:
                self._reduce(u)
            u.pending = 0
        while self._inflight:
            self._inflight.pop(0).complete_reduce()
        for u in self.units:
            u.discard_prefetch()

    def shard_params_and_grads(self):
        return [(u.shard, u.grad) for u in self.units]

    @torch.no_grad()
    def get_all_parameters(self):
        for u in self.units:
            u.gather()

    def release_all(self):
        for u in self.units:
            u.release()

    def state_dict(self, *a, **k):
        self.get_all_parameters()
        sd = {kk: v.clone() for kk, v in self._layer.state_dict().items()}
        self.release_all()
        return sd

    def parameters(self, recurse=True):
        return self._layer.parameters(recurse)


class _Stage3Optimizer:
    """AdamW (Paddle semantics) over the rank-local f32 shards of a GroupShardedStage3 model: ONE
    device-side global grad norm (weighted shard squares, all-reduced over the sharding, tensor-
    and pipeline-parallel groups) drives the clip coefficient, which the fused flat AdamW kernel
    applies as its grad scale. Offloaded units update on the host copy."""

    def __init__(self, model: GroupShardedStage3, inner):
        from ..ops.optim import adamw_flat, sumsq
        self._adamw, self._sumsq = adamw_flat, sumsq
        self.model, self.inner = model, inner
        self.t = 0
        clip = getattr(inner, "_grad_clip", None)
        self.clip_norm = getattr(clip, "clip_norm", None)
        self.wd = inner._decay_coeff() if getattr(inner, "_decoupled", False) else 0.0
        fn = getattr(inner, "_apply_decay_param_fun", None)
        if fn is not None:
            model.set_decay_fn(fn)

    @torch.no_grad()
    def _grad_norm_sq(self):
        units = self.model.units
        tot = torch.zeros((), dtype=torch.float32, device=units[0].grad.device)
        for u in units:
            for a, b, w in u.norm_segs:
                if w == 1.0:
                    self._sumsq(u.grad[a:b], out=tot, accumulate=True)
                elif w:
                    tot.add_(self._sumsq(u.grad[a:b]), alpha=w)
        for g in (self.model.group if self.model.world > 1 else None, self.model.mp_group,
                  self.model.pp_group):
            if g is not None and dist.get_world_size(g) > 1:
                dist.all_reduce(tot, group=g)
        return tot

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
            tot = self._grad_norm_sq()
            coef = torch.clamp(self.clip_norm / (tot.sqrt() + 1e-6), max=1.0).reshape(1)
        for u in units:
            host = u.master.device != u.grad.device
            g = u._host_grad.copy_(u.grad) if host else u.grad
            c = coef.cpu() if (host and coef is not None) else coef
            for a, b, dec in u.decay_segs:
                self._adamw(u.master[a:b], u.m[a:b], u.v[a:b], g[a:b], lr, b1, b2, eps,
                            self.wd if dec else 0.0, self.t, grad_scale=c)
            u.shard.copy_(u.master, non_blocking=host)
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

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def get_lr(self):
        return self.inner.get_lr()

    def set_lr(self, lr):
        return self.inner.set_lr(lr)

    def __getattr__(self, k):
        if k in ("inner", "model"):
            raise AttributeError(k)
        return getattr(self.inner, k)

    def state_dict(self):
        return {f"{u.name}.{k}": getattr(u, k) for u in self.model.units for k in ("master", "m", "v")} | {"t": self.t}


def group_sharded_parallel(model, optimizer, level, scaler=None, group=None, offload=False,
                           sync_buffers=False, buffer_max_size=2 ** 23, segment_size=2 ** 20,
                           sync_comm=False, dp_group=None, exclude_layer=None):
    assert level in ("os", "os_g", "p_g_os"), level
    if offload and level != "p_g_os":
        raise NotImplementedError("offload is implemented for level 'p_g_os' (ZeRO-3); stage 1/2 keep "
                                  "their f32 states on the device")
    pg = _pg(group) if group is not None else (dist.group.WORLD if dist.is_initialized() else None)
    if level == "p_g_os":
        m = GroupShardedStage3(model, optimizer, pg, segment_size=segment_size, exclude_layer=exclude_layer,
                               apply_decay_param_fun=getattr(optimizer, "_apply_decay_param_fun", None),
                               offload=offload, sync_comm=sync_comm,
                               replica_group=_pg(dp_group) if dp_group is not None else None)
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
