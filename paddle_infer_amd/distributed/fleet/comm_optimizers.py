"""Communication-reducing data-parallel meta-optimizers: LocalSGD, adaptive LocalSGD and DGC.

Reference: `python/paddle/distributed/fleet/meta_optimizers/localsgd_optimizer.py:26` (LocalSGD and
AdaptiveLocalSGD as static-program rewrites), `dgc_optimizer.py:21` + `fluid/optimizer.py:1545`
(DGCMomentumOptimizer) with the kernels `operators/dgc_op.h`, `dgc_clip_by_norm_op.h` and
`optimizers/dgc_momentum_op.h`. Here they are dygraph optimizer wrappers over torch.distributed
(RCCL on the GPU, gloo on the CPU); `fleet.distributed_model` leaves the model without a gradient
reducer when one of them is on, because they own all data-parallel communication:

* LocalSGD: every rank steps on its own gradients; parameters are averaged over the data-parallel
  group every step up to ``begin_step`` and every ``k_steps`` steps after it (the reference's
  snapshot form ``p = s − allreduce(s − p)/n`` is the same average when the snapshots agree, as
  they do after every average).
* Adaptive LocalSGD: the same, with the interval re-chosen at each average from the
  group-averaged loss: ``k = clamp(ceil(sqrt(lr₀·loss / (lr·loss₀) · init_k_steps)), 1, 16)``.
* DGC: momentum correction + local accumulation + top-k sparsification. Parameters with ≥ 16384
  fp32 elements, after ``rampup_begin_step``: ``u = m·u + g`` (Nesterov: ``u = m·(u + g)``,
  ``v += u + g``), ``v += u``; the k = numel·(1 − sparsity(step)) largest-|v| entries are sent
  (indices + values, all-gathered), ``u`` and ``v`` are zeroed there, and the parameter takes an
  SGD step on the gathered sum / nranks (the momentum is already in ``u``). ``sparsity`` ramps
  over ``rampup_step`` steps through the configured list. Before the ramp and for small
  parameters: dense all-reduce (mean) + the inner Momentum update on the same velocity ``u``.
  A ``ClipGradByNorm(c)`` clips the local gradient at ``c·nranks^-½`` once DGC is active
  (`dgc_clip_by_norm`).
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist


def _world(group):
    return dist.get_world_size(group) if dist.is_initialized() else 1


@torch.no_grad()
def _average_params(params, group):
    n = _world(group)
    if n <= 1:
        return
    by_dtype = {}
    for p in params:
        by_dtype.setdefault((p.dtype, p.device), []).append(p)
    for ps in by_dtype.values():
        flat = torch.cat([p.detach().reshape(-1) for p in ps])
        dist.all_reduce(flat, group=group)
        flat.div_(n)
        off = 0
        for p in ps:
            k = p.numel()
            p.copy_(flat[off:off + k].view_as(p))
            off += k


@torch.no_grad()
def _average_grads(params, group):
    n = _world(group)
    gs = [p.grad for p in params if p.grad is not None]
    if n <= 1 or not gs:
        return
    by_dtype = {}
    for g in gs:
        by_dtype.setdefault((g.dtype, g.device), []).append(g)
    for ts in by_dtype.values():
        flat = torch.cat([g.reshape(-1) for g in ts])
        dist.all_reduce(flat, group=group)
        flat.div_(n)
        off = 0
        for g in ts:
            k = g.numel()
            g.copy_(flat[off:off + k].view_as(g))
            off += k


class _Wrapper:
    def __init__(self, inner, group):
        self._inner, self.group = inner, group

    def __getattr__(self, k):
        if k == "_inner":
            raise AttributeError(k)
        return getattr(self._inner, k)

    def clear_grad(self, set_to_zero=True):
        self._inner.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step(loss=loss)

    def state_dict(self):
        return self._inner.state_dict()

    def set_state_dict(self, sd):
        return self._inner.set_state_dict(sd)


class LocalSGDOptimizer(_Wrapper):
    def __init__(self, inner, group=None, k_steps=1, begin_step=1):
        if int(k_steps) < 1:
            raise ValueError("localsgd_configs.k_steps must be >= 1")
        super().__init__(inner, group)
        self.k_steps, self.begin_step = int(k_steps), int(begin_step)
        self._step_no = 0
        self._last = 0

    def _params(self):
        return [p for p in self._inner._parameter_list if p.requires_grad]

    def _communicate(self):
        _average_params(self._params(), self.group)
        self._last = self._step_no

    def step(self, loss=None):
        self._inner.step()
        self._step_no += 1
        if self._step_no <= self.begin_step:
            self._communicate()
        elif self._step_no - self._last == self.k_steps:
            self._communicate()


class AdaptiveLocalSGDOptimizer(LocalSGDOptimizer):
    MAX_K, MIN_K = 16, 1

    def __init__(self, inner, group=None, init_k_steps=1, begin_step=1):
        super().__init__(inner, group, init_k_steps, begin_step)
        self.init_k_steps = int(init_k_steps)
        self._lr0 = self._loss0 = None

    def _avg_loss(self, loss):
        if loss is None:
            raise ValueError("adaptive LocalSGD needs the loss: call minimize(loss) or step(loss=loss)")
        t = loss.detach().float().reshape(1).clone()
        if _world(self.group) > 1:
            dist.all_reduce(t, group=self.group)
            t.div_(_world(self.group))
        return float(t)

    def step(self, loss=None):
        self._inner.step()
        self._step_no += 1
        if self._lr0 is None:  # reference `initialize`: first step records lr₀ and the mean loss₀
            self._loss0 = self._avg_loss(loss)
            self._lr0 = float(self._inner.get_lr())
        if self._step_no <= self.begin_step:
            self._communicate()
        elif self._step_no - self._last == self.k_steps:
            self._communicate()
            avg = self._avg_loss(loss)
            lr = float(self._inner.get_lr())
            ratio = self._lr0 * avg / (lr * self._loss0) if lr > 0 and self._loss0 else 1.0
            k = math.ceil(math.sqrt(max(ratio, 0.0) * self.init_k_steps))
            self.k_steps = min(max(k, self.MIN_K), self.MAX_K)


def _sparsity_at(sparsity, cur, rampup_step):
    """`get_period_sparcity` (dgc_op.h): the ramp walks the list over rampup_step steps."""
    idx = int(cur * len(sparsity) / max(rampup_step, 1e-12))
    return sparsity[min(idx, len(sparsity) - 1)]


class DGCMomentumOptimizer(_Wrapper):
    MIN_NUMEL = 16384

    def __init__(self, inner, group=None, rampup_begin_step=0, rampup_step=1, sparsity=(0.999,)):
        from ...optimizer import Momentum
        if not isinstance(inner, Momentum):
            raise TypeError(f"strategy.dgc needs a Momentum optimizer, got {type(inner).__name__}")
        super().__init__(inner, group)
        self.rampup_begin_step, self.rampup_step = int(rampup_begin_step), max(int(rampup_step), 1)
        self.sparsity = [float(s) for s in sparsity] or [0.999]
        for s in self.sparsity:
            if not 0.0 <= s < 1.0:
                raise ValueError(f"dgc sparsity {s} outside [0, 1)")
        self._step_no = 0
        self._v = {}
        self.last_k = {}

    def _use_dgc(self, p):
        return p.numel() >= self.MIN_NUMEL and p.dtype == torch.float32

    @torch.no_grad()
    def step(self, loss=None):
        inner = self._inner
        params = [p for p in inner._parameter_list if p.requires_grad and p.grad is not None]
        n = _world(self.group)
        active = self._step_no >= self.rampup_begin_step and n > 1
        dgc_ps = [p for p in params if active and self._use_dgc(p)]
        dense = [p for p in params if not (active and self._use_dgc(p))]
        _average_grads(dense, self.group)
        if dgc_ps:
            ratio = 1.0 - _sparsity_at(self.sparsity, self._step_no - self.rampup_begin_step,
                                       self.rampup_step)
            clip = getattr(inner, "_grad_clip", None)
            cn = getattr(clip, "clip_norm", None) if type(clip).__name__ == "ClipGradByNorm" else None
            lr = float(inner.get_lr())
            mu, nest = float(inner._momentum), bool(inner._nesterov)
            for p in dgc_ps:
                g = p.grad.float()
                if cn is not None:  # dgc_clip_by_norm: local clip at c·n^-½
                    nrm = g.norm()
                    lim = cn * n ** -0.5
                    if nrm > lim:
                        g = g * (lim / nrm)
                g = inner._l2(p, g)
                u = inner._acc("velocity", p)
                v = self._v.get(id(p))
                if v is None:
                    v = self._v[id(p)] = torch.zeros_like(p, dtype=torch.float32)
                if nest:
                    u.add_(g).mul_(mu)
                    v.add_(u).add_(g)
                else:
                    u.mul_(mu).add_(g)
                    v.add_(u)
                k = max(1, int(p.numel() * ratio))
                self.last_k[id(p)] = k
                vf, uf = v.view(-1), u.view(-1)
                idx = torch.topk(vf.abs(), k, sorted=False).indices
                vals = vf[idx].clone()
                vf[idx] = 0
                uf[idx] = 0
                gi = [torch.empty_like(idx) for _ in range(n)]
                gv = [torch.empty_like(vals) for _ in range(n)]
                dist.all_gather(gi, idx, group=self.group)
                dist.all_gather(gv, vals, group=self.group)
                G = torch.zeros(p.numel(), dtype=torch.float32, device=p.device)
                G.index_add_(0, torch.cat(gi), torch.cat(gv))
                p.sub_((lr * G / n).view_as(p).to(p.dtype))
            saved = {id(p): p.grad for p in dgc_ps}
            for p in dgc_ps:
                p.grad = None
            try:
                inner.step()  # the dense / small parameters (momentum on the same velocity)
            finally:
                for p in dgc_ps:
                    p.grad = saved[id(p)]
        else:
            inner.step()
        self._step_no += 1
