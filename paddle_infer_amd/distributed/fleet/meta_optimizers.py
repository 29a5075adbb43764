"""DistributedStrategy switches applied to the model and optimizer (reference
`python/paddle/distributed/fleet/meta_optimizers/`: `amp_optimizer.py:20`, `recompute_optimizer.py:20`,
`gradient_merge_optimizer.py:20`, `lamb_optimizer.py`, `lars_optimizer.py`, `asp_optimizer.py`,
`raw_program_optimizer.py` for static data parallelism).

Every switch is either honoured here or rejected by `check_strategy` — none is accepted and
ignored:

* ``amp``: the model's forward runs under ``auto_cast`` (bf16 unless ``use_bf16`` is False); O2
  (``use_pure_fp16``) casts the weights (norms stay fp32); fp16 gets a dynamic ``GradScaler`` that
  ``minimize`` / ``train_batch`` drive.
* ``recompute``: GPT-style models switch their per-layer recompute on, a ``PipelineLayer`` gets
  ``recompute_interval`` 1, otherwise every ``recompute_configs.checkpoints`` sub-layer (default:
  every element of every LayerList / Sequential) re-runs its forward in backward.
* ``gradient_merge``: ``step()`` applies the update every ``k_steps`` calls (grads averaged when
  ``avg``); ``clear_grad()`` between updates keeps the accumulation.
* ``lamb`` / ``lars``: the Adam / Momentum optimizer is replaced by Lamb / LarsMomentum with the
  configured coefficients (reference meta-optimizers swap the same way).
* ``asp``: the optimizer re-applies the 2:4 masks after each update (``incubate.asp.decorate``).
* ``sync_batch_norm``: BatchNorm layers become SyncBatchNorm.
* ``localsgd`` / ``adaptive_localsgd`` / ``dgc``: the optimizer owns the data-parallel
  communication (periodic parameter averaging, or top-k sparsified momentum-corrected gradients;
  `comm_optimizers.py`) and the model gets no gradient reducer.
* Static mode: ``distributed_optimizer(opt).minimize(loss)`` appends backward + optimizer ops and
  inserts one ``c_allreduce_sum`` + ``scale`` per gradient before the first optimizer op (data
  parallel over ring 0), so the saved program carries its collectives like the reference's.
"""
from __future__ import annotations

import torch

# switches this framework does not implement (parameter server, quantisation-aware training,
# auto-parallel search): setting one raises instead of being ignored
REJECTED = {
    "a_sync": "parameter-server training is out of scope",
    "qat": "use paddle_infer_amd.quantization for quantization-aware training",
    "auto": "use paddle_infer_amd.distributed.auto_parallel (Engine) for auto-parallel",
    "semi_auto": "use paddle_infer_amd.distributed.auto_parallel (Engine) for semi-auto parallel",
    "auto_search": "auto-parallel search is not implemented",
    "heter_ccl_mode": "heterogeneous collectives are not implemented",
    "is_fl_ps_mode": "federated parameter server is out of scope",
    "is_with_coordinator": "parameter-server coordinator is out of scope",
    "elastic": "use paddle_infer_amd.distributed.launch --elastic for elastic training",
}


COMM_REDUCING = ("localsgd", "adaptive_localsgd", "dgc")


def comm_reducing(st):
    """The switch (if any) whose optimizer owns the data-parallel communication."""
    for f in COMM_REDUCING:
        if getattr(st, f, False):
            return f
    return None


def check_comm_reducing(st, hcg):
    f = comm_reducing(st)
    if f is None or hcg is None:
        return
    if (hcg.get_model_parallel_world_size() > 1 or hcg.get_pipe_parallel_world_size() > 1
            or hcg.get_sharding_parallel_world_size() > 1 or st.sharding):
        raise NotImplementedError(f"DistributedStrategy.{f}: pure data parallelism only "
                                  "(no tensor / pipeline / sharding axes)")


def wrap_comm_reducing(opt, st, hcg):
    """localsgd / adaptive_localsgd / dgc around the inner optimizer (they replace the gradient
    all-reduce: `comm_optimizers.py`)."""
    from . import comm_optimizers as C
    g = hcg.get_data_parallel_group() if hcg is not None else None
    if st.localsgd:
        c = st.localsgd_configs or {}
        return C.LocalSGDOptimizer(opt, g, c.get("k_steps", 1), c.get("begin_step", 1))
    if st.adaptive_localsgd:
        c = st.adaptive_localsgd_configs or {}
        return C.AdaptiveLocalSGDOptimizer(opt, g, c.get("init_k_steps", 1), c.get("begin_step", 1))
    c = st.dgc_configs or {}
    return C.DGCMomentumOptimizer(opt, g, c.get("rampup_begin_step", 0), c.get("rampup_step", 1),
                                  c.get("sparsity", [0.999]))


def check_strategy(st):
    for f, why in REJECTED.items():
        if getattr(st, f, False):
            raise NotImplementedError(f"DistributedStrategy.{f} = True: {why}")
    if st.lamb and st.lars:
        raise ValueError("DistributedStrategy: lamb and lars are mutually exclusive")
    if sum(bool(getattr(st, f, False)) for f in COMM_REDUCING) > 1:
        raise ValueError("DistributedStrategy: localsgd, adaptive_localsgd and dgc are mutually exclusive")
    if int(st.nccl_comm_num) != 1:
        raise NotImplementedError("nccl_comm_num > 1: one RCCL communicator per group is used")
    scale = (st.gradient_scale_configs or {}).get("scale_strategy", "avg")
    if scale != "avg":
        raise NotImplementedError(f"gradient_scale_configs.scale_strategy={scale!r}: only 'avg'")


# ------------------------------------------------------------------------------- model side
def _amp_dtype(cfg):
    return "bfloat16" if cfg.get("use_bf16", True) else "float16"


def apply_model_strategy(model, st):
    if st.sync_batch_norm:
        from ...nn.layer.layers import SyncBatchNorm
        SyncBatchNorm.convert_sync_batchnorm(model)
    if st.recompute:
        _apply_recompute(model, st.recompute_configs or {})
    if st.amp:
        cfg = st.amp_configs or {}
        from ... import amp
        level = "O2" if cfg.get("use_pure_fp16", False) else "O1"
        if level == "O2":
            amp.decorate(model, level="O2", dtype=_amp_dtype(cfg))
        orig = model.forward
        white, black = cfg.get("custom_white_list"), cfg.get("custom_black_list")

        def forward(*a, **k):
            with amp.auto_cast(True, white, black, level=level, dtype=_amp_dtype(cfg)):
                return orig(*a, **k)
        model.forward = forward
        model._fleet_amp = cfg
    return model


def _apply_recompute(model, cfg):
    from .pipeline import PipelineLayer
    from .recompute import recompute
    names = list(cfg.get("checkpoints") or [])
    if not names:
        if hasattr(getattr(model, "cfg", None), "recompute"):
            model.cfg.recompute = True  # the model's own per-layer recompute (GPT)
            return
        if isinstance(model, PipelineLayer):
            model.recompute_interval = model.recompute_interval or 1
            return
    mods = dict(model.named_modules())
    if names:
        targets = []
        for n in names:
            if n not in mods:
                raise ValueError(f"recompute_configs.checkpoints: no sub-layer named {n!r}")
            targets.append(mods[n])
    else:
        targets = [c for m in model.modules() if isinstance(m, (torch.nn.ModuleList, torch.nn.Sequential))
                   for c in m.children()]
    for t in targets:
        orig = t.forward

        def fwd(*a, _f=orig, **k):
            if torch.is_grad_enabled() and any(isinstance(x, torch.Tensor) and x.requires_grad for x in a):
                return recompute(_f, *a, **k)
            return _f(*a, **k)
        t.forward = fwd
        t._fleet_recompute = True


# --------------------------------------------------------------------------- optimizer side
def _lamb(opt, cfg):
    from ... import optimizer as O
    if not isinstance(opt, O.Adam):
        raise TypeError(f"strategy.lamb replaces an Adam optimizer, got {type(opt).__name__}")
    excl = list(cfg.get("exclude_from_weight_decay", []) or [])
    names = {id(p): getattr(p, "pd_name", "") for p in opt._parameter_list}
    fn = (lambda p: any(e in names.get(id(p), "") for e in excl)) if excl else None
    return O.Lamb(learning_rate=opt._learning_rate, lamb_weight_decay=cfg.get("lamb_weight_decay", 0.01),
                  beta1=getattr(opt, "_beta1", 0.9), beta2=getattr(opt, "_beta2", 0.999),
                  epsilon=getattr(opt, "_epsilon", 1e-6), parameters=opt._parameter_list,
                  grad_clip=opt._grad_clip, exclude_from_weight_decay_fn=fn)


def _lars(opt, cfg):
    from ... import optimizer as O
    if not isinstance(opt, O.Momentum):
        raise TypeError(f"strategy.lars replaces a Momentum optimizer, got {type(opt).__name__}")
    return O.LarsMomentum(learning_rate=opt._learning_rate, momentum=opt._momentum,
                          lars_coeff=cfg.get("lars_coeff", 0.001),
                          lars_weight_decay=cfg.get("lars_weight_decay", 0.0005),
                          epsilon=cfg.get("epsilon", 0.0), parameters=opt._parameter_list,
                          grad_clip=opt._grad_clip,
                          exclude_from_weight_decay=cfg.get("exclude_from_weight_decay", None))


def swap_optimizer(opt, st):
    """lamb / lars meta-optimizers: the inner optimizer they replace."""
    if st.lamb:
        return _lamb(opt, st.lamb_configs or {})
    if st.lars:
        return _lars(opt, st.lars_configs or {})
    return opt


def wrap_optimizer(opt, st):
    """gradient_merge / asp / amp(fp16) around the (hybrid) optimizer."""
    from ... import in_dynamic_mode
    if not in_dynamic_mode():  # static mode: the meta-optimizers are Program rewrites (static_minimize)
        return opt
    if st.asp:
        from ...incubate import asp
        opt = asp.decorate(opt)
    if st.gradient_merge:
        cfg = st.gradient_merge_configs or {}
        opt = GradientMergeOptimizer(opt, int(cfg.get("k_steps", 1)), bool(cfg.get("avg", True)))
    if st.amp and _amp_dtype(st.amp_configs or {}) == "float16":
        opt = AMPOptimizer(opt, st.amp_configs or {})
    return opt


def _params(opt):
    while not hasattr(opt, "_parameter_list") and hasattr(opt, "_inner"):
        opt = opt._inner
    return getattr(opt, "_parameter_list", [])


@torch.no_grad()
def scale_grads(opt, s):
    """Multiply the pending gradients of ``opt`` (any wrapper: flat engine, ZeRO-3 shards or
    per-parameter grads) by ``s``."""
    from ..sharding import _Stage3Optimizer
    o = opt
    while True:
        if isinstance(o, _Stage3Optimizer):
            for u in o.model.units:
                u.grad.mul_(s)
                for p in u.params:
                    if p.grad is not None:
                        p.grad.mul_(s)
            return
        flat = o.__dict__.get("_flat") if hasattr(o, "__dict__") else None
        if flat is not None:
            for g in flat.groups:
                g.gflat.mul_(s)
            return
        nxt = o.__dict__.get("_inner") if hasattr(o, "__dict__") else None
        if nxt is None:
            break
        o = nxt
    for p in _params(opt):
        if p.grad is not None:
            p.grad.mul_(s)


class GradientMergeOptimizer:
    """Reference `gradient_merge_optimizer.py`: ``k_steps`` backward passes accumulate before one
    update (averaged with ``avg``)."""

    def __init__(self, inner, k_steps, avg=True):
        if k_steps < 1:
            raise ValueError("gradient_merge_configs.k_steps must be >= 1")
        self._inner, self.k_steps, self.avg = inner, k_steps, avg
        self._count = 0

    def step(self):
        self._count += 1
        if self._count % self.k_steps:
            return
        if self.avg and self.k_steps > 1:
            scale_grads(self._inner, 1.0 / self.k_steps)
        self._inner.step()

    def clear_grad(self, set_to_zero=True):
        if self._count % self.k_steps == 0:
            self._inner.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def __getattr__(self, k):
        if k == "_inner":
            raise AttributeError(k)
        return getattr(self._inner, k)


class AMPOptimizer:
    """fp16 AMP (reference `amp_optimizer.py`): ``minimize(loss)`` scales the loss, unscales the
    grads, skips the step on inf/nan and updates the dynamic loss scale."""

    def __init__(self, inner, cfg):
        from ...amp import GradScaler
        self._inner = inner
        self.scaler = GradScaler(init_loss_scaling=cfg.get("init_loss_scaling", 32768.0),
                                 incr_ratio=cfg.get("incr_ratio", 2.0), decr_ratio=cfg.get("decr_ratio", 0.5),
                                 incr_every_n_steps=cfg.get("incr_every_n_steps", 1000),
                                 decr_every_n_nan_or_inf=cfg.get("decr_every_n_nan_or_inf", 2),
                                 use_dynamic_loss_scaling=cfg.get("use_dynamic_loss_scaling", True))

    def minimize(self, loss, *a, **k):
        self.scaler.scale(loss).backward()
        self._unscale_step()

    @torch.no_grad()
    def _unscale_step(self):
        s = self.scaler
        scale_grads(self._inner, 1.0 / s.get_loss_scaling())
        bad = torch.zeros((), dtype=torch.bool)
        for p in _params(self._inner):
            if p.grad is not None:
                bad = bad | (~torch.isfinite(p.grad).all()).cpu()
        s._found_inf, s._unscaled = bool(bad), True
        if not s._found_inf:
            self._inner.step()
        s.update()

    def __getattr__(self, k):
        if k == "_inner":
            raise AttributeError(k)
        return getattr(self._inner, k)


# ------------------------------------------------------------------------------ static graph
def static_minimize(opt, loss, st, hcg, startup_program=None, parameters=None, no_grad_set=None):
    """Static-graph fleet ``minimize``: the meta-optimizers as Program rewrites
    (`fleet/static_meta.py`) around backward + the optimizer pass — amp casts (and fp16 loss
    scaling ops), recompute segments re-emitted in backward, data-parallel all-reduce ops (fp16
    with ``fp16_allreduce``), gradient merge as a conditional optimizer block."""
    import torch.distributed as dist
    from . import static_meta as SM
    block = loss.block.program.global_block()
    world = dist.get_world_size() if dist.is_initialized() else 1
    amp_cfg = st.amp_configs or {}
    ls = None
    bwd_loss = loss
    if st.amp:
        dt = _amp_dtype(amp_cfg)
        SM.amp_rewrite_forward(block, dt, amp_cfg.get("custom_white_list"), amp_cfg.get("custom_black_list"))
        if dt == "float16":
            bwd_loss, ls = SM.amp_scale_loss(block, loss, amp_cfg.get("init_loss_scaling", 32768.0))
    res = opt.minimize(bwd_loss, startup_program, parameters, no_grad_set)
    if st.recompute:
        cks = (st.recompute_configs or {}).get("checkpoints") or []
        if not cks:
            raise ValueError("static-graph recompute needs recompute_configs['checkpoints']")
        SM.recompute_rewrite(block, cks)
    gm = st.gradient_merge and int((st.gradient_merge_configs or {}).get("k_steps", 1)) > 1
    if world > 1 and not gm:
        SM.insert_dp_allreduce(block, world, bool(st.fp16_allreduce))
    if ls is not None:
        SM.amp_unscale_and_skip(block, ls, amp_cfg, merged=gm)
    if gm:
        cfg = st.gradient_merge_configs or {}
        SM.gradient_merge_rewrite(block, int(cfg.get("k_steps", 1)), bool(cfg.get("avg", True)),
                                  world, bool(st.fp16_allreduce))
    return res
