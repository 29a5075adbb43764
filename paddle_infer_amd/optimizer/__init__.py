"""``paddle.optimizer`` (reference `python/paddle/optimizer/{optimizer,sgd,momentum,adam,adamw,lamb,
adagrad,rmsprop,adadelta,adamax}.py`) and ``paddle.optimizer.lr``.

MI355X-native design: on GPU, ``Adam``/``AdamW``/``Momentum`` build flat parameter/gradient
buffers at construction (``parallel.flat_engine``) so ``step()`` is ONE fused HIP kernel launch
per dtype/decay group with fp32 master weights (``multi_precision``) and a device-side global-norm
clip — no per-tensor launches, no host sync. Other optimizers (and the CPU path) apply the same
math per parameter with torch ops.
"""
from __future__ import annotations

import math

import torch

from . import lr  # noqa: F401
from .lr import LRScheduler


def _lr_value(lr_):
    return lr_() if isinstance(lr_, LRScheduler) else float(lr_)


class Optimizer:
    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None,
                 name=None, multi_precision=False):
        from ..static.framework import _STATE as _SSTATE
        if parameters is None and not _SSTATE["static"]:
            raise ValueError("parameters must be given in dygraph mode")
        params = list(parameters) if parameters is not None else []
        if params and isinstance(params[0], dict):  # param groups
            self._param_groups = params
            params = [p for g in params for p in g["params"]]
        else:
            self._param_groups = None
        self._parameter_list = params
        self._learning_rate = learning_rate
        self.regularization = weight_decay
        self._grad_clip = grad_clip
        self._multi_precision = multi_precision
        self._accumulators = {}
        self._master = {}
        self._step = 0

    # ---- lr -------------------------------------------------------------------------
    def get_lr(self):
        return _lr_value(self._learning_rate)

    def set_lr(self, value):
        if isinstance(self._learning_rate, LRScheduler):
            raise RuntimeError("optimizer's learning rate is an LRScheduler; call scheduler.step()")
        self._learning_rate = float(value)

    def set_lr_scheduler(self, scheduler):
        self._learning_rate = scheduler

    # ---- grads ----------------------------------------------------------------------
    def clear_grad(self, set_to_zero=True):
        for p in self._parameter_list:
            if p.grad is not None:
                if set_to_zero:
                    p.grad.zero_()
                else:
                    p.grad = None

    clear_gradients = clear_grad

    def _params_grads(self):
        from ..utils import nan_inf
        if nan_inf.enabled():  # FLAGS_check_nan_inf: one host read per step
            nan_inf.check()
        pg = [(p, p.grad) for p in self._parameter_list if p.requires_grad]
        if self._grad_clip is not None:
            pg = self._grad_clip(pg)
        return pg

    def _l2(self, p, g):
        wd = self.regularization
        if wd is None:
            return g
        coeff = wd if isinstance(wd, (int, float)) else getattr(wd, "_coeff", getattr(wd, "coeff", 0.0))
        if isinstance(wd, L1Decay):
            return g + coeff * torch.sign(p)
        return g + coeff * p if coeff else g

    def _master_of(self, p):
        if self._multi_precision and p.dtype in (torch.float16, torch.bfloat16):
            m = self._master.get(id(p))
            if m is None:
                m = self._master[id(p)] = p.detach().float().clone()
            return m
        return p

    def _acc(self, name, p, init=0.0, like=None):
        key = (name, id(p))
        t = self._accumulators.get(key)
        if t is None:
            ref = like if like is not None else self._master_of(p)
            t = self._accumulators[key] = torch.full_like(ref, init, dtype=torch.float32 if ref.is_floating_point() else ref.dtype)
        return t

    # merged (multi-tensor) GPU update: one launch for every parameter (reference
    # merged_momentum / use_multi_tensor); subclasses name their op code
    _merged_op = None

    def _merged_ok(self, pg):
        if self._merged_op is None or self._param_groups is not None or isinstance(self.regularization, L1Decay):
            return False
        def dense(t):
            return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))
        # elementwise over storage: p, grad (and the states, created like p) share one dense layout
        return all(p.is_cuda and p.dtype == torch.float32 and g is not None and dense(p)
                   and g.stride() == p.stride() and g.dtype in (torch.float32, torch.bfloat16)
                   for p, g in pg)

    def _merged_step(self, pg, lr_):
        from ..ops.optim import multi_tensor_update
        wd = self.regularization
        coeff = 0.0 if wd is None else float(wd if isinstance(wd, (int, float)) else getattr(wd, "_coeff", 0.0))
        entries = []
        for p, g in pg:
            s1 = self._acc("velocity", p) if self._merged_op == 1 else None
            entries.append((p, g, s1, None, coeff, getattr(p, "optimize_attr", {}).get("learning_rate", 1.0)))
        cache = self.__dict__.setdefault("_mt_cache", {})
        multi_tensor_update(self._merged_op, entries, lr_, cache, **self._merged_hyper())

    def _merged_hyper(self):
        return {}

    @torch.no_grad()
    def step(self):
        self._step += 1
        from ..ops import autotune as _at
        _at.step()
        lr_ = self.get_lr()
        pg = [(p, g) for p, g in self._params_grads() if g is not None]
        if pg and self._merged_ok(pg):
            self._merged_step(pg, lr_)
            return
        for p, g in pg:
            if g is None:
                continue
            mp = self._master_of(p)
            gf = g.float() if mp.dtype == torch.float32 else g
            plr = lr_ * getattr(p, "optimize_attr", {}).get("learning_rate", 1.0)
            self._update(p, mp, gf, plr)
            if mp is not p:
                p.copy_(mp)

    def _update(self, p, mp, g, lr_):  # pragma: no cover
        raise NotImplementedError

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        from ..static.framework import Variable as _SVar
        if isinstance(loss, _SVar):  # static graph: append backward + optimize ops
            from ..static.backward import minimize as _static_minimize
            return _static_minimize(self, loss, parameters, no_grad_set)
        loss.backward()
        self.step()
        return None, [(p, p.grad) for p in self._parameter_list]

    def backward(self, loss, startup_program=None, parameters=None, no_grad_set=None, callbacks=None):
        loss.backward()
        return [(p, p.grad) for p in self._parameter_list]

    def apply_gradients(self, params_grads):
        self.step()

    # ---- state ----------------------------------------------------------------------
    def state_dict(self):
        sd = {"step": self._step}
        names = {id(p): getattr(p, "pd_name", str(i)) for i, p in enumerate(self._parameter_list)}
        for (n, pid), t in self._accumulators.items():
            sd[f"{names.get(pid, pid)}_{n}_0"] = t
        for pid, t in self._master.items():
            sd[f"master_weights.{names.get(pid, pid)}"] = t
        if isinstance(self._learning_rate, LRScheduler):
            sd["LR_Scheduler"] = self._learning_rate.state_dict()
        return sd

    def set_state_dict(self, state_dict):
        self._step = int(state_dict.get("step", 0))
        names = {getattr(p, "pd_name", str(i)): p for i, p in enumerate(self._parameter_list)}
        for k, v in state_dict.items():
            if k.startswith("master_weights."):
                p = names.get(k[len("master_weights."):])
                if p is not None:
                    self._master[id(p)] = torch.as_tensor(v).to(p.device).float()
                continue
            for pname, p in names.items():
                if k.startswith(pname + "_") and k.endswith("_0"):
                    acc = k[len(pname) + 1:-2]
                    self._accumulators[(acc, id(p))] = torch.as_tensor(v).to(p.device)
        if "LR_Scheduler" in state_dict and isinstance(self._learning_rate, LRScheduler):
            self._learning_rate.set_state_dict(state_dict["LR_Scheduler"])

    load_state_dict = set_state_dict


class L2Decay:
    def __init__(self, coeff=0.0):
        self._coeff = coeff


class L1Decay(L2Decay):
    pass


class SGD(Optimizer):
    _merged_op = 0

    def _update(self, p, mp, g, lr_):
        mp.sub_(lr_ * self._l2(mp, g))


class Momentum(Optimizer):
    def __init__(self, learning_rate=0.001, momentum=0.9, parameters=None, use_nesterov=False,
                 weight_decay=None, grad_clip=None, multi_precision=False, rescale_grad=1.0,
                 name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._momentum, self._nesterov, self._rescale = momentum, use_nesterov, rescale_grad
        self._merged_op = 1 if rescale_grad == 1.0 else None

    def _merged_hyper(self):
        return {"mu": float(self._momentum), "nesterov": bool(self._nesterov)}

    def _update(self, p, mp, g, lr_):
        g = self._l2(mp, g * self._rescale)
        v = self._acc("velocity", p)
        v.mul_(self._momentum).add_(g)
        mp.sub_(lr_ * (g + self._momentum * v if self._nesterov else v))


class LarsMomentum(Momentum):
    """LARS (reference `fluid/optimizer.py` LarsMomentumOptimizer / `lars_momentum` op): per-layer
    local lr = lr · lars_coeff · ‖w‖ / (‖g‖ + lars_weight_decay · ‖w‖ + epsilon), then momentum
    on (g + lars_weight_decay · w). Parameters whose name contains an entry of
    ``exclude_from_weight_decay`` get no decay (and the plain lr)."""

    def __init__(self, learning_rate=0.001, momentum=0.9, lars_coeff=0.001, lars_weight_decay=0.0005,
                 parameters=None, grad_clip=None, name=None, exclude_from_weight_decay=None,
                 epsilon=0.0, multi_precision=False, rescale_grad=1.0):
        super().__init__(learning_rate, momentum, parameters, False, None, grad_clip, multi_precision,
                         rescale_grad, name)
        self._lars_coeff, self._lars_wd, self._lars_eps = lars_coeff, lars_weight_decay, epsilon
        self._exclude = list(exclude_from_weight_decay or [])
        self._merged_op = None

    def _update(self, p, mp, g, lr_):
        g = g * self._rescale
        excluded = any(e in getattr(p, "pd_name", "") for e in self._exclude)
        wd = 0.0 if excluded else self._lars_wd
        v = self._acc("velocity", p)
        if excluded:
            local = lr_
        else:
            wn, gn = mp.norm(), g.norm()
            ratio = self._lars_coeff * wn / (gn + wd * wn + self._lars_eps)
            local = lr_ * torch.where((wn > 0) & (gn > 0), ratio, torch.ones_like(wn))
        v.mul_(self._momentum).add_(local * (g + wd * mp))
        mp.sub_(v)


class Adam(Optimizer):
    _decoupled = False

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None,
                 weight_decay=None, grad_clip=None, lazy_mode=False, multi_precision=False,
                 use_multi_tensor=False, name=None, **kw):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._beta1, self._beta2, self._epsilon = float(beta1), float(beta2), float(epsilon)
        self._flat = None
        self._maybe_flat(kw)

    # ----- fused flat-buffer path on GPU ------------------------------------------------
    def _flat_ok(self):
        ps = [p for p in self._parameter_list if p.requires_grad]
        return (ps and all(p.is_cuda for p in ps) and self._param_groups is None
                and (self._decoupled or self.regularization is None)
                and (self._grad_clip is None or type(self._grad_clip).__name__ == "ClipGradByGlobalNorm"))

    def _maybe_flat(self, kw):
        if not self._flat_ok():
            return
        from ..distributed import fleet as _fleet
        if _fleet._STATE.get("hcg") is not None:
            # fleet.distributed_optimizer builds the engine on the hybrid groups (building it here
            # too would hold two copies of every fp32 master / moment buffer until then)
            self._flat_pending = True
            return
        from ..parallel.flat_engine import FlatTrainer
        wd = self._decay_coeff() if self._decoupled else 0.0
        apply = getattr(self, "_apply_decay_param_fun", None)
        clip = getattr(self._grad_clip, "clip_norm", None)
        named = [(getattr(p, "pd_name", str(i)), p) for i, p in enumerate(self._parameter_list)]
        self._flat = FlatTrainer(None, lr=self.get_lr(), betas=(self._beta1, self._beta2),
                                 eps=self._epsilon, weight_decay=wd, grad_clip=clip,
                                 named_params=named,
                                 no_decay_fn=(lambda n, p: not apply(n)) if apply else (lambda n, p: False))

    def _decay_coeff(self):
        return 0.0

    @torch.no_grad()
    def step(self):
        if self._flat is not None:
            from ..ops import autotune as _at
            _at.step()
            self._step += 1
            self._flat.step(self.get_lr())
            return
        super().step()

    def clear_grad(self, set_to_zero=True):
        if self._flat is not None:
            self._flat.zero_grad()
            return
        super().clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def _update(self, p, mp, g, lr_):
        if not self._decoupled:
            g = self._l2(mp, g)
        else:
            mp.mul_(1.0 - lr_ * self._coeff_for(p))
        m = self._acc("moment1", p)
        v = self._acc("moment2", p)
        t = self._step
        m.mul_(self._beta1).add_(g, alpha=1 - self._beta1)
        v.mul_(self._beta2).addcmul_(g, g, value=1 - self._beta2)
        bc2 = math.sqrt(1 - self._beta2 ** t)
        step = lr_ * bc2 / (1 - self._beta1 ** t)
        mp.addcdiv_(m, v.sqrt().add_(self._epsilon * bc2), value=-step)

    def _coeff_for(self, p):
        return 0.0

    def state_dict(self):
        if self._flat is not None:
            sd = self._flat.state_dict()
            if isinstance(self._learning_rate, LRScheduler):
                sd["LR_Scheduler"] = self._learning_rate.state_dict()
            return sd
        return super().state_dict()

    def set_state_dict(self, state_dict):
        if self._flat is not None:
            self._flat.set_state_dict(state_dict)
            self._step = self._flat.step_count
            if "LR_Scheduler" in state_dict and isinstance(self._learning_rate, LRScheduler):
                self._learning_rate.set_state_dict(state_dict["LR_Scheduler"])
            return
        super().set_state_dict(state_dict)


class AdamW(Adam):
    _decoupled = True

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None,
                 weight_decay=0.01, lr_ratio=None, apply_decay_param_fun=None, grad_clip=None,
                 lazy_mode=False, multi_precision=False, name=None):
        self._wd = float(weight_decay if not isinstance(weight_decay, L2Decay) else weight_decay._coeff)
        self._apply_decay_param_fun = apply_decay_param_fun
        super().__init__(learning_rate, beta1, beta2, epsilon, parameters, None, grad_clip, lazy_mode,
                         multi_precision, name=name)

    def _decay_coeff(self):
        return self._wd

    def _coeff_for(self, p):
        if self._apply_decay_param_fun is not None and not self._apply_decay_param_fun(getattr(p, "pd_name", "")):
            return 0.0
        return self._wd


class Adamax(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._beta1, self._beta2, self._epsilon = beta1, beta2, epsilon

    def _update(self, p, mp, g, lr_):
        g = self._l2(mp, g)
        m = self._acc("moment", p)
        u = self._acc("inf_norm", p)
        m.mul_(self._beta1).add_(g, alpha=1 - self._beta1)
        torch.maximum(u * self._beta2, g.abs() + self._epsilon, out=u)
        mp.sub_(lr_ / (1 - self._beta1 ** self._step) * m / u)


class Adagrad(Optimizer):
    def __init__(self, learning_rate, epsilon=1e-6, parameters=None, weight_decay=None,
                 grad_clip=None, name=None, initial_accumulator_value=0.0):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._epsilon, self._init = epsilon, initial_accumulator_value

    def _update(self, p, mp, g, lr_):
        g = self._l2(mp, g)
        acc = self._acc("moment", p, self._init)
        acc.addcmul_(g, g)
        mp.addcdiv_(g, acc.sqrt().add_(self._epsilon), value=-lr_)


class RMSProp(Optimizer):
    def __init__(self, learning_rate, rho=0.95, epsilon=1e-6, momentum=0.0, centered=False,
                 parameters=None, weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._rho, self._eps, self._mom, self._centered = rho, epsilon, momentum, centered

    def _update(self, p, mp, g, lr_):
        g = self._l2(mp, g)
        ms = self._acc("mean_square", p)
        ms.mul_(self._rho).addcmul_(g, g, value=1 - self._rho)
        if self._centered:
            mg = self._acc("mean_grad", p)
            mg.mul_(self._rho).add_(g, alpha=1 - self._rho)
            denom = (ms - mg * mg).add_(self._eps).sqrt()
        else:
            denom = ms.add(self._eps).sqrt()
        mom = self._acc("momentum", p)
        mom.mul_(self._mom).addcdiv_(g, denom, value=lr_)
        mp.sub_(mom)


class Adadelta(Optimizer):
    def __init__(self, learning_rate=0.001, epsilon=1e-6, rho=0.95, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._eps, self._rho = epsilon, rho

    def _update(self, p, mp, g, lr_):
        g = self._l2(mp, g)
        eg = self._acc("avg_squared_grad", p)
        ex = self._acc("avg_squared_update", p)
        eg.mul_(self._rho).addcmul_(g, g, value=1 - self._rho)
        upd = g * (ex + self._eps).sqrt() / (eg + self._eps).sqrt()
        ex.mul_(self._rho).addcmul_(upd, upd, value=1 - self._rho)
        mp.sub_(lr_ * upd)


class Lamb(Optimizer):
    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999,
                 epsilon=1e-6, parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None,
                 multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name, multi_precision)
        self._wd, self._b1, self._b2, self._eps = lamb_weight_decay, beta1, beta2, epsilon
        self._exclude = exclude_from_weight_decay_fn

    def _update(self, p, mp, g, lr_):
        m = self._acc("moment1", p)
        v = self._acc("moment2", p)
        t = self._step
        m.mul_(self._b1).add_(g, alpha=1 - self._b1)
        v.mul_(self._b2).addcmul_(g, g, value=1 - self._b2)
        mh = m / (1 - self._b1 ** t)
        vh = v / (1 - self._b2 ** t)
        wd = 0.0 if (self._exclude and self._exclude(p)) else self._wd
        r = mh / (vh.sqrt() + self._eps) + wd * mp
        wn, rn = mp.norm(), r.norm()
        trust = torch.where((wn > 0) & (rn > 0), wn / rn, torch.ones_like(wn))
        mp.sub_(lr_ * trust * r)


__all__ = ["Optimizer", "SGD", "Momentum", "Adam", "AdamW", "Adamax", "Adagrad", "RMSProp",
           "Adadelta", "Lamb", "LarsMomentum", "L1Decay", "L2Decay", "lr"]
