"""``paddle.amp`` — auto_cast (O1/O2), GradScaler, decorate (reference `python/paddle/amp/`).

bf16 is the native MI355X training dtype (no loss scaling needed); fp16 O1/O2 with dynamic loss
scaling is supported for parity. O1 = per-op autocast (white list ops such as matmul/conv run in
low precision); O2 = parameters cast to the low dtype with fp32 master weights in the optimizer
(``multi_precision``), norms kept in fp32.
"""
from __future__ import annotations

import contextlib

import torch

from ..framework.dtype import to_torch_dtype as _dt

WHITE_LIST = {"matmul", "conv2d", "linear", "mul", "bmm", "einsum"}
BLACK_LIST = {"softmax_with_cross_entropy", "layer_norm", "exp", "log", "mean", "sum"}


@contextlib.contextmanager
def auto_cast(enable=True, custom_white_list=None, custom_black_list=None, level="O1",
              dtype="float16", use_promote=True):
    if not enable or level == "O0":
        yield
        return
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    d = _dt(dtype)
    if dev == "cpu" and d == torch.float16:
        d = torch.bfloat16
    with torch.autocast(device_type=dev, dtype=d):
        yield


amp_guard = auto_cast


def _is_norm(m):
    n = type(m).__name__
    return "Norm" in n


def decorate(models, optimizers=None, level="O1", dtype="float16", master_weight=None,
             save_dtype=None, master_grad=False, excluded_layers=None):
    if level != "O2":
        return (models, optimizers) if optimizers is not None else models
    d = _dt(dtype)
    single = not isinstance(models, (list, tuple))
    ms = [models] if single else list(models)
    for m in ms:
        for sub in m.modules():
            if _is_norm(sub) or (excluded_layers and isinstance(sub, tuple(excluded_layers))):
                continue
            for p in sub.parameters(recurse=False):
                p.data = p.data.to(d)
    if optimizers is not None:
        os_ = [optimizers] if not isinstance(optimizers, (list, tuple)) else list(optimizers)
        for o in os_:
            o._multi_precision = True if master_weight is None else bool(master_weight)
        return (ms[0] if single else ms), optimizers
    return ms[0] if single else ms


class GradScaler:
    """Dynamic loss scaling (reference `python/paddle/amp/grad_scaler.py`)."""

    def __init__(self, enable=True, init_loss_scaling=2.0 ** 15, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=1000, decr_every_n_nan_or_inf=2, use_dynamic_loss_scaling=True):
        self._enable = enable
        self._scale = float(init_loss_scaling)
        self._incr_ratio, self._decr_ratio = incr_ratio, decr_ratio
        self._incr_every, self._decr_every = incr_every_n_steps, decr_every_n_nan_or_inf
        self._dynamic = use_dynamic_loss_scaling
        self._good = 0
        self._bad = 0
        self._found_inf = False
        self._unscaled = False

    def is_enable(self):
        return self._enable

    def is_use_dynamic_loss_scaling(self):
        return self._dynamic

    def get_loss_scaling(self):
        return self._scale

    def set_loss_scaling(self, v):
        self._scale = float(v)

    def scale(self, var):
        return var * self._scale if self._enable else var

    def unscale_(self, optimizer):
        if not self._enable or self._unscaled:
            return
        found = torch.zeros((), dtype=torch.bool)
        inv = 1.0 / self._scale
        for p in optimizer._parameter_list:
            if p.grad is not None:
                p.grad.mul_(inv)
                found = found | (~torch.isfinite(p.grad).all()).cpu()
        self._found_inf = bool(found)
        self._unscaled = True

    def step(self, optimizer):
        if not self._enable:
            optimizer.step()
            return
        self.unscale_(optimizer)
        if not self._found_inf:
            optimizer.step()

    def minimize(self, optimizer, *args, **kwargs):
        self.step(optimizer)
        self.update()
        return None, None

    def update(self):
        if not self._enable:
            return
        if self._dynamic:
            if self._found_inf:
                self._bad += 1
                self._good = 0
                if self._bad >= self._decr_every:
                    self._scale = max(1.0, self._scale * self._decr_ratio)
                    self._bad = 0
            else:
                self._good += 1
                self._bad = 0
                if self._good >= self._incr_every:
                    self._scale *= self._incr_ratio
                    self._good = 0
        self._found_inf = False
        self._unscaled = False

    def state_dict(self):
        return {"scale": self._scale, "incr_count": self._good, "decr_count": self._bad,
                "incr_ratio": self._incr_ratio, "decr_ratio": self._decr_ratio,
                "incr_every_n_steps": self._incr_every, "decr_every_n_nan_or_inf": self._decr_every,
                "use_dynamic_loss_scaling": self._dynamic}

    def load_state_dict(self, sd):
        self._scale = sd["scale"]
        self._good, self._bad = sd.get("incr_count", 0), sd.get("decr_count", 0)

    set_state_dict = load_state_dict


AmpScaler = GradScaler


def is_float16_supported(device=None):
    return torch.cuda.is_available()


def is_bfloat16_supported(device=None):
    return True
