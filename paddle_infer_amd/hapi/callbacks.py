"""hapi callbacks (reference `python/paddle/hapi/callbacks.py`)."""
from __future__ import annotations

import os
import time

import numpy as np


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_params(self, params):
        self.params = params

    def set_model(self, model):
        self.model = model

    def on_begin(self, mode, logs=None):
        getattr(self, f"on_{mode}_begin")(logs)

    def on_end(self, mode, logs=None):
        getattr(self, f"on_{mode}_end")(logs)

    def on_batch_begin(self, mode, step, logs=None):
        getattr(self, f"on_{mode}_batch_begin")(step, logs)

    def on_batch_end(self, mode, step, logs=None):
        getattr(self, f"on_{mode}_batch_end")(step, logs)

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_eval_begin(self, logs=None): pass
    def on_eval_end(self, logs=None): pass
    def on_predict_begin(self, logs=None): pass
    def on_predict_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_train_batch_begin(self, step, logs=None): pass
    def on_train_batch_end(self, step, logs=None): pass
    def on_eval_batch_begin(self, step, logs=None): pass
    def on_eval_batch_end(self, step, logs=None): pass
    def on_predict_batch_begin(self, step, logs=None): pass
    def on_predict_batch_end(self, step, logs=None): pass


class CallbackList:
    def __init__(self, callbacks):
        self.callbacks = list(callbacks)

    def __getattr__(self, name):
        def call(*args, **kwargs):
            for c in self.callbacks:
                getattr(c, name)(*args, **kwargs)
        return call


def _rank0():
    try:
        import torch.distributed as dist
        return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
    except Exception:  # noqa: BLE001
        return True


class ProgBarLogger(Callback):
    def __init__(self, log_freq=1, verbose=2):
        super().__init__()
        self.log_freq, self.verbose = log_freq, verbose

    def on_train_begin(self, logs=None):
        self._t0 = time.time()

    def on_epoch_begin(self, epoch, logs=None):
        self.epoch = epoch
        self._tstep = time.time()
        if self.verbose and _rank0():
            print(f"Epoch {epoch + 1}/{self.params.get('epochs', '?')}")

    def _fmt(self, logs):
        parts = []
        for k in self.params.get("metrics", []):
            if k in logs:
                v = logs[k]
                v = v[0] if isinstance(v, (list, tuple)) and len(v) == 1 else v
                parts.append(f"{k}: {v:.4f}" if isinstance(v, float) else f"{k}: {v}")
        return " - ".join(parts)

    def on_train_batch_end(self, step, logs=None):
        if self.verbose and _rank0() and (step + 1) % self.log_freq == 0:
            dt = (time.time() - self._tstep) / self.log_freq
            self._tstep = time.time()
            print(f"step {step + 1}/{self.params.get('steps', '?')} - {self._fmt(logs or {})} - {dt * 1e3:.0f}ms/step")

    def on_eval_end(self, logs=None):
        if self.verbose and _rank0():
            print(f"Eval - {self._fmt(logs or {})}")


class ModelCheckpoint(Callback):
    def __init__(self, save_freq=1, save_dir=None):
        super().__init__()
        self.save_freq, self.save_dir = save_freq, save_dir

    def on_epoch_end(self, epoch, logs=None):
        if self.save_dir and (epoch + 1) % self.save_freq == 0 and _rank0():
            self.model.save(os.path.join(self.save_dir, str(epoch)))

    def on_train_end(self, logs=None):
        if self.save_dir and _rank0():
            self.model.save(os.path.join(self.save_dir, "final"))


class LRScheduler(Callback):
    def __init__(self, by_step=True, by_epoch=False):
        super().__init__()
        self.by_step, self.by_epoch = by_step, by_epoch

    def _step(self):
        opt = self.model._optimizer
        sched = getattr(opt, "_learning_rate", None)
        if sched is not None and hasattr(sched, "step"):
            sched.step()

    def on_train_batch_end(self, step, logs=None):
        if self.by_step:
            self._step()

    def on_epoch_end(self, epoch, logs=None):
        if self.by_epoch:
            self._step()


class EarlyStopping(Callback):
    def __init__(self, monitor="loss", mode="auto", patience=0, verbose=1, min_delta=0,
                 baseline=None, save_best_model=True):
        super().__init__()
        self.monitor, self.patience, self.min_delta = monitor, patience, abs(min_delta)
        self.baseline, self.save_best_model = baseline, save_best_model
        if mode == "auto":
            mode = "max" if "acc" in monitor else "min"
        self.better = (lambda a, b: a < b - self.min_delta) if mode == "min" else (lambda a, b: a > b + self.min_delta)
        self.wait, self.best = 0, None

    def on_eval_end(self, logs=None):
        v = (logs or {}).get(self.monitor)
        if v is None:
            return
        v = float(np.mean(v))
        if self.best is None or self.better(v, self.best):
            self.best, self.wait = v, 0
            save_dir = self.params.get("save_dir")
            if self.save_best_model and save_dir and _rank0():
                self.model.save(os.path.join(save_dir, "best_model"))
        else:
            self.wait += 1
            if self.wait > self.patience:
                self.model.stop_training = True


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor="loss", factor=0.1, patience=10, verbose=1, mode="auto",
                 min_delta=1e-4, cooldown=0, min_lr=0):
        super().__init__()
        self.monitor, self.factor, self.patience = monitor, factor, patience
        self.min_delta, self.min_lr, self.cooldown = min_delta, min_lr, cooldown
        self.mode = ("max" if "acc" in monitor else "min") if mode == "auto" else mode
        self.best, self.wait, self.cool = None, 0, 0

    def on_eval_end(self, logs=None):
        v = (logs or {}).get(self.monitor)
        if v is None:
            return
        v = float(np.mean(v))
        better = self.best is None or (v < self.best - self.min_delta if self.mode == "min" else v > self.best + self.min_delta)
        if better:
            self.best, self.wait = v, 0
        elif self.cool > 0:
            self.cool -= 1
        else:
            self.wait += 1
            if self.wait >= self.patience:
                opt = self.model._optimizer
                opt.set_lr(max(opt.get_lr() * self.factor, self.min_lr))
                self.wait, self.cool = 0, self.cooldown


class VisualDL(Callback):
    """VisualDL is not available in this environment; scalars are appended to a JSONL file."""

    def __init__(self, log_dir):
        super().__init__()
        self.log_dir = log_dir
        os.makedirs(log_dir, exist_ok=True)

    def on_train_batch_end(self, step, logs=None):
        import json
        with open(os.path.join(self.log_dir, "scalars.jsonl"), "a") as f:
            f.write(json.dumps({"step": step, **{k: (v if isinstance(v, (int, float)) else float(np.mean(v)))
                                                 for k, v in (logs or {}).items()
                                                 if k not in ("batch_size",)}}) + "\n")


def config_callbacks(callbacks=None, model=None, batch_size=None, epochs=None, steps=None,
                     log_freq=2, verbose=2, save_freq=1, save_dir=None, metrics=None, mode="train"):
    cbs = list(callbacks or [])
    if not any(isinstance(c, ProgBarLogger) for c in cbs) and verbose:
        cbs = [ProgBarLogger(log_freq, verbose)] + cbs
    if not any(isinstance(c, ModelCheckpoint) for c in cbs):
        cbs.append(ModelCheckpoint(save_freq, save_dir))
    if not any(isinstance(c, LRScheduler) for c in cbs):
        cbs.append(LRScheduler())
    cl = CallbackList(cbs)
    cl.set_model(model)
    cl.set_params({"batch_size": batch_size, "epochs": epochs, "steps": steps, "verbose": verbose,
                   "metrics": metrics or [], "save_dir": save_dir})
    return cl
