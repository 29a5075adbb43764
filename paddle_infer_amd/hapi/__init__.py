"""``paddle.Model`` high-level API + callbacks (reference `python/paddle/hapi/model.py`,
`hapi/callbacks.py`, `hapi/model_summary.py`).

Training steps run the dygraph path (HIP kernels + the framework optimizers, AMP via
``amp.auto_cast`` when ``amp_configs`` is given); data comes from ``io.DataLoader`` (device
prefetch on a side HIP stream). Distributed: when launched with several ranks the network is
wrapped in ``DataParallel`` and the loader shards with ``DistributedBatchSampler``.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from .. import io as _io
from ..framework import io as _fio
from ..metric import Metric
from . import callbacks as cbks
from .callbacks import (Callback, ProgBarLogger, ModelCheckpoint, EarlyStopping,  # noqa: F401
                        LRScheduler, ReduceLROnPlateau, VisualDL)


def _to_list(x):
    if x is None:
        return []
    return list(x) if isinstance(x, (list, tuple)) else [x]


def _device():
    from ..device import _resolve
    return _resolve()


class Model:
    def __init__(self, network, inputs=None, labels=None):
        self.network = network
        self._inputs, self._labels = _to_list(inputs), _to_list(labels)
        self._optimizer = self._loss = None
        self._metrics = []
        self._amp = None
        self.stop_training = False
        self._dist = None
        dev = _device()
        self.network.to(dev)

    # ------------------------------------------------------------------------------ setup
    def prepare(self, optimizer=None, loss=None, metrics=None, amp_configs=None):
        self._optimizer, self._loss = optimizer, loss
        self._metrics = _to_list(metrics)
        for m in self._metrics:
            assert isinstance(m, Metric), f"{m} is not a paddle.metric.Metric"
        if amp_configs is not None:
            level = amp_configs if isinstance(amp_configs, str) else amp_configs.get("level", "O1")
            self._amp = {"level": level, "dtype": (amp_configs.get("dtype", "bfloat16")
                                                   if isinstance(amp_configs, dict) else "bfloat16")}
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1 and self._dist is None:
            from ..distributed.parallel import DataParallel
            self._dist = DataParallel(self.network)

    def parameters(self, *args, **kwargs):
        return self.network.parameters(*args, **kwargs)

    @property
    def _net(self):
        return self._dist if self._dist is not None else self.network

    # ------------------------------------------------------------------------------ batches
    def _split(self, data):
        data = _to_list(data)
        n_in = len(self._inputs) if self._inputs else max(len(data) - (len(self._labels) or (1 if self._loss else 0)), 1)
        return data[:n_in], data[n_in:]

    def _move(self, xs):
        dev = _device()
        out = []
        for x in xs:
            if isinstance(x, np.ndarray):
                x = torch.from_numpy(x)
            out.append(x.to(dev, non_blocking=True) if isinstance(x, torch.Tensor) else x)
        return out

    def _forward(self, inputs):
        if self._amp is not None:
            from ..amp import auto_cast
            with auto_cast(level=self._amp["level"], dtype=self._amp["dtype"]):
                return self._net(*inputs)
        return self._net(*inputs)

    def _metric_updates(self, outputs, labels):
        res = []
        for m in self._metrics:
            r = m.compute(*(_to_list(outputs) + list(labels)))
            res.append(m.update(*_to_list(r)))
        return res

    def train_batch(self, inputs, labels=None, update=True):
        self.network.train()
        inputs, labels = self._move(_to_list(inputs)), self._move(_to_list(labels))
        outputs = self._forward(inputs)
        losses = _to_list(self._loss(*(_to_list(outputs) + labels))) if self._loss else []
        total = losses[0] if len(losses) == 1 else sum(losses)
        total.backward()
        if update:
            self._optimizer.step()
            self._optimizer.clear_grad()
        metrics = self._metric_updates(outputs, labels)
        loss_np = [float(l.detach().float()) for l in losses]
        return (loss_np, metrics) if self._metrics else loss_np

    @torch.no_grad()
    def eval_batch(self, inputs, labels=None):
        self.network.eval()
        inputs, labels = self._move(_to_list(inputs)), self._move(_to_list(labels))
        outputs = self._forward(inputs)
        losses = _to_list(self._loss(*(_to_list(outputs) + labels))) if self._loss else []
        metrics = self._metric_updates(outputs, labels)
        loss_np = [float(l.detach().float()) for l in losses]
        return (loss_np, metrics) if self._metrics else loss_np

    @torch.no_grad()
    def predict_batch(self, inputs):
        self.network.eval()
        outputs = self._forward(self._move(_to_list(inputs)))
        return [o.detach().cpu().numpy() for o in _to_list(outputs)]

    # ------------------------------------------------------------------------------ loops
    def _loader(self, data, batch_size, shuffle, drop_last, num_workers):
        if data is None or isinstance(data, (_io.DataLoader,)) or not isinstance(data, _io.Dataset):
            return data
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            bs = _io.DistributedBatchSampler(data, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last)
            return _io.DataLoader(data, batch_sampler=bs, num_workers=num_workers)
        return _io.DataLoader(data, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last,
                              num_workers=num_workers)

    def _metrics_names(self):
        names = ["loss"]
        for m in self._metrics:
            names.extend(_to_list(m.name()))
        return names

    def _logs(self, outs):
        logs = {}
        if self._metrics:
            losses, mets = outs
        else:
            losses, mets = outs, []
        logs["loss"] = losses if len(losses) != 1 else losses[0]
        for m in self._metrics:
            acc = m.accumulate()
            for n, v in zip(_to_list(m.name()), _to_list(acc)):
                logs[n] = v
        return logs

    def fit(self, train_data=None, eval_data=None, batch_size=1, epochs=1, eval_freq=1,
            log_freq=10, save_dir=None, save_freq=1, verbose=2, drop_last=False, shuffle=True,
            num_workers=0, callbacks=None, accumulate_grad_batches=1, num_iters=None):
        loader = self._loader(train_data, batch_size, shuffle, drop_last, num_workers)
        eval_loader = self._loader(eval_data, batch_size, False, False, num_workers)
        steps = len(loader) if hasattr(loader, "__len__") else None
        cb = cbks.config_callbacks(callbacks, model=self, epochs=epochs, steps=steps,
                                   log_freq=log_freq, save_freq=save_freq, save_dir=save_dir,
                                   verbose=verbose, metrics=self._metrics_names())
        self.stop_training = False
        cb.on_begin("train")
        it = 0
        for epoch in range(epochs):
            cb.on_epoch_begin(epoch)
            for m in self._metrics:
                m.reset()
            logs = {}
            for step, data in enumerate(loader):
                cb.on_batch_begin("train", step, logs)
                ins, labs = self._split(data)
                update = (step + 1) % accumulate_grad_batches == 0
                outs = self.train_batch(ins, labs, update=update)
                logs = self._logs(outs)
                logs["step"], logs["batch_size"] = step, batch_size
                cb.on_batch_end("train", step, logs)
                it += 1
                if num_iters is not None and it >= num_iters:
                    self.stop_training = True
                    break
            cb.on_epoch_end(epoch, logs)
            if eval_loader is not None and (epoch + 1) % eval_freq == 0:
                self.evaluate(eval_loader, batch_size, log_freq, verbose, num_workers, callbacks=cb)
            if self.stop_training:
                break
        cb.on_end("train", logs)
        return logs

    def evaluate(self, eval_data, batch_size=1, log_freq=10, verbose=2, num_workers=0,
                 callbacks=None, num_iters=None):
        loader = self._loader(eval_data, batch_size, False, False, num_workers)
        cb = callbacks if isinstance(callbacks, cbks.CallbackList) else cbks.config_callbacks(
            callbacks, model=self, log_freq=log_freq, verbose=verbose, metrics=self._metrics_names(),
            steps=len(loader) if hasattr(loader, "__len__") else None)
        for m in self._metrics:
            m.reset()
        cb.on_begin("eval")
        logs, losses = {}, []
        for step, data in enumerate(loader):
            cb.on_batch_begin("eval", step, logs)
            ins, labs = self._split(data)
            outs = self.eval_batch(ins, labs)
            logs = self._logs(outs)
            losses.append(logs.get("loss"))
            cb.on_batch_end("eval", step, logs)
            if num_iters is not None and step + 1 >= num_iters:
                break
        if losses and losses[0] is not None and not isinstance(losses[0], list):
            logs["loss"] = [float(np.mean(losses))]
        cb.on_end("eval", logs)
        return logs

    def predict(self, test_data, batch_size=1, num_workers=0, stack_outputs=False, verbose=1,
                callbacks=None):
        loader = self._loader(test_data, batch_size, False, False, num_workers)
        outputs = []
        for data in loader:
            ins, _ = self._split(data)
            outputs.append(self.predict_batch(ins))
        outs = list(zip(*outputs))
        if stack_outputs:
            return [np.concatenate(o, 0) for o in outs]
        return [list(o) for o in outs]

    # ------------------------------------------------------------------------------ io
    def save(self, path, training=True):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if training:
            _fio.save(self.network.state_dict(), path + ".pdparams")
            if self._optimizer is not None:
                _fio.save(self._optimizer.state_dict(), path + ".pdopt")
        else:
            from .. import jit
            spec = self._inputs or None
            jit.save(self.network, path, input_spec=spec)

    def load(self, path, skip_mismatch=False, reset_optimizer=False):
        state = _fio.load(path + ".pdparams" if not path.endswith(".pdparams") else path)
        if skip_mismatch:
            own = self.network.state_dict()
            state = {k: v for k, v in state.items() if k in own and tuple(own[k].shape) == tuple(v.shape)}
        self.network.set_state_dict(state)
        opt_path = (path[:-len(".pdparams")] if path.endswith(".pdparams") else path) + ".pdopt"
        if not reset_optimizer and self._optimizer is not None and os.path.exists(opt_path):
            self._optimizer.set_state_dict(_fio.load(opt_path))

    def summary(self, input_size=None, dtype=None):
        from .. import summary
        return summary(self.network, input_size, dtype)


time  # noqa
