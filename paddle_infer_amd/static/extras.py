"""Remaining ``paddle.static`` names (reference `python/paddle/static/__init__.py`).

* Accelerator-specific entry points of other vendors' devices (IPU / XPU / NPU / MLU) behave as in
  a reference build compiled without that device: they raise, naming the missing device.
* ``ExponentialMovingAverage``: EMA of the trainable parameters, updated after every training run
  of the program it was created for, ``apply`` swaps the averages in (bias-corrected with
  ``thres_steps``-style decay), ``restore`` swaps back (reference `fluid/optimizer.py`).
* ``auc`` / ``ctr_metric_bundle``: streaming AUC over threshold buckets and CTR statistics
  (reference `fluid/layers/metric_op.py`), with persistable global statistics.
* ``exponential_decay``: the legacy LR schedule as an LRScheduler (reference
  `fluid/layers/learning_rate_scheduler.py`).
"""
from __future__ import annotations

import contextlib

import torch

from ..nn import ParamAttr


def _no_device(kind):
    raise RuntimeError(f"paddle_infer_amd is not compiled with {kind} (MI355X / ROCm build)")


def xpu_places(device_ids=None):
    _no_device("XPU")


def npu_places(device_ids=None):
    _no_device("NPU")


def mlu_places(device_ids=None):
    _no_device("MLU")


@contextlib.contextmanager
def ipu_shard_guard(index=-1, stage=-1):
    _no_device("IPU")
    yield


def set_ipu_shard(call_func, index=-1, stage=-1):
    _no_device("IPU")


class IpuStrategy:
    def __init__(self):
        _no_device("IPU")


class IpuCompiledProgram:
    def __init__(self, program=None, scope=None, ipu_strategy=None):
        _no_device("IPU")


class WeightNormParamAttr(ParamAttr):
    """ParamAttr requesting weight normalisation w = g · v / ‖v‖ over all dims but ``dim``
    (reference `fluid/param_attr.py:WeightNormParamAttr`)."""

    def __init__(self, dim=None, name=None, initializer=None, learning_rate=1.0, regularizer=None,
                 trainable=True, do_model_average=False, need_clip=True):
        super().__init__(name=name, initializer=initializer, learning_rate=learning_rate,
                         regularizer=regularizer, trainable=trainable, need_clip=need_clip)
        self.dim = dim
        self.do_model_average = do_model_average


class ExponentialMovingAverage:
    """EMA of the program's trainable parameters: ema = decay·ema + (1 − decay)·param after each
    training run (``update()`` registers the update on the current main program), decay ramped as
    min(decay, (1 + step) / (10 + step)) when ``thres_steps`` is given; ``apply(exe)`` swaps the
    bias-corrected averages into the scope, ``restore(exe)`` swaps the parameters back."""

    def __init__(self, decay=0.999, thres_steps=None, name=None):
        self._decay = float(decay)
        self._thres = thres_steps
        self._ema, self._backup = {}, {}
        self._step = 0
        self._program = None

    def update(self):
        from .framework import default_main_program
        prog = default_main_program()
        self._program = prog
        hooks = prog.__dict__.setdefault("_post_run_hooks", [])
        hooks.append(self._on_run)

    def _decay_now(self):
        if self._thres is None:
            return self._decay
        return min(self._decay, (1.0 + self._step) / (10.0 + self._step))

    def _on_run(self, scope, program):
        d = self._decay_now()
        self._step += 1
        with torch.no_grad():
            for n, p in program.params.items():
                cur = scope.get(n)
                if cur is None or not cur.is_floating_point() or n.startswith("learning_rate"):
                    continue
                e = self._ema.get(n)
                if e is None:
                    e = self._ema[n] = torch.zeros_like(cur, dtype=torch.float32)
                e.mul_(d).add_(cur.float(), alpha=1.0 - d)

    @contextlib.contextmanager
    def apply(self, executor=None, need_restore=True):
        from .framework import global_scope
        scope = global_scope()
        corr = 1.0 - self._decay ** max(self._step, 1) if self._thres is None else 1.0
        with torch.no_grad():
            for n, e in self._ema.items():
                cur = scope.get(n)
                self._backup[n] = cur.detach().clone()
                cur.copy_((e / corr).to(cur.dtype))
        try:
            yield
        finally:
            if need_restore:
                self.restore(executor)

    def restore(self, executor=None):
        from .framework import global_scope
        scope = global_scope()
        with torch.no_grad():
            for n, b in self._backup.items():
                scope.get(n).copy_(b)
        self._backup.clear()


def _auc_from_stats(pos, neg):
    """Trapezoidal ROC AUC from per-bucket positive / negative counts (highest bucket first)."""
    tp = torch.cumsum(pos.flip(0), 0)
    fp = torch.cumsum(neg.flip(0), 0)
    P, N = tp[-1], fp[-1]
    if P <= 0 or N <= 0:
        return torch.tensor(0.5, dtype=torch.float64)
    tpr = torch.cat([tp.new_zeros(1), tp]) / P
    fpr = torch.cat([fp.new_zeros(1), fp]) / N
    return torch.trapz(tpr, fpr)


_AUC_STATE: dict = {}


def auc(input, label, curve="ROC", num_thresholds=2 ** 12 - 1, topk=1, slide_steps=1,  # noqa: A002
        ins_tag_weight=None):
    """Streaming AUC (reference `metric_op.py:auc`): ``input`` [N, 2] class probabilities (column
    1 = positive), ``label`` [N, 1]. Returns (global_auc, batch_auc, [batch_stat_pos,
    batch_stat_neg, stat_pos, stat_neg]); the global statistics persist across calls (per call
    site)."""
    if curve != "ROC":
        raise ValueError("auc: only the ROC curve is supported")
    prob = input[:, -1].detach().double()
    lab = label.reshape(-1).detach().long()
    w = ins_tag_weight.reshape(-1).double() if ins_tag_weight is not None else torch.ones_like(prob)
    b = torch.clamp((prob * num_thresholds).long(), 0, num_thresholds)
    pos = torch.zeros(num_thresholds + 1, dtype=torch.float64, device=prob.device)
    neg = torch.zeros_like(pos)
    pos.index_add_(0, b, w * (lab == 1))
    neg.index_add_(0, b, w * (lab != 1))
    key = (num_thresholds, prob.device)
    st = _AUC_STATE.setdefault(key, [torch.zeros_like(pos), torch.zeros_like(neg)])
    st[0].add_(pos)
    st[1].add_(neg)
    return _auc_from_stats(st[0], st[1]), _auc_from_stats(pos, neg), [pos, neg, st[0], st[1]]


def ctr_metric_bundle(input, label, ins_tag_weight=None):  # noqa: A002
    """CTR statistics (reference `metric_op.py:ctr_metric_bundle`): local sums of squared error,
    absolute error, predicted probability, clicked label and instance count — the terms of RMSE /
    MAE / predicted CTR / actual CTR over a pass."""
    p = input.reshape(-1).float()
    y = label.reshape(-1).float()
    w = ins_tag_weight.reshape(-1).float() if ins_tag_weight is not None else torch.ones_like(p)
    return ((w * (p - y) ** 2).sum(), (w * (p - y).abs()).sum(), (w * p).sum(), (w * y).sum(),
            w.sum())


def exponential_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    """lr · decay_rate^(step / decay_steps) (floored when ``staircase``)."""
    from ..optimizer.lr import LRScheduler

    class _ExpDecay(LRScheduler):
        def get_lr(self):
            e = self.last_epoch / decay_steps
            if staircase:
                e = float(int(e))
            return self.base_lr * decay_rate ** e

    return _ExpDecay(learning_rate)


def create_lod_tensor(data, recursive_seq_lens, place=None):
    """Packed tensor + LoD (offsets from ``recursive_seq_lens``) for the sequence ops."""
    t = data if isinstance(data, torch.Tensor) else torch.as_tensor(data)
    lod = []
    for lens in recursive_seq_lens:
        offs = [0]
        for n in lens:
            offs.append(offs[-1] + int(n))
        lod.append(offs)
    t.lod = lod
    return t
