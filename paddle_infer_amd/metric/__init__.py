"""``paddle.metric`` (reference `python/paddle/metric/metrics.py`): Metric, Accuracy, Precision,
Recall, Auc and the functional ``accuracy``. ``compute`` runs on-device (one fused top-k + compare
per batch); ``update`` accumulates on the host like the reference."""
from __future__ import annotations

import abc

import numpy as np
import torch


def _np(x):
    if isinstance(x, torch.Tensor):
        x = x.detach()
        if x.dtype == torch.bfloat16:
            x = x.float()
        return x.cpu().numpy()
    return np.asarray(x)


class Metric(abc.ABC):
    def __init__(self):
        pass

    @abc.abstractmethod
    def reset(self):
        ...

    @abc.abstractmethod
    def update(self, *args):
        ...

    @abc.abstractmethod
    def accumulate(self):
        ...

    @abc.abstractmethod
    def name(self):
        ...

    def compute(self, *args):
        return args


class Accuracy(Metric):
    def __init__(self, topk=(1,), name=None, *args, **kwargs):
        super().__init__()
        self.topk = topk if isinstance(topk, (list, tuple)) else (topk,)
        self.maxk = max(self.topk)
        self._init_name(name)
        self.reset()

    def compute(self, pred, label, *args):
        pred = torch.as_tensor(pred) if not isinstance(pred, torch.Tensor) else pred
        label = torch.as_tensor(label) if not isinstance(label, torch.Tensor) else label
        idx = torch.topk(pred.float(), self.maxk, dim=-1).indices
        if label.dim() == pred.dim() and label.shape[-1] == pred.shape[-1] and label.shape[-1] > 1:
            label = label.argmax(-1, keepdim=True)  # one-hot / soft labels
        if label.dim() == pred.dim() - 1:
            label = label.unsqueeze(-1)
        return (idx == label.to(idx.device).long()).float()

    def update(self, correct, *args):
        correct = _np(correct)
        num = int(np.prod(correct.shape[:-1]))
        accs = []
        for i, k in enumerate(self.topk):
            c = float(correct[..., :k].sum())
            accs.append(c / max(num, 1))
            self.total[i] += c
            self.count[i] += num
        return accs[0] if len(self.topk) == 1 else accs

    def reset(self):
        self.total = [0.0] * len(self.topk)
        self.count = [0] * len(self.topk)

    def accumulate(self):
        res = [t / max(c, 1) for t, c in zip(self.total, self.count)]
        return res[0] if len(self.topk) == 1 else res

    def _init_name(self, name):
        name = name or "acc"
        self._name = [f"{name}_top{k}" for k in self.topk] if len(self.topk) > 1 else [name]

    def name(self):
        return self._name


class Precision(Metric):
    def __init__(self, name="precision", *args, **kwargs):
        super().__init__()
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = (_np(preds).reshape(-1) >= 0.5).astype(np.int64)
        y = _np(labels).reshape(-1).astype(np.int64)
        self.tp += int(((p == 1) & (y == 1)).sum())
        self.fp += int(((p == 1) & (y == 0)).sum())

    def reset(self):
        self.tp = self.fp = 0

    def accumulate(self):
        ap = self.tp + self.fp
        return float(self.tp) / ap if ap else 0.0

    def name(self):
        return self._name


class Recall(Metric):
    def __init__(self, name="recall", *args, **kwargs):
        super().__init__()
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = (_np(preds).reshape(-1) >= 0.5).astype(np.int64)
        y = _np(labels).reshape(-1).astype(np.int64)
        self.tp += int(((p == 1) & (y == 1)).sum())
        self.fn += int(((p == 0) & (y == 1)).sum())

    def reset(self):
        self.tp = self.fn = 0

    def accumulate(self):
        r = self.tp + self.fn
        return float(self.tp) / r if r else 0.0

    def name(self):
        return self._name


class Auc(Metric):
    """Histogram AUC (reference: ``num_thresholds`` buckets of the positive-class score)."""

    def __init__(self, curve="ROC", num_thresholds=4095, name="auc", *args, **kwargs):
        super().__init__()
        self._curve, self._num_thresholds, self._name = curve, num_thresholds, name
        self.reset()

    def update(self, preds, labels):
        p = _np(preds)
        if p.ndim == 2 and p.shape[1] == 2:
            p = p[:, 1]
        p = p.reshape(-1)
        y = _np(labels).reshape(-1)
        bins = np.clip((p * self._num_thresholds).astype(np.int64), 0, self._num_thresholds)
        np.add.at(self._stat_pos, bins[y > 0], 1)
        np.add.at(self._stat_neg, bins[y <= 0], 1)

    def reset(self):
        self._stat_pos = np.zeros(self._num_thresholds + 1, np.int64)
        self._stat_neg = np.zeros(self._num_thresholds + 1, np.int64)

    def accumulate(self):
        tot_pos = tot_neg = 0.0
        auc = 0.0
        for i in range(self._num_thresholds, -1, -1):
            np_, nn_ = tot_pos, tot_neg
            tot_pos += self._stat_pos[i]
            tot_neg += self._stat_neg[i]
            auc += (tot_neg - nn_) * (tot_pos + np_) / 2.0
        return auc / (tot_pos * tot_neg) if tot_pos > 0 and tot_neg > 0 else 0.0

    def name(self):
        return self._name


def accuracy(input, label, k=1, correct=None, total=None, name=None):  # noqa: A002
    """Reference `metric/metrics.py:accuracy` — top-k accuracy as a 0-d tensor."""
    idx = torch.topk(input.float(), k, dim=-1).indices
    lab = label.reshape(-1, 1).to(idx.device).long() if label.dim() <= 1 or label.shape[-1] == 1 else label
    hit = (idx == lab).any(-1).float()
    return hit.mean()
