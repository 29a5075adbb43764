"""``paddle.text`` (reference `python/paddle/text/`): Viterbi decoding for CRF-style sequence
labelling, and the dataset classes (`datasets.py`: the reference's parsers over the archives it
downloads — without network access they read a local ``data_file``)."""
from __future__ import annotations

import torch

from ..nn.layer.base import Layer

__all__ = ["Conll05st", "Imdb", "Imikolov", "Movielens", "UCIHousing", "WMT14", "WMT16",
           "ViterbiDecoder", "viterbi_decode"]


def viterbi_decode(potentials, transition_params, lengths, include_bos_eos_tag=True, name=None):
    """potentials [B, T, N] emission scores, transition_params [N, N], lengths [B]. Returns
    (scores [B], paths [B, T_max]) — batched max-product dynamic programming on the device.
    With ``include_bos_eos_tag`` the last two tags are BOS / EOS (reference convention)."""
    B, T, N = potentials.shape
    if potentials.is_cuda:
        return _viterbi_device(potentials, transition_params, lengths, include_bos_eos_tag)
    trans = transition_params
    lengths = lengths.long()
    alpha = potentials[:, 0].clone()
    if include_bos_eos_tag:
        alpha = alpha + trans[N - 2].unsqueeze(0)  # from BOS
    hist = []
    for t in range(1, T):
        s = alpha.unsqueeze(2) + trans.unsqueeze(0)  # [B, from, to]
        best, arg = s.max(1)
        nxt = best + potentials[:, t]
        live = (t < lengths).unsqueeze(1)
        alpha = torch.where(live, nxt, alpha)
        hist.append(torch.where(live, arg, torch.arange(N, device=arg.device).expand_as(arg)))
    if include_bos_eos_tag:
        alpha = alpha + trans[:, N - 1].unsqueeze(0)  # to EOS
    scores, last = alpha.max(1)
    Tm = int(lengths.max().item()) if B else 0
    path = [last]
    for t in range(T - 2, -1, -1):
        last = hist[t].gather(1, last.unsqueeze(1)).squeeze(1)
        path.append(last)
    path = torch.stack(path[::-1], 1)[:, :Tm]
    mask = torch.arange(Tm, device=path.device)[None, :] < lengths[:, None]
    return scores, torch.where(mask, path, torch.zeros_like(path))


def _viterbi_device(potentials, transition_params, lengths, include_bos_eos_tag):
    """One launch of `csrc/kernels/viterbi.hip` (workgroup per sequence, scores in LDS, device
    backtrace); the only host read is max(lengths) for the output width."""
    from ..ops import _lib
    pot = potentials.float().contiguous()
    tr = transition_params.to(device=pot.device, dtype=torch.float32).contiguous()
    ln = lengths.to(device=pot.device, dtype=torch.int64).contiguous()
    B, T, N = pot.shape
    scores = torch.empty(B, device=pot.device, dtype=torch.float32)
    path = torch.empty(B, T, device=pot.device, dtype=torch.int64)
    hist = torch.empty(B, max(T, 1), N, device=pot.device, dtype=torch.int32)
    _lib.call("piamd_viterbi_decode", pot.data_ptr(), tr.data_ptr(), ln.data_ptr(), B, T, N,
              int(bool(include_bos_eos_tag)), scores.data_ptr(), path.data_ptr(), hist.data_ptr(),
              _lib.stream())
    Tm = int(ln.max().item()) if B else 0
    return scores, path[:, :Tm]


class ViterbiDecoder(Layer):
    def __init__(self, transitions, include_bos_eos_tag=True, name=None):
        super().__init__()
        self.transitions, self.include_bos_eos_tag = transitions, include_bos_eos_tag

    def forward(self, potentials, lengths):
        return viterbi_decode(potentials, self.transitions, lengths, self.include_bos_eos_tag)


class _OfflineDataset:
    """Base for the reference's downloadable text datasets: loads ``data_file`` if given."""
    NAME = ""

    def __init__(self, data_file=None, mode="train", download=False, **kw):
        if data_file is None:
            raise RuntimeError(f"{self.NAME}: no network access in this environment; pass data_file=")
        self.data_file, self.mode = data_file, mode
        self._load()

    def _load(self):
        with open(self.data_file) as f:
            self.data = [line.rstrip("\n") for line in f]

    def __getitem__(self, i):
        return self.data[i]

    def __len__(self):
        return len(self.data)


class UCIHousing(_OfflineDataset):
    NAME = "UCIHousing"
    FEATURE_NUM = 14

    def _load(self):
        import numpy as np
        d = np.loadtxt(self.data_file, dtype=np.float32).reshape(-1, self.FEATURE_NUM)
        mx, mn, avg = d.max(0), d.min(0), d.mean(0)
        d[:, :-1] = (d[:, :-1] - avg[:-1]) / np.maximum(mx[:-1] - mn[:-1], 1e-12)
        n = int(len(d) * 0.8)
        self.data = d[:n] if self.mode == "train" else d[n:]

    def __getitem__(self, i):
        return self.data[i][:-1], self.data[i][-1:]


from . import datasets  # noqa: E402
from .datasets import Conll05st, Imdb, Imikolov, Movielens, WMT14, WMT16  # noqa: E402,F401
