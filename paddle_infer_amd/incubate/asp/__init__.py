"""``paddle.incubate.asp`` — automatic 2:4 structured sparsity (reference `incubate/asp/`).

``prune_model`` computes n:m masks (default 2:4, magnitude-based along the reduction dimension,
``mask_1d`` / ``mask_2d_greedy`` / ``mask_2d_best`` algorithms) for every supported layer weight
and applies them; ``decorate(optimizer)`` re-applies the masks after each optimizer step so the
sparsity pattern survives training. 2:4 patterns are the layout CDNA's sparse MFMA (smfmac)
instructions consume. Excluded layers are managed by name."""
from __future__ import annotations

import itertools

import torch

__all__ = ["calculate_density", "decorate", "prune_model", "set_excluded_layers",
           "reset_excluded_layers", "add_supported_layer"]

_EXCLUDED: set = set()
_MASKS: dict = {}
_SUPPORTED = {"Linear", "Conv2D", "Conv1D", "Conv3D", "ColumnParallelLinear", "RowParallelLinear",
              "FC"}


def calculate_density(x):
    x = x if isinstance(x, torch.Tensor) else torch.as_tensor(x)
    return float((x != 0).sum()) / max(1, x.numel())


def set_excluded_layers(param_names=None, main_program=None):
    _EXCLUDED.update(param_names or [])


def reset_excluded_layers(main_program=None):
    _EXCLUDED.clear()


def add_supported_layer(layer, pruning_func=None):
    _SUPPORTED.add(layer if isinstance(layer, str) else layer.__name__)


def _mask_1d(w2, n, m):
    """Keep the n largest |w| of every m consecutive elements of each row."""
    R, C = w2.shape
    pad = (-C) % m
    a = torch.nn.functional.pad(w2.abs(), (0, pad)).reshape(R, -1, m)
    idx = a.topk(n, -1).indices
    mask = torch.zeros_like(a, dtype=torch.bool).scatter_(-1, idx, True)
    return mask.reshape(R, -1)[:, :C]


def _mask_2d(w2, n, m, best):
    """m×m blocks with n non-zeros in every row AND column (greedy or exhaustive best)."""
    R, C = w2.shape
    pr, pc = (-R) % m, (-C) % m
    a = torch.nn.functional.pad(w2.abs(), (0, pc, 0, pr))
    Rb, Cb = a.shape[0] // m, a.shape[1] // m
    blocks = a.reshape(Rb, m, Cb, m).permute(0, 2, 1, 3).reshape(-1, m, m)
    out = torch.zeros_like(blocks, dtype=torch.bool)
    if best:
        rows = [r for r in itertools.product([0, 1], repeat=m) if sum(r) == n]
        pats = [torch.tensor(p, dtype=torch.bool) for p in itertools.product(rows, repeat=m)
                if all(sum(col) == n for col in zip(*p))]
        P = torch.stack(pats).to(a.device)  # [np, m, m]
        score = (blocks[:, None] * P[None]).sum((-1, -2))
        out = P[score.argmax(1)]
    else:
        for bi in range(blocks.shape[0]):
            b = blocks[bi]
            order = torch.argsort(b.reshape(-1), descending=True)
            rc, cc = [0] * m, [0] * m
            for f in order.tolist():
                r, c = divmod(f, m)
                if rc[r] < n and cc[c] < n:
                    out[bi, r, c] = True
                    rc[r] += 1
                    cc[c] += 1
    mask = out.reshape(Rb, Cb, m, m).permute(0, 2, 1, 3).reshape(Rb * m, Cb * m)
    return mask[:R, :C]


def _compute_mask(w, n, m, algo):
    # reduction dimension last: Linear [in, out] → transpose to [out, in]; conv [O, I, kh, kw]
    w2 = w.detach().t() if w.dim() == 2 else w.detach().reshape(w.shape[0], -1)
    if algo == "mask_1d":
        mk = _mask_1d(w2, n, m)
    else:
        mk = _mask_2d(w2, n, m, algo == "mask_2d_best")
    return mk.t() if w.dim() == 2 else mk.reshape(w.shape)


def prune_model(model, n=2, m=4, mask_algo="mask_1d", with_mask=True):
    masks = {}
    for lname, layer in model.named_modules():
        if type(layer).__name__ not in _SUPPORTED:
            continue
        for pname, p in layer.named_parameters(recurse=False):
            full = f"{lname}.{pname}" if lname else pname
            if pname != "weight" or full in _EXCLUDED:
                continue
            mk = _compute_mask(p, n, m, mask_algo)
            with torch.no_grad():
                p.mul_(mk.to(p.dtype))
            if with_mask:
                _MASKS[id(p)] = (p, mk)
            masks[full] = mk
    return masks


class _ASPOptimizer:
    def __init__(self, optimizer):
        self._opt = optimizer

    def __getattr__(self, k):
        return getattr(self._opt, k)

    @torch.no_grad()
    def step(self):
        self._opt.step()
        for p, mk in _MASKS.values():
            p.mul_(mk.to(p.dtype))

    def minimize(self, loss, *a, **kw):
        loss.backward()
        self.step()


def decorate(optimizer):
    return _ASPOptimizer(optimizer)
