"""Activation recomputation (reference `python/paddle/distributed/fleet/recompute/recompute.py`).

Forward runs ``function`` without saving activations; backward re-runs it with autograd and
back-propagates. The framework's kernel-dropout generator state (seed/offset counters) and the
torch RNG state are captured before the first run and restored for the re-run, so dropout masks
are identical (``preserve_rng_state``).
"""
from __future__ import annotations

import torch

from ...framework import random as _random


def _detach(x):
    if isinstance(x, torch.Tensor):
        d = x.detach()
        d.requires_grad_(x.requires_grad)
        return d
    return x


class _RecomputeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, function, preserve, *args):
        ctx.function = function
        ctx.preserve = preserve
        ctx.rng = _random.get_rng_state()
        ctx.torch_rng = torch.get_rng_state()
        ctx.cuda_rng = torch.cuda.get_rng_state() if torch.cuda.is_available() and any(
            isinstance(a, torch.Tensor) and a.is_cuda for a in args) else None
        tensor_idx = [i for i, a in enumerate(args) if isinstance(a, torch.Tensor)]
        ctx.tensor_idx = tensor_idx
        ctx.others = [None if i in tensor_idx else a for i, a in enumerate(args)]
        ctx.save_for_backward(*[args[i] for i in tensor_idx])
        with torch.no_grad():
            out = function(*args)
        return out

    @staticmethod
    def backward(ctx, *grads):
        saved = ctx.saved_tensors
        args = list(ctx.others)
        for i, t in zip(ctx.tensor_idx, saved):
            args[i] = _detach(t)
        cur = _random.get_rng_state()
        cur_t = torch.get_rng_state()
        cur_c = torch.cuda.get_rng_state() if ctx.cuda_rng is not None else None
        if ctx.preserve:
            _random.set_rng_state(ctx.rng)
            torch.set_rng_state(ctx.torch_rng)
            if ctx.cuda_rng is not None:
                torch.cuda.set_rng_state(ctx.cuda_rng)
        with torch.enable_grad():
            out = ctx.function(*args)
        if ctx.preserve:
            _random.set_rng_state(cur)
            torch.set_rng_state(cur_t)
            if cur_c is not None:
                torch.cuda.set_rng_state(cur_c)
        outs = out if isinstance(out, tuple) else (out,)
        pairs = [(o, g) for o, g in zip(outs, grads) if isinstance(o, torch.Tensor) and o.requires_grad and g is not None]
        if pairs:
            torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
        arg_grads = [a.grad if isinstance(a, torch.Tensor) and a.requires_grad else None for a in args]
        return (None, None, *arg_grads)


def recompute(function, *args, preserve_rng_state=True, use_reentrant=True, **kwargs):
    if kwargs:
        fn = function
        function = lambda *a: fn(*a, **kwargs)  # noqa: E731
    return _RecomputeFn.apply(function, preserve_rng_state, *args)


def recompute_sequential(ctx, functions, *args, **kwargs):
    segments = ctx.get("segments", 1) if isinstance(ctx, dict) else 1
    fs = list(functions.children()) if isinstance(functions, torch.nn.Module) else list(functions)
    per = max(1, len(fs) // segments)
    x = args[0] if len(args) == 1 else args
    for i in range(0, len(fs), per):
        chunk = fs[i:i + per]

        def run(inp, _c=chunk):
            for f in _c:
                inp = f(inp)
            return inp
        x = recompute(run, x, **kwargs)
    return x
