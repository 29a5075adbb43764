"""Random seeds for the stateless-hash dropout kernels and the model-parallel RNG tracker.

Parity: ``paddle.seed`` (reference `python/paddle/framework/random.py`) and
``fleet.meta_parallel.get_rng_state_tracker`` (`fleet/meta_parallel/parallel_layers/random.py`):
regions whose activations are replicated across the tensor-parallel group must draw the same mask
on every mp rank ("global_seed"), sharded regions a different one per rank ("local_seed").

Kernel dropout is counter based: a launch gets ``(seed, offset)``, folded into a per-launch key
``k = H(seed, offset)``, and the pair of elements ``(2j, 2j+1)`` takes the two 16-bit halves of
``lowbias32(lowbias32(j + k) ^ H'(k))`` (`csrc/kernels/common.h` ``hash_uniform8``; the second
keyed round keeps masks of different launches from being index-shifted copies of each other). The
offset advances by the element count, so no RNG state lives on the GPU and backward / recompute
regenerate the identical mask.
"""
from __future__ import annotations

import contextlib
import threading

import torch

_state = threading.local()


class _Gen:
    def __init__(self, seed: int):
        self.seed = int(seed) & 0xFFFFFFFFFFFF
        self.offset = 0

    def next(self, n: int):
        o = self.offset
        self.offset += (int(n) + 3) & ~3
        return self.seed, o


_GLOBAL = {"default": _Gen(2024)}
_ACTIVE = ["default"]


def seed(s: int):
    """``paddle.seed``: reseeds torch and the kernel dropout generator."""
    torch.manual_seed(s)
    _GLOBAL["default"] = _Gen(s)
    return s


def next_seed_offset(n: int):
    return _GLOBAL[_ACTIVE[-1]].next(n)


def get_rng_state():
    return {k: (g.seed, g.offset) for k, g in _GLOBAL.items()}


def set_rng_state(state):
    for k, (s, o) in state.items():
        g = _Gen(s)
        g.offset = o
        _GLOBAL[k] = g


def get_cuda_rng_state():
    """Per-GPU generator states: torch's (for torch-side sampling) plus the kernel dropout
    generator's (seed, offset) — restoring both replays dropout masks exactly."""
    states = torch.cuda.get_rng_state_all() if torch.cuda.is_available() else []
    return {"torch": states, "kernel": get_rng_state()}


def set_cuda_rng_state(state):
    if isinstance(state, dict):
        if state.get("torch") and torch.cuda.is_available():
            torch.cuda.set_rng_state_all(state["torch"])
        set_rng_state(state.get("kernel", {}))
    elif state and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(state)


class RNGStatesTracker:
    """Named generators; ``rng_state(name)`` makes kernel dropout inside the block draw from it."""

    def add(self, name: str, s: int):
        if name in _GLOBAL and name != "default":
            raise ValueError(f"rng state {name} already exists")
        _GLOBAL[name] = _Gen(s)

    def reset(self):
        for k in list(_GLOBAL):
            if k != "default":
                del _GLOBAL[k]

    @contextlib.contextmanager
    def rng_state(self, name: str = "global_seed"):
        if name not in _GLOBAL:
            raise ValueError(f"rng state {name} not added")
        _ACTIVE.append(name)
        try:
            yield
        finally:
            _ACTIVE.pop()


_TRACKER = RNGStatesTracker()


def get_rng_state_tracker() -> RNGStatesTracker:
    return _TRACKER


def model_parallel_random_seed(seed_: int = 2048, mp_rank: int = 0, pp_rank: int = 0):
    """Reference: `parallel_layers/random.py:model_parallel_random_seed`."""
    local = seed_ + 1024 + mp_rank * 100 + pp_rank * 10
    _TRACKER.reset()
    _TRACKER.add("global_seed", seed_)
    _TRACKER.add("local_seed", local)
    seed(seed_)
