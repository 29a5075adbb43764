"""Runtime autotuning of the framework's own HIP kernel plans (tile width, split-K factor).

Parity: reference `paddle/phi/kernels/autotune/` (``AutoTuneCache`` keyed by op + shape, an
``AutoTuneStatus`` step counter, tuning only inside ``tuning_range``) behind
``paddle.incubate.autotune.set_config({"kernel": {"enable": True, "tuning_range": [a, b]}})``.

A kernel call site asks :func:`choose` for a plan with its cache key, the candidate plans, the
heuristic default and a ``run(plan)`` closure. Outside tuning (disabled, or the step counter out of
range) the cached winner — else the heuristic — is returned at once; inside, each candidate is timed
on the live operands (one warm-up + ``REPS`` timed launches between HIP events, interleaved) and the
fastest is cached (and appended to ``cache_file`` as JSON, so a later process replays it without
tuning). The step counter advances on every optimizer step (``Optimizer.step``).
"""
from __future__ import annotations

import json
import os
import threading

import torch

REPS = 3
_LOCK = threading.Lock()
_STATE = {"enable": False, "range": (0, 1 << 62), "step": 0, "cache_file": None}
CACHE: dict = {}
STATS = {"tuned": 0, "hits": 0}


def configure(enable=True, tuning_range=None, cache_file=None):
    _STATE["enable"] = bool(enable)
    if tuning_range is not None:
        a, b = tuning_range
        _STATE["range"] = (int(a), int(b))
    if cache_file is not None:
        _STATE["cache_file"] = cache_file
        load(cache_file)


def load(path):
    if path and os.path.exists(path):
        with open(path) as f:
            for k, v in json.load(f).items():
                CACHE[k] = tuple(v) if isinstance(v, list) else v


def save(path=None):
    path = path or _STATE["cache_file"]
    if not path:
        return
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump({k: list(v) if isinstance(v, tuple) else v for k, v in CACHE.items()}, f)
    os.replace(tmp, path)


def step():
    """Advance the tuning step counter (called once per training step)."""
    _STATE["step"] += 1


def tuning_active() -> bool:
    a, b = _STATE["range"]
    return _STATE["enable"] and a <= _STATE["step"] < b


def key_of(op, *shape) -> str:
    return op + ":" + ",".join(str(s) for s in shape)


def _time(run, plan):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        run(plan)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / REPS


def choose(key, candidates, default, run):
    """Plan for ``key``: cached winner, else (tuning active) the measured best of ``candidates``,
    else ``default``. ``run(plan)`` must launch the kernel with that plan (outputs are rewritten by
    the caller's final launch)."""
    hit = CACHE.get(key)
    if hit is not None:
        STATS["hits"] += 1
        return hit
    if not tuning_active() or not torch.cuda.is_available():
        return default
    cands = [c for c in dict.fromkeys(candidates)]
    if default not in cands:
        cands.insert(0, default)
    with _LOCK:
        for c in cands:  # warm-up (first-launch costs out of the timing)
            run(c)
        t = {c: [] for c in cands}
        for _ in range(2):  # interleaved rounds
            for c in cands:
                t[c].append(_time(run, c))
        best = min(cands, key=lambda c: min(t[c]))
        CACHE[key] = best
        STATS["tuned"] += 1
    if _STATE["cache_file"]:
        save()
    return best
