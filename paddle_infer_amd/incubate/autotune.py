"""``paddle.incubate.autotune`` — kernel autotuning (reference
`python/paddle/incubate/autotune.py:set_config`, backed by `phi/kernels/autotune/`).

MI355X design: GEMM autotuning is PyTorch TunableOp over the hipBLASLt + rocBLAS solution
spaces (every candidate kernel for a GEMM shape is timed once, the winner cached per
shape/layout/dtype). Tuned tables ship in-tree (``paddle_infer_amd/tuning/*.csv``) keyed by
the GPU arch + ROCm/hipBLASLt versions (TunableOp validators), so production runs replay the
winners with tuning OFF (no first-step stall). The framework's own HIP kernels pick their launch
plans (tile width, split-K) at run time through ``ops/autotune.py`` (heuristic by default, measured
per shape inside ``tuning_range`` when enabled).
"""
from __future__ import annotations

import os

_TUNING_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")
_STATE = {"loaded": None}


def default_table():
    return os.path.join(_TUNING_DIR, "tunableop_gfx950.csv")


def use_tuned_gemms(path=None, tune_missing=False):
    """Enable TunableOp with a shipped table (tuning of unseen shapes only if ``tune_missing``).
    Returns True when a table was found and loaded."""
    import torch
    if not torch.cuda.is_available():
        return False
    import torch.cuda.tunable as tun
    path = path or default_table()
    tun.enable(True)
    tun.tuning_enable(bool(tune_missing))
    if os.path.exists(path):
        tun.set_filename(path, insert_device_ordinal=False)
        ok = tun.read_file(path)
        _STATE["loaded"] = path if ok else None
        return bool(ok)
    return False


def set_config(config=None):
    """Reference-compatible: ``{"kernel": {"enable": bool, "tuning_range": [a, b]},
    "layout": {...}, "dataloader": {...}}``. ``kernel.enable`` turns GEMM autotuning on
    (tuning new shapes, results written to ``kernel.table`` or the in-tree default) AND the
    runtime plan tuning of the framework's own HIP kernels (``ops/autotune.py``: conv tile /
    split-K plans, measured on the live operands during ``tuning_range`` steps, cached per shape,
    persisted to ``kernel.cache_file`` when given)."""
    import torch
    from ..ops import autotune as _own
    cfg = config or {"kernel": {"enable": True}}
    k = cfg.get("kernel", {})
    _own.configure(enable=k.get("enable", False), tuning_range=k.get("tuning_range"),
                   cache_file=k.get("cache_file"))
    if not torch.cuda.is_available():
        return
    import torch.cuda.tunable as tun
    if k.get("enable", False):
        tun.enable(True)
        tun.tuning_enable(True)
        table = k.get("table", default_table())
        os.makedirs(os.path.dirname(table), exist_ok=True)
        tun.set_filename(table, insert_device_ordinal=False)
        if os.path.exists(table):
            tun.read_file(table)
        if "max_tuning_duration_ms" in k:
            tun.set_max_tuning_duration(int(k["max_tuning_duration_ms"]))
    else:
        tun.enable(False)
