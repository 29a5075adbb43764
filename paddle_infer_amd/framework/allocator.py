"""Device allocator selection (reference ``FLAGS_allocator_strategy``, `paddle/fluid/memory/
allocation/allocator_facade.cc`): ``"auto_growth"`` installs the framework's own auto-growth
best-fit allocator (``csrc/alloc/allocator.cc`` → ``_lib/libpiamd_alloc.so``) as PyTorch-ROCm's
HIP allocator; anything else keeps PyTorch's caching allocator.

Must run before the first device allocation of the process (the package does it at import when
``FLAGS_allocator_strategy=auto_growth`` is in the environment).

Stream safety (reference `stream_safe_cuda_allocator.cc:40`, ``RecordStream``): a freed block is
reused only by allocations on the stream it was allocated on; ``Tensor.record_stream(s)`` — and
the record-stream calls RCCL's process group makes for its collectives — reach the allocator
(``piamd_record_stream``): the block then waits, after its free, for an event on every other
stream that used it before it is reusable.

hipGraph capture: PyTorch's private graph pools map onto the allocator's tagged pools
(``piamd_begin_pool`` / ``piamd_end_pool`` / ``piamd_release_pool``): a captured graph's memory is
never handed to work outside the graph while the graph lives.

With the allocator active, ``torch.cuda.memory_allocated`` / ``max_memory_allocated`` /
``memory_reserved`` / ``max_memory_reserved`` / ``reset_peak_memory_stats`` / ``empty_cache``
report and act on this allocator (PyTorch's pluggable interface has no statistics of its own).
"""
from __future__ import annotations

import ctypes
import os

_STATE = {"active": False, "lib": None, "allocator": None}
STAT_NAMES = ("allocated", "reserved", "peak_allocated", "peak_reserved", "num_alloc", "num_free",
              "num_chunk_alloc", "num_chunk_free")


def lib_path():
    from .. import _build
    return _build.ALLOC_LIB


def _lib():
    if _STATE["lib"] is None:
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(f"allocator library not built ({path}); run paddle_infer_amd._build")
        lib = ctypes.CDLL(path)
        lib.piamd_alloc_stats.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_longlong)]
        lib.piamd_alloc_release.argtypes = [ctypes.c_int]
        lib.piamd_alloc_reset_peak.argtypes = [ctypes.c_int]
        _STATE["lib"] = lib
    return _STATE["lib"]


def active() -> bool:
    return _STATE["active"]


def enable(strategy: str = "auto_growth") -> bool:
    """Install the allocator for ``strategy``; returns whether the framework allocator is active."""
    if strategy != "auto_growth":
        return False
    if _STATE["active"]:
        return True
    from torch.cuda.memory import CUDAPluggableAllocator, change_current_allocator
    lib = _lib()
    alloc = CUDAPluggableAllocator(lib_path(), "piamd_alloc", "piamd_free")

    def fn(name):
        return ctypes.cast(getattr(lib, name), ctypes.c_void_p).value
    a = alloc._allocator
    a.set_record_stream_fn(fn("piamd_record_stream"))
    a.set_begin_allocate_to_pool(fn("piamd_begin_pool"))
    a.set_end_allocate_to_pool_fn(fn("piamd_end_pool"))
    a.set_release_pool(fn("piamd_release_pool"))
    change_current_allocator(alloc)
    _patch_torch_memory_api()
    _STATE["active"] = True
    _STATE["allocator"] = alloc
    return True


def record_stream(t, stream) -> None:
    """``t`` is used on ``stream``: its block is not reused before that stream's work on it."""
    t.record_stream(stream)


def _patch_torch_memory_api():
    import torch

    def dev(d):
        if d is None:
            return torch.cuda.current_device()
        return d.index if isinstance(d, torch.device) and d.index is not None else int(
            d if not isinstance(d, torch.device) else torch.cuda.current_device())
    cm = torch.cuda.memory
    repl = {
        "memory_allocated": lambda device=None: stats(dev(device))["allocated"],
        "max_memory_allocated": lambda device=None: stats(dev(device))["peak_allocated"],
        "memory_reserved": lambda device=None: stats(dev(device))["reserved"],
        "max_memory_reserved": lambda device=None: stats(dev(device))["peak_reserved"],
        "reset_peak_memory_stats": lambda device=None: reset_peak(dev(device)),
        "reset_max_memory_allocated": lambda device=None: reset_peak(dev(device)),
        "empty_cache": lambda: empty_cache(torch.cuda.current_device()),
    }
    for k, f in repl.items():
        _ORIG.setdefault(k, getattr(torch.cuda, k))
        setattr(torch.cuda, k, f)
        if hasattr(cm, k):
            setattr(cm, k, f)


_ORIG: dict = {}


def stats(device: int = 0) -> dict:
    buf = (ctypes.c_longlong * 8)()
    _lib().piamd_alloc_stats(int(device), buf)
    return dict(zip(STAT_NAMES, list(buf)))


def empty_cache(device: int = 0) -> None:
    _lib().piamd_alloc_release(int(device))


def reset_peak(device: int = 0) -> None:
    _lib().piamd_alloc_reset_peak(int(device))


def default_strategy() -> str:
    """``FLAGS_allocator_strategy`` when set; otherwise ``auto_growth`` (the framework allocator),
    for single- and multi-process jobs alike. RCCL's collectives allocate their own staging
    buffers; the user tensors they read and write come from this allocator, and the process
    group's ``record_stream`` calls on them reach ``piamd_record_stream`` (covered by
    `tests/test_allocator_gpu.py` and the 2-rank collective tests)."""
    v = os.environ.get("FLAGS_allocator_strategy")
    if v:
        return v
    return "auto_growth"


def maybe_enable_from_env() -> None:
    """Called at package import: install the framework allocator when it is the strategy and a GPU
    is present (before the first device allocation)."""
    if default_strategy() != "auto_growth":
        return
    import torch
    if not torch.cuda.is_available():
        return
    try:
        enable("auto_growth")
    except Exception as e:  # allocator already initialised / library missing: say so once
        import warnings
        warnings.warn(f"FLAGS_allocator_strategy=auto_growth not applied: {e}", RuntimeWarning)
