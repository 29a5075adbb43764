"""Device allocator selection (reference ``FLAGS_allocator_strategy``, `paddle/fluid/memory/
allocation/allocator_facade.cc`): ``"auto_growth"`` installs the framework's own auto-growth
best-fit allocator (``csrc/alloc/allocator.cc`` → ``_lib/libpiamd_alloc.so``) as PyTorch-ROCm's
HIP allocator; anything else keeps PyTorch's caching allocator.

Must run before the first device allocation of the process (the package does it at import when
``FLAGS_allocator_strategy=auto_growth`` is in the environment).

Stream safety (reference `stream_safe_cuda_allocator.cc:40`, ``RecordStream``): a freed block is
reused only by allocations on the stream it was allocated on (stream-ordered reuse). A tensor used
on ANOTHER stream is covered two ways, because PyTorch's pluggable-allocator interface forwards no
record-stream calls to the allocator:

* ``Tensor.record_stream(s)`` is routed to :func:`record_stream`: an event is recorded on ``s`` and
  the tensor is kept alive until that event has completed, so its block returns to the free list
  only after the other stream's work on it — the reference's deferred free;
* RCCL collectives (whose C++ record-stream calls never reach this allocator) run with
  ``TORCH_NCCL_AVOID_RECORD_STREAMS=1``: the process group stashes every collective's tensors until
  the work has been waited on by the compute stream, which orders the free after the collective.
"""
from __future__ import annotations

import ctypes
import os

_STATE = {"active": False, "lib": None}
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
    _lib()
    import torch
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl":
        raise RuntimeError("FLAGS_allocator_strategy=auto_growth must be set before the RCCL "
                           "process group is created (its collectives must stash tensors instead "
                           "of record_stream)")
    os.environ["TORCH_NCCL_AVOID_RECORD_STREAMS"] = "1"
    change_current_allocator(CUDAPluggableAllocator(lib_path(), "piamd_alloc", "piamd_free"))
    if "record_stream" not in _ORIG:
        _ORIG["record_stream"] = torch.Tensor.record_stream
        torch.Tensor.record_stream = lambda t, s: record_stream(t, s)
    _STATE["active"] = True
    return True


_ORIG: dict = {}
_PENDING: list = []  # (event, tensor): blocks in use on another stream


def record_stream(t, stream) -> None:
    """Defer ``t``'s free until the work queued on ``stream`` so far has completed."""
    import torch
    if not _STATE["active"] or not t.is_cuda:
        return _ORIG.get("record_stream", torch.Tensor.record_stream)(t, stream)
    ev = torch.cuda.Event()
    ev.record(stream)
    _PENDING.append((ev, t))
    purge()


def purge() -> int:
    """Release tensors whose other-stream work has completed; returns how many stay pending."""
    keep = [(e, t) for e, t in _PENDING if not e.query()]
    _PENDING[:] = keep
    return len(keep)


def stats(device: int = 0) -> dict:
    buf = (ctypes.c_longlong * 8)()
    _lib().piamd_alloc_stats(int(device), buf)
    return dict(zip(STAT_NAMES, list(buf)))


def empty_cache(device: int = 0) -> None:
    _lib().piamd_alloc_release(int(device))


def reset_peak(device: int = 0) -> None:
    _lib().piamd_alloc_reset_peak(int(device))


def maybe_enable_from_env() -> None:
    if os.environ.get("FLAGS_allocator_strategy", "") == "auto_growth":
        try:
            enable("auto_growth")
        except Exception as e:  # allocator already initialised / library missing: say so once
            import warnings
            warnings.warn(f"FLAGS_allocator_strategy=auto_growth not applied: {e}", RuntimeWarning)
