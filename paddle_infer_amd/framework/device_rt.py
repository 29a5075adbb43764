"""ctypes binding of the native device runtime ``_lib/libpiamd_device.so`` (``csrc/device``):
device properties, a stream pool with priorities, events, and the host/device range tracer.

Loaded lazily and AFTER ``import torch`` so the HIP runtime is the one torch already mapped: a
stream created here is a plain ``hipStream_t`` that ``torch.cuda.ExternalStream`` adopts, so
PyTorch ops, the framework's HIP kernels (they launch on torch's current stream) and RCCL
collectives all run on it. Reference: `paddle/phi/backends/gpu/gpu_info.cc`,
`gpu_context.cc` (streams with priorities), `platform/device_event*`,
`fluid/platform/profiler/host_tracer.cc`.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (HIP runtime first)

from .. import _build

_LIB = None
_LOCK = threading.Lock()
c_int, c_void_p, c_ll, c_float = ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_float


class DevProps(ctypes.Structure):
    """Mirror of ``struct DevProps`` (csrc/device/device.cc)."""
    _fields_ = [("name", ctypes.c_char * 256), ("arch", ctypes.c_char * 64), ("major", c_int),
                ("minor", c_int), ("cus", c_int), ("clock_khz", c_int), ("mem_clock_khz", c_int),
                ("bus_width", c_int), ("total_mem", c_ll), ("l2_bytes", c_ll),
                ("lds_per_block", c_ll), ("warp", c_int), ("max_threads_per_block", c_int),
                ("regs_per_block", c_int), ("pci_bus", c_int), ("pci_dev", c_int),
                ("pci_domain", c_int), ("cooperative", c_int), ("concurrent_kernels", c_int)]


_SIGS = {
    "piamd_dev_count": [ctypes.POINTER(c_int)],
    "piamd_dev_props": [c_int, ctypes.POINTER(DevProps)],
    "piamd_dev_synchronize": [c_int],
    "piamd_dev_mem_info": [c_int, ctypes.POINTER(c_ll), ctypes.POINTER(c_ll)],
    "piamd_stream_priority_range": [ctypes.POINTER(c_int), ctypes.POINTER(c_int)],
    "piamd_stream_create": [c_int, c_int, c_int, ctypes.POINTER(c_void_p)],
    "piamd_stream_destroy": [c_void_p],
    "piamd_stream_sync": [c_void_p],
    "piamd_stream_query": [c_void_p],
    "piamd_stream_wait_event": [c_void_p, c_void_p],
    "piamd_stream_get_priority": [c_void_p, ctypes.POINTER(c_int)],
    "piamd_event_create": [c_int, c_int, ctypes.POINTER(c_void_p)],
    "piamd_event_destroy": [c_void_p],
    "piamd_event_record": [c_void_p, c_void_p],
    "piamd_event_sync": [c_void_p],
    "piamd_event_query": [c_void_p],
    "piamd_event_elapsed": [c_void_p, c_void_p, ctypes.POINTER(c_float)],
    "piamd_trace_enable": [c_int, c_int, c_void_p],
    "piamd_trace_push": [ctypes.c_char_p, c_void_p],
    "piamd_trace_pop": [c_void_p],
    "piamd_trace_count": [],
    "piamd_trace_dump": [ctypes.c_char_p, c_int],
}
_RESTYPES = {"piamd_trace_count": c_ll, "piamd_trace_dump": c_ll}


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            if not os.path.exists(_build.DEVICE_LIB):
                raise RuntimeError(f"device runtime not built ({_build.DEVICE_LIB}); run "
                                   "`python -m paddle_infer_amd._build`")
            L = ctypes.CDLL(_build.DEVICE_LIB, mode=ctypes.RTLD_GLOBAL)
            for n, a in _SIGS.items():
                f = getattr(L, n)
                f.argtypes = a
                f.restype = _RESTYPES.get(n, c_int)
            _LIB = L
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except (RuntimeError, OSError):
        return False


def check(err: int, what: str) -> None:
    if err != 0:
        raise RuntimeError(f"{what} failed with hipError {err}")


def props(dev: int) -> DevProps:
    p = DevProps()
    check(lib().piamd_dev_props(int(dev), ctypes.byref(p)), "hipGetDeviceProperties")
    return p


def priority_range():
    lo, hi = c_int(), c_int()
    check(lib().piamd_stream_priority_range(ctypes.byref(lo), ctypes.byref(hi)),
          "hipDeviceGetStreamPriorityRange")
    return lo.value, hi.value  # (least, greatest) — greatest is the numerically smallest
