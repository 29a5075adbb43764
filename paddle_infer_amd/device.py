"""Device / place management (reference `python/paddle/device/__init__.py`, `device/cuda/`).

On this framework a "gpu" place is a HIP device (MI355X); ``paddle.set_device('gpu:0')`` selects
the default device for tensor creation. Streams/events are HIP streams/events via torch.cuda.
"""
from __future__ import annotations

import ctypes

import torch

_current = {"device": None}


class Place:
    def __init__(self, kind: str, idx: int = 0):
        self.kind, self.idx = kind, idx

    def torch_device(self):
        return torch.device("cpu") if self.kind == "cpu" else torch.device("cuda", self.idx)

    def is_gpu_place(self):
        return self.kind == "gpu"

    def is_cpu_place(self):
        return self.kind == "cpu"

    def gpu_device_id(self):
        return self.idx

    def __repr__(self):
        return "Place(cpu)" if self.kind == "cpu" else f"Place(gpu:{self.idx})"

    def __eq__(self, other):
        return isinstance(other, Place) and (self.kind, self.idx) == (other.kind, other.idx)


def CPUPlace():
    return Place("cpu")


def CUDAPlace(idx=0):
    return Place("gpu", idx)


CUDAPinnedPlace = CPUPlace
XPUPlace = CUDAPlace


def _no_device(kind):
    def place(idx=0):
        raise RuntimeError(f"{kind} is not available: this framework targets MI355X (HIP) and CPU")
    place.__name__ = kind
    return place


NPUPlace = _no_device("NPUPlace")
IPUPlace = _no_device("IPUPlace")
MLUPlace = _no_device("MLUPlace")


def is_compiled_with_cuda():
    return torch.cuda.is_available()


def is_compiled_with_rocm():
    return torch.version.hip is not None


def is_compiled_with_xpu():
    return False


def is_compiled_with_npu():
    return False


def is_compiled_with_cinn():
    return False


def is_compiled_with_ipu():
    return False


def is_compiled_with_mlu():
    return False


def get_cudnn_version():
    """MIOpen stands in for cuDNN on ROCm; report its version as an int (major*1000+minor*100+patch)."""
    v = getattr(torch.backends.cudnn, "version", lambda: None)()
    return v


def get_all_custom_device_type():
    return []


def get_available_custom_device():
    return []


def _parse(dev) -> torch.device:
    if dev is None:
        return None
    if isinstance(dev, torch.device):
        return dev
    if isinstance(dev, Place):
        return dev.torch_device()
    if isinstance(dev, int):  # a device ordinal (paddle.device.cuda.* accept ints)
        return torch.device("cuda", dev)
    s = str(dev).lower()
    if s == "cpu":
        return torch.device("cpu")
    if s.startswith("gpu") or s.startswith("cuda") or s.startswith("hip"):
        idx = int(s.split(":")[1]) if ":" in s else 0
        return torch.device("cuda", idx)
    raise ValueError(f"unknown device {dev}")


def set_device(device):
    d = _parse(device)
    if d.type == "cuda":
        torch.cuda.set_device(d)
    _current["device"] = d
    return Place("cpu") if d.type == "cpu" else Place("gpu", d.index or 0)


def get_device():
    d = _resolve(None)
    return "cpu" if d.type == "cpu" else f"gpu:{d.index or 0}"


def _resolve(place=None) -> torch.device:
    if place is not None:
        return _parse(place)
    if _current["device"] is None:
        _current["device"] = torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() else torch.device("cpu")
    return _current["device"]


def get_all_device_type():
    return ["cpu", "gpu"] if torch.cuda.is_available() else ["cpu"]


def get_available_device():
    return [f"gpu:{i}" for i in range(torch.cuda.device_count())] if torch.cuda.is_available() else []


class _NativeStream:
    """``paddle.device.cuda.Stream`` on a natively created HIP stream (``csrc/device``: priority
    from the device's range, non-blocking w.r.t. the legacy default stream). ``torch_stream`` is the
    same ``hipStream_t`` adopted by ``torch.cuda.ExternalStream``: entered through
    :func:`cuda.stream_guard` every PyTorch op, framework HIP kernel and collective in the block
    runs on it. Reference: `paddle/fluid/pybind/cuda_streams_py.cc` (priority 1 = high, 2 =
    normal), `phi/backends/gpu/gpu_context.cc`."""

    def __init__(self, device=None, priority=2, *, _torch=None):
        from .framework import device_rt as rt
        if _torch is not None:  # non-owning wrapper of an existing torch stream
            self._t, self._own = _torch, False
            self.device = _torch.device
            self._h = _torch.cuda_stream
            return
        dev = _parse(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        self.priority = int(priority)
        if not rt.available():  # native runtime not built: a torch pool stream of that priority
            self._t = torch.cuda.Stream(device=torch.device("cuda", idx),
                                        priority=-1 if self.priority == 1 else 0)
            self._h, self._own, self.device = self._t.cuda_stream, False, torch.device("cuda", idx)
            return
        self._h, self._own, self.device = _pool_stream(idx, int(priority)), False, torch.device("cuda", idx)
        self._t = torch.cuda.ExternalStream(self._h, device=self.device)

    @property
    def cuda_stream(self) -> int:
        return self._h

    @property
    def torch_stream(self):
        return self._t

    def synchronize(self):
        from .framework import device_rt as rt
        if not rt.available():
            return self._t.synchronize()
        rt.check(rt.lib().piamd_stream_sync(self._h), "hipStreamSynchronize")

    def query(self) -> bool:
        from .framework import device_rt as rt
        if not rt.available():
            return self._t.query()
        r = rt.lib().piamd_stream_query(self._h)
        if r < 0:
            raise RuntimeError(f"hipStreamQuery failed with hipError {-r}")
        return r == 1

    def wait_event(self, event):
        from .framework import device_rt as rt
        if event._tev is not None:
            return self._t.wait_event(event._tev)
        rt.check(rt.lib().piamd_stream_wait_event(self._h, event.handle), "hipStreamWaitEvent")

    def wait_stream(self, stream):
        ev = _NativeEvent()
        ev.record(stream)
        self.wait_event(ev)

    def record_event(self, event=None):
        event = event if event is not None else _NativeEvent()
        event.record(self)
        return event

    def __eq__(self, other):
        return isinstance(other, _NativeStream) and other._h == self._h

    def __hash__(self):
        return hash(self._h)



# Native streams come from a per-(device, priority) pool handed out round-robin and never destroyed
# (the reference's GPU context and PyTorch pool streams the same way): a stream id that torch's
# allocator may still hold an event record for can never dangle.
_POOL_SIZE = 16
_POOL: dict = {}


def _pool_stream(idx: int, priority: int) -> int:
    from .framework import device_rt as rt
    key = (idx, priority)
    ent = _POOL.get(key)
    if ent is None:
        least, greatest = rt.priority_range()
        hip_prio = greatest if priority == 1 else least
        hs = []
        for _ in range(_POOL_SIZE):
            h = ctypes.c_void_p()
            rt.check(rt.lib().piamd_stream_create(idx, hip_prio, 1, ctypes.byref(h)), "hipStreamCreate")
            hs.append(h.value)
        ent = _POOL[key] = [hs, 0]
    hs, i = ent
    ent[1] = (i + 1) % len(hs)
    return hs[i]


class _NativeEvent:
    """``paddle.device.cuda.Event`` on a native HIP event (timing / blocking-sync flags)."""

    def __init__(self, enable_timing=False, blocking=False, interprocess=False):
        from .framework import device_rt as rt
        self._tev = None
        if not rt.available():  # native runtime not built: torch's event
            self._tev = torch.cuda.Event(enable_timing=enable_timing, blocking=blocking,
                                         interprocess=interprocess)
            self.handle, self.enable_timing = None, bool(enable_timing)
            return
        h = ctypes.c_void_p()
        rt.check(rt.lib().piamd_event_create(int(bool(enable_timing)), int(bool(blocking)),
                                             ctypes.byref(h)), "hipEventCreate")
        self.handle, self.enable_timing = h.value, bool(enable_timing)

    def record(self, stream=None):
        from .framework import device_rt as rt
        if self._tev is not None:
            ts = stream.torch_stream if isinstance(stream, _NativeStream) else stream
            return self._tev.record(ts) if ts is not None else self._tev.record()
        h = (stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream)
        rt.check(rt.lib().piamd_event_record(self.handle, h), "hipEventRecord")

    def query(self) -> bool:
        from .framework import device_rt as rt
        if self._tev is not None:
            return self._tev.query()
        r = rt.lib().piamd_event_query(self.handle)
        if r < 0:
            raise RuntimeError(f"hipEventQuery failed with hipError {-r}")
        return r == 1

    def synchronize(self):
        from .framework import device_rt as rt
        if self._tev is not None:
            return self._tev.synchronize()
        rt.check(rt.lib().piamd_event_sync(self.handle), "hipEventSynchronize")

    def elapsed_time(self, end) -> float:
        from .framework import device_rt as rt
        if self._tev is not None:
            return self._tev.elapsed_time(end._tev)
        ms = ctypes.c_float()
        rt.check(rt.lib().piamd_event_elapsed(self.handle, end.handle, ctypes.byref(ms)),
                 "hipEventElapsedTime")
        return ms.value

    def __del__(self):
        if getattr(self, "handle", None):
            try:
                from .framework import device_rt as rt
                rt.lib().piamd_event_destroy(self.handle)
            except Exception:  # noqa: BLE001
                pass
            self.handle = None


class _Props:
    """Device properties from the native runtime (hipGetDeviceProperties), with the attribute
    names of ``paddle.device.cuda.get_device_properties`` / torch's."""

    def __init__(self, p):
        self.name = p.name.decode()
        self.gcnArchName = p.arch.decode()
        self.major, self.minor = p.major, p.minor
        self.multi_processor_count = p.cus
        self.total_memory = p.total_mem
        self.L2_cache_size = p.l2_bytes
        self.shared_memory_per_block = p.lds_per_block
        self.warp_size = p.warp
        self.max_threads_per_block = p.max_threads_per_block
        self.clock_rate_khz = p.clock_khz
        self.memory_clock_rate_khz = p.mem_clock_khz
        self.memory_bus_width = p.bus_width
        self.pci_bus_id, self.pci_device_id, self.pci_domain_id = p.pci_bus, p.pci_dev, p.pci_domain
        self.cooperative_launch = bool(p.cooperative)

    def __repr__(self):
        return (f"_gpuDeviceProperties(name='{self.name}', arch='{self.gcnArchName}', "
                f"total_memory={self.total_memory // (1 << 20)}MB, "
                f"multi_processor_count={self.multi_processor_count})")


_SIDE: dict = {}


def side_stream(device, priority=2, key="side"):
    """A framework-owned side stream (native HIP stream from ``csrc/device``, cached per
    (device, key)), returned as the ``torch.cuda.ExternalStream`` that ``torch.cuda.stream`` /
    ``wait_stream`` / events take. priority 1 = the device's highest (collective streams: their
    kernels are scheduled ahead of queued compute), 2 = normal. Falls back to a torch stream when
    the native runtime is not built."""
    dev = _parse(device) if not isinstance(device, torch.device) else device
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    k = (idx, key, int(priority))
    ent = _SIDE.get(k)
    if ent is None:
        from .framework import device_rt as rt
        if rt.available():
            ent = _SIDE[k] = _NativeStream(torch.device("cuda", idx), priority)  # pool stream
        else:
            ent = _SIDE[k] = _NativeStream(_torch=torch.cuda.Stream(device=torch.device("cuda", idx)))
    return ent.torch_stream


class cuda:  # namespace paddle.device.cuda
    Stream = _NativeStream
    Event = _NativeEvent
    from .framework import cuda_graphs as graphs  # paddle.device.cuda.graphs.CUDAGraph

    @staticmethod
    def device_count():
        return torch.cuda.device_count()

    @staticmethod
    def synchronize(device=None):
        if torch.cuda.is_available():
            from .framework import device_rt as rt
            idx = _parse(device).index if device is not None else None
            if not rt.available():
                return torch.cuda.synchronize(idx)
            rt.check(rt.lib().piamd_dev_synchronize(torch.cuda.current_device() if idx is None else idx),
                     "hipDeviceSynchronize")

    @staticmethod
    def current_stream(device=None):
        return _NativeStream(_torch=torch.cuda.current_stream(_parse(device) if device is not None else None))

    @staticmethod
    def stream_guard(stream):
        return torch.cuda.stream(stream.torch_stream if isinstance(stream, _NativeStream) else stream)

    @staticmethod
    def max_memory_allocated(device=None):
        if _own_alloc():
            return _own_stats(device)["peak_allocated"]
        return torch.cuda.max_memory_allocated(_parse(device) if device is not None else None)

    @staticmethod
    def max_memory_reserved(device=None):
        if _own_alloc():
            return _own_stats(device)["peak_reserved"]
        return torch.cuda.max_memory_reserved(_parse(device) if device is not None else None)

    @staticmethod
    def memory_allocated(device=None):
        if _own_alloc():
            return _own_stats(device)["allocated"]
        return torch.cuda.memory_allocated(_parse(device) if device is not None else None)

    @staticmethod
    def memory_reserved(device=None):
        if _own_alloc():
            return _own_stats(device)["reserved"]
        return torch.cuda.memory_reserved(_parse(device) if device is not None else None)

    @staticmethod
    def empty_cache():
        if _own_alloc():
            from .framework import allocator as _a
            _a.empty_cache(torch.cuda.current_device())
        elif torch.cuda.is_available():
            torch.cuda.empty_cache()

    @staticmethod
    def get_device_properties(device=None):
        from .framework import device_rt as rt
        d = _parse(device) if device is not None else None
        idx = d.index if d is not None and d.index is not None else (
            torch.cuda.current_device() if torch.cuda.is_available() else 0)
        if not rt.available():
            return torch.cuda.get_device_properties(idx)
        return _Props(rt.props(idx))

    @staticmethod
    def mem_get_info(device=None):
        """(free, total) bytes of the device (hipMemGetInfo)."""
        from .framework import device_rt as rt
        d = _parse(device) if device is not None else None
        idx = d.index if d is not None and d.index is not None else torch.cuda.current_device()
        if not rt.available():
            return torch.cuda.mem_get_info(idx)
        f, t = ctypes.c_longlong(), ctypes.c_longlong()
        rt.check(rt.lib().piamd_dev_mem_info(idx, ctypes.byref(f), ctypes.byref(t)), "hipMemGetInfo")
        return f.value, t.value

    @staticmethod
    def get_device_name(device=None):
        return torch.cuda.get_device_name(_parse(device) if device is not None else 0)

    @staticmethod
    def get_device_capability(device=None):
        return torch.cuda.get_device_capability(_parse(device) if device is not None else 0)


def synchronize(device=None):
    cuda.synchronize(device)


def _own_alloc():
    from .framework import allocator as _a
    return _a.active()


def _own_stats(device):
    from .framework import allocator as _a
    if device is None:
        d = torch.cuda.current_device()
    elif isinstance(device, int):
        d = device
    else:
        d = getattr(_parse(device), "index", 0) or 0
    return _a.stats(d)


# paddle.device-level stream API (reference python/paddle/device/__init__.py: Stream, Event,
# current_stream, set_stream, stream_guard) on the native runtime
Stream = _NativeStream
Event = _NativeEvent


def current_stream(device=None):
    return cuda.current_stream(device)


def set_stream(stream):
    """Make ``stream`` the current stream of its device; returns the previous one."""
    prev = cuda.current_stream(stream.device if isinstance(stream, _NativeStream) else None)
    torch.cuda.set_stream(stream.torch_stream if isinstance(stream, _NativeStream) else stream)
    return prev


def stream_guard(stream):
    return cuda.stream_guard(stream)


# ``import paddle.device.cuda.graphs`` / ``from paddle.device.cuda import graphs`` spellings
import sys as _sys  # noqa: E402
_sys.modules.setdefault(__name__ + ".cuda", cuda)  # type: ignore[arg-type]
_sys.modules.setdefault(__name__ + ".cuda.graphs", cuda.graphs)
