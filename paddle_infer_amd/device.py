"""Device / place management (reference `python/paddle/device/__init__.py`, `device/cuda/`).

On this framework a "gpu" place is a HIP device (MI355X); ``paddle.set_device('gpu:0')`` selects
the default device for tensor creation. Streams/events are HIP streams/events via torch.cuda.
"""
from __future__ import annotations

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


class cuda:  # namespace paddle.device.cuda
    Stream = torch.cuda.Stream if hasattr(torch.cuda, "Stream") else object
    Event = torch.cuda.Event if hasattr(torch.cuda, "Event") else object

    @staticmethod
    def device_count():
        return torch.cuda.device_count()

    @staticmethod
    def synchronize(device=None):
        if torch.cuda.is_available():
            torch.cuda.synchronize(_parse(device) if device is not None else None)

    @staticmethod
    def current_stream(device=None):
        return torch.cuda.current_stream(_parse(device) if device is not None else None)

    @staticmethod
    def stream_guard(stream):
        return torch.cuda.stream(stream)

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
        return torch.cuda.get_device_properties(_parse(device) if device is not None else 0)

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
