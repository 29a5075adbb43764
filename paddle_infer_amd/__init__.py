"""paddle_infer_amd — an MI355X-native deep-learning framework with PaddlePaddle's capabilities.

Compute path: PyTorch-ROCm tensors + autograd, hand-written CDNA4 HIP kernels (``ops``) for the
hot fused ops, hipBLASLt for plain GEMMs, RCCL over xGMI for collectives; native C++ runtime
(``csrc/runtime``) for the static-graph scheduler and memory planner.

Use it the way the reference is used: ``import paddle_infer_amd as paddle``.
"""
__version__ = "0.1.0"

import torch as _torch  # noqa: F401  (must load before the HIP kernel library)

from .framework import tensor_patch as _tensor_patch  # noqa: F401
from .framework import allocator as _allocator
_allocator.maybe_enable_from_env()  # FLAGS_allocator_strategy=auto_growth: own HIP allocator
from .framework import random as _random
from .framework.random import seed, get_rng_state, set_rng_state, get_cuda_rng_state, set_cuda_rng_state  # noqa: F401,E501
from .framework.dtype import (float32, float64, float16, bfloat16, int8, uint8, int16, int32,  # noqa: F401
                              int64, bool_ as bool, set_default_dtype, get_default_dtype,
                              complex64, complex128, dtype, iinfo, finfo)
from .framework.io import save, load  # noqa: F401
from .framework import flags as _flags
from .framework.flags import set_flags, get_flags  # noqa: F401
from .tensor import *  # noqa: F401,F403
from .tensor import Tensor  # noqa: F401
from . import linalg  # noqa: F401
from . import tensor  # noqa: F401
from .device import (set_device, get_device, CPUPlace, CUDAPlace, CUDAPinnedPlace,  # noqa: F401
                     is_compiled_with_cuda, is_compiled_with_rocm, is_compiled_with_xpu,
                     is_compiled_with_npu, is_compiled_with_cinn, NPUPlace, XPUPlace,
                     IPUPlace, MLUPlace)
from . import device  # noqa: F401
from . import ops  # noqa: F401
from . import nn  # noqa: F401
from . import optimizer  # noqa: F401
from . import amp  # noqa: F401
from . import autograd  # noqa: F401
from .autograd import grad, no_grad, enable_grad, set_grad_enabled, is_grad_enabled  # noqa: F401
from . import io  # noqa: F401
from .nn import ParamAttr  # noqa: F401

disable_static = lambda place=None: None  # noqa: E731  (dygraph is the default mode)


class LazyGuard:
    """Defer parameter materialisation (reference `fluid/lazy_init.py:LazyGuard`): layers built
    inside the guard are created on the ``meta`` device; ``Layer.to(device)`` / ``to_empty`` or
    loading a state dict materialises them."""

    def __enter__(self):
        self._ctx = _torch.device("meta")
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        return self._ctx.__exit__(*exc)


def set_printoptions(precision=None, threshold=None, edgeitems=None, sci_mode=None, linewidth=None):
    _torch.set_printoptions(precision=precision, threshold=threshold, edgeitems=edgeitems,
                            sci_mode=sci_mode, linewidth=linewidth)


def disable_signal_handler():
    """The reference unhooks its C++ fatal-signal handler; Python's defaults are already in place."""
    return None


def in_dynamic_mode():
    from . import static as _s
    return not _s._STATE["static"]


def enable_static():
    from . import static as _s
    _s._STATE["static"] = True


def disable_static(place=None):  # noqa: F811
    from . import static as _s
    _s._STATE["static"] = False


def create_parameter(shape, dtype="float32", name=None, attr=None, is_bias=False, default_initializer=None):
    from .nn.layer.base import Layer
    return Layer().create_parameter(shape, attr, dtype, is_bias, default_initializer)


def summary(net, input_size=None, dtypes=None, input=None):
    n = sum(p.numel() for p in net.parameters())
    t = sum(p.numel() for p in net.parameters() if p.requires_grad)
    print(f"Total params: {n:,}\nTrainable params: {t:,}")
    return {"total_params": n, "trainable_params": t}


def flops(net, input_size, custom_ops=None, print_detail=False):
    from .utils.flops import count_flops
    return count_flops(net, input_size)


def __getattr__(name):
    import importlib
    lazy = {"distributed", "static", "inference", "jit", "incubate", "vision", "metric", "hapi",
            "profiler", "utils", "models", "parallel", "text", "fft", "signal", "sparse", "callbacks",
            "distribution", "geometric", "audio", "onnx", "regularizer", "sysconfig", "hub",
            "reader", "quantization"}
    if name == "batch":
        return importlib.import_module(".reader", __name__).batch
    if name in lazy:
        return importlib.import_module(f".{name}", __name__)
    if name in ("Model",):
        return importlib.import_module(".hapi", __name__).Model
    if name == "DataParallel":
        return importlib.import_module(".distributed", __name__).DataParallel
    raise AttributeError(f"module 'paddle_infer_amd' has no attribute {name!r}")
