"""``paddle.set_flags`` / ``get_flags`` (reference `paddle/fluid/platform/flags.cc`).

Flags honoured by this framework: FLAGS_check_nan_inf (NaN/Inf checker on every op output through
``utils.nan_inf``), FLAGS_cudnn_deterministic (torch deterministic algorithms),
FLAGS_use_hipgraph (inference predictor graph capture), FLAGS_allocator_strategy ("auto_growth"
in the environment or set before the first device allocation installs the framework's own
auto-growth best-fit HIP allocator, ``framework/allocator.py``; the in-process default stays
PyTorch's caching allocator; ``get_flags`` reports the allocator actually installed),
FLAGS_fraction_of_gpu_memory_to_use (the per-process memory fraction of the caching allocator).
Setting a flag that is not registered raises, as the reference's ``set_flags`` does.
"""
from __future__ import annotations

import os

import torch

_FLAGS = {
    "FLAGS_check_nan_inf": False,
    "FLAGS_cudnn_deterministic": False,
    "FLAGS_use_hipgraph": True,
    "FLAGS_fraction_of_gpu_memory_to_use": 0.92,
    "FLAGS_allocator_strategy": "auto_growth",
    "FLAGS_eager_delete_tensor_gb": 0.0,
    "FLAGS_benchmark": False,
    "FLAGS_embedding_deterministic": 0,
    "FLAGS_conv_workspace_size_limit": 512,
    "FLAGS_cudnn_exhaustive_search": False,
    "FLAGS_use_autotune": False,
    "FLAGS_max_inplace_grad_add": 0,
    "FLAGS_enable_gpu_memory_usage_log": False,
    "FLAGS_call_stack_level": 1,
    "FLAGS_sort_sum_gradient": False,
    "FLAGS_gpu_allocator_retry_time": 10000,
    "FLAGS_initial_gpu_memory_in_mb": 0,
    "FLAGS_reallocate_gpu_memory_in_mb": 0,
    "FLAGS_use_stream_safe_cuda_allocator": True,
    "FLAGS_new_executor_use_cuda_graph": False,
    "FLAGS_tracer_profile_fname": "",
    "FLAGS_print_ir": False,
    "FLAGS_low_precision_op_list": 0,
    "FLAGS_selected_gpus": "",
}
for k in list(_FLAGS):
    if k in os.environ:
        v = os.environ[k]
        d = _FLAGS[k]
        _FLAGS[k] = (v.lower() in ("1", "true")) if isinstance(d, bool) else type(d)(v)


def set_flags(flags: dict):
    for k in flags:
        if k not in _FLAGS:
            raise ValueError(f"Flag {k} is not registered in this framework's flag registry")
    for k, v in flags.items():
        _FLAGS[k] = v
        if k == "FLAGS_cudnn_deterministic":
            torch.use_deterministic_algorithms(bool(v), warn_only=True)
        if k == "FLAGS_check_nan_inf":
            from ..utils import nan_inf
            nan_inf.enable(bool(v))
        if k == "FLAGS_cudnn_exhaustive_search" or k == "FLAGS_use_autotune":
            from ..ops import autotune
            autotune.configure(enable=bool(v))
        if k == "FLAGS_fraction_of_gpu_memory_to_use" and torch.cuda.is_available():
            from . import allocator
            if allocator.active():  # the auto-growth allocator grows on demand: no fixed pool
                import warnings
                warnings.warn("FLAGS_fraction_of_gpu_memory_to_use has no effect under the "
                              "auto_growth allocator", RuntimeWarning)
            else:
                torch.cuda.set_per_process_memory_fraction(float(v))
        if k == "FLAGS_allocator_strategy" and v == "auto_growth":
            from . import allocator
            try:
                allocator.enable("auto_growth")
            except RuntimeError as e:  # device memory already in use by the caching allocator
                import warnings
                warnings.warn(f"FLAGS_allocator_strategy=auto_growth not applied: {e}", RuntimeWarning)


def get_flags(flags):
    names = [flags] if isinstance(flags, str) else list(flags)
    out = {}
    for k in names:
        if k not in _FLAGS:
            raise ValueError(f"Flag {k} is not registered in this framework's flag registry")
        v = _FLAGS[k]
        if k == "FLAGS_allocator_strategy":
            from . import allocator
            v = "auto_growth" if allocator.active() else "torch_caching"
        out[k] = v
    return out


def flag(name, default=None):
    return _FLAGS.get(name, default)
