"""``paddle.static`` — static-graph Programs, Executor, save/load of inference models.

Parity: reference `python/paddle/static/__init__.py`. Programs are recorded by running the user's
model code on meta-backed :class:`Variable` tensors (every torch call is captured as an Operator);
:class:`Executor` runs them with the native C++ dependency/GC plan. ``save_inference_model``
writes a Paddle-wire-compatible ``.pdmodel`` (framework.proto ProgramDesc) + ``.pdiparams``
(combined LoDTensor stream), and Programs loaded from real Paddle ``.pdmodel`` files execute
through the op registry (`static/ops_registry.py`).
"""
from .framework import (Program, Variable, Block, Operator, program_guard, name_scope, data,  # noqa: F401
                        default_main_program, default_startup_program, Scope, global_scope,
                        scope_guard, InputSpec, _STATE)
from .executor import Executor, CompiledProgram, BuildStrategy, ExecutionStrategy  # noqa: F401
from .backward import append_backward, gradients  # noqa: F401
from .io import (save_inference_model, load_inference_model, serialize_program,  # noqa: F401
                 deserialize_program, serialize_persistables, deserialize_persistables, save, load,
                 load_program_state, set_program_state)
from . import nn  # noqa: F401
from .nn import create_parameter, py_func  # noqa: F401

ParallelExecutor = CompiledProgram


def cpu_places(device_count=None):
    from ..device import CPUPlace
    return [CPUPlace()] * (device_count or 1)


def cuda_places(device_ids=None):
    import torch
    from ..device import CUDAPlace
    ids = device_ids if device_ids is not None else range(max(torch.cuda.device_count(), 1))
    return [CUDAPlace(i) for i in ids]


class device_guard:  # noqa: N801
    """Reference `paddle.static.device_guard`: ops recorded inside carry ``op_device`` (e.g.
    ``"gpu:1"`` — the pipeline stage HybridParallelInferenceHelper places them on, ``"gpu:all"``
    for every stage). The executor itself runs every op on the program's device."""

    def __init__(self, device=None):
        self.device = device

    def __enter__(self):
        from . import framework as _fw
        self._prev = _fw._OP_DEVICE[0]
        _fw._OP_DEVICE[0] = self.device
        return self

    def __exit__(self, *a):
        from . import framework as _fw
        _fw._OP_DEVICE[0] = self._prev
        return False


def save_to_file(path, content):
    with open(path, "wb") as f:
        f.write(content)


def load_from_file(path):
    with open(path, "rb") as f:
        return f.read()


def normalize_program(program, feed_vars, fetch_vars):
    from .io import prune
    fetches = [v.var_name if isinstance(v, Variable) else v for v in
               (fetch_vars if isinstance(fetch_vars, (list, tuple)) else [fetch_vars])]
    p = program.clone(for_test=True)
    p.global_block().ops = prune(p, fetches)
    p._version += 1
    return p


def create_global_var(shape, value, dtype, persistable=False, force_cpu=False, name=None):
    import torch
    from ..framework.dtype import to_torch_dtype
    t = torch.full(list(shape), value, dtype=to_torch_dtype(dtype))
    prog = default_main_program()
    n = prog.param_var(t)
    return prog.global_block().vars[n]


def accuracy(input, label, k=1, correct=None, total=None):  # noqa: A002
    from ..metric import accuracy as _acc
    return _acc(input, label, k)


def Print(input, first_n=-1, message=None, summarize=20, print_tensor_name=True,  # noqa: N802,A002
          print_tensor_type=True, print_tensor_shape=True, print_tensor_lod=True,
          print_phase="both"):
    return input
from .extras import (xpu_places, npu_places, mlu_places, ipu_shard_guard, set_ipu_shard,  # noqa: E402,F401
                     IpuStrategy, IpuCompiledProgram, WeightNormParamAttr, ExponentialMovingAverage,
                     auc, ctr_metric_bundle, exponential_decay, create_lod_tensor)
