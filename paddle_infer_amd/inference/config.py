"""Inference ``Config`` (reference `paddle/fluid/inference/api/paddle_analysis_config.h`,
bound in `pybind/inference_api.cc`). Backends that do not exist on MI355X (TensorRT, MKLDNN,
Lite, XPU/NPU/IPU, ONNXRuntime) keep their switches for API compatibility; enabling them logs a
notice and the HIP path is used. MI355X-specific: :meth:`enable_hip_graph`."""
from __future__ import annotations

import enum
import os


class PrecisionType(enum.IntEnum):
    Float32 = 0
    Int8 = 1
    Half = 2
    Bfloat16 = 3


class PlaceType(enum.IntEnum):
    UNK = -1
    CPU = 0
    GPU = 1
    XPU = 2
    NPU = 3
    IPU = 4
    CUSTOM = 5


class DataType(enum.IntEnum):
    FLOAT32 = 0
    INT64 = 1
    INT32 = 2
    UINT8 = 3
    INT8 = 4
    FLOAT16 = 5
    BOOL = 6
    FLOAT64 = 7
    BFLOAT16 = 8


_NBYTES = {DataType.FLOAT32: 4, DataType.INT64: 8, DataType.INT32: 4, DataType.UINT8: 1,
           DataType.INT8: 1, DataType.FLOAT16: 2, DataType.BOOL: 1, DataType.FLOAT64: 8,
           DataType.BFLOAT16: 2}


def get_num_bytes_of_data_type(dtype):
    return _NBYTES[DataType(dtype)]


class _PassBuilder:
    def __init__(self, passes):
        self._passes = list(passes)

    def all_passes(self):
        return list(self._passes)

    def append_pass(self, name):
        self._passes.append(name)

    def insert_pass(self, idx, name):
        self._passes.insert(idx, name)

    def delete_pass(self, name):
        self._passes = [p for p in self._passes if p != name]

    def set_passes(self, passes):
        self._passes = list(passes)

    def turn_on_debug(self):
        pass

    def debug_string(self):
        return "\n".join(self._passes)


class Config:
    def __init__(self, model_dir_or_prog_file=None, params_file=None):
        from .passes import GPU_PASSES
        self._model_dir = None
        self._prog_file = None
        self._params_file = params_file
        if model_dir_or_prog_file is not None:
            if params_file is None and os.path.isdir(model_dir_or_prog_file):
                self._model_dir = model_dir_or_prog_file
            else:
                self._prog_file = model_dir_or_prog_file
        self._model_buffer = None
        self._use_gpu = False
        self._device_id = 0
        self._memory_pool_mb = 0
        self._precision = PrecisionType.Float32
        self._ir_optim = True
        self._memory_optim = False
        self._hip_graph = False
        self._profile = False
        self._glog = True
        self._threads = 1
        self._exec_stream = None
        self._pass_builder = _PassBuilder(GPU_PASSES)
        self._mixed_black_list = set()
        self._notes = []
        self._save_optim = False
        self._optim_cache_dir = None

    # ---- optimised-model cache (reference AnalysisConfig::EnableSaveOptimModel) ---------------
    def enable_save_optim_model(self, x=True):
        """Write the IR-optimised, precision-converted model as ``_optimized.pdmodel`` /
        ``.pdiparams`` (into ``set_optim_cache_dir`` or the model's directory) when the predictor
        is created — the input of the native C++ predictor's GPU path."""
        self._save_optim = bool(x)

    def set_optim_cache_dir(self, d):
        self._optim_cache_dir = d

    def optim_model_prefix(self):
        d = self._optim_cache_dir or self._model_dir or os.path.dirname(self.prog_file() or ".") or "."
        return os.path.join(d, "_optimized")

    # ---- model location -------------------------------------------------------------------
    def set_model(self, model_dir_or_prog_file, params_file=None):
        self.__init__(model_dir_or_prog_file, params_file)

    def set_prog_file(self, f):
        self._prog_file = f

    def set_params_file(self, f):
        self._params_file = f

    def set_model_buffer(self, prog_buffer, prog_size, params_buffer, params_size):
        self._model_buffer = (bytes(prog_buffer[:prog_size]) if prog_size else bytes(prog_buffer),
                              bytes(params_buffer[:params_size]) if params_size else bytes(params_buffer))

    def model_from_memory(self):
        return self._model_buffer is not None

    def model_dir(self):
        return self._model_dir

    def prog_file(self):
        if self._prog_file:
            return self._prog_file
        if self._model_dir:
            for cand in ("inference.pdmodel", "model.pdmodel", "__model__"):
                p = os.path.join(self._model_dir, cand)
                if os.path.exists(p):
                    return p
            for f in sorted(os.listdir(self._model_dir)):
                if f.endswith(".pdmodel"):
                    return os.path.join(self._model_dir, f)
        return None

    def params_file(self):
        if self._params_file:
            return self._params_file
        pf = self.prog_file()
        if pf and pf.endswith(".pdmodel"):
            return pf[:-len(".pdmodel")] + ".pdiparams"
        return None

    # ---- device / precision --------------------------------------------------------------
    def enable_use_gpu(self, memory_pool_init_size_mb=100, device_id=0,
                       precision_mode=PrecisionType.Float32):
        self._use_gpu, self._memory_pool_mb, self._device_id = True, memory_pool_init_size_mb, device_id
        self._precision = PrecisionType(precision_mode)

    def disable_gpu(self):
        self._use_gpu = False

    def use_gpu(self):
        return self._use_gpu

    def gpu_device_id(self):
        return self._device_id

    def memory_pool_init_size_mb(self):
        return self._memory_pool_mb

    def fraction_of_gpu_memory_for_pool(self):
        return 0.0

    def exp_enable_mixed_precision(self, precision=PrecisionType.Bfloat16, black_list=None):
        self._precision = PrecisionType(precision)
        self._mixed_black_list = set(black_list or ())

    def enable_hip_graph(self, enable=True):
        """Capture the whole forward as a hipGraph per input-shape set and replay it."""
        self._hip_graph = bool(enable)

    enable_cuda_graph = enable_hip_graph

    def hip_graph_enabled(self):
        return self._hip_graph

    def set_exec_stream(self, stream):
        self._exec_stream = stream

    # ---- optimisation switches ------------------------------------------------------------
    def switch_ir_optim(self, x=True):
        self._ir_optim = bool(x)

    def ir_optim(self):
        return self._ir_optim

    def enable_memory_optim(self, x=True):
        self._memory_optim = bool(x)

    def enable_memory_optimize(self):
        return self._memory_optim

    def switch_use_feed_fetch_ops(self, x=True):
        pass

    def switch_specify_input_names(self, x=True):
        pass

    def switch_ir_debug(self, x=True):
        self._ir_debug = bool(x)

    def pass_builder(self):
        return self._pass_builder

    def delete_pass(self, name):
        self._pass_builder.delete_pass(name)

    def enable_profile(self):
        self._profile = True

    def disable_glog_info(self):
        self._glog = False

    def glog_info_disabled(self):
        return not self._glog

    def set_cpu_math_library_num_threads(self, n):
        self._threads = int(n)

    def cpu_math_library_num_threads(self):
        return self._threads

    def _unsupported(self, what):
        self._notes.append(what)

    # ---- backends absent on MI355X (accepted, HIP path used) --------------------------------
    def enable_tensorrt_engine(self, *a, **k):
        self._unsupported("tensorrt")

    def tensorrt_engine_enabled(self):
        return False

    def set_trt_dynamic_shape_info(self, *a, **k):
        pass

    def enable_mkldnn(self):
        self._unsupported("mkldnn")

    def mkldnn_enabled(self):
        return False

    def enable_mkldnn_bfloat16(self):
        self._unsupported("mkldnn_bf16")

    def enable_xpu(self, *a, **k):
        self._unsupported("xpu")

    def enable_npu(self, *a, **k):
        self._unsupported("npu")

    def enable_ipu(self, *a, **k):
        self._unsupported("ipu")

    def enable_lite_engine(self, *a, **k):
        self._unsupported("lite")

    def enable_onnxruntime(self):
        self._unsupported("onnxruntime")

    def summary(self):
        rows = [("model", self.prog_file() or "<memory>"), ("params", self.params_file()),
                ("use_gpu", self._use_gpu), ("device_id", self._device_id),
                ("precision", self._precision.name), ("ir_optim", self._ir_optim),
                ("memory_optim", self._memory_optim), ("hip_graph", self._hip_graph),
                ("passes", ",".join(self._pass_builder.all_passes()))]
        w = max(len(k) for k, _ in rows)
        return "\n".join(f"{k.ljust(w)} : {v}" for k, v in rows)
