"""Predictor (reference `paddle/fluid/inference/api/analysis_predictor.cc`).

Load → (IR passes) → precision cast → run on the static Executor (native dependency/GC plan).
With ``Config.enable_hip_graph()`` each distinct set of input shapes is captured once into a
``torch.cuda.CUDAGraph`` (hipGraph on ROCm) over static input buffers and replayed afterwards —
the MI355X replacement for the reference's CUDA-graph predictor mode.
"""
from __future__ import annotations

import copy
import os

import numpy as np
import torch

from .. import static as _static
from ..static import io as _sio
from .config import Config, DataType, PrecisionType

_NP2DT = {np.dtype("float32"): DataType.FLOAT32, np.dtype("int64"): DataType.INT64,
          np.dtype("int32"): DataType.INT32, np.dtype("uint8"): DataType.UINT8,
          np.dtype("int8"): DataType.INT8, np.dtype("float16"): DataType.FLOAT16,
          np.dtype("bool"): DataType.BOOL, np.dtype("float64"): DataType.FLOAT64}


def get_version():
    from .. import __version__
    return f"paddle_infer_amd {__version__} (MI355X / gfx950, HIP)"


def get_trt_compile_version():
    return (0, 0, 0)


def get_trt_runtime_version():
    return (0, 0, 0)


class Tensor:
    """Input/output handle (reference `paddle_tensor.h` ZeroCopyTensor / paddle_infer::Tensor)."""

    def __init__(self, name, predictor, is_input):
        self._name, self._pred, self._is_input = name, predictor, is_input
        self._shape = None
        self._lod = []

    def name(self):
        return self._name

    def reshape(self, shape):
        self._shape = list(shape)

    def copy_from_cpu(self, data):
        arr = np.ascontiguousarray(data)
        t = torch.from_numpy(arr)
        if self._shape is not None and list(t.shape) != self._shape and t.numel() == int(np.prod(self._shape)):
            t = t.reshape(self._shape)
        self._pred._inputs[self._name] = t.to(self._pred._device, non_blocking=True)

    def share_external_data(self, data):
        t = data if isinstance(data, torch.Tensor) else torch.as_tensor(np.asarray(data))
        self._pred._inputs[self._name] = t.to(self._pred._device)

    def copy_to_cpu(self):
        t = self._tensor()
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.detach().cpu().numpy()

    def to_torch(self):
        return self._tensor()

    def _tensor(self):
        d = self._pred._inputs if self._is_input else self._pred._outputs
        if self._name not in d:
            raise RuntimeError(f"tensor {self._name} has no data yet")
        return d[self._name]

    def shape(self):
        if self._is_input and self._name not in self._pred._inputs:
            return list(self._shape or [])
        return list(self._tensor().shape)

    def type(self):
        t = self._tensor()
        if t.dtype == torch.bfloat16:
            return DataType.BFLOAT16
        return _NP2DT.get(np.dtype(str(t.dtype).replace("torch.", "")), DataType.FLOAT32)

    def set_lod(self, lod):
        self._lod = lod

    def lod(self):
        return self._lod


class Predictor:
    def __init__(self, config: Config, _shared=None):
        self._config = config
        use_gpu = config.use_gpu() and torch.cuda.is_available()
        self._device = torch.device(f"cuda:{config.gpu_device_id()}" if use_gpu else "cpu")
        self._scope = _static.Scope()
        self._exe = _static.Executor(self._device)
        self._graphs = {}
        self._inputs, self._outputs = {}, {}
        self._cast_dtype = None
        prec = config._precision
        if self._device.type == "cuda" and prec in (PrecisionType.Half, PrecisionType.Bfloat16):
            self._cast_dtype = torch.bfloat16 if prec == PrecisionType.Bfloat16 else torch.float16
        if _shared is not None:
            self._program, self._feed_names, self._fetch_names, src_scope = _shared
            self._scope.vars = src_scope.vars  # weights shared between clones
            return
        with _static.scope_guard(self._scope):
            if config.model_from_memory():
                prog = _sio.deserialize_program(config._model_buffer[0])
                _sio.deserialize_persistables(prog, config._model_buffer[1], self._exe)
                feeds, fetches = prog.feed_names, prog.fetch_names
            else:
                pf = config.prog_file()
                if pf is None or not os.path.exists(pf):
                    raise FileNotFoundError(f"inference model not found: {pf}")
                prog, feeds, fetch_vars = _static.load_inference_model(
                    pf[:-len(".pdmodel")] if pf.endswith(".pdmodel") else pf, self._exe,
                    model_filename=pf, params_filename=config.params_file())
                fetches = [v.var_name for v in fetch_vars]
        self._program, self._feed_names, self._fetch_names = prog, list(feeds), list(fetches)
        if config.ir_optim():
            from .passes import apply_passes
            self.pass_stats = apply_passes(prog, config.pass_builder().all_passes(), fetches,
                                           debug=getattr(config, "_ir_debug", False))
            # parameters created by passes (folded conv-bn weights) into the scope
            for n, t in prog.params.items():
                if self._scope.get(n) is None:
                    self._scope.set(n, t.to(self._device))
        if self._cast_dtype is not None:
            for n, t in list(self._scope.vars.items()):
                if t is not None and t.is_floating_point() and n not in config._mixed_black_list:
                    self._scope.set(n, t.to(self._cast_dtype))
        if getattr(config, "_save_optim", False):
            self.save_optimized_model(config.optim_model_prefix())

    # ---- handles --------------------------------------------------------------------------
    def get_input_names(self):
        return list(self._feed_names)

    def get_output_names(self):
        return list(self._fetch_names)

    def get_input_handle(self, name):
        return Tensor(name, self, True)

    def get_output_handle(self, name):
        return Tensor(name, self, False)

    get_input_tensor = get_input_handle
    get_output_tensor = get_output_handle

    def get_input_tensor_shape(self):
        b = self._program.global_block()
        return {n: list(b.vars[n].declared_shape or []) for n in self._feed_names}

    # ---- execution ------------------------------------------------------------------------
    def _feed(self):
        feed = {}
        for n in self._feed_names:
            if n not in self._inputs:
                raise RuntimeError(f"input {n} not set")
            t = self._inputs[n]
            if self._cast_dtype is not None and t.is_floating_point():
                t = t.to(self._cast_dtype)
            feed[n] = t
        return feed

    def _run_eager(self, feed):
        with _static.scope_guard(self._scope), torch.no_grad():
            return self._exe.run(self._program, feed=feed, fetch_list=self._fetch_names,
                                 return_numpy=False)

    def _run_graph(self, feed):
        key = tuple((n, tuple(t.shape), t.dtype) for n, t in feed.items())
        ent = self._graphs.get(key)
        if ent is None:
            static_in = {n: t.clone() for n, t in feed.items()}
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):  # warm-up: lazy allocations / library handles
                    self._run_eager(static_in)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                static_out = self._run_eager(static_in)
            ent = self._graphs[key] = (g, static_in, static_out)
        g, static_in, static_out = ent
        for n, t in feed.items():
            static_in[n].copy_(t, non_blocking=True)
        g.replay()
        return static_out

    def run(self, inputs=None):
        if inputs is not None:  # new-style API: run(list of tensors) -> list of outputs
            for n, v in zip(self._feed_names, inputs):
                self.get_input_handle(n).share_external_data(v)
        feed = self._feed()
        if self._config.hip_graph_enabled() and self._device.type == "cuda":
            outs = self._run_graph(feed)
        else:
            outs = self._run_eager(feed)
        self._outputs = dict(zip(self._fetch_names, outs))
        if inputs is not None:
            return [self._outputs[n] for n in self._fetch_names]
        return True

    def clone(self, stream=None):
        return Predictor(self._config, (self._program, self._feed_names, self._fetch_names, self._scope))

    def clear_intermediate_tensor(self):
        self._outputs = {}

    def try_shrink_memory(self):
        self._graphs.clear()
        if self._device.type == "cuda":
            torch.cuda.empty_cache()
        return 0

    def save_optimized_model(self, path_prefix):
        """Write the IR-optimised program (fused ops after the passes) and its parameters in the
        predictor's compute dtype (bf16 / fp16 under mixed precision) as ``path_prefix``
        ``.pdmodel`` / ``.pdiparams`` — the model the native C++ predictor (``libpiamd_infer.so``,
        ``pd_infer_run``) runs on the framework's GPU kernels. Reference: the analysis predictor's
        optimised-model cache (``Config.enable_save_optim_model``)."""
        blk = self._program.global_block()
        with _static.scope_guard(self._scope):
            _static.save_inference_model(path_prefix, [blk.vars[n] for n in self._feed_names],
                                         [blk.vars[n] for n in self._fetch_names], self._exe,
                                         program=self._program)

    def get_serialized_program(self):
        return _sio.serialize_program([self._program.global_block().vars[n] for n in self._feed_names],
                                      [self._program.global_block().vars[n] for n in self._fetch_names],
                                      self._program)

    @property
    def program(self):
        return self._program


def create_predictor(config: Config) -> Predictor:
    return Predictor(config)


class PredictorPool:
    def __init__(self, config: Config, size: int = 1):
        first = Predictor(config)
        self._preds = [first] + [first.clone() for _ in range(size - 1)]

    def retrive(self, idx):
        return self._preds[idx]

    retrieve = retrive


def convert_to_mixed_precision(model_file, params_file, mixed_model_file, mixed_params_file,
                               mixed_precision=PrecisionType.Bfloat16, backend=None,
                               keep_io_types=True, black_list=None):
    """Offline conversion: floating persistables → fp16/bf16 (reference
    `convert_to_mixed_precision.cc`); ops run in the stored precision."""
    dt = torch.bfloat16 if PrecisionType(mixed_precision) == PrecisionType.Bfloat16 else torch.float16
    black = set(black_list or ())
    with open(model_file, "rb") as f:
        prog = _sio.deserialize_program(f.read())
    scope = _static.Scope()
    with _static.scope_guard(scope):
        with open(params_file, "rb") as f:
            _sio.deserialize_persistables(prog, f.read())
        for n, t in list(prog.params.items()):
            if t.is_floating_point() and n not in black:
                prog.params[n] = t.to(dt)
                scope.set(n, prog.params[n])
                v = prog.global_block().vars.get(n)
                if v is not None:
                    prog.global_block().create_var(n, v.declared_shape or list(t.shape),
                                                   "bfloat16" if dt == torch.bfloat16 else "float16",
                                                   persistable=True)
        b = prog.global_block()
        feeds = [b.vars[n] for n in prog.feed_names]
        fetches = [b.vars[n] for n in prog.fetch_names]
        with open(mixed_model_file, "wb") as f:
            f.write(_sio.serialize_program(feeds, fetches, prog))
        names = sorted(prog.params)
        with open(mixed_params_file, "wb") as f:
            f.write(_sio.serialize_persistables(feeds, fetches, None, prog, names))


copy  # noqa
