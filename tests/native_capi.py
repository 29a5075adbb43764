"""ctypes binding of the native engine's C API (`libpiamd_infer.so`, reference `capi_exp`
pd_inference_api.h) for in-process tests: no Python runs inside the engine; torch only allocates
the shared device buffers and checks the results."""
import ctypes

import numpy as np

from paddle_infer_amd import _build

PD_PRECISION_FLOAT32, PD_PRECISION_HALF, PD_PRECISION_BFLOAT16 = 0, 2, 3
PD_PLACE_CPU, PD_PLACE_GPU = 0, 1
PD_DATA = {"float32": 0, "int32": 1, "int64": 2, "uint8": 3, "int8": 4, "float16": 5, "bool": 6,
           "bfloat16": 7}

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        L = ctypes.CDLL(_build.NATIVE_LIB)
        vp, sz, i32, i32p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)
        for n, res, args in [
            ("PD_ConfigCreate", vp, []),
            ("PD_ConfigSetModel", None, [vp, ctypes.c_char_p, ctypes.c_char_p]),
            ("PD_ConfigEnableUseGpu", None, [vp, ctypes.c_uint64, i32, i32]),
            ("PD_ConfigEnableHipGraph", None, [vp, ctypes.c_int8]),
            ("PD_PredictorCreate", vp, [vp]),
            ("PD_PredictorDestroy", None, [vp]),
            ("PD_PredictorRun", ctypes.c_int8, [vp]),
            ("PD_PredictorGetInputHandle", vp, [vp, ctypes.c_char_p]),
            ("PD_PredictorGetOutputHandle", vp, [vp, ctypes.c_char_p]),
            ("PD_TensorDestroy", None, [vp]),
            ("PD_TensorReshape", None, [vp, sz, i32p]),
            ("PD_TensorCopyFromCpuFloat", None, [vp, ctypes.POINTER(ctypes.c_float)]),
            ("PD_TensorCopyFromCpuInt32", None, [vp, i32p]),
            ("PD_TensorCopyToCpuFloat", None, [vp, ctypes.POINTER(ctypes.c_float)]),
            ("PD_TensorShareExternalData", None, [vp, vp, sz, i32p, i32, i32]),
            ("PD_TensorGetDataType", i32, [vp]),
        ]:
            f = getattr(L, n)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def _shape(shape):
    return (ctypes.c_int32 * len(shape))(*shape)


class Predictor:
    def __init__(self, prefix, gpu=0, precision=PD_PRECISION_FLOAT32, hip_graph=False):
        L = lib()
        cfg = L.PD_ConfigCreate()
        L.PD_ConfigSetModel(cfg, (prefix + ".pdmodel").encode(), (prefix + ".pdiparams").encode())
        if gpu is not None:
            L.PD_ConfigEnableUseGpu(cfg, 256, gpu, precision)
        if hip_graph:
            L.PD_ConfigEnableHipGraph(cfg, 1)
        self.p = L.PD_PredictorCreate(cfg)
        assert self.p, "native predictor creation failed (see stderr)"
        self._handles = {}

    def _h(self, name, out=False):
        key = (name, out)
        if key not in self._handles:
            L = lib()
            f = L.PD_PredictorGetOutputHandle if out else L.PD_PredictorGetInputHandle
            self._handles[key] = f(self.p, name.encode())
        return self._handles[key]

    def share(self, name, tensor):
        """Zero-copy input: a torch device tensor the predictor reads (and updates in place)."""
        dt = str(tensor.dtype).replace("torch.", "")
        lib().PD_TensorShareExternalData(self._h(name), tensor.data_ptr(), tensor.dim(),
                                         _shape(list(tensor.shape)),
                                         PD_PLACE_GPU if tensor.is_cuda else PD_PLACE_CPU, PD_DATA[dt])

    def feed(self, name, arr):
        arr = np.ascontiguousarray(arr)
        L = lib()
        h = self._h(name)
        L.PD_TensorReshape(h, arr.ndim, _shape(list(arr.shape)))
        if arr.dtype == np.float32:
            L.PD_TensorCopyFromCpuFloat(h, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        elif arr.dtype == np.int32:
            L.PD_TensorCopyFromCpuInt32(h, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        else:
            raise TypeError(arr.dtype)

    def run(self):
        assert lib().PD_PredictorRun(self.p), "native Run failed (see stderr)"

    def fetch_float(self, name, shape):
        out = np.empty(shape, dtype=np.float32)
        lib().PD_TensorCopyToCpuFloat(self._h(name, True), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        return out

    def close(self):
        L = lib()
        for h in self._handles.values():
            L.PD_TensorDestroy(h)
        self._handles = {}
        if self.p:
            L.PD_PredictorDestroy(self.p)
            self.p = None
