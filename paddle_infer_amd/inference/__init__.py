"""``paddle.inference`` — Config / Predictor / Tensor handles, IR fusion passes, hipGraph replay,
and LLM serving (``generation``).

Parity: reference `python/paddle/inference/__init__.py`, `paddle/fluid/inference/api/
analysis_predictor.cc`, `paddle_analysis_config.h`, `paddle_pass_builder.cc`.
"""
from .config import Config, DataType, PlaceType, PrecisionType, get_num_bytes_of_data_type  # noqa: F401
from .predictor import (Predictor, Tensor, create_predictor, PredictorPool, get_version,  # noqa: F401
                        convert_to_mixed_precision, get_trt_compile_version,
                        get_trt_runtime_version)
from . import passes  # noqa: F401


def __getattr__(name):
    if name == "generation":
        import importlib
        return importlib.import_module(".generation", __name__)
    raise AttributeError(name)


def _get_phi_kernel_name(op_name):
    """Reference `inference/__init__.py:_get_phi_kernel_name` (fluid op name → PHI kernel name);
    here the Paddle-op registry names its kernels after the op types themselves."""
    return {"matmul_v2": "matmul", "elementwise_add": "add", "elementwise_sub": "subtract",
            "elementwise_mul": "multiply", "elementwise_div": "divide", "reshape2": "reshape",
            "transpose2": "transpose", "lookup_table_v2": "embedding", "fill_any_like": "full_like",
            "softmax_with_cross_entropy": "cross_entropy_with_softmax",
            "flatten_contiguous_range": "flatten", "expand_v2": "expand"}.get(op_name, op_name)
