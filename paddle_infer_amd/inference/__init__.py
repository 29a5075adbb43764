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
