"""``paddle.nn.quant`` (reference `python/paddle/nn/quant/`): weight-only / LLM.int8 serving
quantisation (MFMA kernels in ``ops.inference``) and the quantisation-aware-training layers
(fake quant-dequant with straight-through gradients, quantized Linear / Conv / Matmul wrappers,
out-scale observers, quanter stubs, the linear quanter/dequanter export format)."""
from ...ops.inference import (weight_quantize, weight_dequantize, weight_only_linear,  # noqa: F401
                              llm_int8_linear, int8_linear)
from .quant_layers import (FakeQuantAbsMax, FakeQuantMovingAverageAbsMax,  # noqa: F401
                           FakeQuantChannelWiseAbsMax, MovingAverageAbsMaxScale, QuantizedConv2D,
                           QuantizedConv2DTranspose, QuantizedLinear, QuantizedColumnParallelLinear,
                           QuantizedRowParallelLinear, QuantizedMatmul, MAOutputScaleLayer,
                           FakeQuantMAOutputScaleLayer, QuantStub, fake_quant_dequant)
from .functional_layers import (FloatFunctionalLayer, add, subtract, multiply, divide,  # noqa: F401
                                reshape, transpose, concat, flatten, matmul)
from .format import (LinearQuanter, LinearDequanter, LinearQuanterDequanter,  # noqa: F401
                     ConvertibleQuantedLayer)
from .stub import Stub, QuanterStub  # noqa: F401
from . import qat  # noqa: F401

__all__ = ["Stub", "weight_only_linear", "llm_int8_linear", "weight_quantize", "weight_dequantize"]
