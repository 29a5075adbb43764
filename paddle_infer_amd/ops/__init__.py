"""Hand-written CDNA4 HIP kernels exposed as differentiable ops.

GPU tensors run the in-tree HIP library (``_lib/libpiamd_kernels.so``); CPU tensors run the
PyTorch reference composition of the same op.
"""
from .norm import layer_norm, fused_add_layer_norm, rms_norm, fused_add_rms_norm  # noqa: F401
from .attention import (flash_attention, flash_attention_packed, attention_reference,  # noqa: F401
                        flash_attention_varlen)
from .activation import bias_act, gelu, dropout, fused_softmax_mask  # noqa: F401
from .loss import softmax_cross_entropy  # noqa: F401
from .optim import adamw_flat, momentum_flat, sumsq  # noqa: F401
from . import _lib  # noqa: F401
from .inference import (qkv_prep, decode_attention, weight_quantize, weight_dequantize,  # noqa: F401
                        weight_only_linear, llm_int8_linear, int8_linear,
                        quantize_rows)


def _make_recordable():
    """Static-graph capture records these framework ops by name (see static.framework.recordable)."""
    from ..static.framework import recordable
    g = globals()
    for name, ty in (("layer_norm", "layer_norm"), ("fused_add_layer_norm", "skip_layernorm"),
                     ("rms_norm", "rms_norm"), ("flash_attention", "flash_attn"),
                     ("flash_attention_packed", "flash_attn_packed"), ("bias_act", "fused_bias_act"),
                     ("gelu", "gelu"), ("dropout", "dropout"), ("fused_softmax_mask", "softmax_mask_fuse"),
                     ("softmax_cross_entropy", "softmax_with_cross_entropy"),
                     ("weight_only_linear", "weight_only_linear")):
        g[name] = recordable(ty)(g[name])


_make_recordable()
