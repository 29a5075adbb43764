"""``paddle.incubate.nn`` — fused transformer layers (reference `python/paddle/incubate/nn/`)."""
from . import functional  # noqa: F401
from .layer.fused_transformer import (FusedLinear, FusedBiasDropoutResidualLayerNorm,  # noqa: F401
                                      FusedMultiHeadAttention, FusedFeedForward,
                                      FusedTransformerEncoderLayer, FusedTransformer,
                                      FusedMultiTransformer, FusedMultiTransformerWeightOnly,
                                      FusedMultiTransformerINT8, FusedMoELayer,
                                      FusedMultiTransformerMoe, FusedMultiTransformerMoeINT8,
                                      FusedMultiTransformerMoeWeightOnly)
