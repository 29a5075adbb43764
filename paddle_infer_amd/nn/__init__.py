"""``paddle.nn`` — layers, functional, initializers, clipping, quantization."""
from .layer.base import Layer, LayerList, Sequential, LayerDict, ParameterList, ParamAttr  # noqa: F401
from .layer.layers import *  # noqa: F401,F403
from .layer.layers import (  # noqa: F401
    Identity, Linear, Bilinear, Embedding, Dropout, Dropout2D, Dropout3D, AlphaDropout, Flatten,
    Unflatten, Pad1D, Pad2D, Pad3D, Upsample, UpsamplingBilinear2D, UpsamplingNearest2D,
    PixelShuffle, CosineSimilarity, PairwiseDistance, ReLU, ReLU6, GELU, Silu, Swish, Sigmoid, Tanh,
    ELU, SELU, CELU, LeakyReLU, Hardswish, Hardsigmoid, Hardtanh, Hardshrink, Softshrink,
    Tanhshrink, Softplus, Softsign, Mish, LogSigmoid, ThresholdedReLU, Softmax, LogSoftmax, GLU,
    PReLU, Maxout, Conv1D, Conv2D, Conv3D, Conv2DTranspose, Conv1DTranspose, MaxPool1D, MaxPool2D,
    MaxPool3D, AvgPool1D, AvgPool2D, AvgPool3D, AdaptiveAvgPool1D, AdaptiveAvgPool2D,
    AdaptiveAvgPool3D, AdaptiveMaxPool1D, AdaptiveMaxPool2D, LayerNorm, RMSNorm, BatchNorm,
    BatchNorm1D, BatchNorm2D, BatchNorm3D, SyncBatchNorm, GroupNorm, InstanceNorm1D,
    InstanceNorm2D, InstanceNorm3D, LocalResponseNorm, CrossEntropyLoss, MSELoss, L1Loss,
    SmoothL1Loss, BCELoss, BCEWithLogitsLoss, NLLLoss, KLDivLoss, MarginRankingLoss,
    HingeEmbeddingLoss, CosineEmbeddingLoss, TripletMarginLoss, CTCLoss, MultiHeadAttention,
    TransformerEncoderLayer, TransformerEncoder, TransformerDecoderLayer, TransformerDecoder,
    Transformer, SimpleRNN, LSTM, GRU)
from . import functional  # noqa: F401
from . import initializer  # noqa: F401
from .clip import ClipGradByGlobalNorm, ClipGradByNorm, ClipGradByValue  # noqa: F401
from . import utils  # noqa: F401
from . import quant  # noqa: F401,E402
