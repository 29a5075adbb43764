"""``paddle.nn.initializer`` (reference `python/paddle/nn/initializer/*.py`)."""
from __future__ import annotations

import math

import numpy as np
import torch


def _fans(t: torch.Tensor):
    # Paddle convention: Linear weight is [in, out]; conv weight is [out, in, kh, kw].
    if t.dim() < 2:
        return t.numel(), t.numel()
    if t.dim() == 2:
        return t.shape[0], t.shape[1]
    rf = int(np.prod(t.shape[2:]))
    return t.shape[1] * rf, t.shape[0] * rf


class Initializer:
    def __call__(self, t: torch.Tensor, block=None):
        with torch.no_grad():
            self._init(t)
        return t

    def _init(self, t):  # pragma: no cover
        raise NotImplementedError


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def _init(self, t):
        t.fill_(self.value)


class Normal(Initializer):
    def __init__(self, mean=0.0, std=1.0, name=None):
        self.mean, self.std = mean, std

    def _init(self, t):
        if t.dtype in (torch.bfloat16, torch.float16):
            t.copy_(torch.randn(t.shape, dtype=torch.float32, device=t.device) * self.std + self.mean)
        else:
            t.normal_(self.mean, self.std)


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, std=1.0, a=-2.0, b=2.0, name=None):
        self.mean, self.std, self.a, self.b = mean, std, a, b

    def _init(self, t):
        f = torch.empty(t.shape, dtype=torch.float32, device=t.device)
        torch.nn.init.trunc_normal_(f, self.mean, self.std, self.mean + self.a * self.std,
                                    self.mean + self.b * self.std)
        t.copy_(f)


class Uniform(Initializer):
    def __init__(self, low=-1.0, high=1.0, name=None):
        self.low, self.high = low, high

    def _init(self, t):
        f = torch.empty(t.shape, dtype=torch.float32, device=t.device).uniform_(self.low, self.high)
        t.copy_(f)


class XavierUniform(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fi, self.fo, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(t)
        fi, fo = self.fi or fi, self.fo or fo
        lim = self.gain * math.sqrt(6.0 / (fi + fo))
        Uniform(-lim, lim)._init(t)


class XavierNormal(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fi, self.fo, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(t)
        fi, fo = self.fi or fi, self.fo or fo
        Normal(0.0, self.gain * math.sqrt(2.0 / (fi + fo)))._init(t)


class KaimingUniform(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity="relu", name=None):
        self.fi, self.slope, self.nl = fan_in, negative_slope, nonlinearity

    def _init(self, t):
        fi = self.fi or _fans(t)[0]
        gain = math.sqrt(2.0 / (1 + self.slope ** 2)) if self.nl in ("relu", "leaky_relu") else 1.0
        lim = gain * math.sqrt(3.0 / fi)
        Uniform(-lim, lim)._init(t)


class KaimingNormal(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity="relu", name=None):
        self.fi, self.slope, self.nl = fan_in, negative_slope, nonlinearity

    def _init(self, t):
        fi = self.fi or _fans(t)[0]
        gain = math.sqrt(2.0 / (1 + self.slope ** 2)) if self.nl in ("relu", "leaky_relu") else 1.0
        Normal(0.0, gain / math.sqrt(fi))._init(t)


class Assign(Initializer):
    def __init__(self, value, name=None):
        self.value = value

    def _init(self, t):
        v = self.value if isinstance(self.value, torch.Tensor) else torch.as_tensor(np.asarray(self.value))
        t.copy_(v.reshape(t.shape).to(t.dtype))


class Orthogonal(Initializer):
    def __init__(self, gain=1.0, name=None):
        self.gain = gain

    def _init(self, t):
        f = torch.empty(t.shape, dtype=torch.float32)
        torch.nn.init.orthogonal_(f, self.gain)
        t.copy_(f)


class Bilinear(Initializer):
    def _init(self, t):
        shape = t.shape
        f = math.ceil(shape[3] / 2.0)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        w = np.zeros(shape, dtype=np.float32)
        for i in range(int(np.prod(shape))):
            x = i % shape[3]
            y = (i // shape[3]) % shape[2]
            w.flat[i] = (1 - abs(x / f - c)) * (1 - abs(y / f - c))
        t.copy_(torch.from_numpy(w))


class Dirac(Initializer):
    """Identity-preserving conv init (reference `nn/initializer/dirac.py`): weight
    [out, in, *k] gets 1 at the kernel centre of (g·out/groups + i, i) for i < min(out/groups, in)."""

    def __init__(self, groups=1, name=None):
        self.groups = groups

    def _init(self, t):
        if t.dim() not in (3, 4, 5):
            raise ValueError("Dirac initializer needs a 3-D, 4-D or 5-D conv weight")
        out, cin = t.shape[0], t.shape[1]
        if out % self.groups:
            raise ValueError("out channels must be divisible by groups")
        per = out // self.groups
        t.zero_()
        centre = tuple(k // 2 for k in t.shape[2:])
        for g in range(self.groups):
            for i in range(min(per, cin)):
                t[(g * per + i, i) + centre] = 1.0


def calculate_gain(nonlinearity, param=None):
    """Recommended gain per nonlinearity (reference `nn/initializer/__init__.py:calculate_gain`)."""
    linear = ("sigmoid", "linear", "conv1d", "conv2d", "conv3d", "conv1d_transpose",
              "conv2d_transpose", "conv3d_transpose")
    if nonlinearity in linear:
        return 1.0
    if nonlinearity == "tanh":
        return 5.0 / 3
    if nonlinearity == "relu":
        return math.sqrt(2.0)
    if nonlinearity == "leaky_relu":
        slope = 0.01 if param is None else param
        return math.sqrt(2.0 / (1 + slope ** 2))
    if nonlinearity == "selu":
        return 3.0 / 4
    raise ValueError(f"nonlinearity function {nonlinearity} is not supported")


# fluid-style aliases
ConstantInitializer = Constant
NormalInitializer = Normal
UniformInitializer = Uniform
XavierInitializer = XavierUniform
MSRA = KaimingNormal


def set_global_initializer(weight_init, bias_init=None):
    _GLOBAL_INIT[0], _GLOBAL_INIT[1] = weight_init, bias_init


_GLOBAL_INIT = [None, None]
