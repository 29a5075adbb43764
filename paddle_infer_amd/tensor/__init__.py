"""``paddle.*`` tensor API with Paddle semantics over torch tensors.

Parity: reference `python/paddle/tensor/{creation,math,manipulation,search,logic,linalg,random,
stat,einsum,attribute}.py`. Argument names and semantics follow Paddle (``axis`` not ``dim``,
``perm`` for transpose, 0-means-copy in ``reshape``, ``[values, indices]`` from ``topk``, default
float dtype float32 and int dtype int64). The tensor type is ``torch.Tensor`` so every op runs on
PyTorch-ROCm (hipBLASLt / rocBLAS / MIOpen for library ops) and composes with the framework's
hand-written HIP kernels.
"""
from __future__ import annotations

import builtins
import math as _math

import numpy as np
import torch

from ..framework.dtype import to_torch_dtype as _dt, get_default_dtype

Tensor = torch.Tensor

_builtin_sum, _builtin_max, _builtin_min, _builtin_abs = builtins.sum, builtins.max, builtins.min, builtins.abs


def _dev(place=None):
    from .. import device as _device
    return _device._resolve(place)


def _axis(a):
    if a is None:
        return None
    if isinstance(a, torch.Tensor):
        a = a.tolist()
    if isinstance(a, (list, tuple)):
        return tuple(int(i) for i in a)
    return int(a)


def _shape(shape):
    if isinstance(shape, torch.Tensor):
        return [int(s) for s in shape.tolist()]
    if isinstance(shape, (int, np.integer)):
        return [int(shape)]
    return [int(s.item()) if isinstance(s, torch.Tensor) else int(s) for s in shape]


# ------------------------------------------------------------------------------------ creation
def to_tensor(data, dtype=None, place=None, stop_gradient=True):
    if isinstance(data, torch.Tensor):
        t = data.detach().clone()
    else:
        arr = np.asarray(data)
        if arr.dtype == np.float64 and dtype is None:
            arr = arr.astype(np.float32 if get_default_dtype() == "float32" else arr.dtype)
        t = torch.as_tensor(arr)
    if dtype is not None:
        t = t.to(_dt(dtype))
    t = t.to(_dev(place))
    if not stop_gradient and t.is_floating_point():
        t.requires_grad_(True)
    return t


def zeros(shape, dtype=None, name=None):
    return torch.zeros(_shape(shape), dtype=_dt(dtype), device=_dev())


def ones(shape, dtype=None, name=None):
    return torch.ones(_shape(shape), dtype=_dt(dtype), device=_dev())


def full(shape, fill_value, dtype=None, name=None):
    if dtype is None and isinstance(fill_value, bool):
        dtype = "bool"
    return torch.full(_shape(shape), fill_value, dtype=_dt(dtype), device=_dev())


def empty(shape, dtype=None, name=None):
    return torch.empty(_shape(shape), dtype=_dt(dtype), device=_dev())


def zeros_like(x, dtype=None, name=None):
    return torch.zeros_like(x, dtype=_dt(dtype) if dtype else None)


def ones_like(x, dtype=None, name=None):
    return torch.ones_like(x, dtype=_dt(dtype) if dtype else None)


def full_like(x, fill_value, dtype=None, name=None):
    return torch.full_like(x, fill_value, dtype=_dt(dtype) if dtype else None)


def empty_like(x, dtype=None, name=None):
    return torch.empty_like(x, dtype=_dt(dtype) if dtype else None)


def arange(start=0, end=None, step=1, dtype=None, name=None):
    if end is None:
        start, end = 0, start
    vals = [v.item() if isinstance(v, torch.Tensor) else v for v in (start, end, step)]
    if dtype is None:
        dtype = "int64" if builtins.all(isinstance(v, (int, np.integer)) for v in vals) else None
    return torch.arange(*vals, dtype=_dt(dtype), device=_dev())


def linspace(start, stop, num, dtype=None, name=None):
    return torch.linspace(float(start), float(stop), int(num), dtype=_dt(dtype), device=_dev())


def logspace(start, stop, num, base=10.0, dtype=None, name=None):
    return torch.logspace(float(start), float(stop), int(num), base=base, dtype=_dt(dtype), device=_dev())


def eye(num_rows, num_columns=None, dtype=None, name=None):
    return torch.eye(int(num_rows), int(num_columns or num_rows), dtype=_dt(dtype), device=_dev())


def diag(x, offset=0, padding_value=0, name=None):
    if x.dim() == 1 and padding_value != 0:
        n = x.shape[0] + _builtin_abs(offset)
        out = torch.full((n, n), padding_value, dtype=x.dtype, device=x.device)
        return out + torch.diag(x, offset) - torch.diag(torch.full_like(x, padding_value), offset)
    return torch.diag(x, offset)


def diagflat(x, offset=0, name=None):
    return torch.diagflat(x, offset)


def meshgrid(*args, **kwargs):
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = args[0]
    return list(torch.meshgrid(*args, indexing="ij"))


def tril(x, diagonal=0, name=None):
    return torch.tril(x, diagonal)


def triu(x, diagonal=0, name=None):
    return torch.triu(x, diagonal)


def assign(x, output=None):
    x = x if isinstance(x, torch.Tensor) else to_tensor(x)
    if output is None:
        return x.clone()
    with torch.no_grad():
        output.copy_(x)
    return output


def clone(x, name=None):
    return x.clone()


def complex(real, imag, name=None):
    return torch.complex(real, imag)


# ------------------------------------------------------------------------------------ random
def rand(shape, dtype=None, name=None):
    return torch.rand(_shape(shape), dtype=_dt(dtype), device=_dev())


def randn(shape, dtype=None, name=None):
    return torch.randn(_shape(shape), dtype=_dt(dtype), device=_dev())


standard_normal = randn


def randint(low=0, high=None, shape=(1,), dtype=None, name=None):
    if high is None:
        low, high = 0, low
    return torch.randint(int(low), int(high), _shape(shape), dtype=_dt(dtype or "int64"), device=_dev())


def randint_like(x, low=0, high=None, dtype=None, name=None):
    if high is None:
        low, high = 0, low
    return torch.randint(int(low), int(high), x.shape, dtype=_dt(dtype) if dtype else x.dtype, device=x.device)


def uniform(shape, dtype=None, min=-1.0, max=1.0, seed=0, name=None):
    return torch.empty(_shape(shape), dtype=_dt(dtype), device=_dev()).uniform_(min, max)


def normal(mean=0.0, std=1.0, shape=None, name=None):
    if isinstance(mean, torch.Tensor) or isinstance(std, torch.Tensor):
        return torch.normal(mean, std)
    return torch.normal(float(mean), float(std), _shape(shape), device=_dev())


def randperm(n, dtype="int64", name=None):
    return torch.randperm(int(n), dtype=_dt(dtype), device=_dev())


def multinomial(x, num_samples=1, replacement=False, name=None):
    return torch.multinomial(x, num_samples, replacement)


def bernoulli(x, name=None):
    return torch.bernoulli(x)


def poisson(x, name=None):
    return torch.poisson(x)


# ------------------------------------------------------------------------------------ math
def _binary(fn):
    def op(x, y, name=None):
        return fn(x, y)
    return op


add = _binary(torch.add)
subtract = _binary(torch.sub)
multiply = _binary(torch.mul)
divide = _binary(torch.true_divide)
floor_divide = _binary(torch.floor_divide)
remainder = mod = floor_mod = _binary(torch.remainder)
maximum = _binary(torch.maximum)
minimum = _binary(torch.minimum)
fmax = _binary(torch.fmax)
fmin = _binary(torch.fmin)
atan2 = _binary(torch.atan2)
heaviside = _binary(torch.heaviside)
gcd = _binary(torch.gcd)
lcm = _binary(torch.lcm)
bitwise_and = _binary(torch.bitwise_and)
bitwise_or = _binary(torch.bitwise_or)
bitwise_xor = _binary(torch.bitwise_xor)
logical_and = _binary(torch.logical_and)
logical_or = _binary(torch.logical_or)
logical_xor = _binary(torch.logical_xor)
equal = _binary(torch.eq)
not_equal = _binary(torch.ne)
greater_than = _binary(torch.gt)
greater_equal = _binary(torch.ge)
less_than = _binary(torch.lt)
less_equal = _binary(torch.le)
kron = _binary(torch.kron)
inner = _binary(torch.inner)
outer = _binary(torch.outer)
dot = _binary(lambda x, y: (x * y).sum(-1))
mv = _binary(torch.mv)
def mm(input, mat2, name=None):  # noqa: A002
    """2-D matrix product (bf16 / fp16 CUDA: the framework's own GEMMs, ``ops.gemm.matmul``)."""
    from ..ops.gemm import matmul as _mm
    return _mm(input, mat2)


def bmm(x, y, name=None):
    """Batched [B, M, K] · [B, K, N] (bf16 / fp16 CUDA: one batched assembly-GEMM launch)."""
    from ..ops.gemm import matmul as _mm
    return _mm(x, y)
cross = lambda x, y, axis=9, name=None: torch.cross(x, y, dim=-1 if axis == 9 else axis)  # noqa: E731


def pow(x, y, name=None):  # noqa: A001
    return torch.pow(x, y)


def _unary(fn):
    def op(x, name=None):
        return fn(x)
    return op


for _n in ["abs", "acos", "acosh", "asin", "asinh", "atan", "atanh", "ceil", "cos", "cosh",
           "digamma", "erf", "erfinv", "exp", "expm1", "floor", "frac", "lgamma", "log", "log10",
           "log1p", "log2", "neg", "reciprocal", "round", "rsqrt", "sigmoid", "sign", "sin", "sinh",
           "sqrt", "square", "tan", "tanh", "trunc", "logical_not", "bitwise_not", "isnan", "isinf",
           "isfinite", "conj", "real", "imag", "angle", "deg2rad", "rad2deg", "sgn"]:
    globals()[_n] = _unary(getattr(torch, _n))
for _n in ["exp", "sqrt", "rsqrt", "ceil", "floor", "round", "reciprocal", "tanh", "abs", "sigmoid"]:
    globals()[_n + "_"] = (lambda f: (lambda x, name=None: f(x)))(getattr(torch.Tensor, _n + "_"))


def scale(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    out = x * scale + bias if bias_after_scale else (x + bias) * scale
    return out if act is None else getattr(torch, act)(out)


def clip(x, min=None, max=None, name=None):  # noqa: A002
    return torch.clamp(x, min, max)


def lerp(x, y, weight, name=None):
    return torch.lerp(x, y, weight)


def logit(x, eps=None, name=None):
    return torch.logit(x, eps)


def stanh(x, scale_a=0.67, scale_b=1.7159, name=None):
    return scale_b * torch.tanh(scale_a * x)


def add_n(inputs, name=None):
    if isinstance(inputs, torch.Tensor):
        return inputs
    out = inputs[0]
    for t in inputs[1:]:
        out = out + t
    return out


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):  # noqa: A002
    from ..ops.gemm import own_dtype, matmul as _mm
    if own_dtype(x, y) and x.dim() == 2 and y.dim() == 2:
        out = _mm(x, y, alpha=alpha)
        if beta == 0:  # BLAS beta = 0: C is not read (NaN / inf in `input` do not propagate)
            return out.expand(torch.broadcast_shapes(out.shape, input.shape)).clone() \
                if out.shape != torch.broadcast_shapes(out.shape, input.shape) else out
        return out + (input if beta == 1.0 else beta * input)
    return torch.addmm(input, x, y, beta=beta, alpha=alpha)


def matmul(x, y, transpose_x=False, transpose_y=False, name=None):
    """``paddle.matmul`` (reference `python/paddle/tensor/linalg.py` matmul → phi matmul kernel):
    bf16 / fp16 CUDA operands run the framework's own GEMMs forward and backward (skinny MFMA kernel
    for few rows, assembly GEMM otherwise, one batched launch for batched operands); other dtypes
    take PyTorch."""
    from ..ops.gemm import matmul as _mm
    return _mm(x, y, transpose_x, transpose_y)


def einsum(equation, *operands):
    if len(operands) == 1 and isinstance(operands[0], (list, tuple)):
        operands = operands[0]
    return torch.einsum(equation, *operands)


def multi_dot(x, name=None):
    return torch.linalg.multi_dot(x)


def _reduce(fn, x, axis=None, keepdim=False, dtype=None):
    ax = _axis(axis)
    if dtype is not None:
        x = x.to(_dt(dtype))
    if ax is None or ax == ():
        out = fn(x)
        return out.reshape([1] * x.dim()) if keepdim else out
    return fn(x, dim=ax, keepdim=keepdim)


def sum(x, axis=None, dtype=None, keepdim=False, name=None):  # noqa: A001
    if dtype is None and x.dtype == torch.bool:
        dtype = "int64"
    return _reduce(torch.sum, x, axis, keepdim, dtype)


def nansum(x, axis=None, dtype=None, keepdim=False, name=None):
    return _reduce(torch.nansum, x, axis, keepdim, dtype)


def mean(x, axis=None, keepdim=False, name=None):
    return _reduce(torch.mean, x, axis, keepdim)


def nanmean(x, axis=None, keepdim=False, name=None):
    return _reduce(torch.nanmean, x, axis, keepdim)


def prod(x, axis=None, keepdim=False, dtype=None, name=None):
    ax = _axis(axis)
    if dtype is not None:
        x = x.to(_dt(dtype))
    if ax is None:
        return torch.prod(x)
    if isinstance(ax, tuple):
        for a in sorted(ax, reverse=True):
            x = torch.prod(x, a, keepdim=keepdim)
        return x
    return torch.prod(x, ax, keepdim=keepdim)


def _minmax(fn, x, axis, keepdim):
    ax = _axis(axis)
    if ax is None:
        return fn(x)
    if isinstance(ax, tuple):
        return torch.amax(x, ax, keepdim) if fn is torch.max else torch.amin(x, ax, keepdim)
    return fn(x, ax, keepdim=keepdim).values


def max(x, axis=None, keepdim=False, name=None):  # noqa: A001
    return _minmax(torch.max, x, axis, keepdim)


def min(x, axis=None, keepdim=False, name=None):  # noqa: A001
    return _minmax(torch.min, x, axis, keepdim)


def amax(x, axis=None, keepdim=False, name=None):
    return torch.amax(x, _axis(axis) if axis is not None else tuple(range(x.dim())), keepdim)


def amin(x, axis=None, keepdim=False, name=None):
    return torch.amin(x, _axis(axis) if axis is not None else tuple(range(x.dim())), keepdim)


def logsumexp(x, axis=None, keepdim=False, name=None):
    ax = _axis(axis)
    return torch.logsumexp(x, ax if ax is not None else tuple(range(x.dim())), keepdim)


def std(x, axis=None, unbiased=True, keepdim=False, name=None):
    ax = _axis(axis)
    return torch.std(x, dim=ax, unbiased=unbiased, keepdim=keepdim) if ax is not None else torch.std(x, unbiased=unbiased)


def var(x, axis=None, unbiased=True, keepdim=False, name=None):
    ax = _axis(axis)
    return torch.var(x, dim=ax, unbiased=unbiased, keepdim=keepdim) if ax is not None else torch.var(x, unbiased=unbiased)


def median(x, axis=None, keepdim=False, name=None):
    if axis is None:
        return torch.quantile(x.float().flatten(), 0.5)
    return torch.quantile(x.float(), 0.5, dim=axis, keepdim=keepdim)


def quantile(x, q, axis=None, keepdim=False, name=None):
    return torch.quantile(x.float(), torch.as_tensor(q, dtype=torch.float32, device=x.device), dim=axis, keepdim=keepdim)


def cumsum(x, axis=None, dtype=None, name=None):
    if axis is None:
        x, axis = x.flatten(), 0
    return torch.cumsum(x, axis, dtype=_dt(dtype) if dtype else None)


def cumprod(x, dim=None, dtype=None, name=None):
    if dim is None:
        x, dim = x.flatten(), 0
    return torch.cumprod(x, dim, dtype=_dt(dtype) if dtype else None)


def logcumsumexp(x, axis=None, dtype=None, name=None):
    if axis is None:
        x, axis = x.flatten(), 0
    return torch.logcumsumexp(x, axis)


def diff(x, n=1, axis=-1, prepend=None, append=None, name=None):
    return torch.diff(x, n, axis, prepend, append)


def trace(x, offset=0, axis1=0, axis2=1, name=None):
    return torch.diagonal(x, offset, axis1, axis2).sum(-1)


def diagonal(x, offset=0, axis1=0, axis2=1, name=None):
    return torch.diagonal(x, offset, axis1, axis2)


def all(x, axis=None, keepdim=False, name=None):  # noqa: A001
    return _reduce(torch.all, x, axis, keepdim)


def any(x, axis=None, keepdim=False, name=None):  # noqa: A001
    return _reduce(torch.any, x, axis, keepdim)


def count_nonzero(x, axis=None, keepdim=False, name=None):
    return sum(x != 0, axis, keepdim=keepdim)


def allclose(x, y, rtol=1e-5, atol=1e-8, equal_nan=False, name=None):
    return torch.tensor(torch.allclose(x, y, rtol, atol, equal_nan))


def isclose(x, y, rtol=1e-5, atol=1e-8, equal_nan=False, name=None):
    return torch.isclose(x, y, rtol, atol, equal_nan)


def equal_all(x, y, name=None):
    return torch.tensor(torch.equal(x, y))


def increment(x, value=1.0, name=None):
    with torch.no_grad():
        x.add_(value)
    return x


def cast(x, dtype):
    return x.to(_dt(dtype))


def numel(x, name=None):
    return torch.tensor(x.numel(), dtype=torch.int64)


def shape(x):
    return torch.tensor(list(x.shape), dtype=torch.int32)


def rank(x):
    return torch.tensor(x.dim(), dtype=torch.int32)


def is_tensor(x):
    return isinstance(x, torch.Tensor)


def is_floating_point(x):
    return x.is_floating_point()


def is_integer(x):
    return not x.is_floating_point() and not x.is_complex() and x.dtype != torch.bool


def is_complex(x):
    return x.is_complex()


def is_empty(x, name=None):
    return torch.tensor(x.numel() == 0)


def broadcast_shape(x_shape, y_shape):
    return list(torch.broadcast_shapes(tuple(x_shape), tuple(y_shape)))


def broadcast_tensors(input, name=None):  # noqa: A002
    return list(torch.broadcast_tensors(*input))


# ------------------------------------------------------------------------------------ manipulation
def reshape(x, shape, name=None):
    s = _shape(shape)
    s = [x.shape[i] if v == 0 else v for i, v in enumerate(s)]
    return x.reshape(s)


def reshape_(x, shape, name=None):
    return reshape(x, shape)


def transpose(x, perm, name=None):
    return x.permute(*perm)


def moveaxis(x, source, destination, name=None):
    return torch.movedim(x, source, destination)


def t(x, name=None):
    return x.t() if x.dim() == 2 else x


def concat(x, axis=0, name=None):
    return torch.cat(list(x), int(axis))


def stack(x, axis=0, name=None):
    return torch.stack(list(x), axis)


def unstack(x, axis=0, num=None):
    return list(torch.unbind(x, axis))


def unbind(input, axis=0):  # noqa: A002
    return list(torch.unbind(input, axis))


def split(x, num_or_sections, axis=0, name=None):
    axis = int(axis) % x.dim()
    n = x.shape[axis]
    if isinstance(num_or_sections, int):
        return list(torch.split(x, n // num_or_sections, axis))
    secs = list(num_or_sections)
    if -1 in secs:
        i = secs.index(-1)
        secs[i] = n - _builtin_sum(s for s in secs if s != -1)
    return list(torch.split(x, secs, axis))


def chunk(x, chunks, axis=0, name=None):
    return list(torch.chunk(x, chunks, axis))


def squeeze(x, axis=None, name=None):
    if axis is None:
        return x.squeeze()
    ax = _axis(axis)
    ax = ax if isinstance(ax, tuple) else (ax,)
    ax = tuple(a % x.dim() for a in ax if x.shape[a] == 1)
    return x.squeeze(ax) if ax else x


def unsqueeze(x, axis, name=None):
    ax = _axis(axis)
    if isinstance(ax, tuple):
        for a in sorted(a if a >= 0 else a + x.dim() + len(ax) for a in ax):
            x = x.unsqueeze(a)
        return x
    return x.unsqueeze(ax)


squeeze_, unsqueeze_ = squeeze, unsqueeze


def flatten(x, start_axis=0, stop_axis=-1, name=None):
    return torch.flatten(x, start_axis, stop_axis)


def expand(x, shape, name=None):
    s = _shape(shape)
    return x.expand(*[x.shape[i - (len(s) - x.dim())] if v == -1 else v for i, v in enumerate(s)])


def expand_as(x, y, name=None):
    return x.expand_as(y)


def broadcast_to(x, shape, name=None):
    return expand(x, shape)


def tile(x, repeat_times, name=None):
    return x.repeat(*_shape(repeat_times)) if len(_shape(repeat_times)) >= x.dim() else \
        x.repeat(*([1] * (x.dim() - len(_shape(repeat_times))) + _shape(repeat_times)))


def repeat_interleave(x, repeats, axis=None, name=None):
    return torch.repeat_interleave(x, repeats, axis)


def flip(x, axis, name=None):
    ax = _axis(axis)
    return torch.flip(x, ax if isinstance(ax, tuple) else (ax,))


def roll(x, shifts, axis=None, name=None):
    return torch.roll(x, shifts, axis)


def rot90(x, k=1, axes=(0, 1), name=None):
    return torch.rot90(x, k, axes)


def gather(x, index, axis=0, name=None):
    return torch.index_select(x, int(axis), index.reshape(-1).long())


def gather_nd(x, index, name=None):
    idx = index.long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    out = x[tuple(flat[:, i] for i in range(k))]
    return out.reshape(*idx.shape[:-1], *x.shape[k:])


def take_along_axis(arr, indices, axis, broadcast=True):
    return torch.take_along_dim(arr, indices.long(), axis)


def put_along_axis(arr, indices, values, axis, reduce="assign"):
    values = values if isinstance(values, torch.Tensor) else torch.full_like(arr, values)
    values = values.expand_as(indices) if values.shape != indices.shape else values
    if reduce == "assign":
        return arr.scatter(axis, indices.long(), values)
    return arr.scatter_reduce(axis, indices.long(), values, {"add": "sum", "multiply": "prod", "mul": "prod"}[reduce])


def take(x, index, mode="raise", name=None):
    return torch.take(x, index.long())


def index_select(x, index, axis=0, name=None):
    return torch.index_select(x, axis, index.long())


def index_sample(x, index):
    return torch.gather(x, 1, index.long())


def index_add(x, index, axis, value, name=None):
    return x.index_add(axis, index.long(), value)


def scatter(x, index, updates, overwrite=True, name=None):
    idx = index.long().reshape(-1)
    if overwrite:
        out = x.clone()
        out[idx] = updates
        return out
    out = x.clone()
    out[idx] = 0
    return out.index_add(0, idx, updates)


def scatter_(x, index, updates, overwrite=True, name=None):
    with torch.no_grad():
        x.copy_(scatter(x, index, updates, overwrite))
    return x


def scatter_nd_add(x, index, updates, name=None):
    idx = index.long()
    k = idx.shape[-1]
    out = x.clone()
    flat = idx.reshape(-1, k)
    out.index_put_(tuple(flat[:, i] for i in range(k)), updates.reshape(flat.shape[0], *x.shape[k:]), accumulate=True)
    return out


def scatter_nd(index, updates, shape, name=None):
    return scatter_nd_add(torch.zeros(_shape(shape), dtype=updates.dtype, device=updates.device), index, updates)


def slice(input, axes, starts, ends):  # noqa: A001,A002
    sl = [builtins.slice(None)] * input.dim()
    for a, s, e in zip(axes, starts, ends):
        s = int(s.item()) if isinstance(s, torch.Tensor) else int(s)
        e = int(e.item()) if isinstance(e, torch.Tensor) else int(e)
        sl[a] = builtins.slice(s, e)
    return input[tuple(sl)]


def strided_slice(x, axes, starts, ends, strides, name=None):
    sl = [builtins.slice(None)] * x.dim()
    for a, s, e, st in zip(axes, starts, ends, strides):
        sl[a] = builtins.slice(int(s), int(e), int(st))
    if builtins.any(st < 0 for st in strides):
        out = x
        for a, s, e, st in zip(axes, starts, ends, strides):
            idx = torch.arange(int(s), int(e), int(st), device=x.device)
            idx = idx[(idx >= 0) & (idx < x.shape[a])]
            out = out.index_select(a, idx)
        return out
    return x[tuple(sl)]


def masked_select(x, mask, name=None):
    return torch.masked_select(x, mask)


def masked_fill(x, mask, value, name=None):
    return x.masked_fill(mask, value)


def where(condition, x=None, y=None, name=None):
    if x is None and y is None:
        return nonzero(condition, as_tuple=True)
    return torch.where(condition, x, y)


def nonzero(x, as_tuple=False):
    return torch.nonzero(x, as_tuple=as_tuple)


def unique(x, return_index=False, return_inverse=False, return_counts=False, axis=None,
           dtype="int64", name=None):
    out = torch.unique(x, sorted=True, return_inverse=return_inverse or return_index,
                       return_counts=return_counts, dim=axis)
    if not (return_index or return_inverse or return_counts):
        return out
    res = [out[0]] if isinstance(out, tuple) else [out]
    if return_index:
        inv = out[1]
        perm = torch.arange(inv.shape[0], device=inv.device)
        first = torch.full((res[0].shape[0],), inv.shape[0], dtype=torch.long, device=inv.device)
        first = first.scatter_reduce(0, inv, perm, "amin")
        res.append(first)
    if return_inverse:
        res.append(out[1])
    if return_counts:
        res.append(out[-1])
    return tuple(res)


def unique_consecutive(x, return_inverse=False, return_counts=False, axis=None, dtype="int64", name=None):
    return torch.unique_consecutive(x, return_inverse=return_inverse, return_counts=return_counts, dim=axis)


def pad(x, pad, mode="constant", value=0.0, data_format="NCHW", name=None):
    from ..nn import functional as F
    return F.pad(x, pad, mode, value, data_format)


def crop(x, shape=None, offsets=None, name=None):
    offsets = offsets or [0] * x.dim()
    sl = tuple(builtins.slice(o, o + (s if s != -1 else x.shape[i] - o)) for i, (o, s) in enumerate(zip(offsets, shape)))
    return x[sl]


def as_complex(x, name=None):
    return torch.view_as_complex(x)


def as_real(x, name=None):
    return torch.view_as_real(x)


def shard_index(input, index_num, nshards, shard_id, ignore_value=-1):  # noqa: A002
    size = (index_num + nshards - 1) // nshards
    lo = shard_id * size
    inr = (input >= lo) & (input < lo + size)
    return torch.where(inr, input - lo, torch.full_like(input, ignore_value))


# ------------------------------------------------------------------------------------ search / sort
def argmax(x, axis=None, keepdim=False, dtype="int64", name=None):
    if axis is None:
        return torch.argmax(x).to(_dt(dtype))
    return torch.argmax(x, axis, keepdim).to(_dt(dtype))


def argmin(x, axis=None, keepdim=False, dtype="int64", name=None):
    if axis is None:
        return torch.argmin(x).to(_dt(dtype))
    return torch.argmin(x, axis, keepdim).to(_dt(dtype))


def argsort(x, axis=-1, descending=False, name=None):
    return torch.argsort(x, axis, descending)


def sort(x, axis=-1, descending=False, name=None):
    return torch.sort(x, axis, descending).values


def topk(x, k, axis=-1, largest=True, sorted=True, name=None):  # noqa: A002
    k = int(k.item()) if isinstance(k, torch.Tensor) else int(k)
    r = torch.topk(x, k, axis, largest, sorted)
    return r.values, r.indices


def kthvalue(x, k, axis=-1, keepdim=False, name=None):
    r = torch.kthvalue(x, k, axis, keepdim)
    return r.values, r.indices


def mode(x, axis=-1, keepdim=False, name=None):
    r = torch.mode(x, axis, keepdim)
    return r.values, r.indices


def searchsorted(sorted_sequence, values, out_int32=False, right=False, name=None):
    return torch.searchsorted(sorted_sequence, values, out_int32=out_int32, right=right)


def bucketize(x, sorted_sequence, out_int32=False, right=False, name=None):
    return torch.bucketize(x, sorted_sequence, out_int32=out_int32, right=right)


def bincount(x, weights=None, minlength=0, name=None):
    return torch.bincount(x, weights, minlength)


def histogram(input, bins=100, min=0, max=0, name=None):  # noqa: A002
    return torch.histc(input.float(), bins, min, max).long()


# ------------------------------------------------------------------------------------ linalg
def norm(x, p="fro", axis=None, keepdim=False, name=None):
    ax = _axis(axis)
    if p == "fro":
        p = 2 if (ax is None or isinstance(ax, int)) else "fro"
        if ax is None:
            return torch.linalg.vector_norm(x.flatten(), 2)
    if isinstance(p, str):
        return torch.linalg.matrix_norm(x, p, dim=ax if ax is not None else (-2, -1), keepdim=keepdim)
    return torch.linalg.vector_norm(x, float(p), dim=ax, keepdim=keepdim)


def dist(x, y, p=2, name=None):
    return torch.dist(x, y, p)


def inverse(x, name=None):
    return torch.linalg.inv(x)


def cholesky(x, upper=False, name=None):
    return torch.linalg.cholesky(x, upper=upper)


def matrix_power(x, n, name=None):
    return torch.linalg.matrix_power(x, n)


def tensordot(x, y, axes=2, name=None):
    return torch.tensordot(x, y, axes)


class linalg:  # namespace: paddle.linalg
    norm = staticmethod(norm)
    inv = staticmethod(inverse)
    cholesky = staticmethod(cholesky)
    matrix_power = staticmethod(matrix_power)
    multi_dot = staticmethod(multi_dot)
    det = staticmethod(lambda x, name=None: torch.linalg.det(x))
    slogdet = staticmethod(lambda x, name=None: torch.stack(list(torch.linalg.slogdet(x))))
    qr = staticmethod(lambda x, mode="reduced", name=None: tuple(torch.linalg.qr(x, mode)))
    svd = staticmethod(lambda x, full_matrices=False, name=None: tuple(torch.linalg.svd(x, full_matrices)))
    eig = staticmethod(lambda x, name=None: tuple(torch.linalg.eig(x)))
    eigh = staticmethod(lambda x, UPLO="L", name=None: tuple(torch.linalg.eigh(x, UPLO)))
    eigvals = staticmethod(lambda x, name=None: torch.linalg.eigvals(x))
    eigvalsh = staticmethod(lambda x, UPLO="L", name=None: torch.linalg.eigvalsh(x, UPLO))
    solve = staticmethod(lambda x, y, name=None: torch.linalg.solve(x, y))
    lstsq = staticmethod(lambda x, y, rcond=None, driver=None, name=None: tuple(torch.linalg.lstsq(x, y, rcond)))
    pinv = staticmethod(lambda x, rcond=1e-15, hermitian=False, name=None: torch.linalg.pinv(x, rtol=rcond, hermitian=hermitian))
    matrix_rank = staticmethod(lambda x, tol=None, hermitian=False, name=None: torch.linalg.matrix_rank(x, tol=tol, hermitian=hermitian))
    cond = staticmethod(lambda x, p=None, name=None: torch.linalg.cond(x, p))
    cov = staticmethod(lambda x, rowvar=True, ddof=True, fweights=None, aweights=None, name=None: torch.cov(x if rowvar else x.t(), correction=int(ddof), fweights=fweights, aweights=aweights))
    corrcoef = staticmethod(lambda x, rowvar=True, name=None: torch.corrcoef(x if rowvar else x.t()))
    cross = staticmethod(cross)
    lu = staticmethod(lambda x, pivot=True, get_infos=False, name=None: tuple(torch.linalg.lu_factor(x)))
    triangular_solve = staticmethod(lambda x, y, upper=True, transpose=False, unitriangular=False, name=None: torch.linalg.solve_triangular(x.transpose(-1, -2) if transpose else x, y, upper=upper != transpose, unitriangular=unitriangular))
    cholesky_solve = staticmethod(lambda x, y, upper=False, name=None: torch.cholesky_solve(x, y, upper))

    lu_unpack = staticmethod(lambda x, y, unpack_ludata=True, unpack_pivots=True, name=None:
                             tuple(torch.lu_unpack(x, y, unpack_ludata, unpack_pivots)))


# ------------------------------------------------------------------------------------ misc
def nanmedian(x, axis=None, keepdim=True, name=None):
    if axis is None:
        v = torch.nanmedian(x.flatten())
        return v.reshape([1] * x.dim()) if keepdim else v
    return torch.nanmedian(x, dim=axis, keepdim=keepdim).values


def nanquantile(x, q, axis=None, keepdim=False, name=None):
    return torch.nanquantile(x.float(), torch.as_tensor(q, dtype=torch.float32, device=x.device),
                             dim=axis, keepdim=keepdim)


def multiplex(inputs, index, name=None):
    """out[i] = inputs[index[i]][i] (reference `tensor/math.py:multiplex`)."""
    stacked = torch.stack(list(inputs), 0)
    idx = index.reshape(-1).long()
    return stacked[idx, torch.arange(idx.numel(), device=idx.device)]


def renorm(x, p, axis, max_norm):
    return torch.renorm(x, p, axis, max_norm)


def reverse(x, axis, name=None):
    return flip(x, axis)


def tolist(x):
    return x.tolist()


def tril_indices(row, col, offset=0, dtype="int64"):
    return torch.tril_indices(row, col, offset)


def triu_indices(row, col=None, offset=0, dtype="int64"):
    return torch.triu_indices(row, row if col is None else col, offset)


def index_add_(x, index, axis, value, name=None):
    return x.index_add_(axis, index.long(), value)


def check_shape(shape):
    """Validate a shape argument (list/tuple of ints ≥ -1, or an int tensor)."""
    if isinstance(shape, torch.Tensor):
        if shape.dtype not in (torch.int32, torch.int64):
            raise TypeError("shape tensor must be int32 or int64")
        return
    for s in shape:
        if isinstance(s, torch.Tensor):
            continue
        if not isinstance(s, int) or s < -1:
            raise ValueError(f"invalid shape entry {s!r}")


def __getattr__(name):
    raise AttributeError(f"paddle_infer_amd.tensor has no attribute {name}")


_math  # noqa
from ..ops.search import beam_search_softmax  # noqa: E402,F401
