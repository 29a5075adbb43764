"""``paddle.sparse`` (reference `python/paddle/sparse/`): COO / CSR sparse tensors and their
unary, binary and matmul ops, on torch's sparse layouts (rocSPARSE / hipSPARSE kernels for
sparse × dense products on MI355X). Unary ops act on the stored values only (zeros stay zero),
like the reference."""
from __future__ import annotations

import torch

from . import nn  # noqa: F401

__all__ = ["sparse_coo_tensor", "sparse_csr_tensor", "sin", "tan", "asin", "atan", "sinh", "tanh",
           "asinh", "atanh", "sqrt", "square", "log1p", "abs", "pow", "cast", "neg", "deg2rad",
           "rad2deg", "expm1", "mv", "matmul", "masked_matmul", "addmm", "add", "subtract",
           "transpose", "multiply", "divide", "coalesce", "is_same_shape", "reshape", "sum",
           "relu", "isnan", "slice"]


def sparse_coo_tensor(indices, values, shape=None, dtype=None, place=None, stop_gradient=True):
    from ..framework.dtype import to_torch_dtype
    idx = torch.as_tensor(indices).long()
    val = torch.as_tensor(values)
    if dtype is not None:
        val = val.to(to_torch_dtype(dtype))
    t = torch.sparse_coo_tensor(idx, val, size=shape).coalesce()
    return t.requires_grad_(not stop_gradient) if t.is_floating_point() else t


def sparse_csr_tensor(crows, cols, values, shape, dtype=None, place=None, stop_gradient=True):
    from ..framework.dtype import to_torch_dtype
    val = torch.as_tensor(values)
    if dtype is not None:
        val = val.to(to_torch_dtype(dtype))
    return torch.sparse_csr_tensor(torch.as_tensor(crows).long(), torch.as_tensor(cols).long(), val,
                                   size=shape)


def _unary(fn):
    def op(x, name=None):
        if x.layout == torch.sparse_coo:
            x = x.coalesce()
            return torch.sparse_coo_tensor(x.indices(), fn(x.values()), x.shape).coalesce()
        if x.layout == torch.sparse_csr:
            return torch.sparse_csr_tensor(x.crow_indices(), x.col_indices(), fn(x.values()), x.shape)
        return fn(x)
    return op


sin, tan, asin, atan = map(_unary, (torch.sin, torch.tan, torch.asin, torch.atan))
sinh, tanh, asinh, atanh = map(_unary, (torch.sinh, torch.tanh, torch.asinh, torch.atanh))
sqrt, square, log1p, abs = map(_unary, (torch.sqrt, torch.square, torch.log1p, torch.abs))  # noqa: A001
neg, expm1, relu = map(_unary, (torch.neg, torch.expm1, torch.relu))
deg2rad, rad2deg = _unary(torch.deg2rad), _unary(torch.rad2deg)
isnan = _unary(torch.isnan)


def pow(x, factor, name=None):  # noqa: A001
    return _unary(lambda v: torch.pow(v, factor))(x)


def cast(x, index_dtype=None, value_dtype=None, name=None):
    from ..framework.dtype import to_torch_dtype
    x = x.coalesce() if x.layout == torch.sparse_coo else x
    if x.layout == torch.sparse_coo:
        idx = x.indices().to(to_torch_dtype(index_dtype)) if index_dtype else x.indices()
        val = x.values().to(to_torch_dtype(value_dtype)) if value_dtype else x.values()
        return torch.sparse_coo_tensor(idx.long(), val, x.shape)
    val = x.values().to(to_torch_dtype(value_dtype)) if value_dtype else x.values()
    return torch.sparse_csr_tensor(x.crow_indices(), x.col_indices(), val, x.shape)


def coalesce(x, name=None):
    return x.coalesce()


def is_same_shape(x, y):
    return tuple(x.shape) == tuple(y.shape)


def _bin(fn):
    def op(x, y, name=None):
        csr = x.layout == torch.sparse_csr
        a = x.to_sparse_coo() if csr else x
        b = y.to_sparse_coo() if getattr(y, "layout", None) == torch.sparse_csr else y
        r = fn(a, b)
        if r.layout == torch.sparse_coo:
            r = r.coalesce()
        return r.to_sparse_csr() if csr and r.layout == torch.sparse_coo else r
    return op


add = _bin(torch.add)
subtract = _bin(torch.sub)
multiply = _bin(torch.mul)


def divide(x, y, name=None):
    if isinstance(y, (int, float)):
        return _unary(lambda v: v / y)(x)
    # sparse / sparse on the shared pattern (reference semantics: same sparsity)
    xd, yd = x.to_dense(), y.to_dense()
    out = torch.where(xd != 0, xd / yd, torch.zeros_like(xd))
    return out.to_sparse_csr() if x.layout == torch.sparse_csr else out.to_sparse()


def matmul(x, y, name=None):
    return torch.sparse.mm(x, y) if x.layout in (torch.sparse_coo, torch.sparse_csr) else x @ y


def masked_matmul(x, y, mask, name=None):
    """dense x @ dense y evaluated only at ``mask``'s non-zeros (SDDMM)."""
    full = x @ y
    if mask.layout == torch.sparse_csr:
        m = mask.to_sparse_coo().coalesce()
        idx = m.indices()
        return torch.sparse_coo_tensor(idx, full[idx[0], idx[1]], full.shape).to_sparse_csr()
    m = mask.coalesce()
    idx = m.indices()
    return torch.sparse_coo_tensor(idx, full[tuple(idx)], full.shape).coalesce()


def mv(x, vec, name=None):
    return torch.mv(x, vec) if x.layout == torch.sparse_coo else (x @ vec.unsqueeze(-1)).squeeze(-1)


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):  # noqa: A002
    return beta * input + alpha * matmul(x, y)


def transpose(x, perm, name=None):
    d = x.to_dense().permute(*perm)
    return d.to_sparse_csr() if x.layout == torch.sparse_csr else d.to_sparse()


def reshape(x, shape, name=None):
    d = x.to_dense().reshape(shape)
    return d.to_sparse_csr() if x.layout == torch.sparse_csr else d.to_sparse()


def sum(x, axis=None, dtype=None, keepdim=False, name=None):  # noqa: A001
    if axis is None:
        return torch.sparse.sum(x.coalesce() if x.layout == torch.sparse_coo else x.to_sparse_coo())
    return torch.sparse.sum(x.coalesce() if x.layout == torch.sparse_coo else x.to_sparse_coo(), dim=axis)


def slice(x, axes, starts, ends, name=None):  # noqa: A001
    d = x.to_dense()
    for a, s, e in zip(axes, starts, ends):
        d = d.narrow(a, s, min(e, d.shape[a]) - s)
    return d.to_sparse_csr() if x.layout == torch.sparse_csr else d.to_sparse()
