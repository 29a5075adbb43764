"""The long tail of Paddle program op types: the math / linear-algebra / creation / manipulation /
loss / metric ops, the remaining optimizer ops (``adadelta``, ``adagrad``, ``adamax``, ``lamb``,
``rmsprop``, ``lars_momentum``, ``merged_adam``, ``merged_momentum``), static grad clipping
(``squared_l2_norm``, ``clip_by_norm``), the static distributed ops (``c_allgather``,
``c_reducescatter``, ``alltoall``, ``sync_batch_norm``), RNN ops (``cudnn_lstm``, ``lstm``,
``gru``, ``gru_unit``, ``lstm_unit``), interpolation (``linear_interp(_v2)`` /
``trilinear_interp(_v2)``), detection (``matrix_nms``, ``generate_proposals(_v2)``,
``distribute_fpn_proposals``, ``psroi_pool``, ``yolov3_loss``, …) and the fork's serving ops
(``weight_quantize``, ``weight_dequantize``, ``weight_only_linear2``, ``flash_attn_unpadded``,
``fused_moe_kernel``, ``number_count_v2``).

Slot and attribute names follow the reference op makers (fluid ``AddInput`` / ``AddOutput`` /
``AddAttr``) and, for the ops that only exist in `paddle/phi/api/yaml/ops.yaml` (static ops
generated from the yaml: lower-case slot names), the yaml argument names — every kernel reads a
slot under both spellings. Kernels are differentiable compositions of the framework's ops (the
``<type>_grad`` OpDescs run as the forward's VJP, `static/executor.py`), routed to the framework's
HIP kernels where one exists (GEMMs, attention, weight-only GEMM, batch-norm statistics, MoE).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from .ops_registry import REGISTRY, register, _dt, _bcast, _lr, _reg, _skip


# ------------------------------------------------------------------------------------- helpers
def _in(ins, *names, default=None):
    """First tensor present under any of ``names`` (fluid CamelCase or yaml lower-case)."""
    for n in names:
        v = ins.get(n)
        if v:
            return v[0]
    return default


def _inl(ins, *names):
    for n in names:
        v = ins.get(n)
        if v:
            return list(v)
    return []


def _x(ins):
    return _in(ins, "X", "x", "Input", "input")


def _at(a, *names, default=None):
    for n in names:
        if n in a and a[n] is not None:
            return a[n]
    return default


def _out(v, *extra):
    """``{"Out": v, "out": v, ...}``: the op writes whichever slot its desc names."""
    d = {"Out": v, "out": v, "Output": v}
    for e in extra:
        d[e] = v
    return d


def _shape(ins, a, key="shape"):
    if ins.get("ShapeTensor"):
        return [int(v) for v in ins["ShapeTensor"][0].reshape(-1).tolist()]
    if ins.get("ShapeTensorList"):
        return [int(t.reshape(-1)[0]) for t in ins["ShapeTensorList"]]
    return [int(v) for v in (a.get(key) or [])]


def _dtype(a, key="dtype", default="float32"):
    v = a.get(key)
    if v is None or v == -1:
        from ..framework.dtype import to_torch_dtype
        return to_torch_dtype(default)
    if isinstance(v, str):
        from ..framework.dtype import to_torch_dtype
        return to_torch_dtype(v)
    return _dt(v)


def _dev(ins):
    for v in ins.values():
        for t in v:
            if isinstance(t, torch.Tensor):
                return t.device
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def _reduce_dims(x, a, dim_key="dim"):
    if a.get("reduce_all") or a.get(dim_key) in (None, [], ()):
        return tuple(range(x.dim()))
    d = a[dim_key]
    return tuple(int(i) for i in (d if isinstance(d, (list, tuple)) else [d]))


def _unary(name, fn):
    register(name)(lambda ins, a, _f=fn: _out(_f(_x(ins), a)))


# ----------------------------------------------------------------------- unary math / activation
for _n, _f in [("acos", torch.acos), ("acosh", torch.acosh), ("asin", torch.asin), ("asinh", torch.asinh),
               ("atan", torch.atan), ("atanh", torch.atanh), ("cosh", torch.cosh), ("sinh", torch.sinh),
               ("tan", torch.tan), ("expm1", torch.expm1), ("log10", torch.log10), ("log2", torch.log2),
               ("erfinv", torch.erfinv), ("lgamma", torch.lgamma), ("digamma", torch.digamma),
               ("trunc", torch.trunc), ("angle", torch.angle), ("conj", torch.conj_physical),
               ("real", torch.real), ("imag", torch.imag), ("bitwise_not", torch.bitwise_not),
               ("isinf_v2", torch.isinf), ("isnan_v2", torch.isnan), ("sign", torch.sign)]:
    if _n not in REGISTRY:
        _unary(_n, lambda x, a, _f=_f: _f(x))

_unary("logit", lambda x, a: torch.logit(x, float(_at(a, "eps", default=1e-6)) or None))
_unary("celu", lambda x, a: F.celu(x, float(_at(a, "alpha", default=1.0))))
_unary("brelu", lambda x, a: torch.clamp(x, float(_at(a, "t_min", default=0.0)), float(_at(a, "t_max", default=24.0))))
_unary("hard_shrink", lambda x, a: F.hardshrink(x, float(_at(a, "threshold", default=0.5))))
_unary("soft_shrink", lambda x, a: F.softshrink(x, float(_at(a, "lambda", default=0.5))))
_unary("softshrink", lambda x, a: F.softshrink(x, float(_at(a, "lambda", default=0.5))))
_unary("thresholded_relu", lambda x, a: torch.where(x > float(_at(a, "threshold", default=1.0)), x,
                                                     torch.zeros_like(x)))
_unary("selu", lambda x, a: float(_at(a, "scale", default=1.0507009873554805)) *
       torch.where(x > 0, x, float(_at(a, "alpha", default=1.6732632423543772)) * torch.expm1(x)))
_unary("mean_all", lambda x, a: x.mean())
_unary("l1_norm", lambda x, a: x.abs().sum())
_unary("squared_l2_norm", lambda x, a: (x.float() * x.float()).sum().reshape(1).to(x.dtype))
_unary("size", lambda x, a: torch.tensor(x.numel(), dtype=torch.int64, device=x.device))
_unary("is_empty", lambda x, a: torch.tensor(x.numel() == 0, device=x.device))
_unary("isinf", lambda x, a: torch.isinf(x).any().reshape(1))
_unary("isnan", lambda x, a: torch.isnan(x).any().reshape(1))
_unary("isfinite", lambda x, a: torch.isfinite(x).all().reshape(1))
_unary("reverse", lambda x, a: torch.flip(x, [int(i) for i in _at(a, "axis", default=[0])]))
_unary("cumprod", lambda x, a: torch.cumprod(x, int(_at(a, "dim", default=-1))))
_unary("renorm", lambda x, a: torch.renorm(x, float(a.get("p", 2.0)), int(a.get("axis", 0)),
                                            float(a.get("max_norm", 1.0))))
_unary("matrix_power", lambda x, a: torch.linalg.matrix_power(x, int(a.get("n", 1))))
_unary("inverse", lambda x, a: torch.linalg.inv(x))
_unary("cholesky", lambda x, a: torch.linalg.cholesky(x, upper=bool(a.get("upper", False))))
_unary("eigvals", lambda x, a: torch.linalg.eigvals(x))
_unary("exponential", lambda x, a: torch.empty_like(x).exponential_(float(a.get("lambda", 1.0))))
_unary("exponential_", lambda x, a: x.exponential_(float(a.get("lambda", 1.0))))
_unary("bernoulli", lambda x, a: torch.bernoulli(x))
_unary("poisson", lambda x, a: torch.poisson(x))
_unary("dirichlet", lambda x, a: torch.distributions.Dirichlet(x).sample())
_unary("identity_loss", lambda x, a: {0: x.sum(), 1: x.mean(), 2: x}.get(int(a.get("reduction", 1)), x.mean()))


@register("logsumexp")
def _logsumexp(ins, a):
    x = _x(ins)
    dims = tuple(range(x.dim())) if a.get("reduce_all") or not a.get("axis") else tuple(a["axis"])
    return _out(torch.logsumexp(x, dims, keepdim=bool(a.get("keepdim", False))))


@register("logcumsumexp")
def _logcumsumexp(ins, a):
    x = _x(ins)
    if a.get("flatten"):
        x = x.reshape(-1)
    ax = int(a.get("axis", -1))
    if a.get("reverse"):
        x = x.flip(ax)
    y = torch.logcumsumexp(x, ax)
    if a.get("exclusive"):
        y = torch.cat([torch.full_like(y.narrow(ax, 0, 1), -float("inf")), y.narrow(ax, 0, y.shape[ax] - 1)], ax)
    return _out(y.flip(ax) if a.get("reverse") else y)


def _reduce(fn):
    def k(ins, a):
        x = _x(ins)
        dims = _reduce_dims(x, a)
        return _out(fn(x, dims, bool(a.get("keep_dim", a.get("keepdim", False)))))
    return k


register("reduce_amax", "amax")(_reduce(lambda x, d, k: torch.amax(x, d, keepdim=k)))
register("reduce_amin", "amin")(_reduce(lambda x, d, k: torch.amin(x, d, keepdim=k)))
register("frobenius_norm")(_reduce(lambda x, d, k: torch.sqrt((x * x).sum(d, keepdim=k))))
if "max" not in REGISTRY:
    register("max")(_reduce(lambda x, d, k: torch.amax(x, d, keepdim=k)))
if "min" not in REGISTRY:
    register("min")(_reduce(lambda x, d, k: torch.amin(x, d, keepdim=k)))
if "all" not in REGISTRY:
    register("all")(_reduce(lambda x, d, k: torch.all(x.bool(), dim=d, keepdim=k) if d else x.bool()))
if "any" not in REGISTRY:
    register("any")(_reduce(lambda x, d, k: torch.any(x.bool(), dim=d, keepdim=k) if d else x.bool()))


@register("norm")
def _l2_normalize(ins, a):
    """Reference `norm_op.cc` (l2_normalize): Norm = sqrt(Σ x² + ε) along ``axis``, Out = x / Norm."""
    x = _x(ins)
    ax = int(a.get("axis", 1))
    n = torch.sqrt((x * x).sum(ax, keepdim=True) + float(a.get("epsilon", 1e-10)))
    return {"Out": x / n, "Norm": n}


@register("clip_by_norm")
def _clip_by_norm(ins, a):
    """Reference `clip_by_norm_op.h`: Out = X · max_norm / max(‖X‖₂, max_norm)."""
    x = _x(ins)
    mx = float(a.get("max_norm", 1.0))
    n = torch.sqrt((x.float() * x.float()).sum())
    scale = torch.where(n > mx, mx / n, torch.ones_like(n))
    return _out((x.float() * scale).to(x.dtype))


# ----------------------------------------------------------------------------------- binary
def _binary(name, fn, xs=("X", "x"), ys=("Y", "y")):
    register(name)(lambda ins, a, _f=fn: _out(_f(_in(ins, *xs), _in(ins, *ys), a)))


_binary("atan2", lambda x, y, a: torch.atan2(x, y), ("X1", "x"), ("X2", "y"))
for _n in ("elementwise_fmax", "fmax"):
    _binary(_n, lambda x, y, a: torch.fmax(x, _bcast(x, y, a.get("axis", -1))))
for _n in ("elementwise_fmin", "fmin"):
    _binary(_n, lambda x, y, a: torch.fmin(x, _bcast(x, y, a.get("axis", -1))))
_binary("elementwise_heaviside", lambda x, y, a: torch.heaviside(x, _bcast(x, y, a.get("axis", -1))))
_binary("grad_add", lambda x, y, a: x + _bcast(x, y, a.get("axis", -1)))
_binary("minus", lambda x, y, a: x - y)
_binary("kron", lambda x, y, a: torch.kron(x, y))
_binary("complex", lambda x, y, a: torch.complex(x, y))
_binary("bitwise_xor", lambda x, y, a: torch.bitwise_xor(x, y))
_binary("dot", lambda x, y, a: (x * y).sum(-1))
_binary("mv", lambda x, y, a: torch.mv(x, y), ("X", "x"), ("Vec", "vec"))
_binary("cholesky_solve", lambda x, y, a: torch.cholesky_solve(x, y, upper=bool(a.get("upper", False))))
_binary("solve", lambda x, y, a: torch.linalg.solve(x, y))
_binary("triangular_solve", lambda x, y, a: torch.linalg.solve_triangular(
    x.transpose(-1, -2) if a.get("transpose") else x, y,
    upper=bool(a.get("upper", True)) != bool(a.get("transpose", False)),
    unitriangular=bool(a.get("unitriangular", False))))
_binary("dist", lambda x, y, a: torch.linalg.vector_norm(x - y, float(a.get("p", 2.0))))
_binary("equal_all", lambda x, y, a: torch.tensor(x.shape == y.shape and bool(torch.equal(x, y)),
                                                   device=x.device))
_binary("fsp", lambda x, y, a: torch.einsum("nihw,njhw->nij", x, y) / (x.shape[2] * x.shape[3]))
_binary("cross", lambda x, y, a: torch.linalg.cross(
    x, y, dim=int(a["dim"]) if a.get("dim") not in (None, 9) else
    next(i for i, s in enumerate(x.shape) if s == 3)))
_binary("bmm", lambda x, y, a: __import__("paddle_infer_amd.ops.gemm", fromlist=["matmul"]).matmul(x, y))


@register("squared_l2_distance")
def _sq_l2_dist(ins, a):
    x, y = _in(ins, "X"), _in(ins, "Y")
    sub = x.reshape(x.shape[0], -1) - y.reshape(y.shape[0], -1)
    return {"sub_result": sub, "Out": (sub * sub).sum(1, keepdim=True)}


@register("lerp")
def _lerp(ins, a):
    x, y, w = _in(ins, "X", "x"), _in(ins, "Y", "y"), _in(ins, "Weight", "weight")
    return _out(x + w * (y - x))


@register("addmm")
def _addmm(ins, a):
    from ..ops.gemm import matmul
    inp, x, y = _in(ins, "Input", "input"), _in(ins, "X", "x"), _in(ins, "Y", "y")
    al, be = float(_at(a, "Alpha", "alpha", default=1.0)), float(_at(a, "Beta", "beta", default=1.0))
    return _out(be * inp + al * matmul(x, y))


@register("multi_dot")
def _multi_dot(ins, a):
    from ..ops.gemm import matmul
    xs = _inl(ins, "X", "x")
    out = xs[0]
    for t in xs[1:]:
        out = matmul(out, t)
    return _out(out)


@register("trace")
def _trace(ins, a):
    x = _in(ins, "Input", "x", "X")
    return _out(torch.diagonal(x, int(a.get("offset", 0)), int(a.get("axis1", 0)),
                               int(a.get("axis2", 1))).sum(-1))


@register("diagonal")
def _diagonal(ins, a):
    x = _in(ins, "Input", "x", "X")
    return _out(torch.diagonal(x, int(a.get("offset", 0)), int(a.get("axis1", 0)), int(a.get("axis2", 1))))


@register("diag")
def _diag_v1(ins, a):
    return _out(torch.diag(_in(ins, "Diagonal", "X", "x")))


@register("diag_embed")
def _diag_embed(ins, a):
    return _out(torch.diag_embed(_in(ins, "Input", "X", "x"), int(a.get("offset", 0)), int(a.get("dim1", -2)),
                                 int(a.get("dim2", -1))))


@register("determinant", "det")
def _det(ins, a):
    return _out(torch.linalg.det(_in(ins, "Input", "x", "X")))


@register("slogdeterminant", "slogdet")
def _slogdet(ins, a):
    s, l = torch.linalg.slogdet(_in(ins, "Input", "x", "X"))
    return _out(torch.stack([s, l]))


@register("eig")
def _eig(ins, a):
    w, v = torch.linalg.eig(_x(ins))
    return {"Eigenvalues": w, "Eigenvectors": v, "out_w": w, "out_v": v}


@register("eigh")
def _eigh(ins, a):
    w, v = torch.linalg.eigh(_x(ins), UPLO=a.get("UPLO", "L"))
    return {"Eigenvalues": w, "Eigenvectors": v, "out_w": w, "out_v": v}


@register("eigvalsh")
def _eigvalsh(ins, a):
    w, v = torch.linalg.eigh(_x(ins), UPLO=a.get("UPLO", "L"))
    return {"Eigenvalues": w, "Eigenvectors": v}


@register("qr")
def _qr(ins, a):
    mode = a.get("mode", "reduced")
    q, r = torch.linalg.qr(_x(ins), mode="r" if mode == "r" else mode)
    return {"Q": q, "R": r, "q": q, "r": r}


@register("svd")
def _svd(ins, a):
    u, s, vh = torch.linalg.svd(_x(ins), full_matrices=bool(a.get("full_matrices", False)))
    return {"U": u, "S": s, "VH": vh, "u": u, "s": s, "vh": vh}


@register("lstsq")
def _lstsq(ins, a):
    x, y = _in(ins, "X", "x"), _in(ins, "Y", "y")
    r = torch.linalg.lstsq(x, y, rcond=a.get("rcond"), driver=a.get("driver") or None)
    return {"Solution": r.solution, "Residuals": r.residuals, "Rank": r.rank, "SingularValues": r.singular_values}


@register("lu")
def _lu(ins, a):
    lu, piv = torch.linalg.lu_factor(_x(ins), pivot=bool(a.get("pivots", True)))
    return {"Out": lu, "Pivots": piv.to(torch.int32), "Infos": torch.zeros(lu.shape[:-2] or (1,), dtype=torch.int32,
                                                                              device=lu.device)}


@register("lu_unpack")
def _lu_unpack(ins, a):
    p, l, u = torch.lu_unpack(_in(ins, "X", "x"), _in(ins, "Pivots", "y").int(),
                              bool(a.get("unpack_ludata", True)), bool(a.get("unpack_pivots", True)))
    return {"Pmat": p, "L": l, "U": u}


@register("matrix_rank")
def _matrix_rank(ins, a):
    x = _x(ins)
    tol = _in(ins, "TolTensor")
    if tol is None and not a.get("use_default_tol", True):
        tol = torch.tensor(float(a.get("tol", 0.0)), device=x.device)
    return _out(torch.linalg.matrix_rank(x, atol=tol, hermitian=bool(a.get("hermitian", False))))


@register("allclose")
def _allclose(ins, a):
    x, y = _in(ins, "Input", "x"), _in(ins, "Other", "y")
    rt = float(_in(ins, "Rtol").reshape(-1)[0]) if _in(ins, "Rtol") is not None else float(a.get("rtol", 1e-5))
    at = float(_in(ins, "Atol").reshape(-1)[0]) if _in(ins, "Atol") is not None else float(a.get("atol", 1e-8))
    return _out(torch.tensor(torch.allclose(x, y, rt, at, bool(a.get("equal_nan", False))), device=x.device))


@register("isclose")
def _isclose(ins, a):
    x, y = _in(ins, "Input", "x"), _in(ins, "Other", "y")
    rt = float(_in(ins, "Rtol").reshape(-1)[0]) if _in(ins, "Rtol") is not None else float(a.get("rtol", 1e-5))
    at = float(_in(ins, "Atol").reshape(-1)[0]) if _in(ins, "Atol") is not None else float(a.get("atol", 1e-8))
    return _out(torch.isclose(x, y, rt, at, bool(a.get("equal_nan", False))))


# ---------------------------------------------------------------------------------- creation
@register("arange")
def _arange(ins, a):
    s, e, st = (_in(ins, n, n.lower()) for n in ("Start", "End", "Step"))
    return _out(torch.arange(s.reshape(-1)[0].item(), e.reshape(-1)[0].item(), st.reshape(-1)[0].item(),
                             dtype=s.dtype, device=s.device))


@register("empty")
def _empty(ins, a):
    return _out(torch.empty(_shape(ins, a), dtype=_dtype(a), device=_dev(ins)))


@register("empty_like")
def _empty_like(ins, a):
    x = _x(ins)
    return _out(torch.empty_like(x, dtype=_dtype(a, default=str(x.dtype).split(".")[-1]) if a.get("dtype") not in
                                 (None, -1) else x.dtype))


@register("full_like", "fill_any_like_v2")
def _full_like(ins, a):
    x = _x(ins)
    dt = _dtype(a) if a.get("dtype") not in (None, -1) else x.dtype
    return _out(torch.full_like(x, float(_at(a, "value", default=0.0)), dtype=dt))


@register("ones_like")
def _ones_like(ins, a):
    x = _x(ins)
    return _out(torch.ones_like(x, dtype=_dtype(a) if a.get("dtype") not in (None, -1) else x.dtype))


@register("zeros_like", "fill_zeros_like2")
def _zeros_like(ins, a):
    x = _x(ins)
    return _out(torch.zeros_like(x, dtype=_dtype(a) if a.get("dtype") not in (None, -1) else x.dtype))


def _mk_full(val):
    def k(ins, a):
        v = float(_at(a, "value", default=0.0)) if val is None else val
        return _out(torch.full(_shape(ins, a), v, dtype=_dtype(a), device=_dev(ins)))
    return k


register("ones")(_mk_full(1.0))
register("zeros")(_mk_full(0.0))
register("full", "full_")(_mk_full(None))


def _batch_like(kind):
    def k(ins, a):
        ref = _in(ins, "Input", "input")
        shape = list(_shape(ins, a))
        shape[int(a.get("output_dim_idx", 0))] = ref.shape[int(a.get("input_dim_idx", 0))]
        dt, dev = _dtype(a), ref.device
        if kind == "full":
            return _out(torch.full(shape, float(a.get("value", 0.0)), dtype=dt, device=dev))
        if kind == "gauss":
            return _out(torch.randn(shape, device=dev).mul_(float(a.get("std", 1.0))).add_(float(a.get("mean", 0.0))).to(dt))
        lo, hi = float(a.get("min", -1.0)), float(a.get("max", 1.0))
        return _out((torch.rand(shape, device=dev) * (hi - lo) + lo).to(dt))
    return k


register("full_batch_size_like")(_batch_like("full"))
register("gaussian_random_batch_size_like")(_batch_like("gauss"))
register("uniform_random_batch_size_like")(_batch_like("uniform"))


@register("eye")
def _eye(ins, a):
    r = int(a.get("num_rows", 1))
    c = int(a.get("num_columns", -1))
    return _out(torch.eye(r, r if c < 0 else c, dtype=_dtype(a), device=_dev(ins)))


@register("fill_any")
def _fill_any(ins, a):
    x = _x(ins)
    v = float(a.get("value_float", 0.0)) if x.dtype.is_floating_point else int(a.get("value_int", 0))
    return _out(torch.full_like(x, v))


@register("fill")
def _fill(ins, a):
    vals = a.get("value", [])
    return _out(torch.tensor(vals, dtype=_dtype(a), device=_dev(ins)).reshape(_shape(ins, a)))


@register("fill_diagonal")
def _fill_diagonal(ins, a):
    x = _x(ins).clone()
    v, off, wrap = float(a.get("value", 0.0)), int(a.get("offset", 0)), bool(a.get("wrap", False))
    if x.dim() == 2:
        n = x.shape[0] if wrap else min(x.shape)
        idx = torch.arange(n, device=x.device)
        cols = idx + off
        ok = (cols >= 0) & (cols < x.shape[1])
        if wrap:
            flat = x.reshape(-1)
            step = x.shape[1] + 1
            pos = torch.arange(max(off, 0) if off >= 0 else -off * x.shape[1], flat.numel(), step, device=x.device)
            flat[pos] = v
            return _out(flat.reshape(x.shape))
        x[idx[ok], cols[ok]] = v
    else:
        n = min(x.shape)
        i = torch.arange(n, device=x.device)
        x[tuple([i] * x.dim())] = v
    return _out(x)


@register("fill_diagonal_tensor")
def _fill_diagonal_tensor(ins, a):
    x, y = _in(ins, "X", "x").clone(), _in(ins, "Y", "y")
    d = torch.diagonal(x, int(a.get("offset", 0)), int(a.get("dim1", 0)), int(a.get("dim2", 1)))
    d.copy_(y)
    return _out(x)


@register("randint")
def _randint(ins, a):
    return _out(torch.randint(int(a.get("low", 0)), int(a.get("high", 2)), _shape(ins, a),
                              dtype=_dtype(a, default="int64"), device=_dev(ins)))


@register("randperm")
def _randperm(ins, a):
    return _out(torch.randperm(int(a.get("n", 1)), dtype=_dtype(a, default="int64"), device=_dev(ins)))


@register("multinomial")
def _multinomial(ins, a):
    x = _x(ins)
    return _out(torch.multinomial(x.float(), int(a.get("num_samples", 1)), bool(a.get("replacement", False))))


@register("uniform_random_inplace")
def _uniform_inplace(ins, a):
    x = _x(ins)
    lo, hi = float(a.get("min", -1.0)), float(a.get("max", 1.0))
    return _out(torch.rand_like(x.float()).mul_(hi - lo).add_(lo).to(x.dtype))


@register("truncated_gaussian_random")
def _trunc_gauss(ins, a):
    shape = _shape(ins, a)
    mean, std = float(a.get("mean", 0.0)), float(a.get("std", 1.0))
    t = torch.empty(shape, device=_dev(ins))
    torch.nn.init.trunc_normal_(t, mean, std, mean - 2 * std, mean + 2 * std)
    return _out(t.to(_dtype(a)))


@register("seed")
def _seed(ins, a):
    s = int(a.get("seed", 0)) or int(torch.randint(1, 2 ** 31 - 1, ()).item())
    return _out(torch.tensor([s], dtype=torch.int32, device=_dev(ins)))


@register("tril_indices")
def _tril_indices(ins, a):
    return _out(torch.tril_indices(int(a.get("rows", 1)), int(a.get("cols", 1)), int(a.get("offset", 0)),
                                   device=_dev(ins)).to(_dtype(a, default="int64")))


@register("triu_indices")
def _triu_indices(ins, a):
    return _out(torch.triu_indices(int(a.get("row", 1)), int(a.get("col", 1)), int(a.get("offset", 0)),
                                   device=_dev(ins)).to(_dtype(a, default="int64")))


@register("logspace")
def _logspace(ins, a):
    s, e, n, b = (_in(ins, k, k.lower()) for k in ("Start", "Stop", "Num", "Base"))
    return _out(torch.logspace(float(s.reshape(-1)[0]), float(e.reshape(-1)[0]), int(n.reshape(-1)[0]),
                               float(b.reshape(-1)[0]), dtype=_dtype(a), device=s.device))


@register("one_hot")
def _one_hot_v1(ins, a):
    """Reference `one_hot_op.cc` (v1): X [N, 1] int → [N, depth] (depth_tensor overrides)."""
    x = _x(ins)
    d = int(_in(ins, "depth_tensor").reshape(-1)[0]) if _in(ins, "depth_tensor") is not None else int(a.get("depth", 1))
    lab = x.reshape(x.shape[:-1] if x.dim() > 1 and x.shape[-1] == 1 else x.shape).long()
    if a.get("allow_out_of_range"):
        ok = (lab >= 0) & (lab < d)
        oh = F.one_hot(lab.clamp(0, d - 1), d) * ok.unsqueeze(-1)
    else:
        oh = F.one_hot(lab, d)
    return _out(oh.to(_dtype(a)))


# ------------------------------------------------------------------------------ manipulation
@register("unsqueeze")
def _unsqueeze_v1(ins, a):
    x = _x(ins)
    axes = [int(v) for v in (_in(ins, "AxesTensor").reshape(-1).tolist() if _in(ins, "AxesTensor") is not None
                             else a.get("axes", []))]
    for ax in sorted(axes):
        x = x.unsqueeze(ax if ax >= 0 else ax + x.dim() + 1)
    return _out(x)


@register("unstack")
def _unstack(ins, a):
    x = _x(ins)
    return {"Y": list(torch.unbind(x, int(a.get("axis", 0)))), "out": list(torch.unbind(x, int(a.get("axis", 0))))}


@register("broadcast_tensors")
def _broadcast_tensors(ins, a):
    return _out(list(torch.broadcast_tensors(*_inl(ins, "X", "input"))))


@register("expand_as")
def _expand_as_v1(ins, a):
    x = _x(ins)
    t = _in(ins, "target_tensor", "Y", "y")
    shape = a.get("target_shape") or list(t.shape)
    return _out(x.expand(*shape) if x.dim() == len(shape) else x.expand(*shape))


@register("crop", "crop_tensor")
def _crop(ins, a):
    x = _x(ins)
    if _in(ins, "Y") is not None:
        shape = list(_in(ins, "Y").shape)
    elif _in(ins, "Shape", "ShapeTensor") is not None:
        shape = [int(v) for v in _in(ins, "Shape", "ShapeTensor").reshape(-1).tolist()]
    elif ins.get("ShapeTensorList"):
        shape = [int(t.reshape(-1)[0]) for t in ins["ShapeTensorList"]]
    else:
        shape = [int(v) for v in a.get("shape", [])]
    if _in(ins, "Offsets", "OffsetsTensor") is not None:
        offs = [int(v) for v in _in(ins, "Offsets", "OffsetsTensor").reshape(-1).tolist()]
    elif ins.get("OffsetsTensorList"):
        offs = [int(t.reshape(-1)[0]) for t in ins["OffsetsTensorList"]]
    else:
        offs = [int(v) for v in (a.get("offsets") or [0] * x.dim())]
    sl = tuple(slice(o, o + (s if s != -1 else x.shape[i] - o)) for i, (o, s) in enumerate(zip(offs, shape)))
    return _out(x[sl])


@register("pad")
def _pad_v1(ins, a):
    x = _x(ins)
    p = [int(v) for v in a.get("paddings", [])]
    tp = []
    for i in reversed(range(x.dim())):
        tp += [p[2 * i], p[2 * i + 1]]
    return _out(F.pad(x, tp, value=float(a.get("pad_value", 0.0))))


@register("pad2d")
def _pad2d(ins, a):
    x = _x(ins)
    p = [int(v) for v in (_in(ins, "Paddings").reshape(-1).tolist() if _in(ins, "Paddings") is not None
                          else a.get("paddings", [0, 0, 0, 0]))]
    nhwc = a.get("data_format", "NCHW") == "NHWC"
    if nhwc:
        x = x.permute(0, 3, 1, 2)
    mode = {"constant": "constant", "reflect": "reflect", "edge": "replicate"}[a.get("mode", "constant")]
    kw = {"value": float(a.get("pad_value", 0.0))} if mode == "constant" else {}
    y = F.pad(x, [p[2], p[3], p[0], p[1]], mode=mode, **kw)
    return _out(y.permute(0, 2, 3, 1) if nhwc else y)


@register("pad_constant_like")
def _pad_constant_like(ins, a):
    x, y = _in(ins, "X"), _in(ins, "Y")
    tp = []
    for i in reversed(range(x.dim())):
        tp += [0, x.shape[i] - y.shape[i]]
    return _out(F.pad(y, tp, value=float(a.get("pad_value", 0.0))))


@register("repeat_interleave", "repeat_interleave_with_tensor_index")
def _repeat_interleave(ins, a):
    x = _x(ins)
    r = _in(ins, "RepeatsTensor", "repeats")
    rep = r if r is not None else int(_at(a, "Repeats", "repeats", default=1))
    dim = _at(a, "dim", "axis")
    if dim is None:
        return _out(torch.repeat_interleave(x.reshape(-1), rep))
    return _out(torch.repeat_interleave(x, rep, dim=int(dim)))


def _nchw(x, a, key="data_format"):
    return a.get(key, "NCHW") in ("NHWC", "NLC", "NDHWC")


@register("pixel_shuffle")
def _pixel_shuffle(ins, a):
    x = _x(ins)
    r = int(a.get("upscale_factor", 1))
    if _nchw(x, a):
        return _out(F.pixel_shuffle(x.permute(0, 3, 1, 2), r).permute(0, 2, 3, 1))
    return _out(F.pixel_shuffle(x, r))


@register("pixel_unshuffle")
def _pixel_unshuffle(ins, a):
    x = _x(ins)
    r = int(a.get("downscale_factor", 1))
    if _nchw(x, a):
        return _out(F.pixel_unshuffle(x.permute(0, 3, 1, 2), r).permute(0, 2, 3, 1))
    return _out(F.pixel_unshuffle(x, r))


@register("channel_shuffle", "shuffle_channel")
def _channel_shuffle(ins, a):
    x = _x(ins)
    g = int(_at(a, "groups", "group", default=1))
    nhwc = _nchw(x, a)
    if nhwc:
        x = x.permute(0, 3, 1, 2)
    N, C, H, W = x.shape
    y = x.reshape(N, g, C // g, H, W).transpose(1, 2).reshape(N, C, H, W)
    return _out(y.permute(0, 2, 3, 1) if nhwc else y)


@register("space_to_depth")
def _space_to_depth(ins, a):
    """Reference `space_to_depth_op.cc`: output channel = ((by·b + bx)·C + c)."""
    x = _x(ins)
    b = int(a.get("blocksize", 1))
    N, C, H, W = x.shape
    y = x.reshape(N, C, H // b, b, W // b, b).permute(0, 3, 5, 1, 2, 4)
    return _out(y.reshape(N, C * b * b, H // b, W // b))


@register("temporal_shift")
def _temporal_shift(ins, a):
    from ..nn.functional import temporal_shift
    x = _x(ins)
    return _out(temporal_shift(x, int(a.get("seg_num", 1)), float(a.get("shift_ratio", 0.25)),
                               data_format=a.get("data_format", "NCHW")))


@register("fold")
def _fold(ins, a):
    x = _x(ins)
    y = F.fold(x, list(a["output_sizes"]), list(a["kernel_sizes"]), dilation=list(a.get("dilations", [1, 1])),
               padding=list(a.get("paddings", [0, 0, 0, 0]))[:2], stride=list(a.get("strides", [1, 1])))
    return {"Y": y, "out": y}


@register("unfold")
def _unfold(ins, a):
    x = _x(ins)
    p = list(a.get("paddings", [0, 0, 0, 0]))
    if len(p) == 4 and (p[0] != p[2] or p[1] != p[3]):
        x = F.pad(x, [p[1], p[3], p[0], p[2]])
        p = [0, 0]
    y = F.unfold(x, list(a["kernel_sizes"]), dilation=list(a.get("dilations", [1, 1])), padding=p[:2],
                 stride=list(a.get("strides", [1, 1])))
    return {"Y": y, "out": y}


@register("frame")
def _frame(ins, a):
    from ..signal import frame
    return _out(frame(_x(ins), int(a["frame_length"]), int(a["hop_length"]), int(a.get("axis", -1))))


@register("overlap_add")
def _overlap_add(ins, a):
    from ..signal import overlap_add
    return _out(overlap_add(_x(ins), int(a["hop_length"]), int(a.get("axis", -1))))


@register("index_add")
def _index_add(ins, a):
    x, idx, v = _in(ins, "X", "x"), _in(ins, "Index", "index"), _in(ins, "AddValue", "add_value")
    return _out(torch.index_add(x, int(a.get("axis", 0)), idx.long(), v))


@register("put_along_axis")
def _put_along_axis(ins, a):
    """Reference `put_along_axis_op.cc`: Result = Input with Value scattered at Index along Axis
    (Reduce "assign" / "add" / "multiply"|"mul")."""
    x, idx, v = _in(ins, "Input", "arr"), _in(ins, "Index", "indices"), _in(ins, "Value", "values")
    ax = int(_at(a, "Axis", "axis", default=0))
    red = _at(a, "Reduce", "reduce", default="assign")
    idx = idx.long()
    v = v.expand(idx.shape) if v.shape != idx.shape else v
    if red == "add":
        y = x.scatter_add(ax, idx, v.to(x.dtype))
    elif red in ("mul", "multiply"):
        y = x.scatter_reduce(ax, idx, v.to(x.dtype), "prod")
    else:
        y = x.scatter(ax, idx, v.to(x.dtype))
    return {"Result": y, "out": y}


@register("scatter_nd_add")
def _scatter_nd_add(ins, a):
    x, idx, up = _in(ins, "X", "x"), _in(ins, "Index", "index"), _in(ins, "Updates", "updates")
    k = idx.shape[-1]
    flat_idx = idx.reshape(-1, k).long()
    strides = torch.tensor([int(np.prod(x.shape[i + 1:k])) for i in range(k)], device=x.device)
    lin = (flat_idx * strides).sum(-1)
    xv = x.reshape(int(np.prod(x.shape[:k])) if k else 1, -1)
    y = xv.index_add(0, lin, up.reshape(lin.numel(), -1).to(x.dtype))
    return _out(y.reshape(x.shape))


@register("searchsorted")
def _searchsorted(ins, a):
    s, v = _in(ins, "SortedSequence", "sorted_sequence"), _in(ins, "Values", "values")
    return _out(torch.searchsorted(s, v, out_int32=bool(a.get("out_int32", False)), right=bool(a.get("right", False))))


@register("unique")
def _unique(ins, a):
    """Reference `unique_op.cc` (is_sorted=True path): Out sorted unique values, Indices first
    occurrences, Index inverse, Counts; ``axis`` [] flattens. Legacy (is_sorted False) also sorted."""
    x = _x(ins)
    axis = a.get("axis") or []
    dt = _dtype(a, default="int64")
    dim = int(axis[0]) if axis else None
    src = x if dim is not None else x.reshape(-1)
    out, inv, cnt = torch.unique(src, sorted=True, return_inverse=True, return_counts=True, dim=dim if dim is not None else None)
    n = src.shape[dim if dim is not None else 0]
    first = torch.full((out.shape[dim if dim is not None else 0],), n, dtype=torch.long, device=x.device)
    first = first.scatter_reduce(0, inv.reshape(-1), torch.arange(n, device=x.device), "amin")
    return {"Out": out, "Index": inv.to(dt), "Indices": first.to(dt), "Counts": cnt.to(dt)}


@register("unique_consecutive")
def _unique_consecutive(ins, a):
    x = _x(ins)
    axis = a.get("axis") or []
    dim = int(axis[0]) if axis else None
    dt = _dtype(a, default="int64")
    out, inv, cnt = torch.unique_consecutive(x if dim is not None else x.reshape(-1), return_inverse=True,
                                             return_counts=True, dim=dim)
    return {"Out": out, "Index": inv.to(dt), "Counts": cnt.to(dt)}


@register("bincount")
def _bincount(ins, a):
    x, w = _x(ins), _in(ins, "Weights", "weights")
    return _out(torch.bincount(x.reshape(-1), w.reshape(-1) if w is not None else None, int(a.get("minlength", 0))))


@register("histogram")
def _histogram(ins, a):
    x = _x(ins).float()
    lo, hi = float(a.get("min", 0)), float(a.get("max", 0))
    if lo == 0 and hi == 0:
        lo, hi = float(x.min()), float(x.max())
    return _out(torch.histc(x, int(a.get("bins", 100)), lo, hi).to(torch.int64))


@register("kthvalue")
def _kthvalue(ins, a):
    v, i = torch.kthvalue(_x(ins), int(a.get("k", 1)), int(a.get("axis", -1)), bool(a.get("keepdim", False)))
    return {"Out": v, "Indices": i, "out": v, "indices": i}


@register("mode")
def _mode(ins, a):
    v, i = torch.mode(_x(ins), int(a.get("axis", -1)), bool(a.get("keepdim", False)))
    return {"Out": v, "Indices": i, "out": v, "indices": i}


@register("nanmedian")
def _nanmedian(ins, a):
    x = _x(ins)
    ax = a.get("axis") or []
    if not ax:
        v = torch.nanmedian(x.reshape(-1))
        return {"Out": v.reshape([1] * x.dim()) if a.get("keepdim") else v, "MedianIndex": torch.zeros(1, dtype=torch.long)}
    v, i = torch.nanmedian(x, int(ax[0]) if len(ax) == 1 else int(ax[0]), bool(a.get("keepdim", True)))
    return {"Out": v, "MedianIndex": i}


@register("maxout")
def _maxout(ins, a):
    x = _x(ins)
    g, ax = int(a.get("groups", 1)), int(a.get("axis", 1))
    ax = ax % x.dim()
    shape = list(x.shape)
    shape[ax:ax + 1] = [shape[ax] // g, g]
    return _out(x.reshape(shape).amax(ax + 1))


@register("multiplex")
def _multiplex(ins, a):
    ids, xs = _in(ins, "Ids", "index"), _inl(ins, "X", "inputs")
    st = torch.stack(xs)
    return _out(st[ids.reshape(-1).long(), torch.arange(st.shape[1], device=st.device)])


@register("partial_concat")
def _partial_concat(ins, a):
    s, ln = int(a.get("start_index", 0)), int(a.get("length", -1))
    xs = _inl(ins, "X")
    return _out(torch.cat([x[:, s:(None if ln < 0 else s + ln)] for x in xs], 1))


@register("partial_sum")
def _partial_sum(ins, a):
    s, ln = int(a.get("start_index", 0)), int(a.get("length", -1))
    xs = _inl(ins, "X")
    return _out(sum(x[:, s:(None if ln < 0 else s + ln)] for x in xs))


@register("segment_pool")
def _segment_pool(ins, a):
    """Reference `segment_pool_op.cc`: SUM / MEAN / MAX / MIN over sorted SegmentIds rows."""
    x, seg = _x(ins), _in(ins, "SegmentIds", "segment_ids").long()
    n = int(seg.max()) + 1 if seg.numel() else 0
    pt = a.get("pooltype", "SUM").upper()
    shape = (n,) + tuple(x.shape[1:])
    idx = seg.reshape(-1, *([1] * (x.dim() - 1))).expand_as(x)
    cnt = torch.bincount(seg, minlength=n).to(x.dtype).clamp_min(1)
    if pt in ("SUM", "MEAN"):
        s = x.new_zeros(shape).scatter_add(0, idx, x)
        out = s / cnt.reshape(-1, *([1] * (x.dim() - 1))) if pt == "MEAN" else s
    else:
        out = x.new_zeros(shape).scatter_reduce(0, idx, x, "amax" if pt == "MAX" else "amin", include_self=False)
    return {"Out": out, "SummedIds": cnt.reshape(-1, 1)}


@register("shard_index")
def _shard_index(ins, a):
    x = _x(ins)
    nshards, sid = int(a["nshards"]), int(a["shard_id"])
    size = (int(a["index_num"]) + nshards - 1) // nshards
    ig = int(a.get("ignore_value", -1))
    ok = (x // size) == sid
    return _out(torch.where(ok, x % size, torch.full_like(x, ig)))


@register("split_with_num")
def _split_with_num(ins, a):
    x = _x(ins)
    return _out(list(torch.chunk(x, int(a.get("num", 1)), int(a.get("axis", 0)))))


@register("sequence_mask")
def _sequence_mask(ins, a):
    x = _x(ins)
    ml = _in(ins, "MaxLenTensor")
    m = int(ml.reshape(-1)[0]) if ml is not None else int(a.get("maxlen", -1))
    if m < 0:
        m = int(x.max())
    y = (torch.arange(m, device=x.device) < x.unsqueeze(-1))
    return {"Y": y.to(_dtype(a, "out_dtype", "int64"))}


@register("einsum")
def _einsum(ins, a):
    return {"Out": torch.einsum(a["equation"], *_inl(ins, "Operands", "x"))}


@register("as_complex")
def _as_complex(ins, a):
    return _out(torch.view_as_complex(_x(ins).contiguous()))


@register("as_real")
def _as_real(ins, a):
    return _out(torch.view_as_real(_x(ins)))


@register("gather_tree")
def _gather_tree(ins, a):
    from ..nn.functional.extra import gather_tree
    return _out(gather_tree(_in(ins, "Ids", "ids"), _in(ins, "Parents", "parents")))


@register("conv_shift")
def _conv_shift(ins, a):
    """Reference `conv_shift_op.cc`: circular correlation Out[i, j] = Σ_k X[i, (j + k − M/2) mod N]·Y[i, k]."""
    x, y = _in(ins, "X"), _in(ins, "Y")
    N, M = x.shape[1], y.shape[1]
    j = torch.arange(N, device=x.device)[:, None]
    k = torch.arange(M, device=x.device)[None, :]
    idx = (j + k - M // 2) % N
    return _out((x[:, idx] * y[:, None, :]).sum(-1))


@register("row_conv")
def _row_conv(ins, a):
    """Reference `row_conv_op.cc` (lookahead conv): Out[t] = Σ_k X[t + k] ∘ Filter[k] (padded batch [B, T, D])."""
    x, f = _x(ins), _in(ins, "Filter")
    K = f.shape[0]
    xp = F.pad(x, (0, 0, 0, K - 1)) if x.dim() == 3 else F.pad(x, (0, 0, 0, K - 1))
    T = x.shape[-2]
    return _out(sum(xp[..., k:k + T, :] * f[k] for k in range(K)))


@register("bilinear_tensor_product")
def _bilinear_tp(ins, a):
    x, y, w, b = _in(ins, "X", "x"), _in(ins, "Y", "y"), _in(ins, "Weight", "weight"), _in(ins, "Bias", "bias")
    out = torch.einsum("bi,kij,bj->bk", x, w, y)
    return _out(out + b.reshape(1, -1) if b is not None else out)


@register("batch_fc")
def _batch_fc(ins, a):
    x, w, b = _in(ins, "Input"), _in(ins, "W"), _in(ins, "Bias")
    return _out(torch.bmm(x, w) + b.unsqueeze(1))


@register("cos_sim")
def _cos_sim(ins, a):
    x, y = _in(ins, "X"), _in(ins, "Y")
    xf, yf = x.reshape(x.shape[0], -1), y.reshape(y.shape[0], -1)
    xn = torch.sqrt((xf * xf).sum(1, keepdim=True))
    yn = torch.sqrt((yf * yf).sum(1, keepdim=True))
    return {"Out": (xf * yf).sum(1, keepdim=True) / (xn * yn), "XNorm": xn, "YNorm": yn}


@register("affine_grid")
def _affine_grid(ins, a):
    from ..nn.functional import affine_grid
    th = _in(ins, "Theta", "input")
    shp = _in(ins, "OutputShape")
    shape = [int(v) for v in shp.reshape(-1).tolist()] if shp is not None else list(_at(a, "output_shape", "outputShape"))
    g = affine_grid(th, shape, bool(a.get("align_corners", True)))
    return {"Output": g, "out": g}


@register("grid_sample")
def _grid_sample(ins, a):
    x, g = _in(ins, "X", "x"), _in(ins, "Grid", "grid")
    return _out(F.grid_sample(x, g, mode=a.get("mode", "bilinear"), padding_mode=a.get("padding_mode", "zeros"),
                              align_corners=bool(a.get("align_corners", True))), "Output")


# ----------------------------------------------------------------------------- interpolation
def _lin_axis(x, ax, O, align, align_mode, scale):
    """Paddle's linear interpolation along one axis (reference `interpolate_function.h`):
    align_corners → src = dst·(I−1)/(O−1); align_mode 0 → half-pixel src = (dst+½)·r − ½ (≥ 0);
    align_mode 1 → src = dst·r, r = 1/scale (scale > 0) else I/O."""
    I = x.shape[ax]
    dev = x.device
    d = torch.arange(O, device=dev, dtype=torch.float32)
    if align:
        r = (I - 1) / (O - 1) if O > 1 else 0.0
        src = d * r
    else:
        r = (1.0 / scale) if scale and scale > 0 else I / O
        src = ((d + 0.5) * r - 0.5).clamp_min(0.0) if align_mode == 0 else d * r
    lo = src.floor().long().clamp(0, I - 1)
    hi = (lo + 1).clamp(max=I - 1)
    w = (src - lo.float()).clamp(0, 1)
    shp = [1] * x.dim()
    shp[ax] = O
    w = w.reshape(shp).to(x.dtype)
    return torch.index_select(x, ax, lo) * (1 - w) + torch.index_select(x, ax, hi) * w


def _interp_nd(ins, a, nd):
    x = _x(ins)
    cl = a.get("data_layout", "NCHW") in ("NWC", "NHWC", "NDHWC")
    if cl:
        x = x.movedim(-1, 1)
    spatial = list(x.shape[2:])
    keys = {1: ["out_w"], 2: ["out_h", "out_w"], 3: ["out_d", "out_h", "out_w"]}[nd]
    size = None
    if ins.get("OutSize"):
        size = [int(v) for v in ins["OutSize"][0].reshape(-1).tolist()]
    elif ins.get("SizeTensor"):
        size = [int(t.reshape(-1)[0]) for t in ins["SizeTensor"]]
    elif all(int(a.get(k, -1) or -1) > 0 for k in keys):
        size = [int(a[k]) for k in keys]
    scales = [0.0] * nd
    if size is None:
        sc = ins["Scale"][0].reshape(-1).tolist() if ins.get("Scale") else a.get("scale", [])
        if isinstance(sc, (int, float)):
            sc = [sc]
        sc = list(sc) or [1.0]
        scales = [float(sc[min(i, len(sc) - 1)]) for i in range(nd)]
        size = [int(s * f) for s, f in zip(spatial, scales)]
    align, am = bool(a.get("align_corners", True)), int(a.get("align_mode", 1))
    y = x
    for i in range(nd):
        y = _lin_axis(y, 2 + i, size[i], align, am, scales[i])
    return _out(y.movedim(1, -1) if cl else y)


register("linear_interp", "linear_interp_v2")(lambda ins, a: _interp_nd(ins, a, 1))
register("trilinear_interp", "trilinear_interp_v2")(lambda ins, a: _interp_nd(ins, a, 3))
_bilinear_prev = REGISTRY.get("bilinear_interp_v2")


def _bilinear_interp(ins, a):
    # torch's bilinear has no asymmetric (align_mode 1) coordinate map: that case runs _lin_axis
    if not a.get("align_corners", True) and int(a.get("align_mode", 1)) == 1:
        return _interp_nd(ins, a, 2)
    return _bilinear_prev(ins, a)


register("bilinear_interp_v2", "bilinear_interp")(_bilinear_interp)


# --------------------------------------------------------------------------------- pooling
@register("max_pool2d_with_index", "max_pool3d_with_index")
def _max_pool_idx(ins, a):
    x = _x(ins)
    nd = x.dim() - 2
    k = list(a.get("ksize", [1] * nd))
    if a.get("global_pooling"):
        k = list(x.shape[2:])
        pad = [0] * nd
    else:
        pad = list(a.get("paddings", [0] * nd))[:nd]
    st = list(a.get("strides", k))
    if a.get("adaptive"):
        fn = F.adaptive_max_pool2d if nd == 2 else F.adaptive_max_pool3d
        y, m = fn(x, k, return_indices=True)
    else:
        fn = F.max_pool2d if nd == 2 else F.max_pool3d
        y, m = fn(x, k, st, pad, return_indices=True)
    return {"Out": y, "Mask": m.to(torch.int32), "out": y, "mask": m.to(torch.int32)}


@register("unpool", "unpool3d")
def _unpool(ins, a):
    x, idx = _x(ins), _in(ins, "Indices", "indices").long()
    nd = x.dim() - 2
    k = list(a.get("ksize", [2] * nd))
    st = list(a.get("strides", k))
    pad = list(a.get("paddings", [0] * nd))
    os_ = a.get("output_size")
    fn = F.max_unpool2d if nd == 2 else F.max_unpool3d
    y = fn(x, idx, k, st, pad, output_size=list(os_)[-nd:] if os_ else None)
    return _out(y)


@register("lrn")
def _lrn(ins, a):
    x = _x(ins)
    n, k, al, be = int(a.get("n", 5)), float(a.get("k", 2.0)), float(a.get("alpha", 1e-4)), float(a.get("beta", 0.75))
    nhwc = a.get("data_format", "NCHW") == "NHWC"
    if nhwc:
        x = x.permute(0, 3, 1, 2)
    sq = F.pad((x * x).unsqueeze(1), (0, 0, 0, 0, n // 2, (n - 1) // 2)).squeeze(1)
    s = sum(sq[:, i:i + x.shape[1]] for i in range(n))
    mid = k + al * s
    y = x * mid.pow(-be)
    if nhwc:
        y, mid = y.permute(0, 2, 3, 1), mid.permute(0, 2, 3, 1)
    return {"Out": y, "MidOut": mid}


@register("spp")
def _spp(ins, a):
    x = _x(ins)
    N, C, H, W = x.shape
    outs = []
    for p in range(int(a.get("pyramid_height", 1))):
        bins = 2 ** p
        kh, kw = math.ceil(H / bins), math.ceil(W / bins)
        ph, pw = (kh * bins - H + 1) // 2, (kw * bins - W + 1) // 2
        if a.get("pooling_type", "max") == "max":
            y = F.max_pool2d(F.pad(x, (pw, pw, ph, ph), value=-float("inf")), (kh, kw), (kh, kw))
        else:
            y = F.avg_pool2d(F.pad(x, (pw, pw, ph, ph)), (kh, kw), (kh, kw))
        outs.append(y.reshape(N, -1))
    return _out(torch.cat(outs, 1))


# ----------------------------------------------------------------------------------- losses
def _sce(x, t):
    return torch.clamp(x, min=0) - x * t + torch.log1p(torch.exp(-x.abs()))


@register("sigmoid_cross_entropy_with_logits")
def _sigmoid_xent(ins, a):
    """Reference `sigmoid_cross_entropy_with_logits_op.cc`: max(x,0) − x·z + log(1 + e^{−|x|}),
    0 where Label == ignore_index; ``normalize`` divides by the count of non-ignored labels."""
    x, z = _in(ins, "X", "x"), _in(ins, "Label", "label")
    ig = float(a.get("ignore_index", -100))
    keep = z != ig
    loss = torch.where(keep, _sce(x, z.to(x.dtype)), torch.zeros_like(x))
    if a.get("normalize"):
        loss = loss / keep.sum().clamp_min(1).to(x.dtype)
    return _out(loss)


@register("sigmoid_focal_loss")
def _sigmoid_focal(ins, a):
    """Reference `sigmoid_focal_loss_op.cc`: Label [N, 1] in 0..C (0 = background), X [N, C]."""
    x, lab, fg = _in(ins, "X"), _in(ins, "Label"), _in(ins, "FgNum")
    g, al = float(a.get("gamma", 2.0)), float(a.get("alpha", 0.25))
    C = x.shape[1]
    t = (lab.reshape(-1, 1).long() == torch.arange(1, C + 1, device=x.device)[None]).to(x.dtype)
    p = torch.sigmoid(x)
    fgn = fg.reshape(-1)[0].to(x.dtype).clamp_min(1)
    pos = -al * (1 - p).pow(g) * torch.log(p.clamp_min(1e-38))
    neg = -(1 - al) * p.pow(g) * torch.log((1 - p).clamp_min(1e-38))
    valid = (lab.reshape(-1, 1) >= 0).to(x.dtype)
    return _out((t * pos + (1 - t) * neg) * valid / fgn)


@register("bce_loss")
def _bce(ins, a):
    x, lab = _in(ins, "X", "input"), _in(ins, "Label", "label")
    return _out(-(lab * torch.log(x.clamp_min(1e-12)) + (1 - lab) * torch.log((1 - x).clamp_min(1e-12))))


@register("kldiv_loss")
def _kldiv(ins, a):
    x, t = _in(ins, "X", "x"), _in(ins, "Target", "label")
    l = torch.where(t > 0, t * (torch.log(t.clamp_min(1e-38)) - x), torch.zeros_like(x))
    red = a.get("reduction", "mean")
    if red == "mean":
        l = l.mean()
    elif red == "sum":
        l = l.sum()
    elif red == "batchmean":
        l = l.sum() / x.shape[0]
    return {"Loss": l, "out": l}


@register("log_loss")
def _log_loss(ins, a):
    p, lab = _in(ins, "Predicted", "input"), _in(ins, "Labels", "label")
    e = float(a.get("epsilon", 1e-4))
    l = -lab * torch.log(p + e) - (1 - lab) * torch.log(1 - p + e)
    return {"Loss": l, "out": l}


@register("smooth_l1_loss")
def _smooth_l1(ins, a):
    x, y = _in(ins, "X"), _in(ins, "Y")
    iw, ow = _in(ins, "InsideWeight"), _in(ins, "OutsideWeight")
    s2 = float(a.get("sigma", 1.0)) ** 2
    d = x - y
    if iw is not None:
        d = d * iw
    ad = d.abs()
    v = torch.where(ad < 1.0 / s2, 0.5 * d * d * s2, ad - 0.5 / s2)
    if ow is not None:
        v = v * ow
    return {"Diff": d, "Out": v.reshape(v.shape[0], -1).sum(1, keepdim=True)}


@register("huber_loss")
def _huber(ins, a):
    x, y = _in(ins, "X", "input"), _in(ins, "Y", "label")
    dl = float(a.get("delta", 1.0))
    r = y - x
    ar = r.abs()
    out = torch.where(ar <= dl, 0.5 * r * r, dl * (ar - 0.5 * dl))
    return {"Residual": r, "Out": out, "out": out}


@register("hinge_loss")
def _hinge(ins, a):
    x, lab = _in(ins, "Logits"), _in(ins, "Labels")
    return {"Loss": torch.clamp(1 - x * (2 * lab - 1), min=0)}


@register("modified_huber_loss")
def _mod_huber(ins, a):
    x, y = _in(ins, "X"), _in(ins, "Y")
    iv = x * (2 * y - 1)
    out = torch.where(iv < -1, -4 * iv, torch.where(iv < 1, (1 - iv) ** 2, torch.zeros_like(iv)))
    return {"IntermediateVal": iv, "Out": out}


@register("margin_rank_loss")
def _margin_rank(ins, a):
    x1, x2, lab = _in(ins, "X1"), _in(ins, "X2"), _in(ins, "Label")
    act = -lab * (x1 - x2) + float(a.get("margin", 0.0))
    return {"Activated": (act > 0).to(x1.dtype), "Out": torch.clamp(act, min=0)}


@register("rank_loss")
def _rank_loss(ins, a):
    lab, l, r = _in(ins, "Label"), _in(ins, "Left"), _in(ins, "Right")
    o = l - r
    return _out(torch.log1p(torch.exp(o)) - lab * o)


@register("bpr_loss")
def _bpr(ins, a):
    x, lab = _in(ins, "X"), _in(ins, "Label").reshape(-1).long()
    pos = x.gather(1, lab[:, None])
    mask = torch.ones_like(x, dtype=torch.bool)
    mask[torch.arange(x.shape[0]), lab] = False
    l = -torch.log(torch.sigmoid(pos - x).clamp_min(1e-38))
    return {"Y": (l * mask).sum(1, keepdim=True) / max(x.shape[1] - 1, 1)}


@register("nll_loss")
def _nll(ins, a):
    x, lab, w = _in(ins, "X", "input"), _in(ins, "Label", "label"), _in(ins, "Weight", "weight")
    ig = int(a.get("ignore_index", -100))
    red = a.get("reduction", "mean")
    out = F.nll_loss(x, lab.long(), weight=w, ignore_index=ig, reduction=red)
    wt = (w[lab.long().clamp_min(0)] if w is not None else torch.ones_like(lab, dtype=x.dtype)) * (lab != ig)
    return {"Out": out, "Total_weight": wt.sum().reshape(1), "out": out}


@register("cross_entropy", "cross_entropy2")
def _cross_entropy_v1(ins, a):
    """Reference `cross_entropy_op.cc`: X holds probabilities; Y = −log X[label] (hard, ignore_index
    rows 0) or −Σ label·log X (soft); ``cross_entropy2`` also emits MatchX = X[label]."""
    x, lab = _in(ins, "X"), _in(ins, "Label")
    if a.get("soft_label"):
        y = -(lab * torch.log(x)).sum(-1, keepdim=True)
        return {"Y": y}
    ig = int(a.get("ignore_index", -100))
    li = lab.long().reshape(*x.shape[:-1], 1)
    mx = x.gather(-1, li.clamp_min(0))
    y = torch.where(li == ig, torch.zeros_like(mx), -torch.log(mx))
    return {"Y": y, "MatchX": mx, "XShape": torch.empty(0)}


@register("cross_entropy_with_softmax")
def _xent_softmax_yaml(ins, a):
    return REGISTRY["softmax_with_cross_entropy"]({"Logits": [_in(ins, "Logits", "input")],
                                                   "Label": [_in(ins, "Label", "label")]}, a)


@register("margin_cross_entropy")
def _margin_xent(ins, a):
    from ..nn.functional.extra import margin_cross_entropy
    logits, lab = _in(ins, "Logits", "logits"), _in(ins, "Label", "label")
    from .ops_registry import _ring_group
    loss, sm = margin_cross_entropy(logits, lab, float(a.get("margin1", 1.0)), float(a.get("margin2", 0.5)),
                                    float(a.get("margin3", 0.0)), float(a.get("scale", 64.0)),
                                    group=_ring_group(a), return_softmax=True, reduction=None)
    return {"Softmax": sm, "Loss": loss.reshape(-1, 1)}


@register("warpctc")
def _warpctc(ins, a):
    """Reference `warpctc_op.cc` (padded form): Logits [T, B, C] unnormalised, Label [B, L]."""
    lg, lab = _in(ins, "Logits", "logits"), _in(ins, "Label", "label")
    ll, bl = _in(ins, "LogitsLength", "logits_length"), _in(ins, "LabelLength", "labels_length")
    lp = torch.log_softmax(lg.float(), -1)
    loss = F.ctc_loss(lp, lab.long(), ll.long(), bl.long(), blank=int(a.get("blank", 0)), reduction="none",
                      zero_infinity=False)
    if a.get("norm_by_times"):
        loss = loss / ll.to(loss.dtype)
    return {"Loss": loss.reshape(-1, 1).to(lg.dtype), "WarpCTCGrad": torch.zeros_like(lg)}


@register("teacher_student_sigmoid_loss")
def _ts_sigmoid(ins, a):
    """Reference `teacher_student_sigmoid_loss_op.h`: label < −1 → click 0, no teacher; −1 ≤ label
    < 0 → click 1, no teacher; 0 ≤ label < 1 → click 0, teacher label; label ≥ 1 → click 1,
    teacher label − 1. Loss = sce(x, click) + sce(x, teacher) when a teacher exists."""
    x, lab = _in(ins, "X"), _in(ins, "Label")
    click = ((lab >= -1) & (lab < 0)) | (lab >= 1)
    teacher = torch.where(lab >= 1, lab - 1, lab)
    y = _sce(x, click.to(x.dtype)) + torch.where(lab >= 0, _sce(x, teacher), torch.zeros_like(x))
    return {"Y": y}


@register("center_loss")
def _center_loss(ins, a):
    x, lab, cen, rate = _in(ins, "X"), _in(ins, "Label").reshape(-1).long(), _in(ins, "Centers"), _in(ins, "CenterUpdateRate")
    diff = x - cen[lab]
    loss = 0.5 * (diff * diff).sum(1, keepdim=True)
    cout = cen.clone()
    if a.get("need_update", True):
        with torch.no_grad():
            acc = torch.zeros_like(cen).index_add(0, lab, diff.detach())
            cnt = torch.bincount(lab, minlength=cen.shape[0]).to(cen.dtype)
            cout = cen + float(rate.reshape(-1)[0]) * acc / (1.0 + cnt[:, None])
    return {"CentersOut": cout, "SampleCenterDiff": diff, "Loss": loss}


# ---------------------------------------------------------------------------------- metrics
@register("accuracy")
def _accuracy(ins, a):
    idx, lab = _in(ins, "Indices", "indices"), _in(ins, "Label", "label")
    correct = (idx == lab.reshape(-1, 1)).any(1).sum()
    total = torch.tensor(idx.shape[0], device=idx.device)
    acc = (correct.float() / total.clamp_min(1).float()).reshape(1)
    return {"Accuracy": acc, "Correct": correct.reshape(1).int(), "Total": total.reshape(1).int()}


@register("auc")
def _auc(ins, a):
    """Reference `metrics/auc_op.cc` (ROC, sliding stats): bucketised positive / negative counts,
    trapezoidal area; StatPos / StatNeg carry the histogram across batches."""
    pred, lab = _in(ins, "Predict"), _in(ins, "Label").reshape(-1).long()
    sp, sn = _in(ins, "StatPos"), _in(ins, "StatNeg")
    nt = int(a.get("num_thresholds", 2 ** 12 - 1))
    p = pred[:, -1] if pred.dim() == 2 else pred.reshape(-1)
    b = (p.float() * nt).long().clamp(0, nt)
    pos = torch.bincount(b[lab > 0], minlength=nt + 1).to(sp.dtype)
    neg = torch.bincount(b[lab <= 0], minlength=nt + 1).to(sn.dtype)
    spo = sp.reshape(-1)[-(nt + 1):] + pos if sp.numel() >= nt + 1 else pos
    sno = sn.reshape(-1)[-(nt + 1):] + neg if sn.numel() >= nt + 1 else neg
    tp = torch.cumsum(spo.flip(0).double(), 0)
    fp = torch.cumsum(sno.flip(0).double(), 0)
    tp0, fp0 = F.pad(tp, (1, 0))[:-1], F.pad(fp, (1, 0))[:-1]
    area = ((fp - fp0) * (tp + tp0) / 2).sum()
    tot = tp[-1] * fp[-1]
    auc = (area / tot if tot > 0 else torch.zeros((), dtype=torch.float64)).reshape(1)
    return {"AUC": auc, "StatPosOut": spo.reshape(sp.shape) if sp.numel() == spo.numel() else spo,
            "StatNegOut": sno.reshape(sn.shape) if sn.numel() == sno.numel() else sno}


@register("mean_iou")
def _mean_iou(ins, a):
    p, lab = _in(ins, "Predictions").reshape(-1).long(), _in(ins, "Labels").reshape(-1).long()
    C = int(a.get("num_classes", 2))
    wrong = torch.bincount(p[p != lab], minlength=C) + torch.bincount(lab[p != lab], minlength=C)
    correct = torch.bincount(p[p == lab], minlength=C)
    for t in _inl(ins, "InWrongs"):
        wrong = wrong + t.long()
    for t in _inl(ins, "InCorrects"):
        correct = correct + t.long()
    denom = wrong + correct
    valid = denom > 0
    miou = (correct[valid].float() / denom[valid].float()).sum() / valid.sum().clamp_min(1)
    return {"OutMeanIou": miou.reshape(1), "OutWrong": wrong.int(), "OutCorrect": correct.int()}


@register("edit_distance")
def _edit_distance(ins, a):
    hyps, refs = _in(ins, "Hyps"), _in(ins, "Refs")
    hl, rl = _in(ins, "HypsLength"), _in(ins, "RefsLength")
    B = hyps.shape[0]
    out = []
    for b in range(B):
        h = hyps[b, :int(hl[b])].tolist() if hl is not None else hyps[b].tolist()
        r = refs[b, :int(rl[b])].tolist() if rl is not None else refs[b].tolist()
        d = list(range(len(r) + 1))
        for i, hc in enumerate(h, 1):
            prev, d[0] = d[0], i
            for j, rc in enumerate(r, 1):
                cur = min(d[j] + 1, d[j - 1] + 1, prev + (hc != rc))
                prev, d[j] = d[j], cur
        dist = float(d[-1])
        out.append(dist / max(len(r), 1) if a.get("normalized") else dist)
    return {"Out": torch.tensor(out, dtype=torch.float32, device=hyps.device).reshape(-1, 1),
            "SequenceNum": torch.tensor([B], dtype=torch.int64, device=hyps.device)}


@register("ctc_align")
def _ctc_align(ins, a):
    x, xl = _in(ins, "Input"), _in(ins, "InputLength")
    blank, merge, padv = int(a.get("blank", 0)), bool(a.get("merge_repeated", True)), int(a.get("padding_value", 0))
    rows, lens = [], []
    for b in range(x.shape[0]):
        seq = x[b, :int(xl[b])].reshape(-1).tolist() if xl is not None else x[b].reshape(-1).tolist()
        o, prev = [], None
        for t in seq:
            if t != blank and not (merge and t == prev):
                o.append(t)
            prev = t
        rows.append(o)
        lens.append(len(o))
    L = x.shape[1]
    out = torch.full((x.shape[0], L), padv, dtype=x.dtype, device=x.device)
    for b, o in enumerate(rows):
        if o:
            out[b, :len(o)] = torch.tensor(o, dtype=x.dtype)
    return {"Output": out, "OutputLength": torch.tensor(lens, dtype=torch.int64, device=x.device).reshape(-1, 1)}


@register("viterbi_decode")
def _viterbi(ins, a):
    from ..text import viterbi_decode
    s, p = viterbi_decode(_in(ins, "Input"), _in(ins, "Transition"), _in(ins, "Length"),
                          bool(a.get("include_bos_eos_tag", True)))
    return {"Scores": s, "Path": p}


# --------------------------------------------------------------------------- misc framework
@register("depend")
def _depend(ins, a):
    return _out(_x(ins))


@register("share_data", "share_buffer", "memcpy", "memcpy_h2d", "memcpy_d2h", "copy_to", "assign_out_",
          "c_wait_comm", "c_wait_compute", "print", "transfer_layout")
def _passthrough(ins, a):
    xs = _inl(ins, "X", "x", "In")
    v = xs[0] if len(xs) == 1 else xs
    return {"Out": v, "out": v, "XOut": v}


@register("transfer_dtype")
def _transfer_dtype(ins, a):
    return _out(_x(ins).to(_dtype(a, "out_dtype")))


@register("assert")
def _assert(ins, a):
    c = _in(ins, "Cond")
    if c is not None and not bool(c.reshape(-1).all()):
        raise AssertionError("assert op: condition is False")
    return {}


@register("delete_var")
def _delete_var(ins, a):
    return {}


@register("alloc_float_status")
def _alloc_float_status(ins, a):
    return {"FloatStatus": torch.zeros(8, dtype=torch.float32, device=_dev(ins))}


@register("clear_float_status")
def _clear_float_status(ins, a):
    return {"FloatStatusOut": torch.zeros_like(_in(ins, "FloatStatus"))}


@register("get_float_status")
def _get_float_status(ins, a):
    return {"FloatStatusOut": _in(ins, "FloatStatus")}


@register("coalesce_tensor")
def _coalesce_tensor(ins, a):
    """Reference `coalesce_tensor_op.cc`: one fused buffer, Output[i] views into it (copy_data /
    set_constant fill it)."""
    xs = _inl(ins, "Input", "input")
    dt = _dtype(a) if a.get("dtype") not in (None, -1) else xs[0].dtype
    total = sum(t.numel() for t in xs)
    fused = torch.empty(total, dtype=dt, device=xs[0].device)
    if a.get("set_constant"):
        fused.fill_(float(a.get("constant", 0.0)))
    outs, off = [], 0
    for t in xs:
        v = fused[off:off + t.numel()].view(t.shape)
        if a.get("copy_data"):
            v.copy_(t)
        outs.append(v)
        off += t.numel()
    return {"Output": outs, "FusedOutput": fused}


@register("dropout_nd")
def _dropout_nd(ins, a):
    x = _x(ins)
    p = float(a.get("dropout_prob", 0.5))
    up = a.get("dropout_implementation", "downgrade_in_infer") == "upscale_in_train"
    if a.get("is_test"):
        return {"Out": x if up else x * (1 - p)}
    axes = a.get("axis") or list(range(x.dim()))
    ms = [x.shape[i] if i in axes else 1 for i in range(x.dim())]
    m = (torch.rand(ms, device=x.device) >= p).to(x.dtype)
    y = x * m / (1 - p) if up else x * m
    return {"Out": y, "Mask": m.to(torch.uint8).expand_as(x)}


@register("gumbel_softmax")
def _gumbel_softmax(ins, a):
    from ..nn.functional import gumbel_softmax
    return _out(gumbel_softmax(_x(ins), float(a.get("temperature", 1.0)), bool(a.get("hard", False)),
                               int(a.get("axis", -1))))


@register("rrelu")
def _rrelu(ins, a):
    x = _x(ins)
    lo, up = float(a.get("lower", 1 / 8)), float(a.get("upper", 1 / 3))
    if a.get("is_test", False):
        noise = torch.full_like(x, (lo + up) / 2)
    else:
        noise = torch.empty_like(x).uniform_(lo, up)
    noise = torch.where(x >= 0, torch.ones_like(x), noise)
    return {"Out": x * noise, "Noise": noise}


@register("label_smooth")
def _label_smooth(ins, a):
    x, pd = _in(ins, "X", "label"), _in(ins, "PriorDist", "prior_dist")
    e = float(a.get("epsilon", 0.0))
    return _out((1 - e) * x + e * (pd if pd is not None else 1.0 / x.shape[-1]))


@register("spectral_norm")
def _spectral_norm_op(ins, a):
    """Reference `spectral_norm_op.cc`: power iterations on U / V, Out = W / σ."""
    w, u, v = _in(ins, "Weight", "weight"), _in(ins, "U", "u"), _in(ins, "V", "v")
    dim, it, eps = int(a.get("dim", 0)), int(a.get("power_iters", 1)), float(a.get("eps", 1e-12))
    wm = w.permute([dim] + [d for d in range(w.dim()) if d != dim]) if dim != 0 else w
    wm = wm.reshape(wm.shape[0], -1)
    u, v = u.reshape(-1), v.reshape(-1)
    with torch.no_grad():
        for _ in range(it):
            v = wm.t() @ u
            v = v / (v.norm() + eps)
            u = wm @ v
            u = u / (u.norm() + eps)
    sigma = torch.dot(u, wm @ v)
    return _out(w / sigma)


@register("add_position_encoding")
def _add_pos_enc(ins, a):
    """Reference `add_position_encoding_op.h`: out = α·x + β·PE, PE[pos, k] = sin(pos / 10000^{k/(half−1)})
    for k < half, cos(…) for the second half."""
    x = _x(ins)
    al, be = float(a.get("alpha", 1.0)), float(a.get("beta", 1.0))
    B, T, D = x.shape
    half = D // 2
    pos = torch.arange(T, device=x.device, dtype=torch.float32)[:, None]
    k = torch.arange(half, device=x.device, dtype=torch.float32)[None]
    ang = pos / torch.pow(10000.0, k / max(half - 1, 1))
    pe = torch.cat([torch.sin(ang), torch.cos(ang)], 1)
    return _out(al * x + be * pe.to(x.dtype))


@register("polygon_box_transform")
def _polygon_box_transform(ins, a):
    x = _in(ins, "Input")
    N, G, H, W = x.shape
    iw = torch.arange(W, device=x.device, dtype=x.dtype)[None, None, None, :] * 4
    ih = torch.arange(H, device=x.device, dtype=x.dtype)[None, None, :, None] * 4
    even = (torch.arange(G, device=x.device) % 2 == 0)[None, :, None, None]
    return {"Output": torch.where(even, iw - x, ih - x)}


@register("box_clip")
def _box_clip(ins, a):
    b, im = _in(ins, "Input", "input"), _in(ins, "ImInfo", "im_info")
    h = torch.round(im[:, 0] / im[:, 2])
    w = torch.round(im[:, 1] / im[:, 2])
    shp = [-1] + [1] * (b.dim() - 2)
    bw, bh = (w - 1).reshape(shp), (h - 1).reshape(shp)
    out = torch.stack([b[..., 0].clamp(min=0).minimum(bw), b[..., 1].clamp(min=0).minimum(bh),
                       b[..., 2].clamp(min=0).minimum(bw), b[..., 3].clamp(min=0).minimum(bh)], -1)
    return {"Output": out, "out": out}


@register("iou_similarity")
def _iou_similarity(ins, a):
    from ..vision.ops import _jaccard
    x, y = _in(ins, "X", "x"), _in(ins, "Y", "y")
    nrm = bool(a.get("box_normalized", True))
    return _out(torch.stack([_jaccard(x[i], y, nrm) for i in range(x.shape[0])]) if x.shape[0] else
                x.new_zeros((0, y.shape[0])))


@register("anchor_generator")
def _anchor_generator(ins, a):
    """Reference `detection/anchor_generator_op.h`: anchors [H, W, A, 4] per feature-map cell."""
    x = _in(ins, "Input")
    H, W = x.shape[2], x.shape[3]
    sizes = [float(s) for s in a.get("anchor_sizes", [64, 128, 256, 512])]
    ratios = [float(r) for r in a.get("aspect_ratios", [0.5, 1.0, 2.0])]
    sw, sh = [float(s) for s in a.get("stride", [16.0, 16.0])]
    off = float(a.get("offset", 0.5))
    base = []
    for r in ratios:
        for s in sizes:
            area = sw * sh
            bw = round(math.sqrt(area / r))
            bh = round(bw * r)
            aw = (s / sw) * bw
            ah = (s / sh) * bh
            base.append((aw, ah))
    xc = torch.arange(W, dtype=torch.float32, device=x.device) * sw + off * (sw - 1)
    yc = torch.arange(H, dtype=torch.float32, device=x.device) * sh + off * (sh - 1)
    wh = torch.tensor(base, dtype=torch.float32, device=x.device)
    cx, cy = xc[None, :, None], yc[:, None, None]
    anchors = torch.stack([cx - 0.5 * (wh[None, None, :, 0] - 1), cy - 0.5 * (wh[None, None, :, 1] - 1),
                           cx + 0.5 * (wh[None, None, :, 0] - 1), cy + 0.5 * (wh[None, None, :, 1] - 1)], -1)
    var = torch.tensor(a.get("variances", [0.1, 0.1, 0.2, 0.2]), dtype=torch.float32,
                       device=x.device).expand_as(anchors).contiguous()
    return {"Anchors": anchors.to(x.dtype), "Variances": var.to(x.dtype)}


# -------------------------------------------------------------------------------- optimizers
def _mp(ins):
    mp = _in(ins, "MasterParam")
    return mp


def _opt_param(ins, a):
    """(param to update in f32 — the master copy under multi_precision — , the stored param)."""
    p = _in(ins, "Param", "param")
    mp = _mp(ins)
    return (mp if (mp is not None and a.get("multi_precision")) else p), p


def _write_back(p, master):
    if master is not p:
        with torch.no_grad():
            p.copy_(master.to(p.dtype))


@register("adadelta", "adadelta_")
def _adadelta(ins, a):
    """Reference `impl/adadelta_kernel_impl.h`: E[g²] ← ρE[g²] + (1−ρ)g²; Δ = −√((E[Δ²]+ε)/(E[g²]+ε))·g;
    E[Δ²] ← ρE[Δ²] + (1−ρ)Δ²; p += Δ (lr scales Δ when given)."""
    w, p = _opt_param(ins, a)
    g = _in(ins, "Grad", "grad").float()
    sg, su = _in(ins, "AvgSquaredGrad", "avg_squared_grad"), _in(ins, "AvgSquaredUpdate", "avg_squared_update")
    rho, eps = float(a.get("rho", 0.95)), float(a.get("epsilon", 1e-6))
    sg.mul_(rho).add_((1 - rho) * g * g)
    upd = -torch.sqrt((su + eps) / (sg + eps)) * g
    su.mul_(rho).add_((1 - rho) * upd * upd)
    lr = _in(ins, "LearningRate", "learning_rate")
    w.add_((upd * (lr.reshape(()).float() if lr is not None else 1.0)).to(w.dtype))
    _write_back(p, w)
    return {"ParamOut": p, "AvgSquaredGradOut": sg, "AvgSquaredUpdateOut": su, "param_out": p,
            "moment_out": sg, "inf_norm_out": su, "MasterParamOut": w}


@register("adagrad", "adagrad_")
def _adagrad(ins, a):
    """Reference `adagrad` (dense): moment += g²; p −= lr·g / (√moment + ε)."""
    w, p = _opt_param(ins, a)
    g = _reg(w, _in(ins, "Grad", "grad").float(), a)
    m = _in(ins, "Moment", "moment")
    m.add_(g * g)
    w.sub_((_lr(ins) * g / (torch.sqrt(m) + float(a.get("epsilon", 1e-6)))).to(w.dtype))
    _write_back(p, w)
    return {"ParamOut": p, "MomentOut": m, "param_out": p, "moment_out": m, "MasterParamOut": w}


@register("adamax", "adamax_")
def _adamax(ins, a):
    """Reference `impl/adamax_kernel_impl.h`: m ← β1m + (1−β1)g; u ← max(|g|, β2u + ε);
    p −= lr/(1−β1^t)·m/u (Beta1Pow is advanced by the optimizer's own scale op)."""
    w, p = _opt_param(ins, a)
    g = _in(ins, "Grad", "grad").float()
    m, u, b1p = _in(ins, "Moment", "moment"), _in(ins, "InfNorm", "inf_norm"), _in(ins, "Beta1Pow", "beta1_pow")
    b1, b2, eps = float(a.get("beta1", 0.9)), float(a.get("beta2", 0.999)), float(a.get("epsilon", 1e-8))
    m.mul_(b1).add_((1 - b1) * g)
    u.copy_(torch.maximum(g.abs(), b2 * u + eps))
    w.sub_((_lr(ins) / (1 - b1p.reshape(()).float()) * m / u).to(w.dtype))
    _write_back(p, w)
    return {"ParamOut": p, "MomentOut": m, "InfNormOut": u, "param_out": p, "avg_squared_grad_out": m,
            "avg_squared_update_out": u, "MasterParamOut": w}


@register("lamb", "lamb_")
def _lamb(ins, a):
    """Reference `funcs/lamb_functors.h` + `impl/lamb_kernel_impl.h`: r = m̂/(√v̂ + ε) + wd·p,
    trust = ‖p‖/‖r‖ (1 when either is 0), p −= lr·trust·r; beta pows advanced in place."""
    w, p = _opt_param(ins, a)
    if _skip(ins):
        return {"ParamOut": p}
    g = _in(ins, "Grad", "grad").float()
    m1, m2 = _in(ins, "Moment1", "moment1"), _in(ins, "Moment2", "moment2")
    b1p, b2p = _in(ins, "Beta1Pow", "beta1_pow"), _in(ins, "Beta2Pow", "beta2_pow")
    b1, b2 = float(a.get("beta1", 0.9)), float(a.get("beta2", 0.999))
    eps, wd = float(a.get("epsilon", 1e-6)), float(a.get("weight_decay", 0.01))
    m1.mul_(b1).add_((1 - b1) * g)
    m2.mul_(b2).add_((1 - b2) * g * g)
    r = (m1 / (1 - b1p.reshape(()).float())) / (torch.sqrt(m2 / (1 - b2p.reshape(()).float())) + eps) + wd * w.float()
    pn, rn = torch.linalg.vector_norm(w.float()), torch.linalg.vector_norm(r)
    trust = torch.where((pn > 0) & (rn > 0), pn / rn, torch.ones_like(pn))
    w.sub_((_lr(ins) * trust * r).to(w.dtype))
    b1p.mul_(b1)
    b2p.mul_(b2)
    _write_back(p, w)
    return {"ParamOut": p, "Moment1Out": m1, "Moment2Out": m2, "Beta1PowOut": b1p, "Beta2PowOut": b2p,
            "MasterParamOut": w}


@register("rmsprop", "rmsprop_")
def _rmsprop(ins, a):
    """Reference `impl/rmsprop_kernel_impl.h` (dense): ms ← ρms + (1−ρ)g²; (centered) mg ← ρmg + (1−ρ)g;
    mom ← μ·mom + lr·g/√(ms [− mg²] + ε); p −= mom."""
    w, p = _opt_param(ins, a)
    g = _in(ins, "Grad", "grad").float()
    ms, mom = _in(ins, "MeanSquare", "mean_square"), _in(ins, "Moment", "moment")
    mg = _in(ins, "MeanGrad", "mean_grad")
    rho, eps, mu = float(a.get("decay", 0.9)), float(a.get("epsilon", 1e-10)), float(a.get("momentum", 0.0))
    ms.mul_(rho).add_((1 - rho) * g * g)
    if a.get("centered"):
        mg.mul_(rho).add_((1 - rho) * g)
        den = torch.sqrt(ms - mg * mg + eps)
    else:
        den = torch.sqrt(ms + eps)
    mom.mul_(mu).add_(_lr(ins) * g / den)
    w.sub_(mom.to(w.dtype))
    _write_back(p, w)
    out = {"ParamOut": p, "MomentOut": mom, "MeanSquareOut": ms, "param_out": p, "moment_out": mom,
           "mean_square_out": ms, "MasterParamOut": w}
    if mg is not None:
        out.update(MeanGradOut=mg, mean_grad_out=mg)
    return out


@register("lars_momentum")
def _lars_momentum(ins, a):
    """Reference `lars_momentum_op.cu`: local_lr = lr·coeff·‖p‖/(‖g‖ + wd·‖p‖ + ε) (lr when a norm is
    0); v ← μv + local_lr·(g + wd·p); p −= v. Param / Grad / Velocity are lists (merged form)."""
    ps, gs, vs = _inl(ins, "Param"), _inl(ins, "Grad"), _inl(ins, "Velocity")
    mps = _inl(ins, "MasterParam")
    lrs = _inl(ins, "LearningRate")
    mu, coeff, eps = float(a.get("mu", 0.9)), float(a.get("lars_coeff", 0.001)), float(a.get("epsilon", 0.0))
    wds = a.get("lars_weight_decay", [0.0005])
    wds = wds if isinstance(wds, (list, tuple)) else [wds]
    rescale = float(a.get("rescale_grad", 1.0))
    outs_p, outs_v, outs_m = [], [], []
    for i, (p, g, v) in enumerate(zip(ps, gs, vs)):
        w = mps[i] if (mps and a.get("multi_precision")) else p
        lr = lrs[min(i, len(lrs) - 1)].reshape(()).float()
        wd = float(wds[min(i, len(wds) - 1)])
        gf = g.float() * rescale
        pn, gn = torch.linalg.vector_norm(w.float()), torch.linalg.vector_norm(gf)
        local = torch.where((pn > 0) & (gn > 0), lr * coeff * pn / (gn + wd * pn + eps), lr)
        v.mul_(mu).add_(local * (gf + wd * w.float()))
        w.sub_(v.to(w.dtype))
        _write_back(p, w)
        outs_p.append(p)
        outs_v.append(v)
        outs_m.append(w)
    return {"ParamOut": outs_p, "VelocityOut": outs_v, "MasterParamOut": outs_m}


@register("merged_adam", "merged_adam_")
def _merged_adam(ins, a):
    """Reference `merged_adam_op`: the adam update over lists of parameters (one fused step)."""
    ps = _inl(ins, "Param", "param")
    n = len(ps)
    outs = {k: [] for k in ("ParamOut", "Moment1Out", "Moment2Out", "Beta1PowOut", "Beta2PowOut", "MasterParamOut")}
    lrs = _inl(ins, "LearningRate", "learning_rate")
    for i in range(n):
        sub = {"Param": [ps[i]], "Grad": [_inl(ins, "Grad", "grad")[i]],
               "LearningRate": [lrs[min(i, len(lrs) - 1)]],
               "Moment1": [_inl(ins, "Moment1", "moment1")[i]], "Moment2": [_inl(ins, "Moment2", "moment2")[i]],
               "Beta1Pow": [_inl(ins, "Beta1Pow", "beta1_pow")[i if not a.get("use_global_beta_pow") else 0]],
               "Beta2Pow": [_inl(ins, "Beta2Pow", "beta2_pow")[i if not a.get("use_global_beta_pow") else 0]]}
        mp = _inl(ins, "MasterParam", "master_param")
        master = mp[i] if (mp and a.get("multi_precision")) else None
        if master is not None:
            sub["Param"] = [master]
        if a.get("use_global_beta_pow") and i > 0:
            b1, b2 = sub["Beta1Pow"][0], sub["Beta2Pow"][0]
            sub["Beta1Pow"], sub["Beta2Pow"] = [b1.clone()], [b2.clone()]
        r = REGISTRY["adam"](sub, a)
        if master is not None:
            _write_back(ps[i], master)
        outs["ParamOut"].append(ps[i])
        outs["Moment1Out"].append(r["Moment1Out"])
        outs["Moment2Out"].append(r["Moment2Out"])
        outs["Beta1PowOut"].append(r["Beta1PowOut"])
        outs["Beta2PowOut"].append(r["Beta2PowOut"])
        outs["MasterParamOut"].append(master if master is not None else ps[i])
    return outs


@register("merged_momentum", "merged_momentum_")
def _merged_momentum(ins, a):
    """Reference `merged_momentum_op`: the momentum update over lists of parameters; per-parameter
    regularization_method / regularization_coeff lists."""
    ps = _inl(ins, "Param", "param")
    lrs = _inl(ins, "LearningRate", "learning_rate")
    meth = a.get("regularization_method") or []
    coef = a.get("regularization_coeff") or []
    mps = _inl(ins, "MasterParam", "master_param")
    po, vo, mo = [], [], []
    for i, p in enumerate(ps):
        master = mps[i] if (mps and a.get("multi_precision")) else None
        sub = {"Param": [master if master is not None else p], "Grad": [_inl(ins, "Grad", "grad")[i]],
               "Velocity": [_inl(ins, "Velocity", "velocity")[i]], "LearningRate": [lrs[min(i, len(lrs) - 1)]]}
        aa = dict(mu=a.get("mu", 0.9), use_nesterov=a.get("use_nesterov", False),
                  rescale_grad=a.get("rescale_grad", 1.0))
        if i < len(meth) and meth[i]:
            aa.update(regularization_method=meth[i], regularization_coeff=coef[i] if i < len(coef) else 0.0)
        r = REGISTRY["momentum"](sub, aa)
        if master is not None:
            _write_back(p, master)
        po.append(p)
        vo.append(r["VelocityOut"])
        mo.append(master if master is not None else p)
    return {"ParamOut": po, "VelocityOut": vo, "MasterParamOut": mo}


@register("sparse_momentum")
def _sparse_momentum(ins, a):
    """Reference `sparse_momentum_op`: the momentum update on the rows ``Index`` along ``axis``."""
    p, g, v, idx = _in(ins, "Param"), _in(ins, "Grad"), _in(ins, "Velocity"), _in(ins, "Index").reshape(-1).long()
    ax = int(_in(ins, "Axis").reshape(-1)[0]) if _in(ins, "Axis") is not None else int(a.get("axis", 0))
    dense = torch.zeros_like(p, dtype=torch.float32).index_add(ax, idx, g.float())
    r = REGISTRY["momentum"]({"Param": [p], "Grad": [dense], "Velocity": [v],
                              "LearningRate": ins["LearningRate"]}, a)
    return {"ParamOut": r["ParamOut"], "VelocityOut": r["VelocityOut"]}


@register("average_accumulates", "average_accumulates_")
def _average_accumulates(ins, a):
    """Reference `average_accumulates_op.h` (ModelAverage): sums of the parameter over windows."""
    p = _in(ins, "param")
    s1, s2, s3 = _in(ins, "in_sum_1"), _in(ins, "in_sum_2"), _in(ins, "in_sum_3")
    na, ona, nu = (_in(ins, k) for k in ("in_num_accumulates", "in_old_num_accumulates", "in_num_updates"))
    aw, mx, mn = float(a.get("average_window", 0)), int(a.get("max_average_window", 10000)), \
        int(a.get("min_average_window", 10000))
    n_upd = int(nu.reshape(-1)[0]) + 1
    n_acc = int(na.reshape(-1)[0]) + 1
    n_old = int(ona.reshape(-1)[0])
    s1 = s1 + p
    if n_upd % 16384 == 0:  # kMaxNumAccumulates: fold sum_1 into sum_2 for precision
        s2, s1 = s2 + s1, torch.zeros_like(s1)
    if n_acc >= mn and n_acc >= min(mx, n_upd * aw):
        s3, s1, s2 = s1 + s2, torch.zeros_like(s1), torch.zeros_like(s2)
        n_old, n_acc = n_acc, 0
    mk = lambda v, t: torch.tensor([v], dtype=t.dtype, device=t.device)  # noqa: E731
    return {"out_sum_1": s1, "out_sum_2": s2, "out_sum_3": s3, "out_num_accumulates": mk(n_acc, na),
            "out_old_num_accumulates": mk(n_old, ona), "out_num_updates": mk(n_upd, nu)}


# ------------------------------------------------------------------------- static collectives
def _pg(a):
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return None, 1
    from .ops_registry_ext import _group
    g = _group(a)
    return g, dist.get_world_size(g)


@register("c_allgather", "partial_allgather")
def _c_allgather(ins, a):
    """Reference `collective/c_allgather_op.cc`: rank-major concatenation along dim 0 (RCCL
    all_gather_into_tensor; ``partial_allgather``: every rank holds the full tensor and contributes
    its 1/nranks slice)."""
    import torch.distributed as dist
    x = _x(ins).contiguous()
    g, W = _pg(a)
    if W == 1:
        return _out(x)
    if "rank" in a and a.get("nranks"):  # partial_allgather
        r = int(a["rank"])
        part = x.reshape(-1).chunk(W)[r].contiguous()
        out = torch.empty(part.numel() * W, dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, part, group=g)
        return _out(out.view(x.shape))
    out = torch.empty((W * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out.view(-1), x.view(-1), group=g)
    return _out(out)


@register("c_reducescatter")
def _c_reducescatter(ins, a):
    """Reference `collective/c_reducescatter_op.cc`: sum over ranks, rank r keeps rows
    [r·n/W, (r+1)·n/W) of dim 0."""
    import torch.distributed as dist
    x = _x(ins).contiguous()
    g, W = _pg(a)
    if W == 1:
        return _out(x)
    out = torch.empty((x.shape[0] // W,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out.view(-1), x.view(-1), group=g)
    return _out(out)


@register("alltoall")
def _alltoall(ins, a):
    """Reference `collective/alltoall_op.cc`: dim 0 split into W equal blocks, block j goes to rank j."""
    import torch.distributed as dist
    x = _x(ins).contiguous()
    g, W = _pg(a)
    if W == 1:
        return _out(x)
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x, group=g)
    return _out(out)


@register("sync_batch_norm", "sync_batch_norm_")
def _sync_batch_norm(ins, a):
    """Reference `sync_batch_norm_op` (batch_norm slots): training statistics over every rank of the
    ring (own Welford kernels + RCCL all-gather, `ops.batchnorm.sync_batch_norm`)."""
    from ..ops.batchnorm import sync_batch_norm
    x = _in(ins, "X", "x")
    rm, rv = _in(ins, "Mean", "mean"), _in(ins, "Variance", "variance")
    train = not a.get("is_test", False) and not a.get("use_global_stats", False)
    g, _ = _pg(a)
    y = sync_batch_norm(x, rm, rv, _in(ins, "Scale", "scale"), _in(ins, "Bias", "bias"), train,
                        float(a.get("momentum", 0.9)), float(a.get("epsilon", 1e-5)), g,
                        a.get("data_layout", "NCHW"))
    return {"Y": y, "out": y, "MeanOut": rm, "VarianceOut": rv, "mean_out": rm, "variance_out": rv}


def _global_exchange(ins, a, gather):
    """Reference `collective/global_scatter_op.cc` / `global_gather_op.cc` (MoE token exchange):
    rows grouped by (rank, expert) counts. scatter sends ``local_count`` rows per rank and receives
    ``global_count``; gather is the inverse exchange."""
    import torch.distributed as dist
    x = _x(ins)
    lc, gc = _in(ins, "local_count"), _in(ins, "global_count")
    g, W = _pg(a)
    if W == 1:
        return _out(x)
    send = [int(v) for v in lc.reshape(W, -1).sum(1).tolist()]
    recv = [int(v) for v in gc.reshape(W, -1).sum(1).tolist()]
    if gather:
        send, recv = recv, send
    out = torch.empty((sum(recv),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_to_all_single(out, x.contiguous(), recv, send, group=g)
    return _out(out)


register("global_scatter")(lambda ins, a: _global_exchange(ins, a, False))
register("global_gather")(lambda ins, a: _global_exchange(ins, a, True))


# --------------------------------------------------------------------- fork serving / MoE ops
@register("weight_quantize")
def _weight_quantize(ins, a):
    """yaml `weight_quantize`: x [K, N] → (out: this framework's MFMA-tile packed int8 [N, K] /
    int4 [N/2, K] — or row-major [N, K] for llm.int8 —, scale [N])."""
    from ..ops.inference import weight_quantize
    x = _x(ins)
    q, s = weight_quantize(x, a.get("algo", "weight_only_int8"))
    return {"out": q.view(torch.int8) if q.dtype == torch.uint8 else q, "scale": s.to(x.dtype),
            "Out": q, "Scale": s}


@register("weight_dequantize")
def _weight_dequantize(ins, a):
    from ..inference.ref_layout import canonical_weight
    from ..ops.inference import weight_dequantize
    x, s = _in(ins, "x", "X"), _in(ins, "scale", "Scale")
    algo = a.get("algo", "weight_only_int8")
    w = canonical_weight(x, s, "int4" if algo == "weight_only_int4" else "int8")
    od = a.get("out_dtype", "float16")
    if not isinstance(od, str):
        od = {v: k for k, v in __import__("paddle_infer_amd.static.proto", fromlist=["VT"]).VT.items()}.get(int(od), "float16")
    return _out(weight_dequantize(w, s.float(), algo, od))


@register("weight_only_linear2")
def _weight_only_linear2(ins, a):
    """yaml `weight_only_linear2` (x, weight, bias, weight_scale, m, n, k): the weight-only GEMM
    with the GEMM extents given as attributes (x viewed [m, k])."""
    x = _in(ins, "x", "X")
    k = int(a.get("k", x.shape[-1]))
    xv = x.reshape(-1, k)
    r = REGISTRY["weight_only_linear"]({"x": [xv], "weight": ins["weight"], "bias": ins.get("bias") or [],
                                        "weight_scale": ins["weight_scale"]},
                                       {"weight_dtype": a.get("weight_dtype", "int8"),
                                        "act_method": a.get("act_method", "none")})
    y = r["out"]
    return _out(y.reshape(*x.shape[:-1], y.shape[-1]))


@register("flash_attn_unpadded")
def _flash_attn_unpadded(ins, a):
    """yaml `flash_attn_unpadded`: packed [total_tokens, H, D] q/k/v with cumulative offsets —
    the variable-length MFMA flash kernel (`ops.attention.flash_attention_varlen`)."""
    from .. import ops
    q, k, v = _in(ins, "q"), _in(ins, "k"), _in(ins, "v")
    cq, ck = _in(ins, "cu_seqlens_q"), _in(ins, "cu_seqlens_k")
    mask = _in(ins, "attn_mask")
    p = 0.0 if a.get("is_test", False) else float(a.get("dropout", 0.0))
    if mask is not None:  # additive mask over the padded [B, H, Sq, Sk] view: the dense path per sequence
        outs = []
        cql, ckl = cq.tolist(), ck.tolist()
        for b in range(len(cql) - 1):
            qs, ks, vs = q[cql[b]:cql[b + 1]], k[ckl[b]:ckl[b + 1]], v[ckl[b]:ckl[b + 1]]
            mb = mask[b] if mask.dim() == 4 else mask
            mb = mb[..., :qs.shape[0], :ks.shape[0]]
            outs.append(ops.flash_attention(qs[None], ks[None], vs[None], causal=bool(a.get("causal", False)),
                                            scale=a.get("scale"), attn_mask=mb[None] if mb.dim() == 3 else mb,
                                            dropout_p=p)[0])
        o = torch.cat(outs, 0)
    else:
        o = ops.flash_attention_varlen(q, k, v, cq, ck, int(a.get("max_seqlen_q", 0)), int(a.get("max_seqlen_k", 0)),
                                       causal=bool(a.get("causal", False)), scale=a.get("scale"), dropout_p=p,
                                       training=not a.get("is_test", False))
    return {"out": o, "Out": o, "softmax": torch.empty(0, device=o.device),
            "softmax_lse": torch.empty(0, device=o.device), "seed_offset": torch.zeros(2, dtype=torch.int64)}


@register("number_count_v2", "number_count")
def _number_count(ins, a):
    """yaml `number_count_v2` (MoE): per-expert counts of the routed expert ids (ids outside
    [0, upper_range) — dropped slots — are not counted)."""
    x = _in(ins, "numbers", "x", "X").reshape(-1).long()
    up = int(a.get("upper_range", 0))
    ok = (x >= 0) & (x < up)
    return _out(torch.bincount(x[ok], minlength=up)[:up].to(torch.int64))


@register("fused_moe_kernel")
def _fused_moe_kernel(ins, a):
    """yaml `fused_moe_kernel` (reference `phi/kernels/gpu/fused_moe_kernel.cu`): h = LN(x) (pre-LN) or
    x; gate = h·Wg + bg; top-k of the RAW gate logits (their values weight the experts, no softmax);
    expert e: GELU(h·W1_e + b1_e)·W2_e + b2_e; out = x + Σ_k gate_k·expert_k(h); post-LN when not
    pre_layer_norm. Tensor-parallel token slicing (mp_size) with an all-gather; expert parallel
    (world_size) through the all-to-all dispatch. Single-rank experts run the framework's grouped
    MFMA GEMMs (`ops.moe.grouped_ffn`) on a sorted-row routing."""
    from ..incubate.nn import functional as IF
    from ..ops import moe as gm
    import torch.distributed as dist
    x = _in(ins, "x", "X")
    gw, gb = _in(ins, "gate_weight"), _in(ins, "gate_bias")
    lns, lnb = _in(ins, "ln_scale"), _in(ins, "ln_bias")
    w1s, b1s = _inl(ins, "experts_weight1"), _inl(ins, "experts_bias1")
    w2s, b2s = _inl(ins, "experts_weight2"), _inl(ins, "experts_bias2")
    pre = bool(a.get("pre_layer_norm", True))
    eps = float(a.get("ln_epsilon", 1e-5))
    topk = int(a.get("topk", 2))
    mp, mpr, ne, ws = int(a.get("mp_size", 1)), int(a.get("mp_rank", 0)), int(a.get("num_expert", len(w1s))), \
        int(a.get("world_size", 1))
    act = "gelu_tanh" if a.get("approximate") else "gelu"
    B, S, Dm = x.shape
    x2 = x.reshape(-1, Dm)
    h = F.layer_norm(x2.float(), (Dm,), lns.float(), lnb.float(), eps).to(x.dtype) if pre else x2
    T = h.shape[0]
    if mp > 1:
        st = T // ws * mpr
        h = h[st:min(st + T // ws, T)]
    logits = h @ gw.to(h.dtype) + gb.to(h.dtype)
    val, idx = torch.topk(logits, topk, -1)
    from .ops_registry import _ring_group
    grp = _ring_group({"ring_id": a.get("moe_ring_id", -1)}) if ws > 1 else None
    if ws > 1 and grp is not None and dist.get_world_size(grp) > 1:
        from ..incubate.moe import dispatch, combine as ep_combine, run_experts
        xs, counts, ctx = dispatch(h, idx, ne, grp)
        experts = [(lambda t, e=e: F.gelu(t @ w1s[e] + b1s[e], approximate="tanh" if act == "gelu_tanh" else "none")
                    @ w2s[e] + b2s[e]) for e in range(ne)]
        y = ep_combine(run_experts(xs, counts, experts), val, ctx)
    else:
        r = gm.permute(idx, ne, align=64 if h.is_cuda else 1)
        w1 = torch.stack(list(w1s))
        w2 = torch.stack(list(w2s))
        b1 = torch.stack([b.reshape(-1) for b in b1s]) if b1s else None
        b2 = torch.stack([b.reshape(-1) for b in b2s]) if b2s else None
        ys = gm.grouped_ffn(gm.gather(h, r), w1, b1, w2, b2, r, act=act)
        y = gm.combine(ys, val, r)
    if mp > 1:
        parts = [torch.empty_like(y) for _ in range(mp)]
        dist.all_gather(parts, y.contiguous(), group=_ring_group({"ring_id": a.get("moe_ring_id", 0)}))
        y = torch.cat(parts, 0)
    out = (x2 + y.to(x.dtype)).reshape(x.shape)
    if not pre:
        out = F.layer_norm(out.float(), (Dm,), lns.float(), lnb.float(), eps).to(x.dtype)
    del IF
    return _out(out)


@register("random_routing")
def _random_routing(ins, a):
    """Reference `random_routing_op.cu` (gshard): the second expert of a token is dropped (−1) when
    2·value < the token's uniform sample."""
    prob, val, idx = _in(ins, "Prob"), _in(ins, "TopK_Value"), _in(ins, "TopK_Idx")
    out = idx.clone()
    drop = 2 * val[:, 1] < prob.reshape(-1)
    out[:, 1] = torch.where(drop, torch.full_like(out[:, 1], -1), out[:, 1])
    return _out(out)


@register("class_center_sample")
def _class_center_sample(ins, a):
    from ..nn.functional.extra import class_center_sample
    from .ops_registry import _ring_group
    lab = _in(ins, "Label", "label")
    rl, sc = class_center_sample(lab, int(a["num_classes"]), int(a["num_samples"]), group=_ring_group(a))
    return {"RemappedLabel": rl, "SampledLocalClassCenter": sc}


# ----------------------------------------------------------------------------------- RNN ops
def _act_by_name(n):
    return {"sigmoid": torch.sigmoid, "tanh": torch.tanh, "relu": torch.relu, "identity": lambda t: t,
            "": lambda t: t, None: lambda t: t}[n]


def _act_by_id(i):
    return {0: lambda t: t, 1: torch.sigmoid, 2: torch.tanh, 3: torch.relu}[int(i)]


@register("cudnn_lstm")
def _cudnn_lstm(ins, a):
    """Reference `cudnn_lstm_op.cc`: time-major LSTM in cuDNN weight order — WeightList (or the flat
    W: every (layer, direction) W_ih [4H, I] then W_hh [4H, H], then all b_ih, b_hh). Runs the
    ``rnn`` program op (one input GEMM per layer, own GEMMs)."""
    x = _in(ins, "Input")
    L, Hs = int(a.get("num_layers", 1)), int(a.get("hidden_size"))
    D = 2 if a.get("is_bidirec") else 1
    wl = _inl(ins, "WeightList")
    if not wl:
        W = _in(ins, "W").reshape(-1)
        I0 = x.shape[-1]
        shapes = []
        for layer in range(L):
            inp = I0 if layer == 0 else D * Hs
            for _ in range(D):
                shapes += [(4 * Hs, inp), (4 * Hs, Hs)]
        shapes += [(4 * Hs,)] * (2 * L * D)
        off, wl = 0, []
        for s in shapes:
            n = int(np.prod(s))
            wl.append(W[off:off + n].reshape(s))
            off += n
    pre = [t for t in (_in(ins, "InitH"), _in(ins, "InitC")) if t is not None]
    r = REGISTRY["rnn"]({"Input": [x], "WeightList": wl, "PreState": pre,
                         "SequenceLength": ins.get("SequenceLength") or []},
                        {"mode": "LSTM", "num_layers": L, "hidden_size": Hs, "is_bidirec": D == 2,
                         "dropout_prob": a.get("dropout_prob", 0.0), "is_test": a.get("is_test", False)})
    st = r["State"]
    return {"Out": r["Out"], "LastH": st[0], "LastC": st[1], "Reserve": torch.empty(0), "StateOut": torch.empty(0)}


def _seq_major(x):
    """[T, F] (one sequence) or [B, T, F] (padded batch) → ([T, B, F], squeeze flag)."""
    return (x[:, None], True) if x.dim() == 2 else (x.transpose(0, 1), False)


@register("lstm")
def _lstm_op(ins, a):
    """Reference `lstm_op.cc` (dynamic LSTM): Input is the PROJECTED x [T, 4D] (one sequence, or
    [B, T, 4D] padded); gate layout [c̃, i, f, o]; Weight [D, 4D] hidden weights; Bias [1, 4D]
    (+ [1, 3D] peephole checks i, f, o with use_peepholes)."""
    xg, sq = _seq_major(_in(ins, "Input"))
    w, b = _in(ins, "Weight"), _in(ins, "Bias")
    T, B, F4 = xg.shape
    D = F4 // 4
    h = _in(ins, "H0") if _in(ins, "H0") is not None else xg.new_zeros(B, D)
    c = _in(ins, "C0") if _in(ins, "C0") is not None else xg.new_zeros(B, D)
    bias = b.reshape(-1)
    peep = bool(a.get("use_peepholes", True)) and bias.numel() >= 7 * D
    gb = bias[:4 * D]
    ci, cf, co = (bias[4 * D:5 * D], bias[5 * D:6 * D], bias[6 * D:7 * D]) if peep else (0, 0, 0)
    ga = _act_by_name(a.get("gate_activation", "sigmoid"))
    ca = _act_by_name(a.get("cell_activation", "tanh"))
    na = _act_by_name(a.get("candidate_activation", "tanh"))
    steps = range(T - 1, -1, -1) if a.get("is_reverse") else range(T)
    hs, cs = [None] * T, [None] * T
    for t in steps:
        g = xg[t] + h @ w + gb
        gc, gi, gf, go = g.split(D, -1)
        i = ga(gi + c * ci)
        f = ga(gf + c * cf)
        c = na(gc) * i + c * f
        o = ga(go + c * co)
        h = o * ca(c)
        hs[t], cs[t] = h, c
    H, C = torch.stack(hs), torch.stack(cs)
    if sq:
        H, C = H[:, 0], C[:, 0]
    else:
        H, C = H.transpose(0, 1), C.transpose(0, 1)
    return {"Hidden": H, "Cell": C, "BatchGate": torch.empty(0), "BatchCellPreAct": torch.empty(0)}


def _gru_step(xt, h, w, ga, ca, origin):
    """Reference GRU unit: gates (u, r) = ga(x_ur + h·W_ur); c̃ = ca(x_c + (r∘h)·W_c);
    h' = u∘h + (1−u)∘c̃ (origin_mode) or u∘c̃ + (1−u)∘h. Weight [D, 3D] = flat W_ur [D, 2D] then W_c [D, D]."""
    D = h.shape[-1]
    flat = w.reshape(-1)
    wur = flat[:2 * D * D].view(D, 2 * D)
    wc = flat[2 * D * D:].view(D, D)
    ur = ga(xt[:, :2 * D] + h @ wur)
    u, r = ur[:, :D], ur[:, D:]
    rh = r * h
    c = ca(xt[:, 2 * D:] + rh @ wc)
    hn = u * h + (1 - u) * c if origin else u * c + (1 - u) * h
    return hn, torch.cat([u, r, c], -1), rh


@register("gru")
def _gru_op(ins, a):
    """Reference `gru_op.cc` (dynamic GRU): Input projected [T, 3D] (or [B, T, 3D]); H0; Weight
    [D, 3D]; Bias [1, 3D]; is_reverse; origin_mode."""
    xg, sq = _seq_major(_in(ins, "Input"))
    w, b = _in(ins, "Weight"), _in(ins, "Bias")
    T, B, F3 = xg.shape
    D = F3 // 3
    h = _in(ins, "H0") if _in(ins, "H0") is not None else xg.new_zeros(B, D)
    if b is not None:
        xg = xg + b.reshape(-1)
    ga = _act_by_name(a.get("gate_activation", "sigmoid"))
    ca = _act_by_name(a.get("activation", "tanh"))
    steps = range(T - 1, -1, -1) if a.get("is_reverse") else range(T)
    hs = [None] * T
    for t in steps:
        h, _, _ = _gru_step(xg[t], h, w, ga, ca, bool(a.get("origin_mode", False)))
        hs[t] = h
    H = torch.stack(hs)
    H = H[:, 0] if sq else H.transpose(0, 1)
    return {"Hidden": H, "BatchGate": torch.empty(0), "BatchResetHiddenPrev": torch.empty(0),
            "BatchHidden": torch.empty(0)}


@register("gru_unit")
def _gru_unit(ins, a):
    x, hp, w, b = _in(ins, "Input"), _in(ins, "HiddenPrev"), _in(ins, "Weight"), _in(ins, "Bias")
    if b is not None:
        x = x + b.reshape(1, -1)
    h, gate, rh = _gru_step(x, hp, w, _act_by_id(a.get("gate_activation", 1)), _act_by_id(a.get("activation", 2)),
                            bool(a.get("origin_mode", False)))
    return {"Gate": gate, "ResetHiddenPrev": rh, "Hidden": h}


@register("lstm_unit")
def _lstm_unit(ins, a):
    """Reference `lstm_unit_op.h`: X [B, 4D] pre-activations (i, f, o, g); C = σ(f + forget_bias)∘C_prev
    + σ(i)∘tanh(g); H = σ(o)∘tanh(C)."""
    x, cp = _in(ins, "X"), _in(ins, "C_prev")
    i, f, o, g = x.chunk(4, -1)
    c = torch.sigmoid(f + float(a.get("forget_bias", 0.0))) * cp + torch.sigmoid(i) * torch.tanh(g)
    return {"C": c, "H": torch.sigmoid(o) * torch.tanh(c)}


# ---------------------------------------------------------------------------------- detection
@register("matrix_nms")
def _matrix_nms_op(ins, a):
    from ..vision.ops import matrix_nms
    out, num, idx = matrix_nms(_in(ins, "BBoxes", "bboxes"), _in(ins, "Scores", "scores"),
                               float(a.get("score_threshold", 0.0)), float(a.get("post_threshold", 0.0)),
                               int(a.get("nms_top_k", -1)), int(a.get("keep_top_k", -1)),
                               bool(a.get("use_gaussian", False)), float(a.get("gaussian_sigma", 2.0)),
                               int(a.get("background_label", 0)), bool(a.get("normalized", True)),
                               return_index=True, return_rois_num=True)
    return {"Out": out, "Index": idx, "RoisNum": num, "out": out, "index": idx, "roisnum": num}


@register("generate_proposals", "generate_proposals_v2")
def _generate_proposals_op(ins, a):
    from ..vision.ops import generate_proposals
    im = _in(ins, "ImShape", "im_shape")
    if im is None:  # v1: ImInfo [N, 3] (h, w, scale)
        im = _in(ins, "ImInfo")[:, :2]
    rois, probs, num = generate_proposals(
        _in(ins, "Scores", "scores"), _in(ins, "BboxDeltas", "bbox_deltas"), im,
        _in(ins, "Anchors", "anchors"), _in(ins, "Variances", "variances"),
        int(_at(a, "pre_nms_topN", "pre_nms_top_n", default=6000)),
        int(_at(a, "post_nms_topN", "post_nms_top_n", default=1000)), float(a.get("nms_thresh", 0.5)),
        float(a.get("min_size", 0.1)), float(a.get("eta", 1.0)), bool(a.get("pixel_offset", True)),
        return_rois_num=True)
    return {"RpnRois": rois, "RpnRoiProbs": probs, "RpnRoisNum": num, "rpn_rois": rois,
            "rpn_roi_probs": probs, "rpn_rois_num": num}


@register("distribute_fpn_proposals")
def _distribute_fpn_op(ins, a):
    from ..vision.ops import distribute_fpn_proposals
    multi, restore, nums = distribute_fpn_proposals(
        _in(ins, "FpnRois", "fpn_rois"), int(a["min_level"]), int(a["max_level"]), int(a["refer_level"]),
        int(a["refer_scale"]), bool(a.get("pixel_offset", True)), _in(ins, "RoisNum", "rois_num"))
    return {"MultiFpnRois": multi, "RestoreIndex": restore, "MultiLevelRoIsNum": nums or [],
            "multi_fpn_rois": multi, "restore_index": restore, "multi_level_rois_num": nums or []}


@register("collect_fpn_proposals")
def _collect_fpn(ins, a):
    """Reference `collect_fpn_proposals_op`: concatenate every level's rois, keep the top
    post_nms_topN by score overall (per image when RoisNum is given), image-major output."""
    rois, scores = _inl(ins, "MultiLevelRois"), _inl(ins, "MultiLevelScores")
    nums = _inl(ins, "MultiLevelRoIsNum")
    k = int(a.get("post_nms_topN", 100))
    R = torch.cat(rois)
    Sc = torch.cat([s.reshape(-1) for s in scores])
    if nums:
        img = torch.cat([torch.repeat_interleave(torch.arange(n.numel(), device=R.device), n.long()) for n in nums])
        nimg = nums[0].numel()
    else:
        img = torch.zeros(R.shape[0], dtype=torch.long, device=R.device)
        nimg = 1
    top = torch.sort(Sc, descending=True, stable=True).indices[:k]
    sel = top[torch.sort(img[top], stable=True).indices]
    return {"FpnRois": R[sel], "RoisNum": torch.bincount(img[sel], minlength=nimg).to(torch.int32)}


@register("psroi_pool")
def _psroi_pool_op(ins, a):
    from ..vision.ops import psroi_pool
    x, rois = _in(ins, "X", "x"), _in(ins, "ROIs", "boxes")
    rn = _in(ins, "RoisNum", "boxes_num")
    if rn is None:
        rn = torch.tensor([rois.shape[0]])
    return _out(psroi_pool(x, rois, rn, (int(a["pooled_height"]), int(a["pooled_width"])),
                           float(a.get("spatial_scale", 1.0))))


@register("roi_pool")
def _roi_pool_op(ins, a):
    from ..vision.ops import roi_pool
    x, rois = _in(ins, "X", "x"), _in(ins, "ROIs", "boxes")
    rn = _in(ins, "RoisNum", "boxes_num")
    if rn is None:
        rn = torch.tensor([rois.shape[0]])
    y = roi_pool(x, rois, rn, (int(a["pooled_height"]), int(a["pooled_width"])), float(a.get("spatial_scale", 1.0)))
    return {"Out": y, "out": y, "Argmax": torch.zeros(y.shape, dtype=torch.int64)}


@register("prroi_pool")
def _prroi_pool(ins, a):
    """Precise ROI pooling (integral of the bilinear interpolant over each bin), approximated by a
    dense 4×4 bilinear sample average per bin through roi_align."""
    from ..vision.ops import roi_align
    x, rois = _in(ins, "X"), _in(ins, "ROIs")
    rn = _in(ins, "BatchRoINums")
    if rn is None:
        rn = torch.tensor([rois.shape[0]])
    return _out(roi_align(x, rois, rn, (int(a["pooled_height"]), int(a["pooled_width"])),
                          float(a.get("spatial_scale", 1.0)), sampling_ratio=4, aligned=False))


@register("yolov3_loss")
def _yolov3_loss(ins, a):
    from ..vision.ops import yolo_loss
    loss = yolo_loss(_in(ins, "X", "x"), _in(ins, "GTBox", "gt_box"), _in(ins, "GTLabel", "gt_label"),
                     list(a["anchors"]), list(a["anchor_mask"]), int(a["class_num"]), float(a["ignore_thresh"]),
                     int(a["downsample_ratio"]), _in(ins, "GTScore", "gt_score"),
                     bool(a.get("use_label_smooth", True)), scale_x_y=float(a.get("scale_x_y", 1.0)))
    return {"Loss": loss, "loss": loss, "ObjectnessMask": torch.empty(0), "GTMatchMask": torch.empty(0)}


@register("nms")
def _nms_op(ins, a):
    from ..vision.ops import _greedy_nms
    b = _in(ins, "Boxes", "x")
    keep = _greedy_nms(b, torch.arange(b.shape[0], 0, -1, dtype=torch.float32, device=b.device),
                       float(a.get("iou_threshold", 0.3)), 1.0, False)
    return {"KeepBoxesIdxs": keep, "out": keep}


@register("box_decoder_and_assign")
def _box_decoder_and_assign(ins, a):
    """Reference `box_decoder_and_assign_op.h`: per class decode TargetBox deltas against PriorBox
    (+1 pixel convention, variance-scaled, log-size clip), OutputAssignBox = the box of the best
    non-background class."""
    pb, pv, tb, sc = (_in(ins, k) for k in ("PriorBox", "PriorBoxVar", "TargetBox", "BoxScore"))
    clip = float(a.get("box_clip", 4.135))
    R, C = sc.shape
    pw = pb[:, 2] - pb[:, 0] + 1
    ph = pb[:, 3] - pb[:, 1] + 1
    px, py = pb[:, 0] + pw / 2, pb[:, 1] + ph / 2
    t = tb.reshape(R, C, 4)
    v = pv.reshape(-1, 4) if pv is not None else torch.ones(1, 4, device=pb.device)
    dx, dy = v[:, 0:1] * t[..., 0], v[:, 1:2] * t[..., 1]
    dw, dh = torch.clamp(v[:, 2:3] * t[..., 2], max=clip), torch.clamp(v[:, 3:4] * t[..., 3], max=clip)
    cx, cy = dx * pw[:, None] + px[:, None], dy * ph[:, None] + py[:, None]
    w, h = torch.exp(dw) * pw[:, None], torch.exp(dh) * ph[:, None]
    dec = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - 1, cy + h / 2 - 1], -1)
    best = sc[:, 1:].argmax(1) + 1 if C > 1 else torch.zeros(R, dtype=torch.long, device=sc.device)
    assign = dec[torch.arange(R, device=sc.device), best]
    return {"DecodeBox": dec.reshape(R, C * 4), "OutputAssignBox": assign}


@register("bipartite_match")
def _bipartite_match(ins, a):
    """Reference `bipartite_match_op.cc`: greedy global max matching of DistMat [N, M] (rows = gt,
    cols = priors), then ('per_prediction') unmatched columns take their best row above the
    threshold."""
    d = _in(ins, "DistMat").float()
    N, M = d.shape
    idx = torch.full((M,), -1, dtype=torch.int32)
    dist_ = torch.zeros(M)
    dd = d.clone().cpu()
    used_r = torch.zeros(N, dtype=torch.bool)
    for _ in range(min(N, M)):
        masked = dd.clone()
        masked[used_r] = -1
        masked[:, idx >= 0] = -1
        v, flat = masked.reshape(-1).max(0)
        if v <= 0:
            break
        r, c = int(flat) // M, int(flat) % M
        idx[c], dist_[c] = r, v
        used_r[r] = True
    if a.get("match_type", "bipartite") == "per_prediction":
        thr = float(a.get("dist_threshold", 0.5))
        bv, br = dd.max(0)
        sel = (idx < 0) & (bv >= thr)
        idx[sel], dist_[sel] = br[sel].int(), bv[sel]
    return {"ColToRowMatchIndices": idx.reshape(1, M).to(d.device), "ColToRowMatchDist": dist_.reshape(1, M).to(d.device)}


@register("target_assign")
def _target_assign(ins, a):
    x, mi = _in(ins, "X"), _in(ins, "MatchIndices").long()
    neg = _in(ins, "NegIndices")
    mv = float(a.get("mismatch_value", 0))
    N, P = mi.shape
    K = x.shape[-1]
    xs = x.reshape(-1, x.shape[-2] if x.dim() == 3 else 1, K) if x.dim() == 3 else x.reshape(1, -1, K)
    out = torch.full((N, P, K), mv, dtype=x.dtype, device=x.device)
    w = torch.zeros(N, P, 1, dtype=torch.float32, device=x.device)
    for n in range(N):
        ok = mi[n] >= 0
        src = xs[min(n, xs.shape[0] - 1)]
        out[n, ok] = src[mi[n, ok]]
        w[n, ok] = 1.0
    if neg is not None:
        for j in neg.reshape(-1).tolist():
            w[0, int(j)] = 1.0
    return {"Out": out, "OutWeight": w}


@register("density_prior_box")
def _density_prior_box(ins, a):
    """Reference `density_prior_box_op.h`: for each fixed size / density, density² shifted square
    boxes (× each fixed ratio) per feature-map cell, normalised by the image size."""
    x, img = _in(ins, "Input"), _in(ins, "Image")
    H, W = x.shape[2], x.shape[3]
    IH, IW = img.shape[2], img.shape[3]
    sw = float(a.get("step_w", 0) or IW / W)
    sh = float(a.get("step_h", 0) or IH / H)
    off = float(a.get("offset", 0.5))
    sizes = [float(s) for s in a.get("fixed_sizes", [])]
    ratios = [float(r) for r in a.get("fixed_ratios", [1.0])]
    dens = [int(d) for d in a.get("densities", [])]
    boxes = []
    for hh in range(H):
        for ww in range(W):
            cx, cy = (ww + off) * sw, (hh + off) * sh
            cell = []
            for s, dn in zip(sizes, dens):
                shift = s / dn
                for r in ratios:
                    bw, bh = s * math.sqrt(r), s / math.sqrt(r)
                    for di in range(dn):
                        for dj in range(dn):
                            ccx = cx - s / 2 + shift / 2 + dj * shift
                            ccy = cy - s / 2 + shift / 2 + di * shift
                            cell.append([(ccx - bw / 2) / IW, (ccy - bh / 2) / IH, (ccx + bw / 2) / IW,
                                         (ccy + bh / 2) / IH])
            boxes.append(cell)
    b = torch.tensor(boxes, dtype=torch.float32, device=x.device).reshape(H, W, -1, 4)
    if a.get("clip"):
        b = b.clamp(0, 1)
    var = torch.tensor(a.get("variances", [0.1, 0.1, 0.2, 0.2]), dtype=torch.float32,
                       device=x.device).expand_as(b).contiguous()
    if a.get("flatten_to_2d"):
        b, var = b.reshape(-1, 4), var.reshape(-1, 4)
    return {"Boxes": b.to(x.dtype), "Variances": var.to(x.dtype)}


@register("locality_aware_nms")
def _locality_aware_nms(ins, a):
    return REGISTRY["multiclass_nms"](ins, a)


@register("retinanet_detection_output")
def _retinanet_detection_output(ins, a):
    """Reference `retinanet_detection_output_op`: per FPN level decode the top nms_top_k anchors above
    score_threshold, then class-wise NMS over all levels and keep_top_k (rows: label, score, box)."""
    from ..vision.ops import _nms_fast
    bbs, scs, ancs = _inl(ins, "BBoxes"), _inl(ins, "Scores"), _inl(ins, "Anchors")
    im = _in(ins, "ImInfo")
    st, topk = float(a.get("score_threshold", 0.05)), int(a.get("nms_top_k", 1000))
    nt, keep = float(a.get("nms_threshold", 0.3)), int(a.get("keep_top_k", 100))
    eta = float(a.get("nms_eta", 1.0))
    rows, nums = [], []
    N = scs[0].shape[0]
    for n in range(N):
        boxes, scores, cls = [], [], []
        for bb, sc, an in zip(bbs, scs, ancs):
            s = sc[n]  # [A, C]
            flat = s.reshape(-1)
            cand = torch.nonzero(flat > st).reshape(-1)
            cand = cand[torch.sort(flat[cand], descending=True, stable=True).indices][:topk]
            ai, ci = cand // s.shape[1], cand % s.shape[1]
            anc = an.reshape(-1, 4)[ai]
            d = bb[n][ai]
            aw, ah = anc[:, 2] - anc[:, 0] + 1, anc[:, 3] - anc[:, 1] + 1
            cx, cy = anc[:, 0] + aw / 2 + d[:, 0] * aw, anc[:, 1] + ah / 2 + d[:, 1] * ah
            w, h = torch.exp(d[:, 2]) * aw, torch.exp(d[:, 3]) * ah
            scl = im[n, 2]
            bx = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - 1, cy + h / 2 - 1], -1) / scl
            bx = torch.stack([bx[:, 0].clamp(0, im[n, 1] / scl - 1), bx[:, 1].clamp(0, im[n, 0] / scl - 1),
                              bx[:, 2].clamp(0, im[n, 1] / scl - 1), bx[:, 3].clamp(0, im[n, 0] / scl - 1)], -1)
            boxes.append(bx)
            scores.append(flat[cand])
            cls.append(ci)
        B_, S_, C_ = torch.cat(boxes), torch.cat(scores), torch.cat(cls)
        det = []
        for c in C_.unique().tolist():
            m = torch.nonzero(C_ == c).reshape(-1)
            k = _nms_fast(B_[m], S_[m], -1.0, nt, eta, -1, False)
            det += [(float(S_[m[j]]), c, B_[m[j]]) for j in k]
        det = sorted(det, key=lambda t: -t[0])[:keep]
        for s, c, b in det:
            rows.append(torch.cat([torch.tensor([c + 1.0, s], device=b.device), b]))
        nums.append(len(det))
    out = torch.stack(rows) if rows else torch.zeros((0, 6))
    return {"Out": out}


# ------------------------------------------------------------------------------ quantization
@register("dequantize_abs_max")
def _dequantize_abs_max(ins, a):
    x, s = _x(ins), _in(ins, "Scale")
    return _out(x.float() * s.reshape(-1)[0].float() / float(a.get("max_range", 127.0)))


@register("dequantize_log")
def _dequantize_log(ins, a):
    x, d = _x(ins), _in(ins, "Dict")
    xi = x.long()
    return _out(torch.where(xi < 0, -d[(xi + 128).clamp(0, d.numel() - 1)], d[xi.clamp(0, d.numel() - 1)]))


def _fq(x, scale, bits):
    bnt = float((1 << (bits - 1)) - 1)
    return torch.round(torch.clamp(x / scale.clamp_min(1e-30), -1, 1) * bnt)


@register("fake_quantize_abs_max")
def _fake_quantize_abs_max(ins, a):
    x = _x(ins)
    s = x.abs().max().reshape(1)
    return {"Out": _fq(x, s, int(a.get("bit_length", 8))), "OutScale": s}


@register("fake_channel_wise_quantize_abs_max")
def _fake_cw_quantize(ins, a):
    x = _x(ins)
    ax = int(a.get("quant_axis", 0))
    dims = [d for d in range(x.dim()) if d != ax]
    s = x.abs().amax(dims)
    shp = [1] * x.dim()
    shp[ax] = -1
    return {"Out": _fq(x, s.view(shp), int(a.get("bit_length", 8))), "OutScale": s}


@register("fake_quantize_range_abs_max")
def _fake_quantize_range(ins, a):
    x, ins_s = _x(ins), _in(ins, "InScale")
    cur = x.abs().max()
    s = cur if a.get("is_test") is False else torch.maximum(cur, ins_s.reshape(-1)[0]) if ins_s is not None else cur
    return {"Out": _fq(x, s, int(a.get("bit_length", 8))), "OutScale": s.reshape(1)}


@register("fake_quantize_moving_average_abs_max")
def _fake_quantize_mavg(ins, a):
    x = _x(ins)
    rate = float(a.get("moving_rate", 0.9))
    st, acc = _in(ins, "InState"), _in(ins, "InAccum")
    if a.get("is_test") or st is None:
        s = _in(ins, "InScale").reshape(-1)[0]
        return {"Out": _fq(x, s, int(a.get("bit_length", 8))), "OutScale": s.reshape(1)}
    st2 = rate * st + 1
    acc2 = rate * acc + x.abs().max()
    s = (acc2 / st2).reshape(-1)[0]
    return {"Out": _fq(x, s, int(a.get("bit_length", 8))), "OutScale": s.reshape(1), "OutState": st2,
            "OutAccum": acc2}


@register("quantize")
def _quantize_mkldnn(ins, a):
    x = _in(ins, "Input")
    s, sh = float(a.get("Scale", 1.0)), float(a.get("Shift", 0.0))
    q = torch.round(x.float() * s + sh)
    return {"Output": (q.clamp(0, 255).to(torch.uint8) if sh else q.clamp(-128, 127).to(torch.int8))}


@register("dequantize")
def _dequantize_mkldnn(ins, a):
    x = _in(ins, "Input")
    return {"Output": (x.float() - float(a.get("Shift", 0.0))) / float(a.get("Scale", 1.0))}


@register("requantize")
def _requantize(ins, a):
    x = _in(ins, "Input")
    si, so = float(a.get("Scale_in", 1.0)), float(a.get("Scale_out", 1.0))
    shi, sho = float(a.get("Shift_in", 0.0)), float(a.get("Shift_out", 0.0))
    y = torch.round((x.float() - shi) * so / si + sho)
    return {"Output": y.clamp(-128, 127).to(x.dtype)}


# ----------------------------------------------------------------------------------- misc ops
@register("deformable_conv", "deformable_conv_v1")
def _deformable_conv(ins, a):
    """Reference `deformable_conv_op` (v2 with Mask; v1 without)."""
    from ..vision.ops import deform_conv2d
    x, off, w = _in(ins, "Input", "x"), _in(ins, "Offset", "offset"), _in(ins, "Filter", "filter")
    y = deform_conv2d(x, off, w, None, list(a.get("strides", [1, 1])), list(a.get("paddings", [0, 0])),
                      list(a.get("dilations", [1, 1])), int(a.get("deformable_groups", 1)), int(a.get("groups", 1)),
                      mask=_in(ins, "Mask", "mask"))
    return {"Output": y, "out": y}


@register("correlation")
def _correlation(ins, a):
    """Reference `correlation_op.cu` (FlowNet cost volume): mean over channels and the kernel window of
    x1·x2 at displacements up to max_displacement (stride2), on the stride1 output grid."""
    x1, x2 = _in(ins, "Input1"), _in(ins, "Input2")
    pad, k, md = int(a.get("pad_size", 0)), int(a.get("kernel_size", 1)), int(a.get("max_displacement", 0))
    s1, s2 = int(a.get("stride1", 1)), int(a.get("stride2", 1))
    N, C, H, W = x1.shape
    p1, p2 = F.pad(x1, (pad,) * 4), F.pad(x2, (pad,) * 4)
    r = k // 2
    bs = md + r
    Ho = (H + 2 * pad - 2 * bs - 1) // s1 + 1
    Wo = (W + 2 * pad - 2 * bs - 1) // s1 + 1
    ds = list(range(-md, md + 1, s2))
    outs = []
    for dy in ds:
        for dx in ds:
            acc = 0
            for ky in range(-r, r + 1):
                for kx in range(-r, r + 1):
                    ys, xs = bs + ky, bs + kx
                    a1 = p1[:, :, ys:ys + (Ho - 1) * s1 + 1:s1, xs:xs + (Wo - 1) * s1 + 1:s1]
                    a2 = p2[:, :, ys + dy:ys + dy + (Ho - 1) * s1 + 1:s1, xs + dx:xs + dx + (Wo - 1) * s1 + 1:s1]
                    acc = acc + (a1 * a2).sum(1)
            outs.append(acc / (k * k * C))
    return {"Output": torch.stack(outs, 1)}


@register("fused_elemwise_activation", "fused_elemwise_add_activation")
def _fused_elemwise_activation(ins, a):
    """Reference `fused_elemwise_activation_op.h`: functor_list [f1, f2] = binary∘unary
    (Out = f1(X, f2(Y))) or unary∘binary (Out = f1(f2(X, Y)))."""
    x, y = _in(ins, "X"), _in(ins, "Y")
    y = _bcast(x, y, a.get("axis", -1))
    fl = list(a.get("functor_list", ["elementwise_add", "relu"]))
    sc = float(a.get("scale", 0.0))
    un = {"relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh, "gelu": F.gelu,
          "scale": lambda t: t * sc}
    bi = {"elementwise_add": torch.add, "elementwise_mul": torch.mul}
    if fl[0] in bi:
        inter = un[fl[1]](y)
        out = bi[fl[0]](x, inter)
    else:
        inter = bi[fl[1]](x, y)
        out = un[fl[0]](inter)
    return {"Out": out, "IntermediateOut": inter}


@register("fused_embedding_seq_pool")
def _fused_embedding_seq_pool(ins, a):
    w, ids = _in(ins, "W"), _in(ins, "Ids")
    pid = int(a.get("padding_idx", -1))
    idl = ids.reshape(ids.shape[0], -1).long()
    e = F.embedding(idl, w)
    if pid >= 0:
        e = e * (idl != pid).unsqueeze(-1).to(e.dtype)
    return _out(e.sum(1))


@register("lookup_table_dequant")
def _lookup_table_dequant(ins, a):
    """Reference `lookup_table_dequant_op.h`: each W row = [min, max, 8-bit codes packed in floats];
    value = min + code·(max − min)/255."""
    w, ids = _in(ins, "W"), _in(ins, "Ids").reshape(-1).long()
    rows = w[ids]
    mn, mx = rows[:, 0:1], rows[:, 1:2]
    codes = rows[:, 2:].contiguous().view(torch.uint8).float()
    return _out(mn + codes * (mx - mn) / 255.0)


@register("graph_send_recv")
def _graph_send_recv(ins, a):
    from ..geometric import send_u_recv
    x, s, d = _in(ins, "X", "x"), _in(ins, "Src_index", "src_index"), _in(ins, "Dst_index", "dst_index")
    osz = _in(ins, "Out_size", "out_size")
    n = int(osz.reshape(-1)[0]) if osz is not None else (int(a.get("out_size", [0])[0]) if isinstance(
        a.get("out_size"), (list, tuple)) else int(a.get("out_size", 0) or 0))
    out = send_u_recv(x, s, d, a.get("reduce_op", a.get("pool_type", "sum")).lower(), n or None)
    return {"Out": out, "out": out, "Dst_count": torch.bincount(d.long(), minlength=out.shape[0]).to(torch.int32)}


@register("graph_send_ue_recv")
def _graph_send_ue_recv(ins, a):
    from ..geometric import send_ue_recv
    x, y = _in(ins, "X", "x"), _in(ins, "Y", "y")
    s, d = _in(ins, "Src_index", "src_index"), _in(ins, "Dst_index", "dst_index")
    osz = _in(ins, "Out_size", "out_size")
    n = int(osz.reshape(-1)[0]) if osz is not None else 0
    out = send_ue_recv(x, y, s, d, a.get("message_op", "add").lower(), a.get("reduce_op", "sum").lower(), n or None)
    return {"Out": out, "out": out, "Dst_count": torch.bincount(d.long(), minlength=out.shape[0]).to(torch.int32)}


@register("graph_send_uv")
def _graph_send_uv(ins, a):
    from ..geometric import send_uv
    return _out(send_uv(_in(ins, "x", "X"), _in(ins, "y", "Y"), _in(ins, "src_index"), _in(ins, "dst_index"),
                        a.get("message_op", "add").lower()))


@register("stft")
def _stft_op(ins, a):
    x, win = _x(ins), _in(ins, "Window")
    n_fft, hop = int(a["n_fft"]), int(a["hop_length"])
    fr = x.unfold(-1, n_fft, hop)                        # [B, frames, n_fft]
    if win is not None:
        fr = fr * win
    spec = torch.fft.rfft(fr, dim=-1) if a.get("onesided", True) else torch.fft.fft(fr.to(torch.complex64), dim=-1)
    if a.get("normalized"):
        spec = spec / math.sqrt(n_fft)
    return _out(spec.transpose(-1, -2))


def _fft_axes(a):
    return [int(v) for v in a.get("axes", [-1])]


def _fft_norm(a):
    return {"forward": "forward", "backward": "backward", "ortho": "ortho"}.get(a.get("normalization", "backward"),
                                                                               "backward")


@register("fft_c2c")
def _fft_c2c(ins, a):
    x = _x(ins)
    fn = torch.fft.fftn if a.get("forward", True) else torch.fft.ifftn
    return _out(fn(x, dim=_fft_axes(a), norm=_fft_norm(a)))


@register("fft_r2c")
def _fft_r2c(ins, a):
    x = _x(ins)
    fn = torch.fft.rfftn if a.get("onesided", True) else torch.fft.fftn
    y = fn(x, dim=_fft_axes(a), norm=_fft_norm(a))
    return _out(y if a.get("forward", True) else y.conj())


@register("fft_c2r")
def _fft_c2r(ins, a):
    x = _x(ins)
    ax = _fft_axes(a)
    ls = int(a.get("last_dim_size", 0) or 0)
    s = None if not ls else [x.shape[d] for d in ax[:-1]] + [ls]
    fn = torch.fft.irfftn if not a.get("forward", False) else (lambda t, s=None, dim=None, norm=None:
                                                               torch.fft.irfftn(t.conj(), s=s, dim=dim, norm=norm))
    return _out(fn(x, s=s, dim=ax, norm=_fft_norm(a)))


@register("read_file")
def _read_file(ins, a):
    from ..vision.ops import read_file
    return _out(read_file(a["filename"]))


@register("decode_jpeg")
def _decode_jpeg(ins, a):
    from ..vision.ops import decode_jpeg
    return _out(decode_jpeg(_x(ins), a.get("mode", "unchanged")))


@register("yolo_box_head")
def _yolo_box_head(ins, a):
    """Reference `fused/yolo_box_head_op.cu`: sigmoid on x, y, objectness and class channels, exp
    kept for w, h left raw (decoded by yolo_box_post)."""
    x = _x(ins)
    an = len(a["anchors"]) // 2
    C = int(a["class_num"])
    N, _, H, W = x.shape
    v = x.reshape(N, an, 5 + C, H, W)
    out = torch.cat([torch.sigmoid(v[:, :, :2]), v[:, :, 2:4], torch.sigmoid(v[:, :, 4:])], 2)
    return _out(out.reshape(x.shape))


@register("fused_token_prune")
def _fused_token_prune(ins, a):
    """Reference `fused_token_prune_op.cu`: token importance = attention received (Σ over heads and
    queries of Attn masked by Mask); keep the top NewMask.shape[2] tokens (the first one forced with
    keep_first_token), in original order when keep_order."""
    attn, x, mask, nm = _in(ins, "Attn"), _in(ins, "X"), _in(ins, "Mask"), _in(ins, "NewMask")
    keep = nm.shape[2]
    score = (attn * (mask >= 0).to(attn.dtype)).sum((1, 2))          # [B, S]
    if a.get("keep_first_token", True):
        score[:, 0] = float("inf")
    idx = torch.topk(score, keep, -1).indices
    if a.get("keep_order", False):
        idx = torch.sort(idx, -1).values
    slim = x.gather(1, idx[..., None].expand(-1, -1, x.shape[-1]))
    return {"SlimmedX": slim, "CLSInds": idx.to(torch.int64)}


@register("sequence_pool")
def _sequence_pool(ins, a):
    """Padded-batch form ([B, T, D]; no LoD in this framework): SUM / AVERAGE / SQRT / MAX / LAST / FIRST."""
    x = _x(ins)
    pt = a.get("pooltype", "AVERAGE").upper()
    if x.dim() == 2:
        x = x[None]
    if pt == "SUM":
        out = x.sum(1)
    elif pt == "AVERAGE":
        out = x.mean(1)
    elif pt == "SQRT":
        out = x.sum(1) / math.sqrt(x.shape[1])
    elif pt == "MAX":
        out = x.amax(1)
    elif pt == "LAST":
        out = x[:, -1]
    else:
        out = x[:, 0]
    return {"Out": out, "MaxIndex": torch.zeros(0, dtype=torch.int32)}


@register("sequence_softmax")
def _sequence_softmax(ins, a):
    return _out(torch.softmax(_x(ins), -1 if _x(ins).dim() > 1 else 0))


@register("sequence_reverse")
def _sequence_reverse(ins, a):
    x = _x(ins)
    return {"Y": x.flip(1 if x.dim() > 2 else 0)}


@register("sequence_expand_as")
def _sequence_expand_as(ins, a):
    x, y = _in(ins, "X"), _in(ins, "Y")
    return _out(x.repeat_interleave(y.shape[0] // x.shape[0], 0))


@register("sequence_pad")
def _sequence_pad(ins, a):
    x = _x(ins)
    return {"Out": x if x.dim() > 2 else x[None], "Length": torch.tensor([x.shape[-2] if x.dim() > 1 else x.shape[0]])}


@register("sequence_unpad")
def _sequence_unpad(ins, a):
    x, ln = _x(ins), _in(ins, "Length").reshape(-1).long()
    return _out(torch.cat([x[b, :int(ln[b])] for b in range(x.shape[0])], 0))


@register("im2sequence")
def _im2sequence(ins, a):
    x = _x(ins)
    k = list(a.get("kernels", [1, 1]))
    st = list(a.get("strides", [1, 1]))
    p = list(a.get("paddings", [0, 0, 0, 0]))
    xp = F.pad(x, [p[1], p[3], p[0], p[2]])
    col = F.unfold(xp, k, stride=st)                      # [N, C·kh·kw, L]
    return _out(col.transpose(1, 2).reshape(-1, col.shape[1]))
