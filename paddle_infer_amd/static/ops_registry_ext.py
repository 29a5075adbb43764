"""Paddle op types beyond the core set of ``ops_registry.py``: the common tensor ops exported
PaddleNLP / PaddleClas programs use, model-parallel collectives as program ops, control-flow
helpers (tensor arrays, select_input / select_output; ``while`` / ``conditional_block`` themselves
run in the Executor, `static/executor.py`), and the fork's LLM ops in program form
(``fused_multi_transformer_int8`` / ``_moe`` / ``_moe_int8`` / ``_moe_weight_only``,
``beam_search_softmax``, ``fused_gemm_epilogue``).

Slot and attribute names follow the reference op makers (`paddle/fluid/operators/*_op.cc`,
`phi/api/yaml/ops.yaml`); every kernel dispatches to the framework's tensor ops / HIP kernels.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .ops_registry import DEVICE, _dt, register


def _one(ins, slot, default=None):
    v = ins.get(slot)
    return v[0] if v else default


def _ival(t):
    return int(t.reshape(-1)[0].item()) if isinstance(t, torch.Tensor) else int(t)


# ------------------------------------------------------------------------------------ indexing
@register("gather")
def _gather(ins, a):
    """Reference `gather_op.cc`: rows of X along ``axis`` (Axis tensor overrides)."""
    x, idx = ins["X"][0], ins["Index"][0]
    ax = _ival(ins["Axis"][0]) if ins.get("Axis") else int(a.get("axis", 0) or 0)
    return {"Out": torch.index_select(x, ax, idx.reshape(-1).long())}


@register("gather_nd")
def _gather_nd(ins, a):
    x, idx = ins["X"][0], ins["Index"][0].long()
    k = idx.shape[-1]
    if k == 0:
        return {"Out": x.expand(*idx.shape[:-1], *x.shape)}
    flat = idx.reshape(-1, k)
    out = x[tuple(flat[:, i] for i in range(k))]
    return {"Out": out.reshape(*idx.shape[:-1], *x.shape[k:])}


@register("index_select")
def _index_select(ins, a):
    return {"Out": torch.index_select(ins["X"][0], int(a.get("dim", 0)), ins["Index"][0].long())}


@register("index_sample")
def _index_sample(ins, a):
    return {"Out": torch.gather(ins["X"][0], 1, ins["Index"][0].long())}


@register("take_along_axis")
def _take_along_axis(ins, a):
    return {"Result": torch.gather(ins["Input"][0], int(a.get("Axis", 0)), ins["Index"][0].long())}


@register("scatter")
def _scatter(ins, a):
    x, ids, upd = ins["X"][0], ins["Ids"][0].reshape(-1).long(), ins["Updates"][0]
    out = x.clone()
    if a.get("overwrite", True):
        out[ids] = upd
    else:
        out[ids] = 0
        out.index_add_(0, ids, upd)
    return {"Out": out}


@register("set_value")
def _set_value(ins, a):
    """Reference `set_value_op.cc`: Out = Input with Input[slices] = value (ValueTensor or the
    typed ``*_values`` attribute, broadcast), slice bounds from attributes or *TensorList inputs."""
    x = ins["Input"][0].clone()
    axes = list(a.get("axes", []))
    starts = [_ival(t) for t in ins["StartsTensorList"]] if ins.get("StartsTensorList") else list(a.get("starts", []))
    ends = [_ival(t) for t in ins["EndsTensorList"]] if ins.get("EndsTensorList") else list(a.get("ends", []))
    steps = [_ival(t) for t in ins["StepsTensorList"]] if ins.get("StepsTensorList") else list(a.get("steps", []) or [1] * len(axes))
    idx = [torch.arange(n, device=x.device) for n in x.shape]
    for ax, s0, e0, st in zip(axes, starts, ends, steps):
        n = x.shape[ax]
        r = range(n)[slice(s0, e0, st)]  # Python slice semantics = the reference's normalisation
        idx[ax] = torch.tensor(list(r), dtype=torch.long, device=x.device)
    if ins.get("ValueTensor"):
        v = ins["ValueTensor"][0].to(x.dtype)
    else:
        vals = []
        for key in ("fp32_values", "int64_values", "int32_values", "fp64_values", "bool_values",
                    "fp16_values"):
            vals = a.get(key) or []
            if vals:
                break
        shape = list(a.get("shape", [])) or [len(vals)]
        v = torch.tensor(vals, dtype=x.dtype, device=x.device).reshape(shape)
    grids = torch.meshgrid(*idx, indexing="ij")
    tgt_shape = grids[0].shape
    if v.numel() == 1:
        v = v.reshape(()).expand(tgt_shape)
    else:
        # values for a slice with decreased axes: re-insert the size-1 dims before broadcasting
        for d in sorted(a.get("decrease_axes", []) or []):
            if v.dim() < len(tgt_shape):
                v = v.unsqueeze(d)
        v = v.expand(tgt_shape)
    x[grids] = v
    return {"Out": x}


@register("tril_triu")
def _tril_triu(ins, a):
    x, d = ins["X"][0], int(a.get("diagonal", 0))
    return {"Out": torch.tril(x, d) if a.get("lower", True) else torch.triu(x, d)}


@register("masked_select")
def _masked_select(ins, a):
    return {"Y": torch.masked_select(ins["X"][0], ins["Mask"][0].bool())}


@register("where_index")
def _where_index(ins, a):
    return {"Out": torch.nonzero(ins["Condition"][0])}


# ------------------------------------------------------------------------------------ creation
@register("range")
def _range(ins, a):
    s, e, st = (ins[k][0].reshape(-1)[0] for k in ("Start", "End", "Step"))
    dt = ins["Start"][0].dtype
    return {"Out": torch.arange(s.item(), e.item(), st.item(), dtype=dt, device=DEVICE[-1])}


@register("linspace")
def _linspace(ins, a):
    s, e, n = (ins[k][0].reshape(-1)[0].item() for k in ("Start", "Stop", "Num"))
    return {"Out": torch.linspace(s, e, int(n), dtype=_dt(a.get("dtype", 5)), device=DEVICE[-1])}


@register("fill_constant_batch_size_like")
def _fill_bsl(ins, a):
    x = ins["Input"][0]
    shape = list(a.get("shape", []))
    shape[int(a.get("output_dim_idx", 0))] = x.shape[int(a.get("input_dim_idx", 0))]
    sv = a.get("str_value") or ""
    val = float(sv) if sv else float(a.get("value", 0.0))
    return {"Out": torch.full(shape, val, dtype=_dt(a.get("dtype", 5)), device=x.device)}


@register("assign_value")
def _assign_value(ins, a):
    for key in ("fp32_values", "int32_values", "int64_values", "bool_values", "fp64_values"):
        vals = a.get(key)
        if vals:
            break
    return {"Out": torch.tensor(vals, dtype=_dt(a.get("dtype", 5)), device=DEVICE[-1]).reshape(list(a.get("shape", [len(vals)])))}


@register("one_hot_v2")
def _one_hot(ins, a):
    x = ins["X"][0].long()
    depth = _ival(ins["depth_tensor"][0]) if ins.get("depth_tensor") else int(a.get("depth", -1))
    if a.get("allow_out_of_range", False):
        valid = (x >= 0) & (x < depth)
        out = F.one_hot(x.clamp(0, depth - 1), depth) * valid.unsqueeze(-1)
    else:
        out = F.one_hot(x, depth)
    return {"Out": out.to(_dt(a.get("dtype", 5)))}


@register("uniform_random")
def _uniform(ins, a):
    shape = [int(s) for s in a.get("shape", [])]
    g = torch.Generator(device=DEVICE[-1])
    g.manual_seed(int(a.get("seed", 0)) or torch.initial_seed())
    return {"Out": torch.empty(shape, dtype=_dt(a.get("dtype", 5)), device=DEVICE[-1]).uniform_(
        float(a.get("min", -1.0)), float(a.get("max", 1.0)), generator=g)}


@register("gaussian_random")
def _gaussian(ins, a):
    shape = [int(s) for s in a.get("shape", [])]
    g = torch.Generator(device=DEVICE[-1])
    g.manual_seed(int(a.get("seed", 0)) or torch.initial_seed())
    return {"Out": torch.empty(shape, dtype=_dt(a.get("dtype", 5)), device=DEVICE[-1]).normal_(
        float(a.get("mean", 0.0)), float(a.get("std", 1.0)), generator=g)}


# ------------------------------------------------------------------------------------ math / reduce
@register("cumsum")
def _cumsum(ins, a):
    x = ins["X"][0]
    if a.get("flatten", False):
        x = x.reshape(-1)
    ax = int(a.get("axis", -1))
    if a.get("reverse", False):
        x = x.flip(ax)
    out = torch.cumsum(x, ax)
    if a.get("exclusive", False):
        out = out - x
    if a.get("reverse", False):
        out = out.flip(ax)
    return {"Out": out}


def _reduce(fn):
    def k(ins, a):
        x = ins["X"][0]
        if a.get("reduce_all", False) or not list(a.get("dim", [])):
            out = fn(x.reshape(-1), 0)
            return {"Out": out.reshape([1] * x.dim()) if a.get("keep_dim") else out}
        dims = [d % x.dim() for d in a.get("dim")]
        out = x
        for d in sorted(dims, reverse=True):
            out = fn(out, d)
            if a.get("keep_dim"):
                out = out.unsqueeze(d)
        return {"Out": out}
    return k


for _n, _f in (("reduce_sum", lambda t, d: t.sum(d)), ("reduce_mean", lambda t, d: t.mean(d)),
               ("reduce_max", lambda t, d: t.amax(d)), ("reduce_min", lambda t, d: t.amin(d)),
               ("reduce_prod", lambda t, d: t.prod(d)), ("reduce_all", lambda t, d: t.bool().all(d)),
               ("reduce_any", lambda t, d: t.bool().any(d))):
    register(_n)(_reduce(_f))


@register("mean")
def _mean(ins, a):
    return {"Out": ins["X"][0].mean().reshape([1])}


@register("p_norm")
def _p_norm(ins, a):
    x = ins["X"][0]
    out = torch.linalg.vector_norm(x, float(a.get("porder", 2.0)), dim=int(a.get("axis", -1)),
                                   keepdim=bool(a.get("keepdim", False)))
    return {"Out": out}


@register("elementwise_floordiv")
def _floordiv(ins, a):
    return {"Out": torch.div(ins["X"][0], ins["Y"][0], rounding_mode="floor")}


@register("elementwise_mod")
def _mod(ins, a):
    return {"Out": torch.remainder(ins["X"][0], ins["Y"][0])}


for _n, _f in (("erf", torch.erf), ("sin", torch.sin), ("cos", torch.cos), ("ceil", torch.ceil),
               ("round", torch.round), ("reciprocal", torch.reciprocal), ("sign", torch.sign),
               ("log1p", torch.log1p), ("softplus", F.softplus), ("softsign", F.softsign),
               ("mish", F.mish), ("logsigmoid", F.logsigmoid), ("tanh_shrink", F.tanhshrink)):
    register(_n)(lambda ins, a, _f=_f: {"Out": _f(ins["X"][0])})


@register("hard_sigmoid")
def _hard_sigmoid(ins, a):
    x = ins["X"][0]
    return {"Out": torch.clamp(x * float(a.get("slope", 0.2)) + float(a.get("offset", 0.5)), 0, 1)}


@register("elu")
def _elu(ins, a):
    return {"Out": F.elu(ins["X"][0], float(a.get("alpha", 1.0)))}


@register("log_softmax")
def _log_softmax(ins, a):
    return {"Out": F.log_softmax(ins["X"][0], int(a.get("axis", -1)))}


@register("prelu")
def _prelu(ins, a):
    x, w = ins["X"][0], ins["Alpha"][0]
    mode = a.get("mode", "all")
    if mode == "channel":
        w = w.reshape([1, -1] + [1] * (x.dim() - 2)) if a.get("data_format", "NCHW") == "NCHW" else w.reshape(-1)
    return {"Out": torch.where(x >= 0, x, x * w)}


# ------------------------------------------------------------------------------------ compare / logic
for _n, _f in (("less_than", torch.lt), ("less_equal", torch.le), ("greater_than", torch.gt),
               ("greater_equal", torch.ge), ("equal", torch.eq), ("not_equal", torch.ne),
               ("logical_and", torch.logical_and), ("logical_or", torch.logical_or),
               ("logical_xor", torch.logical_xor), ("bitwise_and", torch.bitwise_and),
               ("bitwise_or", torch.bitwise_or)):
    register(_n)(lambda ins, a, _f=_f: {"Out": _f(ins["X"][0], ins["Y"][0])})


@register("logical_not")
def _logical_not(ins, a):
    return {"Out": torch.logical_not(ins["X"][0])}


@register("increment")
def _increment(ins, a):
    return {"Out": ins["X"][0] + a.get("step", 1.0)}


@register("isfinite_v2")
def _isfinite(ins, a):
    return {"Out": torch.isfinite(ins["X"][0])}


# ------------------------------------------------------------------------------------ shape ops
@register("tile")
def _tile(ins, a):
    reps = [_ival(t) for t in ins["repeat_times_tensor"]] if ins.get("repeat_times_tensor") else list(a.get("repeat_times", []))
    return {"Out": ins["X"][0].repeat(*reps) if len(reps) >= ins["X"][0].dim() else
            ins["X"][0].tile(reps)}


@register("flip")
def _flip(ins, a):
    return {"Out": torch.flip(ins["X"][0], list(a.get("axis", [])))}


@register("roll")
def _roll(ins, a):
    ax = list(a.get("axis", []))
    return {"Out": torch.roll(ins["X"][0], list(a.get("shifts", [])), ax if ax else None)}


@register("argsort")
def _argsort(ins, a):
    v, i = torch.sort(ins["X"][0], int(a.get("axis", -1)), bool(a.get("descending", False)))
    return {"Out": v, "Indices": i}


@register("unbind")
def _unbind(ins, a):
    return {"Out": list(torch.unbind(ins["X"][0], int(a.get("axis", 0))))}


@register("meshgrid")
def _meshgrid(ins, a):
    return {"Out": list(torch.meshgrid(*ins["X"], indexing="ij"))}


@register("pad3d")
def _pad3d(ins, a):
    p = list(a.get("paddings", [0] * 6))
    mode = {"constant": "constant", "reflect": "reflect", "replicate": "replicate",
            "circular": "circular"}[a.get("mode", "constant")]
    x = ins["X"][0]
    if a.get("data_format", "NCDHW") == "NDHWC":
        x = x.permute(0, 4, 1, 2, 3)
    out = F.pad(x, p, mode=mode, value=float(a.get("value", 0.0))) if mode == "constant" else F.pad(x, p, mode=mode)
    if a.get("data_format", "NCDHW") == "NDHWC":
        out = out.permute(0, 2, 3, 4, 1)
    return {"Out": out}


@register("top_k")
def _top_k(ins, a):
    v, i = torch.topk(ins["X"][0], int(a.get("k", 1)))
    return {"Out": v, "Indices": i}


# ------------------------------------------------------------------------------------ nn
def _interp(ins, a, mode):
    x = ins["X"][0]
    nhwc = a.get("data_layout", "NCHW") == "NHWC"
    if nhwc:
        x = x.permute(0, 3, 1, 2)
    size = None
    if ins.get("OutSize"):
        size = [int(v) for v in ins["OutSize"][0].reshape(-1).tolist()]
    elif ins.get("SizeTensor"):
        size = [_ival(t) for t in ins["SizeTensor"]]
    elif a.get("out_h", -1) > 0 and a.get("out_w", -1) > 0:
        size = [int(a["out_h"]), int(a["out_w"])]
    scale = None
    if size is None:
        sc = ins["Scale"][0].reshape(-1).tolist() if ins.get("Scale") else list(a.get("scale", []))
        scale = [float(sc[0]), float(sc[-1])] if sc else None
    align = bool(a.get("align_corners", False))
    kw = {"align_corners": align} if mode in ("bilinear", "bicubic") else {}
    if mode == "bilinear" and not align and int(a.get("align_mode", 1)) == 0:
        kw["align_corners"] = False  # half-pixel (align_mode 0) is torch's default
    out = F.interpolate(x, size=size, scale_factor=scale, mode=mode, **kw)
    return {"Out": out.permute(0, 2, 3, 1) if nhwc else out}


register("bilinear_interp_v2", "bilinear_interp")(lambda ins, a: _interp(ins, a, "bilinear"))
register("nearest_interp_v2", "nearest_interp")(lambda ins, a: _interp(ins, a, "nearest"))
register("bicubic_interp_v2")(lambda ins, a: _interp(ins, a, "bicubic"))


@register("group_norm")
def _group_norm(ins, a):
    x = ins["X"][0]
    nhwc = a.get("data_layout", "NCHW") == "NHWC"
    if nhwc:
        x = x.movedim(-1, 1)
    G, eps = int(a.get("groups", 1)), float(a.get("epsilon", 1e-5))
    N = x.shape[0]
    xg = x.reshape(N, G, -1).float()
    mean, var = xg.mean(-1), xg.var(-1, unbiased=False)
    y = F.group_norm(x, G, _one(ins, "Scale"), _one(ins, "Bias"), eps)
    return {"Y": y.movedim(1, -1) if nhwc else y, "Mean": mean, "Variance": var}


@register("instance_norm")
def _instance_norm(ins, a):
    x, eps = ins["X"][0], float(a.get("epsilon", 1e-5))
    red = tuple(range(2, x.dim()))
    xf = x.float()
    mean = xf.mean(red)
    var = xf.var(red, unbiased=False)
    y = F.instance_norm(x, weight=_one(ins, "Scale"), bias=_one(ins, "Bias"), eps=eps)
    return {"Y": y, "SavedMean": mean.reshape(-1), "SavedVariance": (1.0 / torch.sqrt(var + eps)).reshape(-1)}


@register("affine_channel")
def _affine_channel(ins, a):
    x, s, b = ins["X"][0], ins["Scale"][0], ins["Bias"][0]
    shp = [1, -1] + [1] * (x.dim() - 2) if a.get("data_layout", "NCHW") == "NCHW" else [-1]
    return {"Out": x * s.reshape(shp) + b.reshape(shp)}


@register("top_p_sampling")
def _top_p_sampling(ins, a):
    """Reference `phi/kernels/gpu/top_p_sampling_kernel.cu`: per row, sample from the smallest
    prefix of the probability-sorted vocabulary whose mass reaches ps[row]."""
    x, ps = ins["x"][0], ins["ps"][0].reshape(-1, 1).float()
    g = None
    if int(a.get("seed", -1)) >= 0:
        g = torch.Generator(device=x.device)
        g.manual_seed(int(a["seed"]))
    prob = x.float()
    sp, si = torch.sort(prob, -1, descending=True)
    cum = torch.cumsum(sp, -1)
    keep = (cum - sp) < ps                                  # the prefix reaching mass ps (>= 1 token)
    if ins.get("threshold"):
        keep &= sp >= ins["threshold"][0].reshape(-1, 1).float()
        keep[:, 0] = True
    sp = sp * keep
    pick = torch.multinomial(sp / sp.sum(-1, keepdim=True), 1, generator=g)
    ids = si.gather(-1, pick)
    return {"out": x.gather(-1, ids), "ids": ids.long()}


# ------------------------------------------------------------------------------------ model parallel
def _group(a):
    """The process group of ``ring_id`` (0 / unknown → the world group)."""
    from ..distributed.collective import get_group
    g = get_group(int(a.get("ring_id", 0) or 0))
    return getattr(g, "pg", None)


@register("c_identity")
def _c_identity(ins, a):
    return {"Out": ins["X"][0]}


def _c_allreduce(op_name):
    def k(ins, a):
        """Reference `c_allreduce_op.h`: all-reduce X over the ring's group (RCCL / gloo)."""
        import torch.distributed as dist
        x = ins["X"][0].clone()
        if dist.is_available() and dist.is_initialized():
            g = _group(a)
            if dist.get_world_size(g) > 1:
                dist.all_reduce(x, op=getattr(dist.ReduceOp, op_name), group=g)
        return {"Out": x}
    return k


for _n, _o in (("c_allreduce_sum", "SUM"), ("mp_allreduce_sum", "SUM"), ("c_allreduce_max", "MAX"),
               ("c_allreduce_min", "MIN"), ("c_allreduce_prod", "PRODUCT")):
    register(_n)(_c_allreduce(_o))


def _peer(a):
    """``peer`` (rank inside the ring's group) → global rank."""
    import torch.distributed as dist
    g = _group(a)
    peer = int(a.get("peer", 0))
    return dist.get_global_rank(g, peer) if g is not None else peer


_P2P_DT = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.bool,
           torch.uint8, torch.int8, torch.float64]


@register("send_v2")
def _send_v2(ins, a):
    """Reference `send_v2_op.cc`: X to ``peer`` of the ring (shape / dtype sent first, so the
    receiving stage needs no static out_shape)."""
    import torch.distributed as dist
    x = ins["X"][0].contiguous()
    peer = _peer(a)
    meta = torch.tensor([x.dim(), _P2P_DT.index(x.dtype)] + list(x.shape) + [0] * (8 - x.dim()),
                        dtype=torch.int64, device=x.device)
    dist.send(meta, peer)
    dist.send(x, peer)
    return {}


@register("recv_v2")
def _recv_v2(ins, a):
    """Reference `recv_v2_op.cc`: Out from ``peer`` of the ring."""
    import torch.distributed as dist
    from .ops_registry import DEVICE
    dev = DEVICE[0]
    peer = _peer(a)
    meta = torch.empty(10, dtype=torch.int64, device=dev)
    dist.recv(meta, peer)
    nd, dt = int(meta[0]), _P2P_DT[int(meta[1])]
    out = torch.empty([int(v) for v in meta[2:2 + nd].tolist()], dtype=dt, device=dev)
    dist.recv(out, peer)
    return {"Out": out}


@register("c_broadcast")
def _c_broadcast(ins, a):
    """Reference `c_broadcast_op.cc`: X from ``root`` (rank inside the ring's group) to the ring.
    Ranks that do not hold X yet (a pipeline stage that did not compute it) receive shape / dtype
    first."""
    import torch.distributed as dist
    from .ops_registry import DEVICE
    g = _group(a)
    root = int(a.get("root", 0))
    src = dist.get_global_rank(g, root) if g is not None else root
    x = (ins.get("X") or [None])[0]
    dev = x.device if x is not None else DEVICE[0]
    meta = torch.zeros(10, dtype=torch.int64, device=dev)
    if dist.get_rank() == src:
        x = x.contiguous()
        meta[0], meta[1] = x.dim(), _P2P_DT.index(x.dtype)
        meta[2:2 + x.dim()] = torch.tensor(list(x.shape), dtype=torch.int64)
    dist.broadcast(meta, src, group=g)
    nd, dt = int(meta[0]), _P2P_DT[int(meta[1])]
    if dist.get_rank() != src:
        x = torch.empty([int(v) for v in meta[2:2 + nd].tolist()], dtype=dt, device=dev)
    else:
        x = x.clone()
    dist.broadcast(x, src, group=g)
    return {"Out": x}


@register("c_concat")
def _c_concat(ins, a):
    """Reference `c_concat_op.cc`: all-gather X over the ring and concatenate on the last dim."""
    import torch.distributed as dist
    x = ins["X"][0].contiguous()
    if not (dist.is_available() and dist.is_initialized()):
        return {"Out": x}
    g = _group(a)
    if dist.get_world_size(g) == 1:
        return {"Out": x}
    parts = [torch.empty_like(x) for _ in range(dist.get_world_size(g))]
    dist.all_gather(parts, x, group=g)
    return {"Out": torch.cat(parts, -1)}


@register("c_split")
def _c_split(ins, a):
    x = ins["X"][0]
    n, r = int(a.get("nranks", 1)), int(a.get("rank", 0))
    return {"Out": x.chunk(n, -1)[r].contiguous()}


@register("c_embedding")
def _c_embedding(ins, a):
    """Reference `c_embedding_op.cc`: vocabulary-parallel lookup — ids outside
    [start_index, start_index + rows) produce zero rows (the all-reduce that follows sums them)."""
    w, ids = ins["W"][0], ins["Ids"][0].long()
    start = int(a.get("start_index", 0))
    local = ids - start
    valid = (local >= 0) & (local < w.shape[0])
    out = F.embedding(local.clamp(0, w.shape[0] - 1), w) * valid.unsqueeze(-1).to(w.dtype)
    return {"Out": out}


# ------------------------------------------------------------------------------------ tensor arrays
@register("write_to_array")
def _write_to_array(ins, a):
    """In place on the array variable ``Out`` (its current value arrives as ``__out__``)."""
    prev = (ins.get("__out__") or [None])[0]
    arr = list(prev) if isinstance(prev, (list, tuple)) else []
    i = _ival(ins["I"][0])
    x = ins["X"][0]
    while len(arr) <= i:
        arr.append(None)
    arr[i] = x
    return {"Out": [arr]}


@register("read_from_array")
def _read_from_array(ins, a):
    arr = ins["X"][0]
    return {"Out": arr[_ival(ins["I"][0])]}


@register("lod_array_length")
def _array_length(ins, a):
    arr = ins["X"][0]
    return {"Out": torch.tensor([len(arr)], dtype=torch.int64, device=DEVICE[-1])}


@register("select_input")
def _select_input(ins, a):
    return {"Out": ins["X"][_ival(ins["Mask"][0])]}


@register("select_output")
def _select_output(ins, a):
    i = _ival(ins["Mask"][0])
    n = len(a.get("_out_names", [])) or 2
    return {"Out": [ins["X"][0] if j == i else None for j in range(n)]}


# ------------------------------------------------------------------------------------ fork LLM ops
@register("fused_gemm_epilogue")
def _fused_gemm_epilogue(ins, a):
    """Reference `fused_gemm_epilogue_op.cc:415`: Out = act(X·Y + Bias) (ReserveSpace = the
    pre-activation when the activation needs it for backward). bf16 CUDA operands run the
    assembly GEMM with the bias / activation in its epilogue."""
    x, y, b = ins["X"][0], ins["Y"][0], ins["Bias"][0]
    if a.get("trans_x", False):
        x = x.transpose(-1, -2)
    if a.get("trans_y", False):
        y = y.transpose(-1, -2)
    act = a.get("activation", "none")
    actk = {"none": "none", "relu": "relu", "gelu": "gelu_tanh"}.get(act, act)
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    from ..ops import gemm as G
    if G.own_dtype(x2, y, b) and actk in ("none", "relu", "gelu_tanh", "gelu"):
        # own GEMM with the bias + activation in its epilogue; the pre-activation (ReserveSpace,
        # kept by the reference for its grad op) is not materialised for inference
        from ..ops.linear import transposed
        wt = transposed(y) if y.is_contiguous() else y.t().contiguous()
        out = G.gemm_nt(x2, wt, bias=b, act=actk)
        return {"Out": out.reshape(*lead, -1), "ReserveSpace": []}
    pre = x2 @ y + b
    out = {"none": lambda t: t, "relu": F.relu, "gelu_tanh": lambda t: F.gelu(t, approximate="tanh"),
           "gelu": F.gelu}[actk](pre)
    return {"Out": out.reshape(*lead, -1), "ReserveSpace": pre if actk != "none" else []}


@register("beam_search_softmax")
def _beam_search_softmax(ins, a):
    from ..ops.search import beam_search_softmax
    outs = beam_search_softmax(
        ins["logits"][0], ins["cum_scores"][0], ins["sequence_lengths"][0], ins["stop_flags"][0],
        ins["end_ids"][0], ins["step_ids"][0], ins["last_cache_ids"][0], ins["last_beam_offsets"][0],
        int(a["beam_size"]), int(a.get("max_seq_len", 0)), int(a["max_dec_len"]),
        bool(a.get("fuse_softmax", True)), bool(a.get("early_stop", False)),
        float(a.get("length_penalty", 0.0)), bool(a.get("one_stage_topk", False)))
    names = ("ids_this_time", "out_cum_scores", "cache_ids", "beam_offsets", "parent_idx",
             "stop_flags_out", "seq_lens_out", "step_ids_out")
    return dict(zip(names, outs))


def _fmt_run(ins, a, layers, moe=False):
    """Shared driver of the program-form fused multi-transformer variants."""
    from ..incubate.nn import functional as IF
    from .ops_registry import _fmt_common
    kw = _fmt_common(ins, a)
    x = ins["X"][0]
    B, S, E = x.shape
    nh = int(a.get("num_head", 0) or a.get("num_heads", 0) or 0)
    dh = int(a.get("dim_head", 0) or 0)
    if not nh:  # from the QKV weight [3, nh, dh, E] (trans) / [E, 3, nh, dh]
        w = ins["QKVW"][0]
        nh = w.shape[1] if w.dim() == 4 and kw["trans_qkvw"] else (w.shape[2] if w.dim() == 4 else E // 64)
    dh = dh or E // nh
    for L in layers:
        L.setdefault("head_dim", dh)
    decode = kw["time_step"] is not None
    pos, lens = IF._positions(B, kw["time_step"], kw["seq_lens"], S, x.device, decode)
    caches = kw["cache_kvs"]
    rope, pre = IF.ext_inputs(kw.get("rotary_embs"), kw.get("rotary_table_dims", 1),
                              kw.get("pre_caches"), B, dh, x.device, decode)
    with torch.no_grad():
        out = IF.multi_transformer_forward(
            x, layers, nh, int(a.get("num_kv_heads", 0) or 0) or None, kw["pre_layer_norm"],
            kw["epsilon"], IF._caches_from(caches), pos, lens, kw["attn_mask"], decode,
            kw["activation"], kw["rotary_emb_dims"], causal=kw["causal"] and kw["attn_mask"] is None,
            rope_table=rope, pre_caches=pre,
            group=kw["group"], moe_fn=True if moe else None)
    return {"Out": out, "CacheKVOut": caches or []}


def _ln_of(ins, i, dt):
    g = lambda s: ins[s][i].to(dt) if ins.get(s) else None  # noqa: E731
    return g("LnScale"), g("LnBias"), g("FFNLnScale"), g("FFNLnBias")


def _bias(ins, slot, i):
    v = ins.get(slot)
    return v[i].reshape(-1) if v and i < len(v) and v[i] is not None else None


@register("fused_multi_transformer_int8")
def _fmt_int8(ins, a):
    """Reference `fused_multi_transformer_int8_op.cc:367`: int8 weights [N, K] (QKVW [3, nh, dh,
    E]) + per-channel dequant ``*OutScale``; activations quantised with the static
    ``*_in_scale`` attributes (q = round(max_bound · in_scale · x)), int32 accumulation. Here
    y = acc · OutScale[n] maps onto the int8 MFMA GEMM's (weight scale, activation scale) pair."""
    from ..incubate.nn import functional as IF
    x = ins["X"][0]
    dt = x.dtype
    bound = float(a.get("quant_max_bound", 127.0))
    out = []

    def lin(w, oscale, in_scales, i):
        wq = w.reshape(w.shape[0] if w.dim() == 2 else -1, w.shape[-1]).view(torch.int8) \
            if w.dtype in (torch.int8, torch.uint8) else w
        ins_ = float(in_scales[i]) if in_scales and i < len(in_scales) else -1.0
        osc = oscale.reshape(-1).float()
        if ins_ > 0:
            return IF._lin(wq, osc * bound * ins_, -8, act_scale=1.0 / (bound * ins_))
        return IF._lin(wq, osc, -8, act_scale=None)
    n = len(ins["QKVW"])
    for i in range(n):
        ln = _ln_of(ins, i, dt)
        out.append(dict(ln_scale=ln[0], ln_bias=ln[1], ffn_ln_scale=ln[2], ffn_ln_bias=ln[3],
                        qkv=lin(ins["QKVW"][i], ins["QKVOutScale"][i], a.get("qkv_in_scale"), i),
                        qkv_bias=_bias(ins, "QKVBias", i),
                        out=lin(ins["OutLinearW"][i], ins["OutLinearOutScale"][i],
                                a.get("out_linear_in_scale"), i),
                        out_bias=_bias(ins, "OutLinearBias", i),
                        ffn1=lin(ins["FFN1Weight"][i], ins["FFN1OutScale"][i], a.get("ffn1_in_scale"), i),
                        ffn1_bias=_bias(ins, "FFN1Bias", i),
                        ffn2=lin(ins["FFN2Weight"][i], ins["FFN2OutScale"][i], a.get("ffn2_in_scale"), i),
                        ffn2_bias=_bias(ins, "FFN2Bias", i)))
    return _fmt_run(ins, a, out)


def _moe_layers(ins, a, expert_lin):
    """Per-layer attention linears + a top-k gated MoE FFN callable (reference
    `fused_multi_transformer_moe_op.cc:313`: GateWeight/GateBias per layer, ExpertWeight1/2 and
    ExpertBias1/2 = num_layers × num_expert tensors in layer-major order)."""
    from ..incubate.nn import functional as IF
    x = ins["X"][0]
    dt = x.dtype
    n = len(ins["QKVW"])
    ne = int(a.get("num_expert", 1))
    topk = int(a.get("topk", 2))
    act = "gelu_tanh" if a.get("approximate", True) else "gelu"
    trans = bool(a.get("trans_qkvw", True))
    layers = []
    for i in range(n):
        ln = _ln_of(ins, i, dt)
        moe = expert_lin(ins, i, ne, topk, act)
        ow = ins["OutLinearW"][i]
        layers.append(dict(ln_scale=ln[0], ln_bias=ln[1], ffn_ln_scale=ln[2], ffn_ln_bias=ln[3],
                           qkv=IF._qkv_linear(ins["QKVW"][i], trans, *(
                               (ins["QKVWScale"][i], 4 if a.get("weight_dtype") == "int4" else 8)
                               if ins.get("QKVWScale") else ())),
                           qkv_bias=_bias(ins, "QKVBias", i),
                           out=IF._lin(ow) if not ins.get("OutLinearWScale") else
                           IF._lin(ow, ins["OutLinearWScale"][i], 4 if a.get("weight_dtype") == "int4" else 8),
                           out_bias=_bias(ins, "OutLinearBias", i), moe=moe))
    return layers


@register("fused_multi_transformer_moe")
def _fmt_moe(ins, a):
    from ..incubate.moe import moe_ffn

    def expert(ins, i, ne, topk, act):
        sl = slice(i * ne, (i + 1) * ne)
        w1, w2 = ins["ExpertWeight1"][sl], ins["ExpertWeight2"][sl]
        b1 = ins["ExpertBias1"][sl] if ins.get("ExpertBias1") else [None] * ne
        b2 = ins["ExpertBias2"][sl] if ins.get("ExpertBias2") else [None] * ne
        gw, gb = ins["GateWeight"][i], _bias(ins, "GateBias", i)
        return lambda h: moe_ffn(h, gw, gb, w1, b1, w2, b2, topk, act, None)
    return _fmt_run(ins, a, _moe_layers(ins, a, expert), moe=True)


def _canon_stacked(w, s, bits):
    """Per-expert reference-layout check / re-pack of a stacked [E, N_packed, K] weight
    (`inference/ref_layout.py`), cached on the stacked tensor."""
    from ..inference.ref_layout import canonical_weight, is_ref_layout
    key = (w.data_ptr(), w._version)
    c = getattr(w, "_piamd_canon", None)
    if c is not None and c[0] == key:
        return c[1]
    out = w
    if w.dim() == 3 and is_ref_layout(w[0], bits):
        wd = "int4" if bits == 4 else "int8"
        out = torch.stack([canonical_weight(w[e].clone(), s[e], wd) for e in range(w.shape[0])])
    w._piamd_canon = (key, out)
    return out


def _grouped_moe(bits, scale_slots, canon=False):
    from ..incubate.moe import topk_gate, stacked
    from ..ops import moe as gm

    def expert(ins, i, ne, topk, act):
        w1, w2 = ins["ExpertWeight1"][i], ins["ExpertWeight2"][i]
        s1, s2 = ins[scale_slots[0]][i], ins[scale_slots[1]][i]
        if canon:  # reference (sm80) bytes → MI355X order
            w1, w2 = _canon_stacked(w1, s1, bits), _canon_stacked(w2, s2, bits)
        sl = slice(i * ne, (i + 1) * ne)
        b1 = stacked(ins["ExpertBias1"][sl]) if ins.get("ExpertBias1") else None
        b2 = stacked(ins["ExpertBias2"][sl]) if ins.get("ExpertBias2") else None
        gw, gb = ins["GateWeight"][i], _bias(ins, "GateBias", i)

        def moe(h):
            logits = torch.matmul(h, gw.to(h.dtype)) + (gb.to(h.dtype) if gb is not None else 0)
            val, idx = topk_gate(logits, topk)
            r = gm.permute(idx, ne, align=1)
            xs = gm.gather(h, r)
            y1 = gm.grouped_weight_only_linear(xs, w1, s1, r.offs, r.rows_cap,
                                               b1.to(h.dtype) if b1 is not None else None, bits, act)
            ys = gm.grouped_weight_only_linear(y1, w2, s2, r.offs, r.rows_cap,
                                               b2.to(h.dtype) if b2 is not None else None, bits)
            return gm.combine(ys, val, r)
        return moe
    return expert


@register("fused_multi_transformer_moe_weight_only")
def _fmt_moe_wo(ins, a):
    """Reference `fused_multi_transformer_moe_weight_only_op.cc:308`: expert weights stacked per
    layer [num_expert, N_packed, K] with ExpertWeight{1,2}Scale [num_expert, N]; one grouped
    weight-only MFMA launch per projection."""
    bits = 4 if a.get("weight_dtype", "int8") == "int4" else 8
    return _fmt_run(ins, a, _moe_layers(ins, a, _grouped_moe(bits, ("ExpertWeight1Scale", "ExpertWeight2Scale"),
                                                             canon=True)), moe=True)


@register("fused_multi_transformer_moe_int8")
def _fmt_moe_int8(ins, a):
    """Reference `fused_multi_transformer_moe_int8_op.cc:387`: int8 expert weights with
    per-channel ``ExpertWeight{1,2}OutScale``; experts run the grouped int8 weight-only path."""
    return _fmt_run(ins, a, _moe_layers(ins, a, _grouped_moe(8, ("ExpertWeight1OutScale", "ExpertWeight2OutScale"))),
                    moe=True)
