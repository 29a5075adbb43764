"""Static auto-parallel: completion (sharding propagation), partition and reshard of a static
``Program`` into per-rank programs with RCCL collectives.

Parity: reference `python/paddle/distributed/auto_parallel/completion.py` (``Completer``:
propagate ``dims_mapping`` from the user's ``shard_tensor`` annotations through every op),
`partitioner.py` (``Partitioner``: per-rank program with local parameter shards and rewritten
shapes), `reshard.py` (``Resharder``: insert all-gather / slice / all-reduce where a producer's
layout differs from what the consumer needs) and the per-op SPMD rules of
`operators/dist_matmul.py`, `dist_embedding.py`, `dist_reshape.py`, `dist_softmax.py`, ...

Model: a tensor's distribution is a ``dims_mapping`` — one entry per tensor dim, the mesh dim it
is split over or -1 (replicated) — on one ``ProcessMesh``. ``complete`` walks the ops once and,
per op type, decides the layout each input must have (resharding it if its producer left another
one), the layout of each output and whether an output is a *partial sum* over a mesh dim (a
contraction over a sharded dim). Partial outputs are reduced right after their producer
(``c_allreduce_sum``), the Megatron row-parallel pattern. Supported SPMD rules:

* ``linear`` / ``matmul_v2``: column-parallel (weight N split: output N split, no collective),
  row-parallel (weight K split: input sliced locally, all-reduce after, bias added once after the
  reduction), batch-split inputs, attention-style batched matmuls with a split head dim;
* ``lookup_table_v2``: vocab-parallel (out-of-shard ids masked, all-reduce) or hidden-split tables;
* elementwise (broadcast-aware), unary activations / casts / dropout / scale, ``softmax`` (its axis
  gathered), ``layer_norm`` (normalised dims gathered), ``reduce_sum`` / ``reduce_mean``,
  ``reshape2`` (a split dim carried to the outermost dim of its reshape group, local target
  shapes rewritten), ``transpose2``, ``split``, ``concat``, ``fused_attention``;
* anything else: inputs gathered to replicated, output replicated (always correct).

Feeds are global tensors; a feed annotated as split is sliced locally at the program start.
Collectives run through ``torch.distributed.nn.functional`` (autograd-aware RCCL / gloo calls) on
one process group per mesh-dim line, created in the same order on every rank.
"""
from __future__ import annotations

import itertools

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ...static.framework import Operator, Program, SymDim, Variable, VarRef, unique_name

__all__ = ["DistAttr", "Completer", "Partitioner", "complete", "partition"]


class DistAttr:
    def __init__(self, dims_mapping, partial=()):
        self.dims_mapping = list(dims_mapping)
        self.partial = tuple(partial)

    def __repr__(self):
        return f"DistAttr({self.dims_mapping}{', partial=' + str(self.partial) if self.partial else ''})"


def _mapping_from_spec(mesh, spec, ndim):
    if spec is None:
        return [-1] * ndim
    return [-1 if s is None else (mesh.dim_names.index(s) if isinstance(s, str) else int(s)) for s in spec]


_UNARY = {"relu", "gelu", "sigmoid", "tanh", "silu", "exp", "log", "sqrt", "rsqrt", "scale", "cast",
          "dropout", "assign", "clip", "leaky_relu", "swish", "hard_swish", "abs", "square", "erf"}
_BINARY = {"elementwise_add", "elementwise_sub", "elementwise_mul", "elementwise_div",
           "elementwise_pow", "elementwise_max", "elementwise_min", "where", "masked_fill",
           "fused_bias_act"}  # act(x + bias): broadcast of the bias over x's rows


def _dim_arg(op, pos, names=("dim", "axis"), default=None):
    for n in names:
        if n in op.kwargs:
            return op.kwargs[n]
    return op.args[pos] if len(op.args) > pos else default


class Completer:
    """Sharding propagation over the global block (``complete_forward_annotation``): returns
    {var: DistAttr} and records per-op plans (required input layouts, output layouts / partials,
    argument rewrites) used by ``Partitioner``."""

    def __init__(self, program: Program, mesh, annotations=None):
        self.program = program
        self.mesh = mesh
        self.block = program.global_block()
        self.attrs: dict = {}
        self.plans: list = []
        self.feed_slices: dict = {}
        self._ann = dict(annotations or {})

    # -- helpers ---------------------------------------------------------------------------
    def shape(self, name):
        v = self.block.vars.get(name)
        if v is None:
            t = self.program.params.get(name)
            return list(t.shape) if t is not None else None
        return list(v.shape)

    def nmesh(self, k):
        return self.mesh.shape[k]

    def mapping(self, name):
        a = self.attrs.get(name)
        if a is None:
            shp = self.shape(name)
            a = self.attrs[name] = DistAttr([-1] * len(shp or []))
        return list(a.dims_mapping)

    def _annotation_of(self, name):
        if name in self._ann:
            return self._ann[name]
        obj = self.program.params.get(name)
        if obj is None:
            obj = self.block.vars.get(name)
        spec = getattr(obj, "shard_spec", None)
        if spec is None:
            return None
        pm = getattr(obj, "process_mesh", None)
        if pm is not None and pm != self.mesh:
            raise ValueError(f"{name}: annotated on another ProcessMesh than the program's")
        return _mapping_from_spec(self.mesh, spec, len(self.shape(name)))

    def _fix_divisible(self, name, m):
        shp = self.shape(name) or []
        out = []
        for d, k in enumerate(m):
            if k != -1 and (d >= len(shp) or shp[d] % self.nmesh(k) != 0):
                k = -1
            out.append(k)
        return out

    @staticmethod
    def _dedup(m):
        seen, out = set(), []
        for k in m:
            if k != -1 and k in seen:
                k = -1
            seen.add(k)
            out.append(k)
        return out

    # -- propagation -----------------------------------------------------------------------
    def complete_forward_annotation(self):
        for name in list(self.program.params) + list(self.block.vars):
            if name in self.attrs:
                continue
            m = self._annotation_of(name)
            if m is not None:
                self.attrs[name] = DistAttr(self._fix_divisible(name, m))
                if name not in self.program.params and any(k != -1 for k in m):
                    self.feed_slices[name] = list(self.attrs[name].dims_mapping)
        for op in self.block.ops:
            self.plans.append(self._plan(op))
        self.program._dist_attrs = self.attrs
        return self.attrs

    def _plan(self, op):
        ins = [n for n in op.input_names()]
        outs = op.output_names()
        if op.func is None or op.type in ("backward", "optimize", "cond", "while"):
            raise NotImplementedError(f"auto_parallel partition: op {op.type} (forward programs only)")
        rule = getattr(self, "_rule_" + op.type, None)
        plan = None
        if rule is not None:
            plan = rule(op, ins, outs)
        if plan is None:
            plan = self._rule_default(op, ins, outs)
        req, out_maps, partial, rewrite = plan
        for n, m in zip(outs, out_maps):
            self.attrs[n] = DistAttr(m)
        return {"op": op, "req": req, "partial": partial, "rewrite": rewrite}

    def _rule_default(self, op, ins, outs):
        req = {n: [-1] * len(self.shape(n) or []) for n in ins}
        return req, [[-1] * len(self.shape(n) or []) for n in outs], {}, None

    def _unary(self, op, ins, outs):
        if len(ins) != 1:
            return None
        m = self.mapping(ins[0])
        return {}, [m for _ in outs], {}, None

    def _binary(self, op, ins, outs):
        out_shape = self.shape(outs[0])
        if out_shape is None:
            return None
        nd = len(out_shape)
        chosen = [-1] * nd
        for n in ins:
            shp, m = self.shape(n), self.mapping(n)
            off = nd - len(shp)
            for d, k in enumerate(m):
                if k != -1 and chosen[off + d] == -1 and shp[d] == out_shape[off + d] and k not in chosen:
                    chosen[off + d] = k
        req = {}
        for n in ins:
            shp = self.shape(n)
            off = nd - len(shp)
            want = [chosen[off + d] if shp[d] == out_shape[off + d] else -1 for d in range(len(shp))]
            if want != self.mapping(n):
                req[n] = want
        return req, [chosen], {}, None

    def _softmax_like(self, op, ins, outs):
        x = ins[0]
        m = self.mapping(x)
        d = _dim_arg(op, 1, default=-1)
        d = (d if d is not None else -1) % len(m)
        req = {}
        if m[d] != -1:
            m[d] = -1
            req[x] = m
        return req, [m], {}, None

    def _rule_layer_norm(self, op, ins, outs):
        x = ins[0]
        m = self.mapping(x)
        w = op.args[1] if len(op.args) > 1 and isinstance(op.args[1], VarRef) else None
        if isinstance(w, VarRef):
            nnorm = len(self.shape(w.name))
        else:
            ns = op.args[1] if len(op.args) > 1 else op.kwargs.get("normalized_shape", [m[-1]])
            nnorm = len(ns) if isinstance(ns, (list, tuple)) else 1
        req = {}
        if any(k != -1 for k in m[-nnorm:]):
            m = m[:-nnorm] + [-1] * nnorm
            req[x] = m
        for n in ins[1:]:
            if any(k != -1 for k in self.mapping(n)):
                req[n] = [-1] * len(self.shape(n))
        return req, [m], {}, None

    def _reduce(self, op, ins, outs):
        x = ins[0]
        m = self.mapping(x)
        d = _dim_arg(op, 1)
        keep = op.kwargs.get("keepdim", op.args[2] if len(op.args) > 2 and isinstance(op.args[2], bool) else False)
        dims = list(range(len(m))) if d is None else ([d] if isinstance(d, int) else list(d))
        dims = [dd % len(m) for dd in dims]
        req = {}
        if any(m[dd] != -1 for dd in dims):
            m = [(-1 if i in dims else k) for i, k in enumerate(m)]
            req[x] = m
        out = [(-1 if i in dims else k) for i, k in enumerate(m)] if keep else \
            [k for i, k in enumerate(m) if i not in dims]
        return req, [out], {}, None

    def _rule_linear(self, op, ins, outs):
        x, w = op.args[0], op.args[1]
        if not (isinstance(x, VarRef) and isinstance(w, VarRef)):
            return None
        b = op.args[2] if len(op.args) > 2 else op.kwargs.get("bias")
        torch_layout = op.func is F.linear  # weight [out, in]
        kd, nd = (1, 0) if torch_layout else (0, 1)
        xm, wm = self.mapping(x.name), self.mapping(w.name)
        kmap, nmap = wm[kd], wm[nd]
        req = {}
        batch = xm[:-1]
        if nmap != -1 and nmap in batch:  # mesh dim already splits the batch: replicate N
            nmap = -1
        if kmap != -1 and kmap in batch:
            kmap = -1
        if [kmap, nmap][::(-1 if torch_layout else 1)] != [wm[0], wm[1]]:
            want = [-1, -1]
            want[kd], want[nd] = kmap, nmap
            req[w.name] = want
        if xm[-1] != kmap:
            req[x.name] = batch + [kmap]
        rewrite = None
        if isinstance(b, VarRef):
            bm = self.mapping(b.name)
            if bm != [nmap]:
                req[b.name] = [nmap]
        partial = {}
        if kmap != -1:
            partial = {0: kmap}
            if isinstance(b, VarRef):  # bias added once, after the reduction
                rewrite = ("linear_rowpar", kmap)
                partial = {}
        return req, [batch + [nmap]], partial, rewrite

    def _rule_matmul_v2(self, op, ins, outs):
        if len(ins) != 2 or op.kwargs:
            return None
        a, b = op.args[0], op.args[1]
        if not (isinstance(a, VarRef) and isinstance(b, VarRef)):
            return None
        sa, sb = self.shape(a.name), self.shape(b.name)
        if len(sa) < 2 or len(sb) < 2:
            return self._rule_default(op, ins, outs)
        if len(sb) == 2 and b.name in self.program.params:  # activation @ weight: the linear rule
            return self._rule_linear(op, ins, outs)
        am, bm = self.mapping(a.name), self.mapping(b.name)
        nd = max(len(sa), len(sb))
        out_batch = [-1] * (nd - 2)
        for shp, m in ((sa, am), (sb, bm)):
            off = nd - len(shp)
            for d in range(len(shp) - 2):
                if m[d] != -1 and out_batch[off + d] == -1 and m[d] not in out_batch:
                    out_batch[off + d] = m[d]
        kmap = am[-1] if am[-1] == bm[-2] else -1
        mm_, nn_ = am[-2], bm[-1]
        used = set(k for k in out_batch if k != -1)
        if kmap in used:
            kmap = -1
        if mm_ in used or mm_ == kmap:
            mm_ = -1
        used.add(mm_)
        if nn_ in used or nn_ == kmap:
            nn_ = -1
        req = {}
        for ref, shp, m, last2 in ((a, sa, am, [mm_, kmap]), (b, sb, bm, [kmap, nn_])):
            off = nd - len(shp)
            want = [out_batch[off + d] if shp[d] != 1 else -1 for d in range(len(shp) - 2)] + last2
            if want != m:
                req[ref.name] = want
        partial = {0: kmap} if kmap != -1 else {}
        return req, [out_batch + [mm_, nn_]], partial, None

    def _rule_lookup_table_v2(self, op, ins, outs):
        ids, w = op.args[0], op.args[1]
        if not (isinstance(ids, VarRef) and isinstance(w, VarRef)):
            return None
        im, wm = self.mapping(ids.name), self.mapping(w.name)
        vmap, hmap = wm
        if hmap in im:
            hmap = -1
        if vmap in im or vmap == hmap:
            vmap = -1
        req = {}
        if [vmap, hmap] != wm:
            req[w.name] = [vmap, hmap]
        if vmap != -1:
            return req, [im + [hmap]], {}, ("vocab_parallel", vmap)
        return req, [im + [hmap]], {}, None

    def _rule_reshape2(self, op, ins, outs):
        x = ins[0]
        sin, sout = self.shape(x), self.shape(outs[0])
        m = self.mapping(x)
        if all(k == -1 for k in m):
            return {}, [[-1] * len(sout)], {}, None
        # group dims by equal cumulative products
        groups, i, j = [], 0, 0
        while i < len(sin) or j < len(sout):
            gi, gj = [i] if i < len(sin) else [], [j] if j < len(sout) else []
            pi = sin[i] if i < len(sin) else 1
            pj = sout[j] if j < len(sout) else 1
            i += 1 if gi else 0
            j += 1 if gj else 0
            while pi != pj:
                if pi < pj and i < len(sin):
                    pi *= sin[i]
                    gi.append(i)
                    i += 1
                elif j < len(sout):
                    pj *= sout[j]
                    gj.append(j)
                    j += 1
                else:
                    return self._rule_default(op, ins, outs)
            groups.append((gi, gj))
        out = [-1] * len(sout)
        want = list(m)
        for gi, gj in groups:
            sh = [d for d in gi if m[d] != -1]
            if not sh:
                continue
            d = sh[0]
            lead_in = [q for q in gi if sin[q] != 1]
            lead_out = [q for q in gj if sout[q] != 1]
            k = m[d]
            if (len(sh) == 1 and lead_in and lead_in[0] == d and lead_out
                    and sout[lead_out[0]] % self.nmesh(k) == 0):
                out[lead_out[0]] = k
            else:
                for q in sh:
                    want[q] = -1
        req = {x: want} if want != m else {}
        return req, [out], {}, ("reshape", out)

    def _rule_transpose2(self, op, ins, outs):
        x = ins[0]
        m = self.mapping(x)
        name = getattr(op.func, "__name__", "")
        if name in ("transpose", "_transpose", "swapaxes"):
            d0, d1 = op.args[1] % len(m), op.args[2] % len(m)
            out = list(m)
            out[d0], out[d1] = m[d1], m[d0]
        else:
            perm = op.args[1] if len(op.args) == 2 and isinstance(op.args[1], (list, tuple)) else op.args[1:]
            perm = op.kwargs.get("dims", perm)
            out = [m[p % len(m)] for p in perm]
        return {}, [out], {}, None

    def _rule_split(self, op, ins, outs):
        x = ins[0]
        m = self.mapping(x)
        d = _dim_arg(op, 2, default=0) % len(m)
        req = {}
        if m[d] != -1:
            m[d] = -1
            req[x] = m
        return req, [list(m) for _ in outs], {}, None

    def _rule_concat(self, op, ins, outs):
        d = _dim_arg(op, 1, default=0)
        m0 = self.mapping(ins[0])
        d %= len(m0)
        want = list(m0)
        want[d] = -1
        req = {n: want for n in ins if self.mapping(n) != want}
        return req, [want], {}, None

    def _rule_fused_attention(self, op, ins, outs):
        m = self.mapping(ins[0])
        want = m[:-2] + [-1, -1]
        req = {n: want for n in ins[:3] if self.mapping(n) != want}
        for n in ins[3:]:
            if any(k != -1 for k in self.mapping(n)):
                req[n] = [-1] * len(self.shape(n))
        return req, [want], {}, None


for _t in _UNARY:
    setattr(Completer, "_rule_" + _t, Completer._unary)
for _t in _BINARY:
    setattr(Completer, "_rule_" + _t, Completer._binary)
for _t in ("softmax", "log_softmax"):
    setattr(Completer, "_rule_" + _t, Completer._softmax_like)
for _t in ("reduce_sum", "reduce_mean"):
    setattr(Completer, "_rule_" + _t, Completer._reduce)


# ---------------------------------------------------------------------------------------------
# collectives (autograd-aware) and per-rank program construction
# ---------------------------------------------------------------------------------------------
_GROUPS: dict = {}


def _coords(mesh, rank):
    ids = mesh.process_ids
    idx = ids.index(rank)
    out = []
    for s in reversed(mesh.shape):
        out.append(idx % s)
        idx //= s
    return list(reversed(out))


def _groups_for(mesh, k):
    """All process groups along mesh dim ``k`` (created in the same order on every rank)."""
    key = (hash(mesh), k)
    if key not in _GROUPS:
        shape = mesh.shape
        ids = mesh.mesh
        others = [range(s) for i, s in enumerate(shape) if i != k]
        gs = {}
        for oc in itertools.product(*others):
            idx = list(oc)
            idx.insert(k, slice(None))
            ranks = ids[tuple(idx)].reshape(-1).tolist()
            g = dist.new_group(ranks) if dist.is_initialized() and dist.get_world_size() > 1 else None
            for r in ranks:
                gs[r] = (g, ranks)
        _GROUPS[key] = gs
    return _GROUPS[key]


# Megatron-style conjugate collectives: SPMD semantics where every rank holds the same loss, so
# a replicated value's gradient is replicated and a sharded value's gradient is sharded.
class _AllReduceFn(torch.autograd.Function):
    """partial -> replicated: forward sum, backward identity."""

    @staticmethod
    def forward(ctx, x, group):
        y = x.contiguous().clone()
        dist.all_reduce(y, group=group)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None


class _CopyToGroupFn(torch.autograd.Function):
    """replicated input of a computation split over the group: forward identity, backward sum of
    the per-shard partial gradients."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        dist.all_reduce(g, group=ctx.group)
        return g, None


class _GatherFn(torch.autograd.Function):
    """sharded -> replicated along ``dim``: forward all-gather, backward keep the local slice."""

    @staticmethod
    def forward(ctx, x, dim, group):
        n = dist.get_world_size(group)
        parts = [torch.empty_like(x.contiguous()) for _ in range(n)]
        dist.all_gather(parts, x.contiguous(), group=group)
        ctx.dim, ctx.idx, ctx.size = dim, dist.get_rank(group), x.shape[dim]
        return torch.cat(parts, dim=dim)

    @staticmethod
    def backward(ctx, g):
        return g.narrow(ctx.dim, ctx.idx * ctx.size, ctx.size).contiguous(), None, None


class _SliceFn(torch.autograd.Function):
    """replicated -> sharded along ``dim`` (local narrow), backward all-gather of the slices'
    gradients (the replicated input's full gradient)."""

    @staticmethod
    def forward(ctx, x, dim, idx, n, group):
        size = x.shape[dim] // n
        ctx.dim, ctx.group, ctx.n = dim, group, n
        return x.narrow(dim, idx * size, size).contiguous()

    @staticmethod
    def backward(ctx, g):
        if ctx.group is None:
            return g, None, None, None, None
        parts = [torch.empty_like(g.contiguous()) for _ in range(ctx.n)]
        dist.all_gather(parts, g.contiguous(), group=ctx.group)
        return torch.cat(parts, dim=ctx.dim), None, None, None, None


def _allreduce(x, group):
    return x if group is None else _AllReduceFn.apply(x, group)


def _allgather(x, dim, group):
    return x if group is None else _GatherFn.apply(x, dim, group)


class _Identity:
    __name__ = "assign"

    def __call__(self, x):
        return x


class _CopyToGroup:
    __name__ = "c_identity"

    def __init__(self, group):
        self.group = group

    def __call__(self, x):
        if self.group is None or not (x.is_floating_point() and torch.is_grad_enabled()):
            return x
        return _CopyToGroupFn.apply(x, self.group)


class _Gather:
    def __init__(self, dim, group):
        self.dim, self.group = dim, group
        self.__name__ = "c_allgather"

    def __call__(self, x):
        return _allgather(x, self.dim, self.group)


class _Slice:
    def __init__(self, dim, idx, n, group):
        self.dim, self.idx, self.n, self.group = dim, idx, n, group
        self.__name__ = "slice"

    def __call__(self, x):
        if x.is_floating_point() and torch.is_grad_enabled():
            return _SliceFn.apply(x, self.dim, self.idx, self.n, self.group)
        size = x.shape[self.dim] // self.n
        return x.narrow(self.dim, self.idx * size, size).contiguous()


class _AllReduce:
    __name__ = "c_allreduce_sum"

    def __init__(self, group):
        self.group = group

    def __call__(self, x):
        return _allreduce(x, self.group)


class _LinearRowParallel:
    """y = all_reduce(linear(x_shard, w_shard)) + b: the bias is added once, after the sum."""

    def __init__(self, func, group):
        self.func, self.group = func, group
        self.__name__ = "linear_row_parallel"

    def __call__(self, x, w, b=None, *a, **k):
        return _allreduce(self.func(x, w, None), self.group) + (b if b is not None else 0)


class _VocabParallelEmbedding:
    """Vocab-split table: ids outside this rank's rows look up row 0 and are zeroed; the partial
    results are summed over the vocab group (reference `dist_embedding.py` / c_embedding)."""

    def __init__(self, func, start, group):
        self.func, self.start, self.group = func, start, group
        self.__name__ = "c_embedding"

    def __call__(self, ids, w, *a, **k):
        n = w.shape[0]
        local = ids - self.start
        ok = (local >= 0) & (local < n)
        out = self.func(torch.where(ok, local, torch.zeros_like(local)), w, *a, **k)
        out = out * ok.unsqueeze(-1).to(out.dtype)
        return _allreduce(out, self.group)


class Partitioner:
    """Per-rank program of a completed serial program (``partition(rank)``)."""

    def __init__(self, completer: Completer):
        self.c = completer
        self.mesh = completer.mesh
        for k in range(self.mesh.ndim):  # collective groups: same creation order on every rank
            _groups_for(self.mesh, k)

    def _is_float(self, name):
        v = self.c.block.vars.get(name)
        t = v if v is not None else self.c.program.params.get(name)
        return t is not None and t.is_floating_point()

    def _local_shape(self, shape, m):
        return [s // self.mesh.shape[k] if k != -1 else s for s, k in zip(shape, m)]

    def _local_param(self, t, m, coords):
        out = t
        for d, k in enumerate(m):
            if k != -1:
                n = self.mesh.shape[k]
                size = out.shape[d] // n
                out = out.narrow(d, coords[k] * size, size)
        out = out.detach().clone().contiguous()
        out.requires_grad_(t.requires_grad)
        return out

    def partition(self, rank, fetch_list=()):
        c = self.c
        coords = _coords(self.mesh, rank)
        src = c.program
        p = Program()
        blk = p.global_block()
        for name, v in src.global_block().vars.items():  # local shapes, owned by the new block
            m = c.attrs[name].dims_mapping if name in c.attrs else [-1] * len(v.shape)
            meta = torch.empty(self._local_shape(list(v.shape), m), dtype=v.dtype, device="meta")
            blk.vars[name] = Variable(meta, name, blk, v.persistable_, v.stop_gradient_,
                                      declared_shape=v.declared_shape)
        p.feed_names, p.fetch_names = list(src.feed_names), list(src.fetch_names)
        cur = {}  # var -> current local mapping in the per-rank program
        for name, t in src.params.items():
            m = c.attrs[name].dims_mapping if name in c.attrs else [-1] * t.dim()
            p.params[name] = self._local_param(t, m, coords)
            p._param_of[id(p.params[name])] = name
            cur[name] = list(m)
        ops = []
        resh_cache = {}

        def add(func, args, out_name, typ, like=None, mapping=None):
            op = Operator(blk, func, args, {}, VarRef(out_name), type=typ)
            op.idx = len(ops)
            ops.append(op)
            if like is not None and out_name not in blk.vars:  # the new var's local meta
                v = src.global_block().vars.get(like)
                t = v if v is not None else src.params[like]
                m = mapping if mapping is not None else [-1] * len(t.shape)
                meta = torch.empty(self._local_shape(list(t.shape), m), dtype=t.dtype, device="meta")
                blk.vars[out_name] = Variable(meta, out_name, blk, False, False)

        def reshard(name, want):
            have = cur.get(name)
            if have is None:
                have = [-1] * len(c.shape(name) or want)
            if have == want:
                return name
            key = (name, tuple(want))
            if key in resh_cache:
                return resh_cache[key]
            x = name
            cur_m = list(have)
            for d, (h, w) in enumerate(zip(have, want)):  # gathers first, then local slices
                if h != -1 and h != w:
                    g, _ = _groups_for(self.mesh, h)[rank]
                    y = unique_name(f"{name}@GATHER")
                    step = [(q if i != d else -1) for i, q in enumerate(cur_m)]
                    add(_Gather(d, g), (VarRef(x),), y, "c_allgather", name, step)
                    cur_m = step
                    x = y
            for d, (h, w) in enumerate(zip(have, want)):
                if w != -1 and h != w:
                    y = unique_name(f"{name}@SLICE")
                    g, _ = _groups_for(self.mesh, w)[rank]
                    step = [(q if i != d else w) for i, q in enumerate(cur_m)]
                    add(_Slice(d, coords[w], self.mesh.shape[w], g), (VarRef(x),), y, "slice", name, step)
                    cur_m = step
                    x = y
            resh_cache[key] = x
            cur[x] = list(want)
            return x

        for name, m in c.feed_slices.items():  # global feeds -> local shards
            have = [-1] * len(m)
            cur[name] = have
            loc = reshard(name, m)
            if loc != name:
                ops[-1].outputs = VarRef(name)  # slice in place of the feed (reads the global feed)
                cur[name] = list(m)
                resh_cache.clear()
        for plan in c.plans:
            op = plan["op"]
            rename = {}
            for n, want in plan["req"].items():
                loc = reshard(n, list(want))
                if loc != n:
                    rename[n] = loc
            # inputs replicated over a mesh dim this op's computation is split over: their
            # gradient is a per-shard partial sum -> c_identity (backward all-reduce) on that dim
            split = {k for n in op.output_names() for k in c.attrs[n].dims_mapping if k != -1}
            split |= set(plan["partial"].values())
            for n in dict.fromkeys(op.input_names()):
                x = rename.get(n, n)
                if not self._is_float(n):
                    continue
                for k in sorted(split - {q for q in cur.get(x, []) if q != -1}):
                    key = ("copy", x, k)
                    if key not in resh_cache:
                        g, _ = _groups_for(self.mesh, k)[rank]
                        y = unique_name(f"{n}@COPY")
                        add(_CopyToGroup(g), (VarRef(x),), y, "c_identity", n, cur.get(x))
                        cur[y] = list(cur.get(x, []))
                        resh_cache[key] = y
                    x = resh_cache[key]
                if x != n:
                    rename[n] = x

            def ren(x):
                if isinstance(x, VarRef) and x.name in rename:
                    return VarRef(rename[x.name])
                return x
            from torch.utils._pytree import tree_map
            args = tree_map(ren, op.args)
            kwargs = tree_map(ren, op.kwargs)
            func = op.func
            rw = plan["rewrite"]
            outs = op.output_names()
            if rw is not None and rw[0] == "reshape":
                out_map = rw[1]
                shp_arg = args[1] if len(args) == 2 and isinstance(args[1], (list, tuple)) else list(args[1:])
                new = []
                for d, s in enumerate(shp_arg):
                    if d < len(out_map) and out_map[d] != -1 and isinstance(s, int) and s > 0:
                        s = s // self.mesh.shape[out_map[d]]
                    elif d < len(out_map) and out_map[d] != -1 and isinstance(s, SymDim):
                        s = _ScaledSym(s, self.mesh.shape[out_map[d]])
                    new.append(s)
                args = (args[0], new) if len(args) == 2 and isinstance(args[1], (list, tuple)) else \
                    (args[0], *new)
            elif rw is not None and rw[0] == "linear_rowpar":
                g, _ = _groups_for(self.mesh, rw[1])[rank]
                func = _LinearRowParallel(op.func, g)
            elif rw is not None and rw[0] == "vocab_parallel":
                g, _ = _groups_for(self.mesh, rw[1])[rank]
                rows = c.shape(op.args[1].name)[0] // self.mesh.shape[rw[1]]
                func = _VocabParallelEmbedding(op.func, coords[rw[1]] * rows, g)
            partial = plan["partial"]
            new_outs = op.outputs
            if partial:
                tmp = unique_name(f"{outs[0]}@PARTIAL")
                new_outs = VarRef(tmp)
            nop = Operator(blk, func, args, kwargs, new_outs, type=op.type, attrs=op.attrs)
            nop.idx = len(ops)
            ops.append(nop)
            for n in outs:
                cur[n] = list(c.attrs[n].dims_mapping)
            if partial:
                g, _ = _groups_for(self.mesh, partial[0])[rank]
                ov = blk.vars[outs[0]]
                blk.vars[tmp] = Variable(torch.empty(list(ov.shape), dtype=ov.dtype, device="meta"),
                                         tmp, blk, False, False)
                add(_AllReduce(g), (VarRef(tmp),), outs[0], "c_allreduce_sum")
            resh_cache = {k: v for k, v in resh_cache.items() if k[0] not in outs}
        for name in fetch_list:  # fetched values gathered to the global tensor
            name = getattr(name, "var_name", name)
            m = cur.get(name)
            if m is not None and any(k != -1 for k in m):
                loc = reshard(name, [-1] * len(m))
                add(_Identity(), (VarRef(loc),), name, "assign")
        blk.ops = ops
        p._version += 1
        p._dist_rank = rank
        p._dist_mesh = self.mesh
        return p


class _ScaledSym(SymDim):
    """A symbolic (feed-bound) reshape size divided by the mesh-dim degree."""

    def __init__(self, sym, n):  # noqa: super().__init__ not needed: resolve() is overridden
        self.sym, self.n = sym, n

    def resolve(self, bind):
        return self.sym.resolve(bind) // self.n


def complete(program, mesh, annotations=None):
    """Sharding propagation (reference ``Completer.complete_forward_annotation``)."""
    c = Completer(program, mesh, annotations)
    c.complete_forward_annotation()
    return c


def partition(program, mesh, rank=None, annotations=None, fetch_list=()):
    """Complete + partition ``program`` for ``rank`` (default: this process's rank): the per-rank
    program with local parameter shards and the collectives its layouts need."""
    if rank is None:
        rank = dist.get_rank() if dist.is_initialized() else 0
    c = complete(program, mesh, annotations)
    return Partitioner(c).partition(rank, fetch_list)
