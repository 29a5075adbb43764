"""Distributed (sharded) checkpoints with resharding on load.

Parity: reference `python/paddle/distributed/sharding/group_sharded.py:save_group_sharded_model`,
`fleet/utils/...` per-rank ``.pdparams``/``.pdopt`` saves and the TP merge utilities; the
load-time resharding follows the later `paddle.distributed.save_state_dict/load_state_dict`
contract (metadata + per-rank shard files, any source world size → any target world size).

Format (directory):
  metadata.json   {key: {"numel", "shape", "dtype", "regions": [[rank, global_off, length, file_off]...]}}
  <rank>.safetensors   one 1-D tensor per key holding that rank's regions back to back
Every tensor is addressed in its flattened global index space; a shard is a list of
(global_offset, length) regions, which covers ZeRO flat shards (one region per bucket),
row / column tensor-parallel slices and plain replicated tensors (one full region, rank 0 only).
safetensors files are memory-mapped on load and never unpickled.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from safetensors.torch import load_file, save_file


class Shard:
    """A local piece of a global tensor: ``regions`` = [(global_off, length)] in flattened global
    order, laid out back to back in ``local`` (1-D view)."""

    def __init__(self, local, global_shape, regions, replicated=False):
        self.local = local
        self.global_shape = list(global_shape)
        self.regions = [(int(o), int(n)) for o, n in regions]
        self.replicated = replicated  # identical on every rank: only the coordinator writes it
        assert sum(n for _, n in self.regions) == local.numel(), "regions must cover the local tensor"


def _rank_world(group):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _as_shard(v, rank, coordinator=0):
    if isinstance(v, Shard):
        if v.replicated and rank != coordinator:
            return Shard(v.local.reshape(-1)[:0], v.global_shape, [])
        return v
    if isinstance(v, torch.Tensor):  # replicated: written by the coordinator only
        if rank != coordinator:
            return Shard(v.reshape(-1)[:0], v.shape, [])
        return Shard(v.reshape(-1), v.shape, [(0, v.numel())])
    raise TypeError(f"unsupported checkpoint value {type(v)}")


def save_state_dict(state_dict, path, process_group=None, coordinator_rank=0):
    """Collective: every rank calls it with its local Shards / replicated tensors."""
    import torch.distributed as dist
    rank, world = _rank_world(process_group)
    os.makedirs(path, exist_ok=True)
    tensors, meta = {}, {}
    for k, v in state_dict.items():
        if not isinstance(v, (Shard, torch.Tensor)):
            continue
        s = _as_shard(v, rank, coordinator_rank)
        if s.regions and s.local.numel():
            tensors[k] = s.local.detach().reshape(-1).contiguous().cpu()
        off, regs = 0, []
        for go, n in s.regions:
            regs.append([rank, go, n, off])
            off += n
        meta[k] = {"numel": int(np.prod(s.global_shape)) if s.global_shape else 1,
                   "shape": s.global_shape, "dtype": str(s.local.dtype).replace("torch.", ""),
                   "regions": regs}
    save_file(tensors, os.path.join(path, f"{rank}.safetensors"))
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, meta, group=process_group)
    else:
        gathered = [meta]
    if rank == coordinator_rank:
        merged = {}
        for m in gathered:
            for k, e in m.items():
                if k not in merged:
                    merged[k] = dict(e, regions=[])
                merged[k]["regions"].extend(e["regions"])
        extra = {k: v for k, v in state_dict.items() if isinstance(v, (int, float, str, bool))}
        with open(os.path.join(path, "metadata.json"), "w") as f:
            json.dump({"tensors": merged, "extra": extra}, f)
    if world > 1:
        dist.barrier(group=process_group)


def load_state_dict(state_dict, path, process_group=None):
    """Fill every Shard / tensor of ``state_dict`` in place from a checkpoint written with any
    world size (resharding by region overlap)."""
    with open(os.path.join(path, "metadata.json")) as f:
        meta = json.load(f)
    tmeta = meta["tensors"]
    rank, _ = _rank_world(process_group)
    files = {}

    def src_file(r):
        if r not in files:
            files[r] = load_file(os.path.join(path, f"{r}.safetensors"))
        return files[r]

    for k, v in state_dict.items():
        if k not in tmeta:
            if isinstance(v, (Shard, torch.Tensor)):
                raise KeyError(f"{k} not in checkpoint {path}")
            continue
        s = v if isinstance(v, Shard) else Shard(v.reshape(-1) if v.is_contiguous() else v.view(-1),
                                                 v.shape, [(0, v.numel())])
        dst = s.local.reshape(-1)
        loff = 0
        for go, n in s.regions:
            for (r, sgo, sn, soff) in tmeta[k]["regions"]:
                lo, hi = max(go, sgo), min(go + n, sgo + sn)
                if lo >= hi:
                    continue
                src = src_file(r)[k]
                piece = src[soff + (lo - sgo): soff + (hi - sgo)]
                dst[loff + (lo - go): loff + (hi - go)].copy_(piece.to(dst.dtype))
            loff += n
    return meta.get("extra", {})


def axis_shard(local, global_shape, axis, rank, world):
    """Shard of a tensor split evenly along ``axis`` (tensor-parallel column / row slices, vocab
    shards). The local slice is rank ``rank``'s chunk; regions are the contiguous runs it occupies
    in the flattened global tensor (one per index of the leading dims)."""
    gs = list(global_shape)
    axis = axis % len(gs)
    assert gs[axis] % world == 0, "axis must divide evenly"
    chunk = gs[axis] // world
    inner = int(np.prod(gs[axis + 1:])) if axis + 1 < len(gs) else 1
    outer = int(np.prod(gs[:axis])) if axis else 1
    run = chunk * inner
    regions = [(o * gs[axis] * inner + rank * run, run) for o in range(outer)]
    return Shard(local.contiguous().reshape(-1), gs, regions)


# ------------------------------------------------------------------------------ engine helpers
def flat_trainer_state(trainer, model=None, prefix="opt"):
    """Per-PARAMETER shards of a FlatTrainer's fp32 master / moments plus the (replicated) model
    parameters, ready for :func:`save_state_dict` / :func:`load_state_dict`. Keys are parameter
    names, coordinates are each parameter's own flattened index space, so a checkpoint written
    with one data-parallel degree (its flat/bucket padding included) loads under any other."""
    named = dict((id(p), n) for n, p in (model or trainer.model).named_parameters())
    out = {f"{prefix}.step": trainer.step_count}
    for g in trainer.groups:
        # this rank's master buffer: per bucket, the slice [b.start + rank*L, +L) of the flat space
        spans, mo = [], 0
        for b in g.buckets:
            L = (b.end - b.start) // trainer.world if trainer.sharding else (b.end - b.start)
            lo = b.start + (trainer.rank * L if trainer.sharding else 0)
            spans.append((lo, lo + L, mo))
            mo += L
        for p in g.params:
            po, pn = g.offsets[id(p)]
            pname = named.get(id(p), f"param{po}")
            for lo, hi, base in spans:
                a, e = max(po, lo), min(po + pn, hi)
                if a >= e:
                    continue
                for name in ("master", "m", "v"):
                    t = getattr(g, name)
                    if t is None:
                        continue
                    out[f"{prefix}.{pname}.{name}"] = Shard(
                        t[base + (a - lo): base + (e - lo)], list(p.shape), [(a - po, e - a)],
                        replicated=not trainer.sharding)
    if model is not None:
        for k, p in model.state_dict().items():
            out[f"model.{k}"] = p
    return out
