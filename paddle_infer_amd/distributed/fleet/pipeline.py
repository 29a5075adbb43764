"""Pipeline parallelism: PipelineLayer / LayerDesc / SharedLayerDesc and the 1F1B schedule.

Parity: reference `python/paddle/distributed/fleet/meta_parallel/parallel_layers/pp_layers.py`
(LayerDesc, SharedLayerDesc, PipelineLayer with ``seg_method`` uniform / ``layer:<Name>``,
shared-weight groups, ``num_virtual_pipeline_stages``) and `meta_parallel/pipeline_parallel.py`
(PipelineParallel.train_batch / eval_batch, 1F1B: warm-up forwards, steady
one-forward-one-backward, cool-down backwards; PipelineParallelWithInterleave at :464 — each rank
holds V model chunks, global chunk g on rank g % S, and the schedule walks virtual micro-batches so
the pipeline bubble shrinks by V; `pp_utils/p2p_communication.py`).

Stage-to-stage activations and gradients travel as point-to-point RCCL send/recv between adjacent
ranks of the pipe group (one xGMI hop when stages are on the same node). Tensor metadata (ndim,
shape, dtype) is exchanged once per ``train_batch``; steady-state exchanges post the activation send
and the gradient receive together (``batch_isend_irecv``) so opposite-direction traffic between
adjacent stages cannot deadlock.
"""
from __future__ import annotations

import math
import re

import torch
import torch.distributed as dist

from ...nn.layer.base import Layer
from ..collective import Group

_DT = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.bool, torch.float64]


class LayerDesc:
    def __init__(self, layer_func, *inputs, **kwargs):
        self.layer_func, self.inputs, self.kwargs = layer_func, inputs, kwargs

    def build_layer(self):
        return self.layer_func(*self.inputs, **self.kwargs)

    def __repr__(self):
        return f"LayerDesc({getattr(self.layer_func, '__name__', self.layer_func)})"


class SharedLayerDesc(LayerDesc):
    def __init__(self, key, layer_func, forward_func=None, shared_weight_attr="weight", *inputs, **kwargs):
        super().__init__(layer_func, *inputs, **kwargs)
        self.layer_name, self.forward_func, self.shared_weight_attr = key, forward_func, shared_weight_attr


def _segment(descs, num_stages, method):
    n = len(descs)
    if isinstance(method, str) and method.startswith("layer:"):
        pat = method.split(":", 1)[1]
        marks = [i for i, d in enumerate(descs)
                 if re.search(pat, getattr(getattr(d, "layer_func", d), "__name__", type(d).__name__))]
        if len(marks) < num_stages:
            raise ValueError(f"{len(marks)} '{pat}' layers cannot fill {num_stages} pipeline chunks "
                             "(stages x virtual stages)")
        per = math.ceil(len(marks) / num_stages)
        bounds = [0]
        for s in range(1, num_stages):
            k = s * per
            bounds.append(marks[k] if k < len(marks) else n)
        bounds.append(n)
        return bounds
    per = n / num_stages
    return [round(i * per) for i in range(num_stages)] + [n]


class PipelineLayer(Layer):
    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seg_method="uniform",
                 recompute_interval=0, recompute_ctx=None, num_virtual_pipeline_stages=None):
        super().__init__()
        from . import get_hybrid_communicate_group
        hcg = get_hybrid_communicate_group()
        if num_stages is None:
            num_stages = hcg.get_pipe_parallel_world_size() if hcg else 1
        self.num_stages = num_stages
        self.stage_id = hcg.get_stage_id() if hcg else 0
        self.loss_fn = loss_fn
        self.recompute_interval = recompute_interval
        self._descs = list(layers)
        V = int(num_virtual_pipeline_stages or 1)
        self._num_virtual = V
        # S * V segments; global chunk g lives on rank g % S as local chunk g // S
        self.segment_parts = _segment(self._descs, num_stages * V, seg_method)
        self.run_function = []
        self._chunk_fns = []
        self._index_layers = []  # (global desc index, built layer) held by this rank
        self.shared_layers = torch.nn.ModuleDict()
        self.shared_weight_attrs = {}
        self._stage_layers = torch.nn.ModuleList()
        for v in range(V):
            g = v * num_stages + self.stage_id
            fns = []
            for i in range(self.segment_parts[g], self.segment_parts[g + 1]):
                fns.append(self._build(i))
            self._chunk_fns.append(fns)
            self.run_function.extend(fns)
        # shared-weight groups: all stages that hold a given shared layer. new_group is a WORLD
        # collective, so every rank creates the group of every pipe group (same order everywhere)
        # and keeps the one it belongs to.
        self._shared_groups = {}
        if hcg is not None and dist.is_initialized() and num_stages > 1:
            me = dist.get_rank()
            pipe_lists = hcg.topology().get_comm_list("pipe")
            for name in sorted({d.layer_name for d in self._descs if isinstance(d, SharedLayerDesc)}):
                stages = sorted({g % num_stages for g in range(num_stages * V)
                                 for i in range(self.segment_parts[g], self.segment_parts[g + 1])
                                 if isinstance(self._descs[i], SharedLayerDesc) and self._descs[i].layer_name == name})
                if len(stages) < 2:
                    continue
                for pl in pipe_lists:
                    ranks = [pl[st] for st in stages]
                    g = dist.new_group(ranks)
                    if me in ranks and name in self.shared_layers:
                        self._shared_groups[name] = g
                        w = getattr(self.shared_layers[name], self.shared_weight_attrs[name])
                        dist.broadcast(w.data, src=ranks[0], group=g)
                        # the global grad norm counts a shared weight once (reference
                        # `pp_layers.py`: is_firstly_shared)
                        w.is_firstly_shared = me == ranks[0]

    def _build(self, i):
        d = self._descs[i]
        if isinstance(d, SharedLayerDesc):
            if d.layer_name not in self.shared_layers:
                self.shared_layers[d.layer_name] = d.build_layer()
                self.shared_weight_attrs[d.layer_name] = d.shared_weight_attr
            lay = self.shared_layers[d.layer_name]
            self._index_layers.append((i, lay))
            if d.forward_func is not None:
                return lambda x, _l=lay, _f=d.forward_func: _f(_l, x)
            return lay
        if isinstance(d, LayerDesc):
            lay = d.build_layer()
            self._stage_layers.append(lay)
            self._index_layers.append((i, lay))
            return lay
        if isinstance(d, torch.nn.Module):
            self._stage_layers.append(d)
            self._index_layers.append((i, d))
        return d

    def allreduce_shared_weight_gradients(self):
        for name, g in self._shared_groups.items():
            w = getattr(self.shared_layers[name], self.shared_weight_attrs[name])
            grad = getattr(w, "main_grad", None)
            grad = grad if grad is not None else w.grad
            if grad is not None:
                dist.all_reduce(grad, group=g)

    def forward(self, x, chunk_id=None):
        """Run this rank's layers (one virtual chunk when ``chunk_id`` is given)."""
        from .recompute import recompute
        fns = self.run_function if chunk_id is None else self._chunk_fns[chunk_id]
        if self.recompute_interval and self.training:
            k = self.recompute_interval
            for i in range(0, len(fns), k):
                chunk = fns[i:i + k]

                def run(inp, _c=chunk):
                    for f in _c:
                        inp = f(inp)
                    return inp
                # a chunk fed by no grad-requiring tensor (token ids into the embedding) runs
                # plainly: recompute's autograd node would cut its parameters off the graph
                x = recompute(run, x) if isinstance(x, torch.Tensor) and x.requires_grad else run(x)
            return x
        for f in fns:
            x = f(x)
        return x

    def get_stage_from_index(self, idx):
        for g in range(self.num_stages * self._num_virtual):
            if self.segment_parts[g] <= idx < self.segment_parts[g + 1]:
                return g % self.num_stages
        raise IndexError(idx)

    def get_num_virtual_stages(self):
        return self._num_virtual


def _send_meta(t, peer):
    meta = torch.tensor([t.dim(), _DT.index(t.dtype), int(t.requires_grad)] + list(t.shape) +
                        [0] * (8 - t.dim()), dtype=torch.int64, device=t.device)
    dist.send(meta, peer)


def _recv_meta(peer, device):
    meta = torch.empty(11, dtype=torch.int64, device=device)
    dist.recv(meta, peer)
    nd, dt, rg = int(meta[0]), int(meta[1]), int(meta[2])
    return [int(v) for v in meta[3:3 + nd].tolist()], _DT[dt], bool(rg)


def _p2p(send=None, send_peer=None, recv_like=None, recv_peer=None):
    """Post an optional send and an optional receive TOGETHER (batch_isend_irecv) so adjacent
    stages exchanging in opposite directions can never deadlock; returns the received tensor."""
    ops = []
    buf = None
    if send is not None:
        ops.append(dist.P2POp(dist.isend, send.detach().contiguous(), send_peer))
    if recv_like is not None:
        shape, dtype, rg, dev = recv_like
        buf = torch.empty(shape, dtype=dtype, device=dev)
        ops.append(dist.P2POp(dist.irecv, buf, recv_peer))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if buf is not None and rg and buf.is_floating_point():
        buf.requires_grad_(True)
    return buf


class PipelineParallel(torch.nn.Module):
    """1F1B pipeline executor over a :class:`PipelineLayer`."""

    def __init__(self, layers: PipelineLayer, hcg, strategy=None):
        super().__init__()
        self._layers = layers
        self.hcg = hcg
        cfg = (strategy.pipeline_configs if strategy is not None else {}) or {}
        self.accumulate_steps = int(cfg.get("accumulate_steps", 1))
        self.micro_batch_size = cfg.get("micro_batch_size", None)
        self.stage_id = hcg.get_stage_id()
        self.num_stages = hcg.get_pipe_parallel_world_size()
        self.pp_ranks = hcg.get_pipe_parallel_ranks()
        self.is_first = self.stage_id == 0
        self.is_last = self.stage_id == self.num_stages - 1
        self.prev = self.pp_ranks[self.stage_id - 1] if not self.is_first else None
        self.next = self.pp_ranks[self.stage_id + 1] if not self.is_last else None
        self.total_loss = None
        # replicas of this stage (dp / sharding axes) start from identical weights
        # (reference `pipeline_parallel.py`: broadcast_dp_parameters / broadcast_sharding_parameters)
        if dist.is_initialized():
            from . import _coalesced_broadcast
            params = list(layers.parameters())
            with torch.no_grad():
                for size, grp, src in ((hcg.get_sharding_parallel_world_size(), hcg.get_sharding_parallel_group(),
                                        hcg.get_sharding_parallel_group_src_rank),
                                       (hcg.get_data_parallel_world_size(), hcg.get_data_parallel_group(),
                                        hcg.get_data_parallel_group_src_rank)):
                    if size > 1 and grp is not None and params:
                        _coalesced_broadcast(params, src(), grp)

    def _device(self):
        for p in self._layers.parameters():
            return p.device
        return torch.device("cpu")

    def _split(self, data):
        if data is None:
            return [None] * self.accumulate_steps
        if isinstance(data, (list, tuple)):
            parts = [self._split(d) for d in data]
            return [type(data)(p[i] for p in parts) for i in range(self.accumulate_steps)]
        if data.shape[0] % self.accumulate_steps:
            raise ValueError(f"batch {data.shape[0]} does not split into accumulate_steps="
                             f"{self.accumulate_steps} equal micro-batches")
        return list(data.chunk(self.accumulate_steps, 0))

    def _forward_step(self, inp, label):
        out = self._layers(inp)
        if self.is_last:
            loss = self._layers.loss_fn(out, label) if self._layers.loss_fn is not None else out
            return loss / self.accumulate_steps
        return out

    def forward_backward_pipeline(self, data, scaler=None):
        if self._layers.get_num_virtual_stages() > 1:
            return self._interleaved(data, scaler)
        inputs, labels = (data[0], data[1]) if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None)
        mins = self._split(inputs) if self.is_first else [None] * self.accumulate_steps
        mlabs = self._split(labels) if self.is_last else [None] * self.accumulate_steps
        dev = self._device()
        n = self.accumulate_steps
        warmup = min(self.num_stages - self.stage_id - 1, n)
        steady = n - warmup
        losses = []
        pending = []  # (input, output) of micro-batches awaiting backward
        meta = {"in": None, "out": None}
        fi = [0]

        def in_spec():
            shape, dtype, rg = meta["in"]
            return (shape, dtype, rg, dev)

        def out_spec(out):
            return (list(out.shape), out.dtype, False, dev)

        def recv_forward():
            if self.is_first:
                return mins[fi[0]]
            if meta["in"] is None:
                meta["in"] = _recv_meta(self.prev, dev)
            return _p2p(recv_like=in_spec(), recv_peer=self.prev)

        def fwd(x):
            out = self._forward_step(x, mlabs[fi[0]])
            fi[0] += 1
            if self.is_last:
                losses.append(out.detach())
            elif meta["out"] is None:
                _send_meta(out, self.next)
                meta["out"] = True
            pending.append((x, out))
            return out

        def bwd(g):
            x, out = pending.pop(0)
            if self.is_last:
                (scaler.scale(out) if scaler is not None else out).backward()
            else:
                torch.autograd.backward(out, g)
            if self.is_first:
                return None
            return x.grad if x.grad is not None else torch.zeros_like(x)

        for _ in range(warmup):
            out = fwd(recv_forward())
            _p2p(send=out, send_peer=self.next)
        x = recv_forward() if steady > 0 else None
        for i in range(steady):
            out = fwd(x)
            g = None
            if not self.is_last:  # send_forward_recv_backward
                g = _p2p(send=out, send_peer=self.next, recv_like=out_spec(out), recv_peer=self.next)
            dx = bwd(g)
            if i == steady - 1:
                if dx is not None:
                    _p2p(send=dx, send_peer=self.prev)
            else:  # send_backward_recv_forward
                if self.is_first:
                    x = recv_forward()
                else:
                    x = _p2p(send=dx, send_peer=self.prev, recv_like=in_spec(), recv_peer=self.prev)
        for _ in range(warmup):
            _, out = pending[0]
            g = None if self.is_last else _p2p(recv_like=out_spec(out), recv_peer=self.next)
            dx = bwd(g)
            if dx is not None:
                _p2p(send=dx, send_peer=self.prev)
        self._layers.allreduce_shared_weight_gradients()
        loss = torch.stack(losses).sum() if self.is_last else torch.zeros((), device=dev)
        if self.num_stages > 1:  # every stage reports the last stage's loss
            loss = loss.float().reshape(1).contiguous()
            dist.broadcast(loss, self.pp_ranks[-1], group=self.hcg.get_pipe_parallel_group())
            loss = loss.reshape(())
        self.total_loss = loss
        return loss

    # ------------------------------------------------------------------ interleaved 1F1B
    def _interleaved(self, data, scaler=None):
        """Interleaved 1F1B over V virtual chunks per rank (reference
        `pipeline_parallel.py:464` PipelineParallelWithInterleave). Virtual step k of the forward
        order runs chunk ((k mod S*V) // S) on micro-batch (k // (S*V)) * S + k mod S; backward walks
        chunks in reverse. Each step posts its sends / receives as ONE batched p2p round in a fixed
        order (forward-direction ops, then backward-direction ops), so with S = 2 (next == prev)
        the two message streams between a pair can never be matched crosswise. Every chunk
        boundary tensor has the shape of stage 0's first chunk output (exchanged once)."""
        inputs, labels = (data[0], data[1]) if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None)
        S, V, r = self.num_stages, self._layers.get_num_virtual_stages(), self.stage_id
        M = self.accumulate_steps
        if M % S:
            raise ValueError(f"interleaved pipeline needs accumulate_steps ({M}) divisible by pp degree ({S})")
        total = M * V
        dev = self._device()
        mins = self._split(inputs) if r == 0 else None
        mlabs = self._split(labels) if r == S - 1 else None
        nxt, prv = self.pp_ranks[(r + 1) % S], self.pp_ranks[(r - 1) % S]
        ins = [[] for _ in range(V)]
        outs = [[] for _ in range(V)]
        ograds = [[] for _ in range(V)]
        losses = []

        def chunk_id(k, forward):
            c = (k % (S * V)) // S
            return c if forward else V - 1 - c

        def mb_id(k):
            grp, within = divmod(k, S * V)
            return grp * S + within % S

        def first(c):
            return r == 0 and c == 0

        def last(c):
            return r == S - 1 and c == V - 1

        def forward_step(k):
            c = chunk_id(k, True)
            if first(c):
                ins[c].append(mins[mb_id(k)])
            out = self._layers(ins[c][-1], chunk_id=c)
            if last(c):
                out = self._layers.loss_fn(out, mlabs[mb_id(k)]) / M if self._layers.loss_fn is not None else out
                losses.append(out.detach())
            outs[c].append(out)
            return out

        def backward_step(k):
            c = chunk_id(k, False)
            x, out = ins[c].pop(0), outs[c].pop(0)
            if last(c):
                (scaler.scale(out) if scaler is not None else out).backward()
            else:
                torch.autograd.backward(out, ograds[c].pop(0))
            if first(c):
                return None
            return x.grad if x.grad is not None else torch.zeros_like(x)

        # boundary spec: stage 0 runs virtual step 0, then the pipe group learns its output shape
        out0 = forward_step(0) if r == 0 else None
        meta = torch.zeros(11, dtype=torch.int64, device=dev)
        if r == 0:
            meta[0], meta[1] = out0.dim(), _DT.index(out0.dtype)
            meta[3:3 + out0.dim()] = torch.tensor(list(out0.shape), dtype=torch.int64)
        dist.broadcast(meta, self.pp_ranks[0], group=self.hcg.get_pipe_parallel_group())
        nd = int(meta[0])
        spec = ([int(v) for v in meta[3:3 + nd].tolist()], _DT[int(meta[1])], True, dev)

        def comm(send_fwd=None, recv_prev=False, send_bwd=None, recv_next=False):
            ops, rf, rb = [], None, None
            if send_fwd is not None:
                ops.append(dist.P2POp(dist.isend, send_fwd.detach().contiguous(), nxt))
            if recv_prev:
                rf = torch.empty(spec[0], dtype=spec[1], device=dev)
                ops.append(dist.P2POp(dist.irecv, rf, prv))
            if send_bwd is not None:
                ops.append(dist.P2POp(dist.isend, send_bwd.detach().contiguous(), prv))
            if recv_next:
                rb = torch.empty(spec[0], dtype=spec[1], device=dev)
                ops.append(dist.P2POp(dist.irecv, rb, nxt))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            if rf is not None and rf.is_floating_point():
                rf.requires_grad_(True)
            return rf, rb

        all_warmup = M == S
        warm = total if all_warmup else min((S - r - 1) * 2 + (V - 1) * S, total)
        remaining = total - warm
        if r != 0:
            ins[0].append(comm(recv_prev=True)[0])
        for k in range(warm):
            out = out0 if (k == 0 and r == 0) else forward_step(k)
            nc = chunk_id(k + 1, True)
            rp = not (r == 0 and nc == 0) and k != total - 1
            if last(chunk_id(k, True)):
                out = None
            if k == warm - 1 and not all_warmup:
                rn = r != S - 1
                xin, og = comm(send_fwd=out, recv_prev=rp, recv_next=rn)
                if rn:
                    ograds[V - 1].append(og)
            else:
                xin, _ = comm(send_fwd=out, recv_prev=rp)
            if rp:
                ins[nc].append(xin)
        for k in range(remaining):
            fk = k + warm
            out = out0 if (fk == 0 and r == 0) else forward_step(fk)
            ig = backward_step(k)
            if last(chunk_id(fk, True)):
                out = None
            if first(chunk_id(k, False)):
                ig = None
            rp = True
            if r == 0:
                nfc = chunk_id(fk - (S - 1), True)
                if nfc == V - 1:
                    rp = False
                nfc += 1
            else:
                nfc = chunk_id(fk + 1, True)
            rn = True
            if r == S - 1:
                nbc = chunk_id(k - (S - 1), False)
                if nbc == 0:
                    rn = False
                nbc -= 1
            else:
                nbc = chunk_id(k + 1, False)
            if k == remaining - 1:
                rp = False
            xin, og = comm(send_fwd=out, recv_prev=rp, send_bwd=ig, recv_next=rn)
            if rp:
                ins[nfc].append(xin)
            if rn:
                ograds[nbc].append(og)
        if all_warmup and r != S - 1:
            ograds[V - 1].append(comm(recv_next=True)[1])
        for k in range(remaining, total):
            ig = backward_step(k)
            if first(chunk_id(k, False)):
                ig = None
            nbc = chunk_id(k + 1, False)
            rn = not (r == S - 1 and nbc == V - 1) and k != total - 1
            _, og = comm(send_bwd=ig, recv_next=rn)
            if rn:
                ograds[nbc].append(og)
        self._layers.allreduce_shared_weight_gradients()
        loss = torch.stack(losses).sum() if r == S - 1 else torch.zeros((), device=dev)
        loss = loss.float().reshape(1).contiguous()
        dist.broadcast(loss, self.pp_ranks[-1], group=self.hcg.get_pipe_parallel_group())
        self.total_loss = loss.reshape(())
        return self.total_loss

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None):
        self._layers.train()
        loss = self.forward_backward_pipeline(data, scaler)
        if scaler is not None:
            scaler.minimize(optimizer, loss)
        else:
            optimizer.step()
        optimizer.clear_grad()
        if lr_scheduler is not None:
            lr_scheduler.step()
        return loss

    @torch.no_grad()
    def eval_batch(self, data, compute_loss=True):
        self._layers.eval()
        inputs, labels = (data[0], data[1]) if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None)
        mins = self._split(inputs) if self.is_first else [None] * self.accumulate_steps
        mlabs = self._split(labels) if self.is_last else [None] * self.accumulate_steps
        dev = self._device()
        outs = []
        for i in range(self.accumulate_steps):
            if self.is_first:
                x = mins[i]
            else:
                shape, dtype, _ = _recv_meta(self.prev, dev)
                x = _p2p(recv_like=(shape, dtype, False, dev), recv_peer=self.prev)
            out = self._layers(x)
            if self.is_last:
                outs.append(self._layers.loss_fn(out, mlabs[i]) if compute_loss and self._layers.loss_fn else out)
            else:
                _send_meta(out, self.next)
                _p2p(send=out, send_peer=self.next)
        return outs

    def forward(self, *args, **kwargs):
        return self._layers(*args, **kwargs)

    def parameters(self, recurse=True):
        return self._layers.parameters()


Group  # noqa
