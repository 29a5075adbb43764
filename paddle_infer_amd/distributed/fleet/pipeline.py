"""Pipeline parallelism: PipelineLayer / LayerDesc / SharedLayerDesc and the 1F1B schedule.

Parity: reference `python/paddle/distributed/fleet/meta_parallel/parallel_layers/pp_layers.py`
(LayerDesc, SharedLayerDesc, PipelineLayer with ``seg_method`` uniform / ``layer:<Name>``,
shared-weight groups) and `meta_parallel/pipeline_parallel.py` (PipelineParallel.train_batch /
eval_batch, 1F1B: warm-up forwards, steady one-forward-one-backward, cool-down backwards,
`pp_utils/p2p_communication.py`).

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
        self.segment_parts = _segment(self._descs, num_stages, seg_method)
        s, e = self.segment_parts[self.stage_id], self.segment_parts[self.stage_id + 1]
        self.run_function = []
        self.shared_layers = torch.nn.ModuleDict()
        self.shared_weight_attrs = {}
        self._stage_layers = torch.nn.ModuleList()
        for i in range(s, e):
            d = self._descs[i]
            if isinstance(d, SharedLayerDesc):
                if d.layer_name not in self.shared_layers:
                    self.shared_layers[d.layer_name] = d.build_layer()
                    self.shared_weight_attrs[d.layer_name] = d.shared_weight_attr
                lay = self.shared_layers[d.layer_name]
                if d.forward_func is not None:
                    self.run_function.append(lambda x, _l=lay, _f=d.forward_func: _f(_l, x))
                else:
                    self.run_function.append(lay)
            elif isinstance(d, LayerDesc):
                lay = d.build_layer()
                self._stage_layers.append(lay)
                self.run_function.append(lay)
            elif isinstance(d, torch.nn.Module):
                self._stage_layers.append(d)
                self.run_function.append(d)
            else:
                self.run_function.append(d)
        # shared-weight groups: all stages that hold a given shared layer
        self._shared_groups = {}
        if hcg is not None and dist.is_initialized() and num_stages > 1:
            pp_ranks = hcg.get_pipe_parallel_ranks()
            for name in sorted({d.layer_name for d in self._descs if isinstance(d, SharedLayerDesc)}):
                stages = sorted({st for st in range(num_stages)
                                 for i in range(self.segment_parts[st], self.segment_parts[st + 1])
                                 if isinstance(self._descs[i], SharedLayerDesc) and self._descs[i].layer_name == name})
                ranks = [pp_ranks[st] for st in stages]
                g = dist.new_group(ranks) if len(ranks) > 1 else None
                if name in self.shared_layers and g is not None:
                    self._shared_groups[name] = g
                    w = getattr(self.shared_layers[name], self.shared_weight_attrs[name])
                    dist.broadcast(w.data, src=ranks[0], group=g)

    def allreduce_shared_weight_gradients(self):
        for name, g in self._shared_groups.items():
            w = getattr(self.shared_layers[name], self.shared_weight_attrs[name])
            grad = getattr(w, "main_grad", None)
            grad = grad if grad is not None else w.grad
            if grad is not None:
                dist.all_reduce(grad, group=g)

    def forward(self, x):
        from .recompute import recompute
        fns = self.run_function
        if self.recompute_interval and self.training:
            k = self.recompute_interval
            for i in range(0, len(fns), k):
                chunk = fns[i:i + k]

                def run(inp, _c=chunk):
                    for f in _c:
                        inp = f(inp)
                    return inp
                x = recompute(run, x)
            return x
        for f in fns:
            x = f(x)
        return x

    def get_stage_from_index(self, idx):
        for s in range(self.num_stages):
            if self.segment_parts[s] <= idx < self.segment_parts[s + 1]:
                return s
        raise IndexError(idx)


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
        return list(data.chunk(self.accumulate_steps, 0))

    def _forward_step(self, inp, label):
        out = self._layers(inp)
        if self.is_last:
            loss = self._layers.loss_fn(out, label) if self._layers.loss_fn is not None else out
            return loss / self.accumulate_steps
        return out

    def forward_backward_pipeline(self, data, scaler=None):
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
