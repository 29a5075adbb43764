"""Expert-parallel MoE layer and gates.

Parity: reference `python/paddle/incubate/distributed/models/moe/` — MoELayer (moe_layer.py:244),
NaiveGate / GShardGate / SwitchGate (gate/*.py), ClipGradForMOEByGlobalNorm (grad_clip.py).
Dispatch/combine are `incubate/moe.py` (argsort + one variable-split RCCL all_to_all_single).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .....nn.layer.base import Layer, LayerList
from .....nn.layer.layers import Linear
from .... import moe as _moe


class BaseGate(Layer):
    def __init__(self, num_expert, world_size):
        super().__init__()
        self.world_size, self.num_expert = world_size, num_expert
        self.tot_expert = world_size * num_expert
        self.loss = None

    def set_loss(self, loss):
        self.loss = loss

    def get_loss(self, clear=True):
        loss = self.loss
        if clear:
            self.loss = None
        return loss


class NaiveGate(BaseGate):
    def __init__(self, d_model, num_expert, world_size, topk=2):
        super().__init__(num_expert, world_size)
        self.gate = Linear(d_model, self.tot_expert)
        self.top_k = topk

    def forward(self, inp, return_all_scores=False):
        g = self.gate(inp)
        val, idx = torch.topk(g, self.top_k, -1)
        return (val, idx, g) if return_all_scores else (val, idx)


class GShardGate(NaiveGate):
    def __init__(self, d_model, num_expert, world_size, topk=2, capacity=(1.2, 2.4),
                 random_routing=True, group=None):
        assert topk == 2, "topk should be 2 in gshard"
        super().__init__(d_model, num_expert, world_size)
        self.capacity, self.random_routing, self.group = capacity, random_routing, group

    def forward(self, x):
        val, idx, score = super().forward(x, return_all_scores=True)
        s = score.shape[0]
        c_e = torch.zeros(self.tot_expert, device=x.device).index_add_(
            0, idx.flatten(), torch.ones(idx.numel(), device=x.device)) / s
        m_e = F.softmax(score.float(), 1).mean(0)
        self.set_loss((c_e * m_e).mean() * self.num_expert ** 2)
        cap = math.ceil(self.capacity[0 if self.training else 1] * x.shape[0])
        idx = _moe.limit_by_capacity(idx, self.tot_expert, cap)
        if self.random_routing:
            # second expert kept with probability 2 * its (softmax-normalised) gate value
            prob = F.softmax(val.float(), -1)[:, 1]
            drop = 2 * prob < torch.rand(prob.shape, device=x.device)
            idx = idx.clone()
            idx[:, 1] = torch.where(drop, torch.full_like(idx[:, 1], -1), idx[:, 1])
        return val, idx


class SwitchGate(NaiveGate):
    def __init__(self, d_model, num_expert, world_size, topk=1, switch_eps=0.1,
                 capacity=(1.2, 2.4), group=None):
        assert topk == 1, "topk should be 1 in switch"
        super().__init__(d_model, num_expert, world_size, topk=1)
        self.switch_eps, self.capacity, self.group = switch_eps, capacity, group

    def forward(self, inp):
        score = self.gate(inp)
        if self.training:
            noise = torch.rand_like(score) * 2 * self.switch_eps + 1.0 - self.switch_eps
            score = score + noise
        score = F.softmax(score.float(), -1)
        val, idx = torch.topk(score, 1, -1)
        cap = math.ceil(self.capacity[0 if self.training else 1] * inp.shape[0])
        idx = _moe.limit_by_capacity(idx, self.tot_expert, cap)
        valid = idx[idx > -1]
        frac = torch.zeros(self.tot_expert, device=inp.device).index_add_(
            0, valid, torch.ones(valid.numel(), device=inp.device)) / max(valid.numel(), 1)
        prob = score.sum(0) / max(valid.numel(), 1)
        self.set_loss((frac * prob).sum() * self.tot_expert)
        return val, idx


class MoELayer(Layer):
    """MoELayer(d_model, experts: LayerList, gate=dict(type=naive|gshard|switch, top_k=k),
    moe_group, mp_group, recompute_interval)."""

    def __init__(self, d_model, experts, gate=None, moe_group=None, mp_group=None,
                 recompute_interval=0, recompute_ctx=None):
        super().__init__()
        gate = gate if gate is not None else {}
        self.group, self.mp_group = moe_group, mp_group
        self.world_size = _moe._ws(moe_group)
        self.experts = experts if isinstance(experts, LayerList) else LayerList(list(experts))
        self.num_expert = len(self.experts)
        self.d_model, self.recompute_interval = d_model, recompute_interval
        if isinstance(gate, dict):
            self.top_k = gate.get("top_k", 2)
            kind = gate.get("type", "gshard")
            if kind in ("naive", None):
                gate = NaiveGate(d_model, self.num_expert, self.world_size, self.top_k)
            elif kind == "gshard":
                gate = GShardGate(d_model, self.num_expert, self.world_size, self.top_k, group=moe_group)
            elif kind == "switch":
                gate = SwitchGate(d_model, self.num_expert, self.world_size, self.top_k, group=moe_group)
            else:
                raise ValueError(f"unsupported gate {kind}")
        elif isinstance(gate, NaiveGate):
            self.top_k = gate.top_k
        else:
            raise TypeError("gate must be a dict or a NaiveGate")
        self.gate = gate

    def forward(self, inp):
        assert inp.dim() == 3
        shape = inp.shape
        x = inp.reshape(-1, shape[-1])
        val, idx = self.gate(x)
        xl, counts, ctx = _moe.dispatch(x, idx, self.num_expert, self.group)
        if self.recompute_interval > 0 and torch.is_grad_enabled():
            from .....distributed.fleet.recompute import recompute
            yl = recompute(lambda t: _moe.run_experts(t, counts, self.experts), xl)
        else:
            yl = _moe.run_experts(xl, counts, self.experts)
        w = val if val.dtype == x.dtype else val.to(x.dtype)
        return _moe.combine(yl, w, ctx).reshape(shape)


class ClipGradForMOEByGlobalNorm:
    """Global-norm clip where expert parameters' squared norms are summed across the MoE group
    (reference grad_clip.py)."""

    def __init__(self, clip_norm, is_expert_param_func=None, moe_group=None, group_name="default_moe_group"):
        self.clip_norm, self.is_expert = clip_norm, is_expert_param_func
        self.moe_group = moe_group

    def __call__(self, params_grads):
        normal, expert = [], []
        for p, g in params_grads:
            if g is None:
                continue
            (expert if self.is_expert and self.is_expert(p) else normal).append(g)
        sq = sum((g.float() ** 2).sum() for g in normal) if normal else torch.zeros(())
        if expert:
            se = sum((g.float() ** 2).sum() for g in expert)
            if self.moe_group is not None and _moe._ws(self.moe_group) > 1:
                torch.distributed.all_reduce(se, group=_moe._pg(self.moe_group))
            sq = sq + se
        norm = torch.sqrt(sq)
        coef = torch.clamp(self.clip_norm / (norm + 1e-6), max=1.0)
        return [(p, g * coef.to(g.dtype) if g is not None else None) for p, g in params_grads]


__all__ = ["MoELayer", "NaiveGate", "GShardGate", "SwitchGate", "BaseGate", "ClipGradForMOEByGlobalNorm"]
