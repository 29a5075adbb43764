"""Parallel-strategy planner for transformer training on MI355X nodes (``Strategy.auto_mode =
"full"``).

Parity: reference `python/paddle/distributed/auto_parallel/tuner/parallel_tuner.py` +
`cost/` (estimate every candidate's time and memory with a cost model, keep the fastest feasible
one) — re-derived here for the hardware this framework targets, with constants calibrated on our
own measurements (``profiles/``):

* compute: 6·P + 12·L·h·S FLOPs per token (+2·P with recompute) at ``sustained_tflops`` per GPU
  (GPT-3 1.3B measured 1.07 PFLOP/s model FLOPs on one MI355X, ``BENCH``), tensor parallelism
  derated by its smaller GEMMs (``tp_efficiency``);
* communication over xGMI (7 point-to-point links/GPU, ~153 GB/s each): ring all-reduce /
  reduce-scatter / all-gather at ``link_gbs × min(group − 1, 7)`` bus bandwidth; TP: 4 activation
  all-reduces per layer per micro-batch (not overlapped); DP / sharding: gradient reduce of the
  local shard, 70 % hidden under backward; stage 3 adds one parameter all-gather per pass;
  PP: 1F1B bubble (pp − 1)/(m + pp − 1) plus boundary activation sends;
* memory per GPU (288 GB HBM3E, ``mem_fraction`` usable): bf16 params 2P, fp32 master + Adam
  moments 12P, bf16 grads 2P — divided by tp·pp and, per sharding stage, by the DP degree —
  plus activations ≈30·S·b·h/tp bytes per layer and in-flight micro-batch (flash attention keeps
  no S² scores; calibrated on the measured GPT-1.3B mb64 peak; 2·S·b·h with full recompute),
  layers/pp per stage, pp micro-batches in flight (1F1B). Calibration points: GPT-3 13B on one
  GPU with recompute (model 214 GB vs measured 224 GB), GPT-3 1.3B mb64 (124 vs 125 GB).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field


@dataclass
class ModelSpec:
    layers: int
    hidden: int
    heads: int
    seq_len: int
    vocab: int
    ffn: int = 0

    @property
    def params(self):
        ffn = self.ffn or 4 * self.hidden
        per_layer = 4 * self.hidden * self.hidden + 2 * self.hidden * ffn + 13 * self.hidden
        return self.layers * per_layer + (self.vocab + self.seq_len) * self.hidden

    @classmethod
    def from_gpt_config(cls, cfg):
        return cls(cfg.num_layers, cfg.hidden_size, cfg.num_heads, cfg.max_position_embeddings,
                   cfg.vocab_size, getattr(cfg, "ffn_hidden_size", 0) or 0)


@dataclass
class ClusterSpec:
    n_gpus: int = 8
    gpus_per_node: int = 8
    hbm_gb: float = 288.0
    mem_fraction: float = 0.92
    sustained_tflops: float = 1070.0
    link_gbs: float = 153.0
    links_per_gpu: int = 7
    inter_node_gbs: float = 50.0
    tp_efficiency: dict = field(default_factory=lambda: {1: 1.0, 2: 0.93, 4: 0.86, 8: 0.78})


@dataclass
class Plan:
    dp: int
    tp: int
    pp: int
    sharding_stage: int
    micro_batch: int
    recompute: bool
    step_ms: float
    mem_gb: float
    tokens_per_s: float
    breakdown: dict

    def hybrid_configs(self):
        """fleet.DistributedStrategy().hybrid_configs for this plan."""
        return {"dp_degree": self.dp if self.sharding_stage == 0 else 1, "mp_degree": self.tp,
                "pp_degree": self.pp, "sharding_degree": self.dp if self.sharding_stage else 1}


ACT_BYTES = 30.0


def _bus_gbs(c: ClusterSpec, group: int, crosses_node: bool) -> float:
    if group <= 1:
        return float("inf")
    if crosses_node:
        return c.inter_node_gbs
    return c.link_gbs * min(group - 1, c.links_per_gpu)


def _ring_s(nbytes, group, gbs, kind="allreduce"):
    if group <= 1:
        return 0.0
    f = 2.0 * (group - 1) / group if kind == "allreduce" else (group - 1) / group
    return f * nbytes / (gbs * 1e9)


def estimate(m: ModelSpec, c: ClusterSpec, global_batch: int, dp: int, tp: int, pp: int,
             stage: int, micro: int, recompute: bool):
    """(step seconds, bytes per GPU, breakdown) of one training step, or None if the layout is
    invalid for the model (heads / layers not divisible, batch not divisible)."""
    if dp * tp * pp != c.n_gpus or m.heads % tp or m.layers % pp:
        return None
    if global_batch % dp or (global_batch // dp) % micro:
        return None
    local = global_batch // dp
    n_micro = local // micro
    if pp > 1 and n_micro < pp:
        return None
    P = m.params
    S, h, L, a = m.seq_len, m.hidden, m.layers, m.heads
    tokens = global_batch * S
    flops_tok = 6 * P + 12 * L * h * S + (2 * P if recompute else 0)
    eff = c.tp_efficiency.get(tp, 0.7)
    eff *= 0.85 + 0.15 * min(1.0, micro * S / 65536)  # small micro-batches: smaller GEMMs
    compute = tokens * flops_tok / c.n_gpus / (c.sustained_tflops * 1e12 * eff)
    bubble = compute * (pp - 1) / (n_micro + pp - 1) if pp > 1 else 0.0
    tp_node = tp <= c.gpus_per_node
    act_bytes = micro * S * h * 2
    tp_comm = 4 * (L // pp) * n_micro * _ring_s(act_bytes, tp, _bus_gbs(c, tp, not tp_node))
    pp_comm = 2 * n_micro * act_bytes / (_bus_gbs(c, 2, pp * tp > c.gpus_per_node) * 1e9) if pp > 1 else 0.0
    shard_bytes = 2 * P / (tp * pp)
    dp_cross = dp * tp * pp > c.gpus_per_node and dp > 1
    gbs = _bus_gbs(c, dp, dp_cross)
    if stage >= 2:
        dp_comm = _ring_s(shard_bytes, dp, gbs, "rs") + _ring_s(shard_bytes, dp, gbs, "ag")
    else:
        dp_comm = _ring_s(shard_bytes, dp, gbs)
    if stage == 3:
        dp_comm += 2 * _ring_s(shard_bytes, dp, gbs, "ag")
    exposed_dp = 0.3 * dp_comm
    step = compute + bubble + tp_comm + pp_comm + exposed_dp
    # memory
    local_p = P / (tp * pp)
    shard = dp if dp > 1 else 1
    weights = 2 * local_p / (shard if stage == 3 else 1)
    optim = 12 * local_p / (shard if stage >= 1 else 1)
    grads = 2 * local_p / (shard if stage >= 2 else 1)
    # flash attention (no S² scores), dropout masks regenerated, bias+act pre-activation not kept:
    # ≈30 bytes per token·hidden per layer (fits the measured 1.3B mb64 peak of 125 GB)
    per_layer_act = (2 * S * micro * h) if recompute else S * micro * h * ACT_BYTES / tp
    in_flight = min(pp, n_micro) if pp > 1 else 1
    acts = per_layer_act * (L // pp) * in_flight
    logits = micro * S * m.vocab * 2 / tp  # bf16 logits (softmax-CE fused, grad in place)
    mem = weights + optim + grads + acts + logits + 3e9  # + workspace / fragmentation
    return step, mem, {"compute_ms": compute * 1e3, "bubble_ms": bubble * 1e3,
                       "tp_comm_ms": tp_comm * 1e3, "pp_comm_ms": pp_comm * 1e3,
                       "dp_comm_exposed_ms": exposed_dp * 1e3, "weights_gb": weights / 1e9,
                       "optimizer_gb": optim / 1e9, "grads_gb": grads / 1e9,
                       "activations_gb": acts / 1e9}


def plan(model: ModelSpec, cluster: ClusterSpec | None = None, global_batch: int = None,
         micro_batches=(1, 2, 4, 8, 16, 32, 64), top_k: int = 1):
    """Fastest feasible plans (list, best first) for training ``model`` on ``cluster`` with
    ``global_batch`` sequences per step. Raises ValueError when nothing fits in memory."""
    c = cluster or ClusterSpec()
    gb = global_batch or 8 * c.n_gpus
    cands = []
    n = c.n_gpus
    for tp in (1, 2, 4, 8):
        for pp in (1, 2, 4, 8, 16):
            if n % (tp * pp):
                continue
            dp = n // (tp * pp)
            for stage, mb, rc in itertools.product((0, 1, 2, 3), micro_batches, (False, True)):
                if stage and dp == 1:
                    continue
                r = estimate(model, c, gb, dp, tp, pp, stage, mb, rc)
                if r is None:
                    continue
                step, mem, bd = r
                if mem > c.hbm_gb * 1e9 * c.mem_fraction:
                    continue
                cands.append(Plan(dp, tp, pp, stage, mb, rc, step * 1e3, mem / 1e9,
                                  gb * model.seq_len / step, bd))
    if not cands:
        raise ValueError("no parallel layout fits in memory; add GPUs or reduce the batch")
    # prefer faster; among near-ties (<1 %) prefer less memory / simpler layouts
    best = min(q.step_ms for q in cands)
    cands.sort(key=lambda p: (round(p.step_ms / best, 2), p.tp * p.pp, p.sharding_stage,
                              p.recompute, p.mem_gb))
    return cands[:top_k]


def apply_to_strategy(p: Plan, strategy, global_batch: int):
    """Write a plan into an auto_parallel ``Strategy`` (sharding / recompute / pipeline /
    gradient_merge groups) and return the fleet hybrid_configs for it."""
    strategy.sharding.enable = p.sharding_stage > 0
    strategy.sharding.stage = max(1, p.sharding_stage)
    strategy.sharding.degree = p.dp
    strategy.recompute.enable = p.recompute
    strategy.pipeline.enable = p.pp > 1
    strategy.pipeline.micro_batch_size = p.micro_batch
    local = global_batch // p.dp
    steps = max(1, local // p.micro_batch)
    strategy.pipeline.accumulate_steps = steps
    strategy.gradient_merge.enable = p.pp == 1 and steps > 1
    strategy.gradient_merge.k_steps = steps if p.pp == 1 else 1
    strategy.amp.enable = True
    strategy.amp.dtype = "bfloat16"
    strategy.plan = p
    return p.hybrid_configs()
