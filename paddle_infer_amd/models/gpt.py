"""GPT (GPT-2/3 family) with Fleet hybrid parallelism (tensor / data / sharding / pipeline).

Parity: the reference's GPT benchmarks/tests — `python/paddle/fluid/tests/unittests/
auto_parallel_gpt_model.py` (GPTModel, GPTDecoderLayer, GPTForPretraining,
GPTPretrainingCriterion) and the hybrid-parallel test models
(`hybrid_parallel_mp_model.py`, `hybrid_parallel_pp_*.py`) built on
`fleet/layers/mpu/mp_layers.py`.

MI355X-first structure of one decoder layer (pre-LN, per rank with mp degree t):
    y, h  = fused_add_ln(prev_out, h, x_bias=prev_bias, dropout)      # 1 HIP kernel
    qkv   = y @ Wqkv[h, 3h/t] + b                                       # hipBLASLt (bias epilogue)
    o     = flash_attention_packed(qkv as [B,S,3H/t,D], causal)         # HIP MFMA kernel, no transposes
    a     = o @ Wo[h/t, h]  → all-reduce over mp (RCCL/xGMI)            # bias folded into next LN
    y, h  = fused_add_ln(a, h, x_bias=bo, dropout)                      # 1 HIP kernel
    f     = gelu(y @ W1[h, 4h/t] + b1)                                   # hipBLASLt + fused bias-GELU kernel
    m     = f @ W2[4h/t, h] → all-reduce over mp                         # bias folded into next LN
Residual adds, biases of the row-parallel projections and hidden dropout all live inside the LN
kernels; LN / bias-GELU backward produce their bias gradients in the same pass.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

from ..nn.layer.base import Layer, LayerList
from ..nn import initializer as I
from ..ops import fused_add_layer_norm, flash_attention_packed, bias_act, softmax_cross_entropy
from ..ops.linear import (_use_transposed, fused_mlp, fused_mlp_supported, mm_nt, transposed,
                          wgrad_into)
from ..ops.linear import linear as _linear
from ..ops.embedding import embedding as ops_embedding
from ..distributed.fleet.mp_layers import (ColumnParallelLinear, RowParallelLinear,
                                           VocabParallelEmbedding, c_identity)


@dataclass
class GPTConfig:
    vocab_size: int = 50304
    hidden_size: int = 2048
    num_layers: int = 24
    num_heads: int = 16
    num_kv_heads: int | None = None
    ffn_hidden_size: int | None = None
    max_position_embeddings: int = 1024
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.0
    layer_norm_eps: float = 1e-5
    initializer_range: float = 0.02
    # tanh-approximate GELU like the reference GPT (auto_parallel_gpt_model.py:542,
    # F.gelu(..., approximate=True)); "gelu" selects the exact erf form
    activation: str = "gelu_tanh"
    tie_word_embeddings: bool = True
    dtype: str = "bfloat16"
    recompute: bool = False
    extra: dict = field(default_factory=dict)

    @property
    def head_dim(self):
        return self.hidden_size // self.num_heads

    @property
    def ffn(self):
        return self.ffn_hidden_size or 4 * self.hidden_size


PRESETS = {
    "gpt3-tiny": dict(vocab_size=1024, hidden_size=256, num_layers=2, num_heads=4,
                      max_position_embeddings=256),
    "gpt3-125m": dict(hidden_size=768, num_layers=12, num_heads=12),
    "gpt3-350m": dict(hidden_size=1024, num_layers=24, num_heads=16),
    "gpt3-760m": dict(hidden_size=1536, num_layers=24, num_heads=16),
    "gpt3-1.3b": dict(hidden_size=2048, num_layers=24, num_heads=16),
    "gpt3-2.7b": dict(hidden_size=2560, num_layers=32, num_heads=32),
    "gpt3-6.7b": dict(hidden_size=4096, num_layers=32, num_heads=32, max_position_embeddings=2048),
    "gpt3-13b": dict(hidden_size=5120, num_layers=40, num_heads=40, max_position_embeddings=2048),
}


def gpt_config(name: str, **over) -> GPTConfig:
    kw = dict(PRESETS[name])
    kw.update(over)
    return GPTConfig(**kw)


def _mp_size(group):
    import torch.distributed as dist
    return dist.get_world_size(group) if group is not None else 1


class GPTAttention(Layer):
    def __init__(self, cfg: GPTConfig, mp_group=None, layer_idx=0):
        super().__init__(dtype=cfg.dtype)
        t = _mp_size(mp_group)
        self.cfg = cfg
        self.heads = cfg.num_heads // t
        self.kv_heads = (cfg.num_kv_heads or cfg.num_heads) // t
        self.head_dim = cfg.head_dim
        qkv_out = (cfg.num_heads + 2 * (cfg.num_kv_heads or cfg.num_heads)) * cfg.head_dim
        std = cfg.initializer_range
        self.qkv_proj = ColumnParallelLinear(cfg.hidden_size, qkv_out, gather_output=False,
                                             mp_group=mp_group, dtype=cfg.dtype,
                                             weight_attr=I.Normal(0.0, std))
        self.out_proj = RowParallelLinear(cfg.hidden_size, cfg.hidden_size, input_is_parallel=True,
                                          mp_group=mp_group, dtype=cfg.dtype,
                                          weight_attr=I.Normal(0.0, std / math.sqrt(2 * cfg.num_layers)))
        self.mp_group = mp_group

    def forward(self, y):
        """Returns the projection output WITHOUT bias (the bias is fused into the next LN)."""
        B, S, _ = y.shape
        x = c_identity(y, self.mp_group)
        qkv = _linear(x, self.qkv_proj.weight, self.qkv_proj.bias)
        qkv = qkv.view(B, S, self.heads + 2 * self.kv_heads, self.head_dim)
        o = flash_attention_packed(qkv, self.heads, self.kv_heads, causal=True)
        o = o.reshape(B, S, self.heads * self.head_dim)
        a = _linear(o, self.out_proj.weight, None)
        from ..distributed.fleet.mp_layers import mp_allreduce
        return mp_allreduce(a, self.mp_group)


class GPTMLP(Layer):
    def __init__(self, cfg: GPTConfig, mp_group=None):
        super().__init__(dtype=cfg.dtype)
        std = cfg.initializer_range
        self.fc1 = ColumnParallelLinear(cfg.hidden_size, cfg.ffn, gather_output=False,
                                        mp_group=mp_group, dtype=cfg.dtype,
                                        weight_attr=I.Normal(0.0, std))
        self.fc2 = RowParallelLinear(cfg.ffn, cfg.hidden_size, input_is_parallel=True,
                                     mp_group=mp_group, dtype=cfg.dtype,
                                     weight_attr=I.Normal(0.0, std / math.sqrt(2 * cfg.num_layers)))
        self.act = "gelu_tanh" if cfg.activation in ("gelu_tanh", "gelu_new") else "gelu"
        self.mp_group = mp_group

    def forward(self, y):
        from ..distributed.fleet.mp_layers import mp_allreduce
        x = c_identity(y, self.mp_group)
        if fused_mlp_supported(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.act):
            # bias+GELU in the FFN1 GEMM epilogue, GELU backward in the FFN2 dgrad epilogue
            m = fused_mlp(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.act)
            return mp_allreduce(m, self.mp_group)
        f = _linear(x, self.fc1.weight, None)
        f = bias_act(f, self.fc1.bias, self.act)
        m = _linear(f, self.fc2.weight, None)
        return mp_allreduce(m, self.mp_group)


class GPTDecoderLayer(Layer):
    def __init__(self, cfg: GPTConfig, mp_group=None, layer_idx=0):
        super().__init__(dtype=cfg.dtype)
        self.cfg = cfg
        self.ln1 = _LNParams(cfg)
        self.attn = GPTAttention(cfg, mp_group, layer_idx)
        self.ln2 = _LNParams(cfg)
        self.mlp = GPTMLP(cfg, mp_group)

    def forward(self, h, prev_out, prev_bias):
        p = self.cfg.hidden_dropout_prob if self.training else 0.0
        eps = self.cfg.layer_norm_eps
        y, h = fused_add_layer_norm(prev_out, h, self.ln1.weight, self.ln1.bias, eps, prev_bias, p,
                                    self.training)
        a = self.attn(y)
        y, h = fused_add_layer_norm(a, h, self.ln2.weight, self.ln2.bias, eps,
                                    self.attn.out_proj.bias, p, self.training)
        m = self.mlp(y)
        if getattr(self, "_zero3", False):
            # ZeRO-3 frees this layer's weights after its forward: fold the row-parallel bias here
            # instead of deferring it into the NEXT layer's LN kernel (another shard unit)
            return h, m + self.mlp.fc2.bias, None
        return h, m, self.mlp.fc2.bias


class _LNParams(Layer):
    def __init__(self, cfg):
        super().__init__(dtype=cfg.dtype)
        self.weight = self.create_parameter([cfg.hidden_size], default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([cfg.hidden_size], is_bias=True)


class GPTEmbeddings(Layer):
    def __init__(self, cfg: GPTConfig, mp_group=None):
        super().__init__(dtype=cfg.dtype)
        self.word_embeddings = VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size,
                                                      weight_attr=I.Normal(0.0, cfg.initializer_range),
                                                      mp_group=mp_group, dtype=cfg.dtype)
        self.position_embeddings = self.create_parameter(
            [cfg.max_position_embeddings, cfg.hidden_size],
            default_initializer=I.Normal(0.0, cfg.initializer_range))

    def forward(self, input_ids, position_ids=None):
        S = input_ids.shape[1]
        if _mp_size(self.word_embeddings.group) == 1:
            # one fused gather+add kernel; sort-based deterministic backward into main_grad
            return ops_embedding(input_ids, self.word_embeddings.weight, 0,
                                 self.position_embeddings, position_ids)
        w = self.word_embeddings(input_ids)
        if position_ids is None:
            pe = self.position_embeddings[:S].unsqueeze(0)
        else:
            pe = F.embedding(position_ids, self.position_embeddings)
        return w + pe


class _LMHeadFn(torch.autograd.Function):
    """logits = y @ Wᵀ with W the (vocab-sharded) embedding table ``[V_local, h]``; the weight
    gradient accumulates into ``W.main_grad`` when present (shared with the embedding lookup)."""

    @staticmethod
    def forward(ctx, y, w):
        shp = y.shape
        y2 = y.reshape(-1, shp[-1])
        ctx.save_for_backward(y2, w)
        ctx.shp = shp
        return mm_nt(y2.contiguous(), w).view(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dl):
        y2, w = ctx.saved_tensors
        dl2 = dl.reshape(-1, w.shape[0])
        # dgrad on the [h, V] copy: both operands V-contiguous (the GEMMs' fast layout, ops/linear.py)
        dl2 = dl2.contiguous()
        if _use_transposed(dl2, w) or (dl2.is_cuda and dl2.dtype == w.dtype
                                       and dl2.dtype in (torch.bfloat16, torch.float16)):
            dy = mm_nt(dl2, transposed(w)).view(ctx.shp)
        else:
            dy = torch.mm(dl2, w).view(ctx.shp)
        mg = getattr(w, "main_grad", None)
        if mg is not None:
            wgrad_into(mg, dl2, y2)
            return dy, None
        return dy, wgrad_into(torch.zeros_like(w), dl2, y2)


class GPTModel(Layer):
    def __init__(self, cfg: GPTConfig, mp_group=None):
        super().__init__(dtype=cfg.dtype)
        self.cfg = cfg
        self.mp_group = mp_group
        self.embeddings = GPTEmbeddings(cfg, mp_group)
        self.layers = LayerList([GPTDecoderLayer(cfg, mp_group, i) for i in range(cfg.num_layers)])
        self.final_ln = _LNParams(cfg)

    def forward(self, input_ids, position_ids=None):
        emb = self.embeddings(input_ids, position_ids)
        p = self.cfg.hidden_dropout_prob if self.training else 0.0
        h = None  # residual stream starts empty: h0 = dropout(emb)
        out, bias = emb, None
        for layer in self.layers:
            if self.cfg.recompute and self.training:
                # fleet recompute saves / restores the kernel-dropout generator (seed, offset) as
                # well as torch's RNG, so the re-run draws the forward's dropout masks
                from ..distributed.fleet.recompute import recompute
                h, out = recompute(lambda hh, oo, bb, _l=layer: _l(hh, oo, bb)[:2], h, out, bias)
                bias = None if getattr(self, "_zero3", False) else layer.mlp.fc2.bias
            else:
                h, out, bias = layer(h, out, bias)
        y, _ = fused_add_layer_norm(out, h, self.final_ln.weight, self.final_ln.bias,
                                    self.cfg.layer_norm_eps, bias, p, self.training)
        return y


class GPTForPretraining(Layer):
    def __init__(self, cfg: GPTConfig, mp_group=None):
        super().__init__(dtype=cfg.dtype)
        self.cfg = cfg
        self.gpt = GPTModel(cfg, mp_group)
        self.mp_group = mp_group
        if not cfg.tie_word_embeddings:
            self.lm_head = self.create_parameter(
                [cfg.vocab_size // _mp_size(mp_group), cfg.hidden_size],
                default_initializer=I.Normal(0.0, cfg.initializer_range))

    @property
    def _stage3_persistent(self):
        """Modules whose weights are used outside their own forward (the tied LM head reads the word
        table): ZeRO-3 keeps them gathered for the whole step."""
        return ["gpt.embeddings.word_embeddings"] if self.cfg.tie_word_embeddings else []

    def head_weight(self):
        if self.cfg.tie_word_embeddings:
            return self.gpt.embeddings.word_embeddings.weight
        return self.lm_head

    def forward(self, input_ids, labels=None, position_ids=None, loss_mask=None):
        y = self.gpt(input_ids, position_ids)
        y = c_identity(y, self.mp_group)
        logits = _LMHeadFn.apply(y, self.head_weight())
        if labels is None:
            return logits
        group = self.mp_group if _mp_size(self.mp_group) > 1 else None
        loss = softmax_cross_entropy(logits, labels, group=group, inplace_backward=True)
        if loss_mask is not None:
            lm = loss_mask.reshape(-1).float()
            return (loss.reshape(-1) * lm).sum() / lm.sum()
        return loss.float().mean()


class GPTPretrainingCriterion(Layer):
    """Reference-API criterion: masked mean of per-token CE."""

    def __init__(self, mp_group=None):
        super().__init__()
        self.mp_group = mp_group

    def forward(self, logits, labels, loss_mask=None):
        group = self.mp_group if _mp_size(self.mp_group) > 1 else None
        loss = softmax_cross_entropy(logits, labels, group=group)
        if loss_mask is None:
            return loss.float().mean()
        lm = loss_mask.reshape(-1).float()
        return (loss.reshape(-1).float() * lm).sum() / lm.sum()


def gpt_flops_per_token(cfg: GPTConfig, seq_len: int) -> float:
    """Training FLOPs/token (fwd+bwd = 3x fwd), incl. attention scores and the LM head."""
    h, L, V = cfg.hidden_size, cfg.num_layers, cfg.vocab_size
    per_layer = 2 * (3 * h * h + h * h + 2 * h * cfg.ffn) + 2 * 2 * seq_len * h / 2  # causal attn
    return 3 * (L * per_layer + 2 * h * V)


# ---------------------------------------------------------------------------------------------
# Tensor-parallel checkpoint conversion (full <-> per-rank shards)
# ---------------------------------------------------------------------------------------------
def _qkv_cols(cfg: GPTConfig):
    hk = cfg.num_kv_heads or cfg.num_heads
    D = cfg.head_dim
    return cfg.num_heads * D, hk * D


def shard_gpt_state_dict(full: dict, cfg: GPTConfig, rank: int, world: int) -> dict:
    """Slice a full (single-device) GPT state dict into tensor-parallel rank ``rank``'s shard.
    QKV columns are regrouped per rank as [q_heads_r | k_heads_r | v_heads_r]."""
    out = {}
    qc, kc = _qkv_cols(cfg)
    for k, v in full.items():
        if k.endswith("qkv_proj.weight") or k.endswith("qkv_proj.bias"):
            q, kk, vv = v.split([qc, kc, kc], dim=-1)
            out[k] = torch.cat([t.chunk(world, dim=-1)[rank] for t in (q, kk, vv)], dim=-1).clone()
        elif k.endswith("fc1.weight") or k.endswith("fc1.bias"):
            out[k] = v.chunk(world, dim=-1)[rank].clone()
        elif k.endswith("out_proj.weight") or k.endswith("fc2.weight"):
            out[k] = v.chunk(world, dim=0)[rank].clone()
        elif k.endswith("word_embeddings.weight") or k == "lm_head":
            out[k] = v.chunk(world, dim=0)[rank].clone()
        else:
            out[k] = v.clone()
    return out


def merge_gpt_state_dicts(shards: list, cfg: GPTConfig) -> dict:
    """Inverse of :func:`shard_gpt_state_dict`."""
    world = len(shards)
    qc, kc = _qkv_cols(cfg)
    out = {}
    for k in shards[0]:
        vs = [s[k] for s in shards]
        if k.endswith("qkv_proj.weight") or k.endswith("qkv_proj.bias"):
            parts = [v.split([qc // world, kc // world, kc // world], dim=-1) for v in vs]
            out[k] = torch.cat([torch.cat([p[i] for p in parts], dim=-1) for i in range(3)], dim=-1)
        elif k.endswith("fc1.weight") or k.endswith("fc1.bias"):
            out[k] = torch.cat(vs, dim=-1)
        elif k.endswith("out_proj.weight") or k.endswith("fc2.weight") or \
                k.endswith("word_embeddings.weight") or k == "lm_head":
            out[k] = torch.cat(vs, dim=0)
        else:
            out[k] = vs[0]
    return out


# ----------------------------------------------------------------------------- pipeline form
class GPTEmbeddingPipe(GPTEmbeddings):
    """First pipeline layer: token + position embeddings. ``weight`` (the word table) is the
    SharedLayerDesc attribute tied to the LM head on the last stage."""

    @property
    def weight(self):
        return self.word_embeddings.weight

    def forward(self, input_ids, position_ids=None):
        return super().forward(input_ids, position_ids)


class GPTDecoderLayerPipe(GPTDecoderLayer):
    """Decoder layer whose input / output is ONE tensor (what a pipeline stage boundary carries):
    the embeddings [B, S, h] (first layer) or the packed residual state [2, B, S, h] = (h, out).
    The row-parallel fc2 bias, which the monolithic model folds into the NEXT layer's LN kernel, is
    added to ``out`` here — the next layer may live on another stage."""

    def forward(self, x):
        if x.dim() == 3:
            h, out = None, x
        else:
            h, out = x[0], x[1]
        h2, m, b = super().forward(h, out, None)
        return torch.stack([h2, m if b is None else m + b])


class GPTFinalNormPipe(Layer):
    def __init__(self, cfg: GPTConfig):
        super().__init__(dtype=cfg.dtype)
        self.cfg = cfg
        self.final_ln = _LNParams(cfg)

    def forward(self, x):
        p = self.cfg.hidden_dropout_prob if self.training else 0.0
        y, _ = fused_add_layer_norm(x[1], x[0], self.final_ln.weight, self.final_ln.bias,
                                    self.cfg.layer_norm_eps, None, p, self.training)
        return y


class GPTLMHeadPipe(Layer):
    """Untied LM head ([V_local, h])."""

    def __init__(self, cfg: GPTConfig, mp_group=None):
        super().__init__(dtype=cfg.dtype)
        self.mp_group = mp_group
        self.weight = self.create_parameter([cfg.vocab_size // _mp_size(mp_group), cfg.hidden_size],
                                            default_initializer=I.Normal(0.0, cfg.initializer_range))

    def forward(self, y):
        return _LMHeadFn.apply(c_identity(y, self.mp_group), self.weight)


def _tied_head(layer, y):
    return _LMHeadFn.apply(c_identity(y, layer.word_embeddings.group), layer.weight)


def gpt_pipe_descs(cfg: GPTConfig, mp_group=None):
    """LayerDesc list of GPT for PipelineLayer: shared embedding, L decoder layers, final LN and the
    (tied: SharedLayerDesc on the embedding table; untied: own weight) LM head."""
    from ..distributed.fleet.pipeline import LayerDesc, SharedLayerDesc
    descs = [SharedLayerDesc("embed", GPTEmbeddingPipe, None, "weight", cfg, mp_group)]
    descs += [LayerDesc(GPTDecoderLayerPipe, cfg, mp_group, i) for i in range(cfg.num_layers)]
    descs.append(LayerDesc(GPTFinalNormPipe, cfg))
    if cfg.tie_word_embeddings:
        descs.append(SharedLayerDesc("embed", GPTEmbeddingPipe, _tied_head, "weight", cfg, mp_group))
    else:
        descs.append(LayerDesc(GPTLMHeadPipe, cfg, mp_group))
    return descs


def GPTForPretrainingPipe(cfg: GPTConfig, mp_group=None, num_stages=None, topology=None,
                          num_virtual_pipeline_stages=None, recompute_interval=0):
    """Reference `hybrid_parallel_pp_*.py` / PaddleNLP GPTForPretrainingPipe: GPT as a
    PipelineLayer, decoder layers split evenly over ``num_stages`` x ``num_virtual_pipeline_stages``
    chunks (seg_method ``layer:GPTDecoderLayerPipe``), loss = GPTPretrainingCriterion."""
    from ..distributed.fleet.pipeline import PipelineLayer
    return PipelineLayer(gpt_pipe_descs(cfg, mp_group), num_stages=num_stages, topology=topology,
                         loss_fn=GPTPretrainingCriterion(mp_group), seg_method="layer:GPTDecoderLayerPipe",
                         recompute_interval=recompute_interval,
                         num_virtual_pipeline_stages=num_virtual_pipeline_stages)


def gpt_pipe_load_full_state(pipe, full_state: dict, cfg: GPTConfig):
    """Copy a (single-process) GPTForPretraining state dict into this rank's pipeline layers."""
    with torch.no_grad():
        for idx, lay in pipe._index_layers:
            pre = _pipe_prefix(idx, cfg)
            for n, p in lay.named_parameters():
                p.copy_(full_state["lm_head" if pre is None else pre + n])


def _pipe_prefix(idx, cfg: GPTConfig):
    L = cfg.num_layers
    if idx == 0 or (idx == L + 2 and cfg.tie_word_embeddings):
        return "gpt.embeddings."
    if idx <= L:
        return f"gpt.layers.{idx - 1}."
    if idx == L + 1:
        return "gpt."
    return None  # untied head: the "lm_head" parameter


def gpt_pipe_state_to_full(pipe, cfg: GPTConfig) -> dict:
    """This rank's pipeline parameters under their single-process GPTForPretraining names."""
    out = {}
    head = cfg.num_layers + 2
    for idx, lay in pipe._index_layers:
        pre = _pipe_prefix(idx, cfg)
        for n, p in lay.named_parameters():
            if idx == head and cfg.tie_word_embeddings and n != "word_embeddings.weight":
                continue  # the tied head uses only the word table of its embedding copy
            out["lm_head" if pre is None else pre + n] = p.detach().clone()
    return out
