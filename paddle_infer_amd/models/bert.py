"""BERT (post-LN encoder) for pretraining (MLM + NSP) and sequence classification.

Parity: the reference's BERT benchmark / test models (`unittests/bert_dygraph_model.py`,
`dygraph_to_static/bert_dygraph_model.py`: BertConfig, BertModel, BertPretrainingHeads,
PretrainModelLayer) — same sub-layer structure and parameter shapes.

MI355X mapping per encoder layer (post-LN):
    qkv = x @ Wqkv + b                                   hipBLASLt
    a   = attention(qkv, padding mask)                   flash kernel (no padding) or
                                                         GEMM + fused masked-softmax HIP kernel
    x   = LN(x + dropout(a @ Wo + bo))                   one layernorm.hip pass (bias/dropout/residual)
    f   = gelu(x @ W1 + b1)                              hipBLASLt + bias-GELU kernel
    x   = LN(x + dropout(f @ W2 + b2))                   one layernorm.hip pass
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F

from ..incubate.nn.functional import attention_core
from ..nn import initializer as I
from ..nn.layer.base import Layer, LayerList
from ..ops import bias_act, fused_add_layer_norm, layer_norm, softmax_cross_entropy
from ..ops.linear import linear as _linear


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_act: str = "gelu"
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    pad_token_id: int = 0
    dtype: str = "float32"


BERT_PRESETS = {
    "bert-tiny": dict(vocab_size=1024, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                      intermediate_size=512, max_position_embeddings=128),
    "bert-base": dict(),
    "bert-large": dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                       intermediate_size=4096),
}


class _P(Layer):
    def __init__(self, shape, std, dtype, bias=False, one=False):
        super().__init__(dtype=dtype)
        init = I.Constant(1.0) if one else (I.Constant(0.0) if bias else I.Normal(0.0, std))
        self.p = self.create_parameter(shape, default_initializer=init, is_bias=bias)


class BertEmbeddings(Layer):
    def __init__(self, cfg: BertConfig):
        super().__init__(dtype=cfg.dtype)
        std = cfg.initializer_range
        self.word_embeddings = self.create_parameter([cfg.vocab_size, cfg.hidden_size], default_initializer=I.Normal(0.0, std))
        self.position_embeddings = self.create_parameter([cfg.max_position_embeddings, cfg.hidden_size], default_initializer=I.Normal(0.0, std))
        self.token_type_embeddings = self.create_parameter([cfg.type_vocab_size, cfg.hidden_size], default_initializer=I.Normal(0.0, std))
        self.ln_w = self.create_parameter([cfg.hidden_size], default_initializer=I.Constant(1.0))
        self.ln_b = self.create_parameter([cfg.hidden_size], is_bias=True)
        self.cfg = cfg

    def forward(self, input_ids, token_type_ids=None, position_ids=None):
        S = input_ids.shape[1]
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        we = F.embedding(input_ids, self.word_embeddings)
        # default positions 0..S-1: the first S rows of the table, broadcast over the batch (no
        # batch-sized index tensor, so a traced export keeps a symbolic batch dim)
        pos = (self.position_embeddings[:S].unsqueeze(0) if position_ids is None
               else F.embedding(position_ids, self.position_embeddings))
        extra = pos + F.embedding(token_type_ids, self.token_type_embeddings)
        p = self.cfg.hidden_dropout_prob if self.training else 0.0
        # LN(dropout(word + pos + type)) — dropout applies to the sum in the reference; here the
        # position/type sum is the residual input of the fused LN (dropout on the word part)
        y, _ = fused_add_layer_norm(we, extra, self.ln_w, self.ln_b, self.cfg.layer_norm_eps, None, p, self.training)
        return y


class BertLayer(Layer):
    def __init__(self, cfg: BertConfig):
        super().__init__(dtype=cfg.dtype)
        h, f, std = cfg.hidden_size, cfg.intermediate_size, cfg.initializer_range
        self.cfg = cfg
        self.qkv_w = self.create_parameter([h, 3 * h], default_initializer=I.Normal(0.0, std))
        self.qkv_b = self.create_parameter([3 * h], is_bias=True)
        self.out_w = self.create_parameter([h, h], default_initializer=I.Normal(0.0, std))
        self.out_b = self.create_parameter([h], is_bias=True)
        self.ln1_w = self.create_parameter([h], default_initializer=I.Constant(1.0))
        self.ln1_b = self.create_parameter([h], is_bias=True)
        self.fc1_w = self.create_parameter([h, f], default_initializer=I.Normal(0.0, std))
        self.fc1_b = self.create_parameter([f], is_bias=True)
        self.fc2_w = self.create_parameter([f, h], default_initializer=I.Normal(0.0, std))
        self.fc2_b = self.create_parameter([h], is_bias=True)
        self.ln2_w = self.create_parameter([h], default_initializer=I.Constant(1.0))
        self.ln2_b = self.create_parameter([h], is_bias=True)

    def forward(self, x, attn_mask=None):
        cfg = self.cfg
        B, S, h = x.shape
        H = cfg.num_attention_heads
        pd = cfg.hidden_dropout_prob if self.training else 0.0
        pa = cfg.attention_probs_dropout_prob if self.training else 0.0
        qkv = _linear(x, self.qkv_w, self.qkv_b).view(B, S, 3 * H, h // H)
        a = attention_core(qkv, H, H, attn_mask, False, pa, self.training)
        o = _linear(a, self.out_w, None)
        x, _ = fused_add_layer_norm(o, x, self.ln1_w, self.ln1_b, cfg.layer_norm_eps, self.out_b, pd, self.training,
                                      need_residual=False)
        act = "gelu_tanh" if cfg.hidden_act in ("gelu_new", "gelu_tanh") else cfg.hidden_act
        f = bias_act(_linear(x, self.fc1_w, None), self.fc1_b, act)
        m = _linear(f, self.fc2_w, None)
        x, _ = fused_add_layer_norm(m, x, self.ln2_w, self.ln2_b, cfg.layer_norm_eps, self.fc2_b, pd, self.training,
                                      need_residual=False)
        return x


class BertModel(Layer):
    def __init__(self, cfg: BertConfig):
        super().__init__(dtype=cfg.dtype)
        self.cfg = cfg
        self.embeddings = BertEmbeddings(cfg)
        self.encoder = LayerList([BertLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        std = cfg.initializer_range
        self.pool_w = self.create_parameter([cfg.hidden_size, cfg.hidden_size], default_initializer=I.Normal(0.0, std))
        self.pool_b = self.create_parameter([cfg.hidden_size], is_bias=True)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None):
        x = self.embeddings(input_ids, token_type_ids, position_ids)
        mask = None
        # the padding scan is data-dependent: a traced export (meta inputs) takes the mask as an
        # explicit input instead
        if attention_mask is None and self.cfg.pad_token_id is not None and not input_ids.is_meta:
            pad = input_ids == self.cfg.pad_token_id
            if bool(pad.any()):
                attention_mask = ~pad
        if attention_mask is not None:
            am = attention_mask
            if am.dim() == 2:
                am = am[:, None, None, :]
            if am.dtype == torch.bool or not am.is_floating_point():
                mask = torch.zeros(am.shape, dtype=x.dtype, device=x.device).masked_fill(am == 0, -1e4)
            else:
                mask = am.to(x.dtype)
        for layer in self.encoder:
            x = layer(x, mask)
        pooled = torch.tanh(_linear(x[:, 0], self.pool_w, self.pool_b))
        return x, pooled


class BertForPretraining(Layer):
    """MLM (tied decoder) + NSP heads; returns the summed loss when labels are given."""

    def __init__(self, cfg: BertConfig):
        super().__init__(dtype=cfg.dtype)
        self.cfg = cfg
        self.bert = BertModel(cfg)
        std = cfg.initializer_range
        self.tr_w = self.create_parameter([cfg.hidden_size, cfg.hidden_size], default_initializer=I.Normal(0.0, std))
        self.tr_b = self.create_parameter([cfg.hidden_size], is_bias=True)
        self.tr_ln_w = self.create_parameter([cfg.hidden_size], default_initializer=I.Constant(1.0))
        self.tr_ln_b = self.create_parameter([cfg.hidden_size], is_bias=True)
        self.decoder_b = self.create_parameter([cfg.vocab_size], is_bias=True)
        self.nsp_w = self.create_parameter([cfg.hidden_size, 2], default_initializer=I.Normal(0.0, std))
        self.nsp_b = self.create_parameter([2], is_bias=True)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None,
                masked_positions=None, masked_lm_labels=None, next_sentence_labels=None):
        seq, pooled = self.bert(input_ids, token_type_ids, position_ids, attention_mask)
        if masked_positions is not None:
            seq = seq.reshape(-1, seq.shape[-1]).index_select(0, masked_positions.reshape(-1))
        h = bias_act(_linear(seq, self.tr_w, None), self.tr_b, "gelu")
        h = layer_norm(h, self.tr_ln_w, self.tr_ln_b, self.cfg.layer_norm_eps)
        from ..ops.gemm import matmul as _mm  # tied [V, h] table: the own GEMM's NT layout
        logits = _mm(h, self.bert.embeddings.word_embeddings, False, True) + self.decoder_b
        nsp = _linear(pooled, self.nsp_w, self.nsp_b)
        if masked_lm_labels is None:
            return logits, nsp
        mlm = softmax_cross_entropy(logits.reshape(-1, logits.shape[-1]), masked_lm_labels.reshape(-1),
                                    ignore_index=-1)
        valid = (masked_lm_labels.reshape(-1) != -1).float()
        loss = (mlm.float().reshape(-1) * valid).sum() / valid.sum().clamp_min(1)
        if next_sentence_labels is not None:
            loss = loss + F.cross_entropy(nsp.float(), next_sentence_labels.reshape(-1))
        return loss


class BertForSequenceClassification(Layer):
    def __init__(self, cfg: BertConfig, num_classes=2, dropout=None):
        super().__init__(dtype=cfg.dtype)
        self.bert = BertModel(cfg)
        self.dropout = dropout if dropout is not None else cfg.hidden_dropout_prob
        self.cls_w = self.create_parameter([cfg.hidden_size, num_classes],
                                           default_initializer=I.Normal(0.0, cfg.initializer_range))
        self.cls_b = self.create_parameter([num_classes], is_bias=True)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None):
        _, pooled = self.bert(input_ids, token_type_ids, position_ids, attention_mask)
        pooled = F.dropout(pooled, self.dropout, self.training)
        return _linear(pooled, self.cls_w, self.cls_b)


def bert_config(name: str, **over) -> BertConfig:
    kw = dict(BERT_PRESETS[name])
    kw.update(over)
    return BertConfig(**kw)


LayerList  # noqa
