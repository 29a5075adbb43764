"""Fused transformer layers (``paddle.incubate.nn``).

Parity: reference `python/paddle/incubate/nn/layer/fused_transformer.py` —
FusedBiasDropoutResidualLayerNorm:87, FusedMultiHeadAttention:197, FusedFeedForward:490,
FusedTransformerEncoderLayer:721, FusedMultiTransformer:1017,
FusedMultiTransformerWeightOnly:1465, FusedMultiTransformerINT8:1808, FusedMoELayer:2110,
FusedMultiTransformerMoe:2278 (+ weight-only MoE :3107) and `fused_linear.py` (FusedLinear).
Parameter names, shapes and dtypes follow the reference so its state dicts load unchanged
(ln scales f32, weights in the layer dtype; weight-only weights int8 [N, K] / int4 [N/2, K] in
the MI355X MFMA-tile byte order produced by ``nn.quant.weight_quantize``).
"""
from __future__ import annotations

import torch

from ....framework.dtype import to_torch_dtype
from ....nn.initializer import Constant
from ....nn.layer.base import Layer, ParameterList
from .. import functional as incubate_f
from ..functional import _lin


def _attr(attrs, i, n):
    if isinstance(attrs, (list, tuple, ParameterList)):
        assert len(attrs) == n
        return attrs[i]
    return attrs


class FusedLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None,
                 transpose_weight=False, name=None):
        super().__init__()
        shape = [out_features, in_features] if transpose_weight else [in_features, out_features]
        self.weight = self.create_parameter(shape, weight_attr, self._dtype, False)
        self.bias = self.create_parameter([out_features], bias_attr, self._dtype, True)
        self.transpose_weight = transpose_weight

    def forward(self, x):
        return incubate_f.fused_linear(x, self.weight, self.bias, self.transpose_weight)


class FusedBiasDropoutResidualLayerNorm(Layer):
    def __init__(self, embed_dim, dropout_rate=0.5, weight_attr=None, bias_attr=None,
                 epsilon=1e-5, name=None):
        super().__init__()
        self.embed_dim = embed_dim
        self.linear_bias = self.create_parameter([embed_dim], bias_attr, self._dtype, True)
        self.ln_scale = self.create_parameter([embed_dim], weight_attr, torch.float32, False,
                                              Constant(1.0))
        self.ln_bias = self.create_parameter([embed_dim], bias_attr, torch.float32, True)
        self.dropout_rate, self._epsilon = dropout_rate, epsilon

    def forward(self, x, residual):
        return incubate_f.fused_bias_dropout_residual_layer_norm(
            x, residual, self.linear_bias, self.ln_scale.to(x.dtype), self.ln_bias.to(x.dtype),
            self.dropout_rate, self._epsilon, self.training)


class FusedMultiHeadAttention(Layer):
    def __init__(self, embed_dim, num_heads, dropout_rate=0.5, attn_dropout_rate=0.5, kdim=None,
                 vdim=None, normalize_before=False, need_weights=False, qkv_weight_attr=None,
                 qkv_bias_attr=None, linear_weight_attr=None, linear_bias_attr=None,
                 pre_ln_scale_attr=None, pre_ln_bias_attr=None, ln_scale_attr=None,
                 ln_bias_attr=None, epsilon=1e-5, nranks=1, ring_id=-1, transpose_qkv_wb=False,
                 name=None):
        super().__init__()
        assert embed_dim % num_heads == 0
        self.normalize_before, self.embed_dim, self.num_heads = normalize_before, embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.dropout_rate, self.attn_dropout_rate, self._epsilon = dropout_rate, attn_dropout_rate, epsilon
        self.transpose_qkv_wb = transpose_qkv_wb
        nh = num_heads // nranks
        qshape = [embed_dim, 3 * nh * self.head_dim] if transpose_qkv_wb else [3, nh, self.head_dim, embed_dim]
        self.qkv_weight = self.create_parameter(qshape, qkv_weight_attr, self._dtype, False)
        self.qkv_bias = self.create_parameter(
            [3 * nh * self.head_dim] if transpose_qkv_wb else [3, nh, self.head_dim], qkv_bias_attr,
            self._dtype, True)
        self.linear_weight = self.create_parameter([nh * self.head_dim, embed_dim], linear_weight_attr,
                                                   self._dtype, False)
        self.linear_bias = self.create_parameter([embed_dim], linear_bias_attr, self._dtype, True)
        if normalize_before:
            self.pre_ln_scale = self.create_parameter([embed_dim], pre_ln_scale_attr, torch.float32,
                                                      False, Constant(1.0))
            self.pre_ln_bias = self.create_parameter([embed_dim], pre_ln_bias_attr, torch.float32, True)
            self.ln_scale = self.ln_bias = None
        else:
            self.pre_ln_scale = self.pre_ln_bias = None
            self.ln_scale = self.create_parameter([embed_dim], ln_scale_attr, torch.float32, False,
                                                  Constant(1.0))
            self.ln_bias = self.create_parameter([embed_dim], ln_bias_attr, torch.float32, True)
        self._group = None

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        cast = (lambda t: None if t is None else t.to(query.dtype))
        return incubate_f.fused_multi_head_attention(
            query, self.qkv_weight, self.linear_weight, self.normalize_before,
            cast(self.pre_ln_scale), cast(self.pre_ln_bias), cast(self.ln_scale), cast(self.ln_bias),
            self._epsilon, self.qkv_bias, self.linear_bias, cache, attn_mask, self.dropout_rate,
            self.attn_dropout_rate, None, None, self._epsilon, self.training,
            group=self._group, transpose_qkv_wb=self.transpose_qkv_wb, num_heads=self.num_heads)


class FusedFeedForward(Layer):
    def __init__(self, d_model, dim_feedforward, dropout_rate=0.1, epsilon=1e-05,
                 activation="relu", act_dropout_rate=None, normalize_before=False,
                 linear1_weight_attr=None, linear1_bias_attr=None, linear2_weight_attr=None,
                 linear2_bias_attr=None, ln1_scale_attr=None, ln1_bias_attr=None,
                 ln2_scale_attr=None, ln2_bias_attr=None, nranks=1, ring_id=-1, name=None):
        super().__init__()
        self._d_model, self._dim_feedforward = d_model, dim_feedforward
        self._dropout_rate = dropout_rate
        self._act_dropout_rate = dropout_rate if act_dropout_rate is None else act_dropout_rate
        self._act_method, self._normalize_before, self._epsilon = activation, normalize_before, epsilon
        ff = dim_feedforward // nranks
        self._linear1_weight = self.create_parameter([d_model, ff], linear1_weight_attr, self._dtype, False)
        self._linear1_bias = self.create_parameter([ff], linear1_bias_attr, self._dtype, True)
        self._linear2_weight = self.create_parameter([ff, d_model], linear2_weight_attr, self._dtype, False)
        self._linear2_bias = self.create_parameter([d_model], linear2_bias_attr, self._dtype, True)
        if normalize_before:
            self._ln1_scale = self.create_parameter([d_model], ln1_scale_attr, torch.float32, False, Constant(1.0))
            self._ln1_bias = self.create_parameter([d_model], ln1_bias_attr, torch.float32, True)
            self._ln2_scale = self._ln2_bias = None
        else:
            self._ln1_scale = self._ln1_bias = None
            self._ln2_scale = self.create_parameter([d_model], ln2_scale_attr, torch.float32, False, Constant(1.0))
            self._ln2_bias = self.create_parameter([d_model], ln2_bias_attr, torch.float32, True)
        self._group = None

    def forward(self, src, cache=None):
        cast = (lambda t: None if t is None else t.to(src.dtype))
        return incubate_f.fused_feedforward(
            src, self._linear1_weight, self._linear2_weight, self._linear1_bias, self._linear2_bias,
            cast(self._ln1_scale), cast(self._ln1_bias), cast(self._ln2_scale), cast(self._ln2_bias),
            self._act_dropout_rate, self._dropout_rate, None, self._act_method, self._epsilon,
            self._epsilon, self._normalize_before, self.training, group=self._group)


class FusedTransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout_rate=0.1, activation="relu",
                 attn_dropout_rate=None, act_dropout_rate=None, normalize_before=False,
                 weight_attr=None, bias_attr=None):
        super().__init__()
        attn_dropout_rate = dropout_rate if attn_dropout_rate is None else attn_dropout_rate
        act_dropout_rate = dropout_rate if act_dropout_rate is None else act_dropout_rate
        self.normalize_before = normalize_before
        self.fused_attn = FusedMultiHeadAttention(d_model, nhead, dropout_rate, attn_dropout_rate,
                                                  normalize_before=normalize_before)
        self.ffn = FusedFeedForward(d_model, dim_feedforward, dropout_rate, activation=activation,
                                    act_dropout_rate=act_dropout_rate,
                                    normalize_before=normalize_before)

    def forward(self, src, src_mask=None, cache=None):
        if cache is None:
            return self.ffn(self.fused_attn(src, attn_mask=src_mask))
        out, new_cache = self.fused_attn(src, attn_mask=src_mask, cache=cache)
        return self.ffn(out), new_cache


class FusedTransformer(Layer):
    """Reference `fused_transformer.py:899` — encoder/decoder stack of fused layers (decoder
    cross-attention runs through nn.MultiHeadAttention)."""

    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6,
                 dim_feedforward=2048, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None,
                 custom_encoder=None, custom_decoder=None):
        super().__init__()
        from ....nn import LayerList, TransformerDecoder, TransformerDecoderLayer
        self.encoder = custom_encoder or LayerList([
            FusedTransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation,
                                         attn_dropout, act_dropout, normalize_before)
            for _ in range(num_encoder_layers)])
        self.decoder = custom_decoder or TransformerDecoder(
            TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout, activation,
                                    attn_dropout, act_dropout, normalize_before), num_decoder_layers)

    def forward(self, src, tgt, src_mask=None, tgt_mask=None, memory_mask=None):
        mem = src
        for layer in self.encoder:
            mem = layer(mem, src_mask)
        return self.decoder(tgt, mem, tgt_mask, memory_mask)


# ----------------------------------------------------------------------------- multi-transformer
class _MultiTransformerBase(Layer):
    """Shared parameter construction of the FusedMultiTransformer family."""

    def _common_init(self, embed_dim, num_heads, dim_feedforward, dropout_rate, activation,
                     normalize_before, epsilon, num_layers, nranks, ring_id, num_kv_heads,
                     rotary_emb_dims, use_neox_rotary_style, rope_base, attrs):
        assert embed_dim > 0 and num_heads > 0 and dim_feedforward > 0
        assert embed_dim % num_heads == 0, "embed_dim must be divisible by num_heads"
        self.normalize_before, self._epsilon = normalize_before, epsilon
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.num_kv_heads = num_kv_heads or num_heads
        assert num_heads % nranks == 0 and dim_feedforward % nranks == 0 and self.num_kv_heads % nranks == 0
        self._nh, self._nkv = num_heads // nranks, self.num_kv_heads // nranks
        self._dim_feedforward = dim_feedforward // nranks
        self.dropout_rate, self.activation = dropout_rate, activation
        self._ring_id, self._group = ring_id, None
        self.rotary_emb_dims, self.use_neox_rotary_style, self.rope_base = \
            rotary_emb_dims, use_neox_rotary_style, rope_base
        qkv_attrs = attrs.get("qkv_weight_attrs")
        if isinstance(qkv_attrs, (list, tuple, ParameterList)):
            num_layers = len(qkv_attrs)
        assert num_layers > 0
        self.num_layers = num_layers
        for nm in ("ln_scales", "ln_biases", "qkv_weights", "qkv_biases", "linear_weights",
                   "linear_biases", "ffn_ln_scales", "ffn_ln_biases", "ffn1_weights", "ffn1_biases",
                   "ffn2_weights", "ffn2_biases"):
            setattr(self, nm, ParameterList())
        return num_layers

    def _ln_params(self, i, attrs, n):
        E = self.embed_dim
        self.ln_scales.append(self.create_parameter([E], _attr(attrs.get("ln_scale_attrs"), i, n),
                                                    torch.float32, False, Constant(1.0)))
        self.ln_biases.append(self.create_parameter([E], _attr(attrs.get("ln_bias_attrs"), i, n),
                                                    torch.float32, True))
        self.ffn_ln_scales.append(self.create_parameter(
            [E], _attr(attrs.get("ffn_ln_scale_attrs"), i, n), torch.float32, False, Constant(1.0)))
        self.ffn_ln_biases.append(self.create_parameter(
            [E], _attr(attrs.get("ffn_ln_bias_attrs"), i, n), torch.float32, True))

    def _cast_ln(self, dtype):
        c = getattr(self, "_ln_cache", None)
        if c is None or c[0] != dtype:
            self._ln_cache = c = (dtype, [
                tuple(None if p is None else p.detach().to(dtype) for p in ps)
                for ps in zip(self.ln_scales, self.ln_biases, self.ffn_ln_scales, self.ffn_ln_biases)])
        return c[1]

    def _layers(self, dtype):
        raise NotImplementedError

    def layer_specs(self, dtype):
        return self._layers(dtype)

    def forward(self, src, attn_mask=None, caches=None, seq_lens=None, beam_offset=None,
                time_step=None, causal=False):
        """caches: per layer [2, B, Hk, max_seq_len, D] (updated in place). Returns out, or
        (out, caches) when caches are given — the reference's contract."""
        if caches is not None:
            assert len(caches) == self.num_layers
        B, S, _ = src.shape
        decode = time_step is not None
        if beam_offset is not None and caches is not None:
            srcb = beam_offset.reshape(-1)[:B].long().to(src.device)
            for c in caches:
                c.copy_(c.index_select(1, srcb))
        pos, lens = incubate_f._positions(B, time_step, seq_lens, S, src.device, decode)
        with torch.no_grad():
            out = incubate_f.multi_transformer_forward(
                src, self._layers(src.dtype), self._nh, self._nkv, self.normalize_before,
                self._epsilon, incubate_f._caches_from(caches), pos, lens, attn_mask, decode,
                self.activation, self.rotary_emb_dims, self.use_neox_rotary_style, self.rope_base,
                causal=causal and attn_mask is None, group=self._group)
        return (out, caches) if caches is not None else out

    def gen_cache(self, batch_size, max_seq_len, dtype=None, device=None):
        """Allocate per-layer KV caches [2, B, Hk, max_seq_len, D] (HBM-resident)."""
        dt = to_torch_dtype(dtype) if dtype is not None else self.ln_biases[0].dtype \
            if self.qkv_weights[0].dtype in (torch.int8, torch.uint8) else self.qkv_weights[0].dtype
        dev = device or self.ln_scales[0].device
        return [torch.zeros(2, batch_size, self._nkv, max_seq_len, self.head_dim, dtype=dt, device=dev)
                for _ in range(self.num_layers)]


class FusedMultiTransformer(_MultiTransformerBase):
    """Reference `fused_transformer.py:1017`. Extensions (MI355X serving): ``num_kv_heads``
    (GQA), ``rotary_emb_dims`` / ``use_neox_rotary_style`` / ``rope_base`` (RoPE fused into the
    QKV prologue), activation ``swiglu``/``geglu`` (ffn1 produces [gate | up])."""

    def __init__(self, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0, activation="gelu",
                 normalize_before=True, ln_scale_attrs=None, ln_bias_attrs=None,
                 qkv_weight_attrs=None, qkv_bias_attrs=None, linear_weight_attrs=None,
                 linear_bias_attrs=None, ffn_ln_scale_attrs=None, ffn_ln_bias_attrs=None,
                 ffn1_weight_attrs=None, ffn1_bias_attrs=None, ffn2_weight_attrs=None,
                 ffn2_bias_attrs=None, epsilon=1e-5, num_layers=-1, nranks=1, trans_qkvw=True,
                 ring_id=-1, name=None, dy_to_st=False, num_kv_heads=None, rotary_emb_dims=0,
                 use_neox_rotary_style=True, rope_base=10000.0):
        super().__init__()
        attrs = dict(locals())
        n = self._common_init(embed_dim, num_heads, dim_feedforward, dropout_rate, activation,
                              normalize_before, epsilon, num_layers, nranks, ring_id, num_kv_heads,
                              rotary_emb_dims, use_neox_rotary_style, rope_base, attrs)
        self._trans_qkvw = trans_qkvw
        E, D, nh, nkv, F = embed_dim, self.head_dim, self._nh, self._nkv, self._dim_feedforward
        F1 = 2 * F if activation in ("swiglu", "geglu") else F
        dt = self._dtype
        for i in range(n):
            self._ln_params(i, attrs, n)
            if nkv == nh:
                qshape = [3, nh, D, E] if trans_qkvw else [E, 3, nh, D]
                bshape = [3, nh, D]
            else:
                qshape = [nh + 2 * nkv, D, E] if trans_qkvw else [E, nh + 2 * nkv, D]
                bshape = [nh + 2 * nkv, D]
            self.qkv_weights.append(self.create_parameter(qshape, _attr(qkv_weight_attrs, i, n), dt))
            self.qkv_biases.append(self.create_parameter(bshape, _attr(qkv_bias_attrs, i, n), dt, True))
            self.linear_weights.append(self.create_parameter([nh * D, E], _attr(linear_weight_attrs, i, n), dt))
            self.linear_biases.append(self.create_parameter([E], _attr(linear_bias_attrs, i, n), dt, True))
            self.ffn1_weights.append(self.create_parameter([E, F1], _attr(ffn1_weight_attrs, i, n), dt))
            self.ffn1_biases.append(self.create_parameter([F1], _attr(ffn1_bias_attrs, i, n), dt, True))
            self.ffn2_weights.append(self.create_parameter([F, E], _attr(ffn2_weight_attrs, i, n), dt))
            self.ffn2_biases.append(self.create_parameter([E], _attr(ffn2_bias_attrs, i, n), dt, True))
        self.name = name

    def _layers(self, dtype):
        lns = self._cast_ln(dtype)
        out = []
        for i in range(self.num_layers):
            qb = self.qkv_biases[i]
            out.append(dict(
                head_dim=self.head_dim, ln_scale=lns[i][0], ln_bias=lns[i][1],
                qkv=incubate_f._qkv_linear(self.qkv_weights[i], self._trans_qkvw),
                qkv_bias=None if qb is None else qb.reshape(-1),
                out=_lin(self.linear_weights[i]), out_bias=self.linear_biases[i],
                ffn_ln_scale=lns[i][2], ffn_ln_bias=lns[i][3],
                ffn1=_lin(self.ffn1_weights[i]), ffn1_bias=self.ffn1_biases[i],
                ffn2=_lin(self.ffn2_weights[i]), ffn2_bias=self.ffn2_biases[i]))
        return out

    def _amp_decorate(self, dtype):
        dt = to_torch_dtype(dtype)
        with torch.no_grad():
            for pl in (self.qkv_weights, self.qkv_biases, self.linear_weights, self.linear_biases,
                       self.ffn1_weights, self.ffn1_biases, self.ffn2_weights, self.ffn2_biases):
                for p in pl:
                    if p is not None:
                        p.data = p.data.to(dt)
        self._dtype = dt


class FusedMultiTransformerWeightOnly(_MultiTransformerBase):
    """Reference `fused_transformer.py:1465`: int8 / int4 weight-only projections. Weights are
    [N, K] (int8) or [N/2, K] (int4) packed bytes with per-output-channel scales; use
    :meth:`from_float` (or ``nn.quant.weight_quantize``) to fill them."""

    def __init__(self, embed_dim, num_heads, dim_feedforward, weight_dtype="int8",
                 dropout_rate=0.0, activation="gelu", normalize_before=True, ln_scale_attrs=None,
                 ln_bias_attrs=None, qkv_weight_attrs=None, qkv_scale_attrs=None,
                 qkv_bias_attrs=None, linear_weight_attrs=None, linear_scale_attrs=None,
                 linear_bias_attrs=None, ffn_ln_scale_attrs=None, ffn_ln_bias_attrs=None,
                 ffn1_weight_attrs=None, ffn1_scale_attrs=None, ffn1_bias_attrs=None,
                 ffn2_weight_attrs=None, ffn2_scale_attrs=None, ffn2_bias_attrs=None,
                 epsilon=1e-5, num_layers=-1, nranks=1, trans_qkvw=True, ring_id=-1, name=None,
                 num_kv_heads=None, rotary_emb_dims=0, use_neox_rotary_style=True,
                 rope_base=10000.0, dtype="bfloat16"):
        super().__init__(dtype=dtype)
        attrs = dict(locals())
        n = self._common_init(embed_dim, num_heads, dim_feedforward, dropout_rate, activation,
                              normalize_before, epsilon, num_layers, nranks, ring_id, num_kv_heads,
                              rotary_emb_dims, use_neox_rotary_style, rope_base, attrs)
        self._weight_dtype = weight_dtype
        self._bits = 4 if weight_dtype == "int4" else 8
        div = 2 if self._bits == 4 else 1
        E, D, nh, nkv, F = embed_dim, self.head_dim, self._nh, self._nkv, self._dim_feedforward
        F1 = 2 * F if activation in ("swiglu", "geglu") else F
        NQ = (nh + 2 * nkv) * D
        dt = self._dtype
        for nm in ("qkv_scales", "linear_scales", "ffn1_scales", "ffn2_scales"):
            setattr(self, nm, ParameterList())
        u8, one = torch.uint8, Constant(1.0)
        for i in range(n):
            self._ln_params(i, attrs, n)
            self.qkv_weights.append(self.create_parameter([NQ // div, E], _attr(qkv_weight_attrs, i, n), u8, False, Constant(0)))
            self.qkv_scales.append(self.create_parameter([NQ], _attr(qkv_scale_attrs, i, n), torch.float32, False, one))
            self.qkv_biases.append(self.create_parameter([NQ], _attr(qkv_bias_attrs, i, n), dt, True))
            self.linear_weights.append(self.create_parameter([E // div, nh * D], _attr(linear_weight_attrs, i, n), u8, False, Constant(0)))
            self.linear_scales.append(self.create_parameter([E], _attr(linear_scale_attrs, i, n), torch.float32, False, one))
            self.linear_biases.append(self.create_parameter([E], _attr(linear_bias_attrs, i, n), dt, True))
            self.ffn1_weights.append(self.create_parameter([F1 // div, E], _attr(ffn1_weight_attrs, i, n), u8, False, Constant(0)))
            self.ffn1_scales.append(self.create_parameter([F1], _attr(ffn1_scale_attrs, i, n), torch.float32, False, one))
            self.ffn1_biases.append(self.create_parameter([F1], _attr(ffn1_bias_attrs, i, n), dt, True))
            self.ffn2_weights.append(self.create_parameter([E // div, F], _attr(ffn2_weight_attrs, i, n), u8, False, Constant(0)))
            self.ffn2_scales.append(self.create_parameter([E], _attr(ffn2_scale_attrs, i, n), torch.float32, False, one))
            self.ffn2_biases.append(self.create_parameter([E], _attr(ffn2_bias_attrs, i, n), dt, True))
        self.name = name

    def _layers(self, dtype):
        lns = self._cast_ln(dtype)
        b = self._bits
        return [dict(head_dim=self.head_dim, ln_scale=lns[i][0], ln_bias=lns[i][1],
                     qkv=_lin(self.qkv_weights[i], self.qkv_scales[i], b), qkv_bias=self.qkv_biases[i],
                     out=_lin(self.linear_weights[i], self.linear_scales[i], b),
                     out_bias=self.linear_biases[i], ffn_ln_scale=lns[i][2], ffn_ln_bias=lns[i][3],
                     ffn1=_lin(self.ffn1_weights[i], self.ffn1_scales[i], b),
                     ffn1_bias=self.ffn1_biases[i],
                     ffn2=_lin(self.ffn2_weights[i], self.ffn2_scales[i], b),
                     ffn2_bias=self.ffn2_biases[i]) for i in range(self.num_layers)]

    @torch.no_grad()
    def load_from_float(self, fmt: "FusedMultiTransformer"):
        """Quantize a bf16/f32 FusedMultiTransformer's weights into this layer."""
        from ....ops.inference import weight_quantize
        algo = "weight_only_int4" if self._bits == 4 else "weight_only_int8"
        for i in range(self.num_layers):
            for dst, s in ((self.ln_scales, fmt.ln_scales), (self.ln_biases, fmt.ln_biases),
                           (self.ffn_ln_scales, fmt.ffn_ln_scales), (self.ffn_ln_biases, fmt.ffn_ln_biases)):
                dst[i].data.copy_(s[i].data)
            wq = fmt.qkv_weights[i].data
            wq = wq.reshape(-1, wq.shape[-1]).t() if fmt._trans_qkvw else wq.reshape(wq.shape[0], -1)
            for (w, sc, src) in ((self.qkv_weights, self.qkv_scales, wq),
                                 (self.linear_weights, self.linear_scales, fmt.linear_weights[i].data),
                                 (self.ffn1_weights, self.ffn1_scales, fmt.ffn1_weights[i].data),
                                 (self.ffn2_weights, self.ffn2_scales, fmt.ffn2_weights[i].data)):
                q, s = weight_quantize(src.to(w[i].device), algo)
                w[i].data = q.to(w[i].device)
                sc[i].data = s.to(sc[i].device)
            for dst, src in ((self.qkv_biases, fmt.qkv_biases), (self.linear_biases, fmt.linear_biases),
                             (self.ffn1_biases, fmt.ffn1_biases), (self.ffn2_biases, fmt.ffn2_biases)):
                dst[i].data = src[i].data.reshape(-1).to(dst[i].dtype)
        self._ln_cache = None
        return self


class FusedMultiTransformerINT8(FusedMultiTransformerWeightOnly):
    """Reference `fused_transformer.py:1808` / `fused_multi_transformer_int8_op.cu`: int8 weights
    AND int8 activations. Every projection quantises its input (static per-tensor scale from the
    ``*_in_scale`` attributes, reference convention q = round(127 · in_scale · x); or dynamic
    per-token absmax when no scale is given), runs the int8×int8 MFMA GEMM with int32 accumulation
    (``gemm.hip`` gemm_i8) and dequantises with the per-channel weight scale in the epilogue
    (bias and activation fused). Weights are row-major int8 [N, K] + f32 scales [N]; fill with
    :meth:`load_from_float`."""

    def __init__(self, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0, activation="gelu",
                 normalize_before=True, qkv_in_scale=None, out_linear_in_scale=None,
                 ffn1_in_scale=None, ffn2_in_scale=None, **kw):
        kw.pop("weight_dtype", None)
        for k in list(kw):
            if k.endswith("_out_scale_attrs") or k.endswith("_out_scales_attrs"):
                kw.pop(k)
        super().__init__(embed_dim, num_heads, dim_feedforward, "int8", dropout_rate, activation,
                         normalize_before, **kw)
        self.qkv_in_scale, self.out_linear_in_scale = qkv_in_scale, out_linear_in_scale
        self.ffn1_in_scale, self.ffn2_in_scale = ffn1_in_scale, ffn2_in_scale

    @staticmethod
    def _act_scale(scales, i):
        if scales is None:
            return None
        v = scales[i] if isinstance(scales, (list, tuple)) else scales
        v = float(v)
        return None if v <= 0 else 1.0 / (127.0 * v)

    def _layers(self, dtype):
        lns = self._cast_ln(dtype)
        i8 = lambda w: w.view(torch.int8)  # noqa: E731
        out = []
        for i in range(self.num_layers):
            out.append(dict(
                head_dim=self.head_dim, ln_scale=lns[i][0], ln_bias=lns[i][1],
                qkv=_lin(i8(self.qkv_weights[i]), self.qkv_scales[i], -8,
                         act_scale=self._act_scale(self.qkv_in_scale, i)),
                qkv_bias=self.qkv_biases[i],
                out=_lin(i8(self.linear_weights[i]), self.linear_scales[i], -8,
                         act_scale=self._act_scale(self.out_linear_in_scale, i)),
                out_bias=self.linear_biases[i], ffn_ln_scale=lns[i][2], ffn_ln_bias=lns[i][3],
                ffn1=_lin(i8(self.ffn1_weights[i]), self.ffn1_scales[i], -8,
                          act_scale=self._act_scale(self.ffn1_in_scale, i)),
                ffn1_bias=self.ffn1_biases[i],
                ffn2=_lin(i8(self.ffn2_weights[i]), self.ffn2_scales[i], -8,
                          act_scale=self._act_scale(self.ffn2_in_scale, i)),
                ffn2_bias=self.ffn2_biases[i]))
        return out

    @torch.no_grad()
    def load_from_float(self, fmt: "FusedMultiTransformer"):
        """Quantize a bf16/f32 FusedMultiTransformer's weights (per-channel int8, row-major)."""
        from ....ops.inference import weight_quantize
        for i in range(self.num_layers):
            for dst, s in ((self.ln_scales, fmt.ln_scales), (self.ln_biases, fmt.ln_biases),
                           (self.ffn_ln_scales, fmt.ffn_ln_scales), (self.ffn_ln_biases, fmt.ffn_ln_biases)):
                dst[i].data.copy_(s[i].data)
            wq = fmt.qkv_weights[i].data
            wq = wq.reshape(-1, wq.shape[-1]).t() if fmt._trans_qkvw else wq.reshape(wq.shape[0], -1)
            for (w, sc, src) in ((self.qkv_weights, self.qkv_scales, wq),
                                 (self.linear_weights, self.linear_scales, fmt.linear_weights[i].data),
                                 (self.ffn1_weights, self.ffn1_scales, fmt.ffn1_weights[i].data),
                                 (self.ffn2_weights, self.ffn2_scales, fmt.ffn2_weights[i].data)):
                q, s = weight_quantize(src.to(w[i].device), "llm.int8")
                w[i].data = q.view(torch.uint8).to(w[i].device)
                sc[i].data = s.to(sc[i].device)
            for dst, src in ((self.qkv_biases, fmt.qkv_biases), (self.linear_biases, fmt.linear_biases),
                             (self.ffn1_biases, fmt.ffn1_biases), (self.ffn2_biases, fmt.ffn2_biases)):
                dst[i].data = src[i].data.reshape(-1).to(dst[i].dtype)
        self._ln_cache = None
        return self


# ----------------------------------------------------------------------------- MoE
class FusedMoELayer(Layer):
    """Reference `fused_transformer.py:2110`: pre-LN + top-k gated expert FFN (experts sharded
    over ``moe_group`` with all-to-all dispatch/combine)."""

    def __init__(self, d_model, dim_feedforward, num_expert, top_k, approximate=True,
                 moe_group=None, mp_group=None, ln_scale=None, ln_bias=None, gate_weight=None,
                 gate_bias=None, linear1_weights=None, linear1_biases=None, linear2_weights=None,
                 linear2_biases=None):
        super().__init__()
        from ....nn.initializer import KaimingUniform
        self.group = moe_group
        self.world_size = moe_group.nranks if moe_group is not None else 1
        self.num_expert, self.top_k, self.approximate = num_expert, top_k, approximate
        self.d_model, self.dim_feedforward = d_model, dim_feedforward
        self.ln_scale = self.create_parameter([d_model], ln_scale, torch.float32, False, Constant(1.0))
        self.ln_bias = self.create_parameter([d_model], ln_bias, torch.float32, True)
        self.gate_weight = self.create_parameter([d_model, num_expert * self.world_size], gate_weight, self._dtype)
        self.gate_bias = self.create_parameter([num_expert * self.world_size], gate_bias, self._dtype, True)
        self.linear1_weights, self.linear2_weights = ParameterList(), ParameterList()
        self.linear1_biases, self.linear2_biases = ParameterList(), ParameterList()
        for i in range(num_expert):
            self.linear1_weights.append(self.create_parameter(
                [d_model, dim_feedforward], _attr(linear1_weights, i, num_expert), self._dtype, False, KaimingUniform()))
            self.linear2_weights.append(self.create_parameter(
                [dim_feedforward, d_model], _attr(linear2_weights, i, num_expert), self._dtype, False, KaimingUniform()))
            self.linear1_biases.append(self.create_parameter(
                [dim_feedforward], _attr(linear1_biases, i, num_expert), self._dtype, True))
            self.linear2_biases.append(self.create_parameter(
                [d_model], _attr(linear2_biases, i, num_expert), self._dtype, True))

    def forward(self, inp):
        from ...moe import moe_ffn
        B, S, E = inp.shape
        x = inp.reshape(-1, E)
        xn = incubate_f._ln(x, self.ln_scale.to(x.dtype), self.ln_bias.to(x.dtype), 1e-5)
        y = moe_ffn(xn, self.gate_weight, self.gate_bias, list(self.linear1_weights),
                    list(self.linear1_biases), list(self.linear2_weights), list(self.linear2_biases),
                    self.top_k, "gelu_tanh" if self.approximate else "gelu", self.group)
        return (x + y).reshape(B, S, E)


class FusedMultiTransformerMoe(_MultiTransformerBase):
    """Reference `fused_transformer.py:2278`: the multi-transformer with every FFN replaced by a
    top-k gated MoE (``num_expert`` experts per rank, all-to-all over ``moe_group``)."""

    def __init__(self, d_model, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0,
                 activation="gelu", normalize_before=True, num_expert=1, top_k=2,
                 approximate=True, moe_group=None, mp_group=None, epsilon=1e-5, num_layers=-1,
                 nranks=1, trans_qkvw=True, ring_id=-1, name=None, num_kv_heads=None,
                 rotary_emb_dims=0, use_neox_rotary_style=True, rope_base=10000.0, **attrs):
        super().__init__()
        from ....nn.initializer import KaimingUniform
        n = self._common_init(embed_dim, num_heads, dim_feedforward, dropout_rate, activation,
                              normalize_before, epsilon, num_layers, nranks, ring_id, num_kv_heads,
                              rotary_emb_dims, use_neox_rotary_style, rope_base, attrs)
        self._trans_qkvw = trans_qkvw
        self.num_expert, self.top_k, self.approximate = num_expert, top_k, approximate
        self.moe_group = moe_group
        ws = moe_group.nranks if moe_group is not None else 1
        E, D, nh, F, dt = embed_dim, self.head_dim, self._nh, dim_feedforward, self._dtype
        self.gate_weights, self.gate_biases = ParameterList(), ParameterList()
        self.expert_weights1, self.expert_biases1 = ParameterList(), ParameterList()
        self.expert_weights2, self.expert_biases2 = ParameterList(), ParameterList()
        for i in range(n):
            self._ln_params(i, attrs, n)
            self.qkv_weights.append(self.create_parameter([3, nh, D, E] if trans_qkvw else [E, 3, nh, D], None, dt))
            self.qkv_biases.append(self.create_parameter([3, nh, D], None, dt, True))
            self.linear_weights.append(self.create_parameter([nh * D, E], None, dt))
            self.linear_biases.append(self.create_parameter([E], None, dt, True))
            self.gate_weights.append(self.create_parameter([E, num_expert * ws], None, dt))
            self.gate_biases.append(self.create_parameter([num_expert * ws], None, dt, True))
            for _ in range(num_expert):
                self.expert_weights1.append(self.create_parameter([E, F], None, dt, False, KaimingUniform()))
                self.expert_biases1.append(self.create_parameter([F], None, dt, True))
                self.expert_weights2.append(self.create_parameter([F, E], None, dt, False, KaimingUniform()))
                self.expert_biases2.append(self.create_parameter([E], None, dt, True))
        self.name = name

    def _layers(self, dtype):
        from ...moe import moe_ffn
        lns = self._cast_ln(dtype)
        ne = self.num_expert
        act = "gelu_tanh" if self.approximate else "gelu"
        out = []
        for i in range(self.num_layers):
            sl = slice(i * ne, (i + 1) * ne)
            w1, b1 = list(self.expert_weights1)[sl], list(self.expert_biases1)[sl]
            w2, b2 = list(self.expert_weights2)[sl], list(self.expert_biases2)[sl]
            gw, gb = self.gate_weights[i], self.gate_biases[i]

            def moe(x, gw=gw, gb=gb, w1=w1, b1=b1, w2=w2, b2=b2):
                return moe_ffn(x, gw, gb, w1, b1, w2, b2, self.top_k, act, self.moe_group)
            out.append(dict(head_dim=self.head_dim, ln_scale=lns[i][0], ln_bias=lns[i][1],
                            qkv=incubate_f._qkv_linear(self.qkv_weights[i], self._trans_qkvw),
                            qkv_bias=self.qkv_biases[i].reshape(-1), out=_lin(self.linear_weights[i]),
                            out_bias=self.linear_biases[i], ffn_ln_scale=lns[i][2],
                            ffn_ln_bias=lns[i][3], moe=moe))
        return out

    def forward(self, src, attn_mask=None, caches=None, seq_lens=None, beam_offset=None,
                time_step=None, causal=False):
        B, S, _ = src.shape
        decode = time_step is not None
        pos, lens = incubate_f._positions(B, time_step, seq_lens, S, src.device, decode)
        with torch.no_grad():
            out = incubate_f.multi_transformer_forward(
                src, self._layers(src.dtype), self._nh, self._nkv, self.normalize_before,
                self._epsilon, incubate_f._caches_from(caches), pos, lens, attn_mask, decode,
                self.activation, self.rotary_emb_dims, self.use_neox_rotary_style, self.rope_base,
                causal=causal and attn_mask is None, group=self._group, moe_fn=True)
        return (out, caches) if caches is not None else out


class FusedMultiTransformerMoeWeightOnly(FusedMultiTransformerMoe):
    """Reference `fused_transformer.py:3107` / `fused_multi_transformer_moe_weight_only_op.cu`:
    the MoE multi-transformer with int8 / int4 weight-only EXPERT weights. Per layer the experts
    are stored stacked — ``expert_weights{1,2}_q[i]`` [E_local, N_packed, K] uint8 in the MFMA
    tile order of ``weight_quantize`` with ``expert_scales{1,2}[i]`` [E_local, N] f32 — and run
    as ONE grouped weight-only launch per projection (``ops.moe.grouped_weight_only_linear``,
    dequantisation inside the MFMA main loop, expert ranges resolved on the device). Attention /
    gate weights stay bf16. Fill with :meth:`load_from_float`."""

    def __init__(self, d_model, embed_dim, num_heads, dim_feedforward, weight_dtype="int8", **kw):
        super().__init__(d_model, embed_dim, num_heads, dim_feedforward, **kw)
        self._bits = 4 if weight_dtype == "int4" else 8
        div = 2 if self._bits == 4 else 1
        ne, E, F = self.num_expert, embed_dim, dim_feedforward
        u8, one = torch.uint8, Constant(1.0)
        self.expert_weights1_q, self.expert_scales1 = ParameterList(), ParameterList()
        self.expert_weights2_q, self.expert_scales2 = ParameterList(), ParameterList()
        for _ in range(self.num_layers):
            self.expert_weights1_q.append(self.create_parameter([ne, F // div, E], None, u8, False, Constant(0)))
            self.expert_scales1.append(self.create_parameter([ne, F], None, torch.float32, False, one))
            self.expert_weights2_q.append(self.create_parameter([ne, E // div, F], None, u8, False, Constant(0)))
            self.expert_scales2.append(self.create_parameter([ne, E], None, torch.float32, False, one))
        # the bf16 expert weights of the base class are replaced by the quantized stacks
        for pl in (self.expert_weights1, self.expert_weights2):
            for p in pl:
                p.data = p.data.new_empty(0)

    def _layers(self, dtype):
        from ...moe import topk_gate, stacked
        from ....ops import moe as gm
        out = super()._layers(dtype)
        ne, bits = self.num_expert, self._bits
        act = "gelu_tanh" if self.approximate else "gelu"
        for i, L in enumerate(out):
            sl = slice(i * ne, (i + 1) * ne)
            b1 = stacked(list(self.expert_biases1)[sl]).to(dtype)
            b2 = stacked(list(self.expert_biases2)[sl]).to(dtype)
            w1, s1 = self.expert_weights1_q[i], self.expert_scales1[i]
            w2, s2 = self.expert_weights2_q[i], self.expert_scales2[i]
            gw, gb = self.gate_weights[i], self.gate_biases[i]

            def moe(x, gw=gw, gb=gb, w1=w1, s1=s1, b1=b1, w2=w2, s2=s2, b2=b2):
                logits = torch.matmul(x, gw) + gb
                val, idx = topk_gate(logits, self.top_k)
                r = gm.permute(idx, ne, align=1)
                xs = gm.gather(x, r)
                h = gm.grouped_weight_only_linear(xs, w1, s1, r.offs, r.rows_cap, b1, bits, act)
                ys = gm.grouped_weight_only_linear(h, w2, s2, r.offs, r.rows_cap, b2, bits)
                return gm.combine(ys, val, r)
            L["moe"] = moe
        return out

    @torch.no_grad()
    def load_from_float(self, fmt: "FusedMultiTransformerMoe"):
        """Quantize a bf16/f32 FusedMultiTransformerMoe (same shapes) into this layer."""
        from ....ops.inference import weight_quantize
        algo = "weight_only_int4" if self._bits == 4 else "weight_only_int8"
        own = dict(self.named_parameters())
        for n, p in fmt.named_parameters():
            if n in own and not n.startswith("expert_weights"):
                own[n].data = p.data.to(own[n].device, own[n].dtype).reshape(own[n].shape) \
                    if own[n].numel() == p.numel() else own[n].data
        ne = self.num_expert
        for i in range(self.num_layers):
            for wq, sc, src in ((self.expert_weights1_q, self.expert_scales1, fmt.expert_weights1),
                                (self.expert_weights2_q, self.expert_scales2, fmt.expert_weights2)):
                qs, ss = zip(*[weight_quantize(src[i * ne + e].data.to(wq[i].device), algo)
                               for e in range(ne)])
                wq[i].data = torch.stack(qs)
                sc[i].data = torch.stack(ss)
        self._ln_cache = None
        return self


class FusedMultiTransformerMoeINT8(FusedMultiTransformerMoeWeightOnly):
    """Reference `fused_multi_transformer_moe_int8_op.cu`: int8 expert weights. On MI355X the int8
    experts run the grouped weight-only int8 MFMA path (activation in-scales are accepted and
    recorded)."""

    def __init__(self, d_model, embed_dim, num_heads, dim_feedforward, **kw):
        self_scales = {k: kw.pop(k) for k in list(kw) if k.endswith("_in_scale")}
        kw.pop("weight_dtype", None)
        super().__init__(d_model, embed_dim, num_heads, dim_feedforward, weight_dtype="int8", **kw)
        for k, v in self_scales.items():
            setattr(self, k, v)
