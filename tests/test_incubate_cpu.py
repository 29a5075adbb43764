"""CPU tests of the fused-transformer family (reference tests:
`python/paddle/fluid/tests/unittests/test_fused_multi_transformer_op.py`,
`test_fused_feedforward_op.py`, `test_fused_attention_op.py`,
`test_fused_bias_dropout_residual_layer_norm_op.py`, `test_weight_only_linear.py`, MoE tests).

Each fused op is checked against a plain-PyTorch fp32 composition written here from the
reference docstrings' pseudo code."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import paddle_infer_amd as paddle
from paddle_infer_amd.incubate.nn import functional as IF
from paddle_infer_amd.incubate.nn import (FusedMultiTransformer, FusedMultiTransformerWeightOnly,
                                          FusedFeedForward, FusedMultiHeadAttention,
                                          FusedBiasDropoutResidualLayerNorm, FusedMoELayer)
from paddle_infer_amd.ops import inference as I


def _ref_fmt(m: FusedMultiTransformer, x, causal=True, mask=None):
    """Reference pseudo-code of fused_multi_transformer (pre-LN)."""
    B, S, E = x.shape
    H, D = m._nh, m.head_dim
    out = x.float()
    for i in range(m.num_layers):
        res = out
        h = F.layer_norm(out, (E,), m.ln_scales[i].float(), m.ln_biases[i].float(), m._epsilon)
        qkv = h @ m.qkv_weights[i].float().reshape(3 * H * D, E).t() + m.qkv_biases[i].float().reshape(-1)
        qkv = qkv.reshape(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        s = q @ k.transpose(-1, -2) / math.sqrt(D)
        if causal:
            s = s.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float("-inf"))
        if mask is not None:
            s = s + mask
        a = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, S, H * D)
        out = res + a @ m.linear_weights[i].float() + m.linear_biases[i].float()
        res = out
        h = F.layer_norm(out, (E,), m.ffn_ln_scales[i].float(), m.ffn_ln_biases[i].float(), m._epsilon)
        h = F.gelu(h @ m.ffn1_weights[i].float() + m.ffn1_biases[i].float())
        out = res + h @ m.ffn2_weights[i].float() + m.ffn2_biases[i].float()
    return out


def _randomize(m, scale=0.05):
    torch.manual_seed(0)
    with torch.no_grad():
        for p in m.parameters():
            if p.is_floating_point():
                p.copy_(torch.randn_like(p) * scale)
        for s in list(m.ln_scales) + list(m.ffn_ln_scales):
            s.add_(1.0)


def test_fused_multi_transformer_context_matches_reference():
    paddle.seed(0)
    m = FusedMultiTransformer(64, 4, 128, num_layers=2)
    _randomize(m)
    x = torch.randn(2, 5, 64)
    got = m(x, causal=True)
    ref = _ref_fmt(m, x, causal=True)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
    # explicit additive mask path (non-causal attention + mask)
    mask = torch.zeros(2, 1, 5, 5)
    mask[:, :, :, -1] = float("-inf")
    got = m(x, attn_mask=mask)
    torch.testing.assert_close(got, _ref_fmt(m, x, causal=False, mask=mask), rtol=1e-4, atol=1e-4)


def test_fused_multi_transformer_decode_matches_full_context():
    m = FusedMultiTransformer(64, 4, 128, num_layers=2)
    _randomize(m)
    B, S = 2, 6
    x = torch.randn(B, S + 2, 64)
    caches = m.gen_cache(B, 16, dtype="float32")
    out_ctx, caches = m(x[:, :S], caches=caches, causal=True)
    outs = [out_ctx]
    for t in range(S, S + 2):
        o, caches = m(x[:, t:t + 1], caches=caches, time_step=torch.tensor([t]))
        outs.append(o)
    got = torch.cat(outs, 1)
    ref = _ref_fmt(m, x, causal=True)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def test_qkv_prep_rope_and_cache():
    B, S, Hq, Hk, D = 2, 3, 4, 2, 64
    qkv = torch.randn(B * S, (Hq + 2 * Hk) * D)
    bias = torch.randn((Hq + 2 * Hk) * D)
    kc = torch.zeros(B, Hk, 8, D)
    vc = torch.zeros(B, Hk, 8, D)
    pos0 = torch.tensor([0, 2], dtype=torch.int32)
    out = I.qkv_prep(qkv.clone(), bias, kc, vc, pos0, B, S, Hq, Hk, D, rot_dim=32, neox=True)
    x = (qkv + bias).view(B, S, Hq + 2 * Hk, D)
    # v unchanged except bias; k rotated and cached at pos0 + s
    torch.testing.assert_close(out.view(B, S, -1, D)[:, :, Hq + Hk:], x[:, :, Hq + Hk:])
    torch.testing.assert_close(vc[1, :, 2:5], x[1, :, Hq + Hk:].transpose(0, 1))
    torch.testing.assert_close(kc[1, :, 2:5], out.view(B, S, -1, D)[1, :, Hq:Hq + Hk].transpose(0, 1))
    # rotation preserves per-pair norms (rotary part) and leaves the tail untouched
    o = out.view(B, S, -1, D)
    torch.testing.assert_close(o[..., :Hq, 32:], x[..., :Hq, 32:])
    n0 = x[..., :Hq, :16] ** 2 + x[..., :Hq, 16:32] ** 2
    n1 = o[..., :Hq, :16] ** 2 + o[..., :Hq, 16:32] ** 2
    torch.testing.assert_close(n0, n1, rtol=1e-4, atol=1e-4)
    # position 0 is the identity rotation
    torch.testing.assert_close(o[0, 0, :Hq], x[0, 0, :Hq])


@pytest.mark.parametrize("algo", ["weight_only_int8", "weight_only_int4"])
def test_weight_only_linear_cpu(algo):
    torch.manual_seed(0)
    w = torch.randn(128, 64)  # [K, N]
    x = torch.randn(3, 128)
    q, s = I.weight_quantize(w, algo)
    assert q.dtype == torch.uint8 and s.shape == (64,)
    assert q.shape == ((64, 128) if algo.endswith("int8") else (32, 128))
    wd = I.weight_dequantize(q, s, algo, "float32")
    b = torch.randn(64)
    y = I.weight_only_linear(x, q, b, s, "int4" if algo.endswith("int4") else "int8", "relu")
    torch.testing.assert_close(y, F.relu(x @ wd + b), rtol=1e-4, atol=1e-4)
    tol = 0.02 if algo.endswith("int8") else 0.3
    assert (wd - w).abs().max() < tol


def test_weight_only_fmt_matches_dequantized():
    m = FusedMultiTransformer(64, 2, 128, num_layers=1)
    _randomize(m)
    wo = FusedMultiTransformerWeightOnly(64, 2, 128, "int8", num_layers=1, dtype="float32")
    wo.load_from_float(m)
    x = torch.randn(1, 4, 64)
    got = wo(x, causal=True)
    # reference: the bf16 layer with dequantized weights
    with torch.no_grad():
        m.qkv_weights[0].copy_(I.weight_dequantize(wo.qkv_weights[0], wo.qkv_scales[0], out_dtype="float32").t().reshape(m.qkv_weights[0].shape))
        m.linear_weights[0].copy_(I.weight_dequantize(wo.linear_weights[0], wo.linear_scales[0], out_dtype="float32"))
        m.ffn1_weights[0].copy_(I.weight_dequantize(wo.ffn1_weights[0], wo.ffn1_scales[0], out_dtype="float32"))
        m.ffn2_weights[0].copy_(I.weight_dequantize(wo.ffn2_weights[0], wo.ffn2_scales[0], out_dtype="float32"))
    torch.testing.assert_close(got, m(x, causal=True), rtol=1e-4, atol=1e-4)


def test_fused_feedforward_and_bias_dropout_residual_ln():
    paddle.seed(1)
    ff = FusedFeedForward(32, 64, dropout_rate=0.0, activation="relu", normalize_before=False)
    x = torch.randn(2, 3, 32)
    got = ff(x)
    h = F.relu(x @ ff._linear1_weight + ff._linear1_bias) @ ff._linear2_weight + ff._linear2_bias
    ref = F.layer_norm(x + h, (32,), ff._ln2_scale, ff._ln2_bias, 1e-5)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
    ln = FusedBiasDropoutResidualLayerNorm(32, dropout_rate=0.0)
    r = torch.randn(2, 3, 32)
    torch.testing.assert_close(ln(x, r), F.layer_norm(r + x + ln.linear_bias, (32,), ln.ln_scale,
                                                      ln.ln_bias, 1e-5), rtol=1e-5, atol=1e-5)


def test_fused_multi_head_attention():
    paddle.seed(2)
    mha = FusedMultiHeadAttention(32, 4, dropout_rate=0.0, attn_dropout_rate=0.0, normalize_before=True)
    x = torch.randn(2, 5, 32)
    got = mha(x)
    h = F.layer_norm(x, (32,), mha.pre_ln_scale, mha.pre_ln_bias, 1e-5)
    qkv = (h @ mha.qkv_weight.reshape(96, 32).t() + mha.qkv_bias.reshape(-1)).reshape(2, 5, 3, 4, 8)
    q, k, v = qkv.permute(2, 0, 3, 1, 4)
    a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(8), -1) @ v
    ref = x + a.transpose(1, 2).reshape(2, 5, 32) @ mha.linear_weight + mha.linear_bias
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


def test_moe_layer_matches_dense_loop():
    paddle.seed(3)
    moe = FusedMoELayer(16, 32, num_expert=4, top_k=2, approximate=False)
    x = torch.randn(2, 5, 16)
    got = moe(x)
    xf = x.reshape(-1, 16)
    xn = F.layer_norm(xf, (16,), moe.ln_scale, moe.ln_bias, 1e-5)
    probs = torch.softmax(xn @ moe.gate_weight + moe.gate_bias, -1)
    val, idx = probs.topk(2, -1)
    val = val / val.sum(-1, keepdim=True)
    ref = torch.zeros_like(xf)
    for t in range(xf.shape[0]):
        for j in range(2):
            e = int(idx[t, j])
            h = F.gelu(xn[t] @ moe.linear1_weights[e] + moe.linear1_biases[e])
            ref[t] += val[t, j] * (h @ moe.linear2_weights[e] + moe.linear2_biases[e])
    torch.testing.assert_close(got, (xf + ref).reshape(2, 5, 16), rtol=1e-4, atol=1e-5)


def test_moe_gates_and_layer_backward():
    from paddle_infer_amd.incubate.distributed.models.moe import MoELayer
    from paddle_infer_amd import nn
    experts = nn.LayerList([nn.Sequential(nn.Linear(8, 16), nn.ReLU(), nn.Linear(16, 8)) for _ in range(4)])
    for gate in ("naive", "gshard", "switch"):
        layer = MoELayer(8, experts, gate={"type": gate, "top_k": 1 if gate == "switch" else 2})
        x = torch.randn(2, 6, 8, requires_grad=True)
        y = layer(x)
        y.sum().backward()
        assert y.shape == x.shape and x.grad is not None
