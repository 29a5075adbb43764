"""fused_multi_transformer program op with the reference's RotaryPosEmb (external cos / sin table,
rotary_emb_dims head-dim chunks) and PreCaches (prefix K/V) inputs — `fused_multi_transformer_op.cc
:166,170` — against a plain fp32 composition: context stage (prefix attended ahead of the prompt,
written to cache slots [0, P + S)), then one decode step reading the table of the new position."""
import math

import pytest
import torch
import torch.nn.functional as F

from paddle_infer_amd.static.ops_registry import REGISTRY

E, H, D, FF, B, S, P, MAXS = 64, 4, 16, 128, 2, 5, 3, 16


def _weights(L, g):
    def r(*s, sc=0.2):
        return sc * torch.randn(*s, generator=g)
    return [dict(ln_s=1 + r(E, sc=0.1), ln_b=r(E, sc=0.1), qkvw=r(3, H, D, E), qkvb=r(3, H, D, sc=0.1),
                 ow=r(E, E), ob=r(E, sc=0.1), fln_s=1 + r(E, sc=0.1), fln_b=r(E, sc=0.1),
                 f1w=r(E, FF), f1b=r(FF, sc=0.1), f2w=r(FF, E), f2b=r(E, sc=0.1)) for _ in range(L)]


def _rot_ref(x, cos, sin, chunks, decode):
    # x [B, S, H, D]; cos / sin [B, S, D]; element-wise loops mirror the reference kernels
    out = x.clone()
    Lw = D // chunks
    h = Lw // 2
    for c in range(chunks):
        for t in range(h):
            i, j = c * Lw + t, c * Lw + t + h
            cl, sl = cos[:, :, None, i], sin[:, :, None, i]
            cr, sr = (cos[:, :, None, j], sin[:, :, None, j]) if decode else (cl, sl)
            out[..., i] = x[..., i] * cl - x[..., j] * sl
            out[..., j] = x[..., j] * cr + x[..., i] * sr
    return out


def _ref_layer(x, W, K_prev, V_prev, cos, sin, chunks, decode, mask=None):
    """x [B, S, E]; K_prev / V_prev [B, H, T0, D] keys attended ahead (prefix or cache)."""
    h = F.layer_norm(x, (E,), W["ln_s"], W["ln_b"], 1e-5)
    qkv = h @ W["qkvw"].reshape(3 * H * D, E).t() + W["qkvb"].reshape(-1)
    qkv = qkv.reshape(B, -1, 3, H, D)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    q, k = _rot_ref(q, cos, sin, chunks, decode), _rot_ref(k, cos, sin, chunks, decode)
    Kf = torch.cat([K_prev, k.transpose(1, 2)], 2)
    Vf = torch.cat([V_prev, v.transpose(1, 2)], 2)
    s = q.transpose(1, 2) @ Kf.transpose(-1, -2) / math.sqrt(D)
    if mask is not None:
        s = s + mask
    a = (torch.softmax(s, -1) @ Vf).transpose(1, 2).reshape(B, -1, E)
    x = x + a @ W["ow"] + W["ob"]
    h = F.layer_norm(x, (E,), W["fln_s"], W["fln_b"], 1e-5)
    x = x + F.gelu(h @ W["f1w"] + W["f1b"]) @ W["f2w"] + W["f2b"]
    return x, Kf, Vf


def _ins(x, Ws, caches, extra):
    d = {"X": [x], "LnScale": [w["ln_s"] for w in Ws], "LnBias": [w["ln_b"] for w in Ws],
         "QKVW": [w["qkvw"] for w in Ws], "QKVBias": [w["qkvb"] for w in Ws],
         "OutLinearW": [w["ow"] for w in Ws], "OutLinearBias": [w["ob"] for w in Ws],
         "FFNLnScale": [w["fln_s"] for w in Ws], "FFNLnBias": [w["fln_b"] for w in Ws],
         "FFN1Weight": [w["f1w"] for w in Ws], "FFN1Bias": [w["f1b"] for w in Ws],
         "FFN2Weight": [w["f2w"] for w in Ws], "FFN2Bias": [w["f2b"] for w in Ws],
         "CacheKV": caches}
    d.update(extra)
    return d


@pytest.mark.parametrize("chunks", [1, 2])
@pytest.mark.parametrize("with_prefix", [False, True])
def test_fmt_rotary_table_and_prefix(chunks, with_prefix):
    g = torch.Generator().manual_seed(chunks * 10 + with_prefix)
    L = 2
    Ws = _weights(L, g)
    x = torch.randn(B, S, E, generator=g)
    Pn = P if with_prefix else 0
    pre = [0.5 * torch.randn(2, B, H, Pn, D, generator=g) for _ in range(L)]
    # a non-standard table (angles per position and dim, cos[i + half] != cos[i]) so the context /
    # decode index conventions are both exercised
    ang = torch.randn(B, S + 1, D, generator=g)
    cos, sin = torch.cos(ang), torch.sin(ang)
    rot_ctx = torch.stack([cos[:, :S], sin[:, :S]])[:, :, None]            # [2, B, 1, S, D]
    rot_dec = torch.stack([cos[:, S:S + 1], sin[:, S:S + 1]])[:, :, None]  # [2, B, 1, 1, D]
    caches = [torch.zeros(2, B, H, MAXS, D) for _ in range(L)]
    attrs = {"pre_layer_norm": True, "epsilon": 1e-5, "act_method": "gelu", "trans_qkvw": True,
             "rotary_emb_dims": chunks}
    extra = {"RotaryPosEmb": [rot_ctx]}
    if with_prefix:
        extra["PreCaches"] = pre
    out = REGISTRY["fused_multi_transformer"](_ins(x, Ws, caches, extra), attrs)["Out"]
    # reference: context with the prefix ahead of the prompt
    ref, Ks, Vs = x, [], []
    for li, W in enumerate(Ws):
        ref, Kf, Vf = _ref_layer(ref, W, pre[li][0], pre[li][1], cos[:, :S], sin[:, :S], chunks, False)
        Ks.append(Kf)
        Vs.append(Vf)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    for li in range(L):  # cache slots [0, P + S)
        torch.testing.assert_close(caches[li][0, :, :, :Pn + S], Ks[li], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(caches[li][1, :, :, :Pn + S], Vs[li], rtol=1e-5, atol=1e-5)
    # decode step at position P + S (time_step), mask over the Pn + S + 1 valid keys
    x1 = torch.randn(B, 1, E, generator=g)
    T = Pn + S
    mask = torch.zeros(B, 1, 1, T + 1)
    ext = {"RotaryPosEmb": [rot_dec], "TimeStep": [torch.tensor([T], dtype=torch.int32)],
           "SrcMask": [mask]}
    out1 = REGISTRY["fused_multi_transformer"](_ins(x1, Ws, caches, ext), attrs)["Out"]
    ref1 = x1
    for li, W in enumerate(Ws):
        ref1, _, _ = _ref_layer(ref1, W, Ks[li], Vs[li], cos[:, S:S + 1], sin[:, S:S + 1], chunks, True,
                                mask)
    torch.testing.assert_close(out1, ref1, rtol=1e-4, atol=1e-4)


def test_fmt_rotary_dims_without_table_refused():
    g = torch.Generator().manual_seed(0)
    Ws = _weights(1, g)
    x = torch.randn(B, S, E, generator=g)
    with pytest.raises(ValueError, match="RotaryPosEmb"):
        REGISTRY["fused_multi_transformer"](_ins(x, Ws, [], {}), {"rotary_emb_dims": 1})
