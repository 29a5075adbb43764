"""MoE routing (sorted, 64-aligned expert segments) and the grouped expert FFN contract on CPU:
permute/gather/combine against a dense per-token loop, gradients of the grouped FFN against
autograd through the dense loop, and the weight-only MoE multi-transformer against its bf16
original (reference tests: `test_fused_moe_op.py`, `test_fused_multi_transformer_moe_op.py`)."""
import torch
import torch.nn.functional as F

from paddle_infer_amd.ops import moe as gm


def _dense(x, idx, val, W1, B1, W2, B2, act):
    out = torch.zeros_like(x)
    for t in range(x.shape[0]):
        for j in range(idx.shape[1]):
            e = int(idx[t, j])
            if e < 0:
                continue
            h = x[t] @ W1[e] + B1[e]
            h = F.gelu(h, approximate="tanh") if act == "gelu_tanh" else F.relu(h)
            out[t] = out[t] + val[t, j] * (h @ W2[e] + B2[e])
    return out


def test_permute_layout():
    torch.manual_seed(0)
    T, k, E = 37, 2, 5
    idx = torch.randint(0, E, (T, k))
    idx[3, 1] = -1  # a dropped assignment
    r = gm.permute(idx, E, align=64)
    offs = r.offs.tolist()
    assert offs[0] == 0 and all((offs[e + 1] - offs[e]) % 64 == 0 for e in range(E))
    assert r.rows_cap >= offs[-1]
    for t in range(T):
        for j in range(k):
            s = int(r.slot[t, j])
            if idx[t, j] < 0:
                assert s == -1
                continue
            e = int(idx[t, j])
            assert offs[e] <= s < offs[e + 1]
            assert int(r.src[s]) == t
    # padding rows point nowhere; each expert's used rows come first in its segment
    for e in range(E):
        n = int((idx == e).sum())
        seg = r.src[offs[e]:offs[e + 1]]
        assert (seg[:n] >= 0).all() and (seg[n:] == -1).all()


def test_grouped_ffn_forward_backward_matches_dense():
    torch.manual_seed(1)
    T, H, Fd, E, k = 19, 16, 24, 4, 2
    x = torch.randn(T, H, dtype=torch.float64, requires_grad=True)
    W1 = torch.randn(E, H, Fd, dtype=torch.float64, requires_grad=True)
    B1 = torch.randn(E, Fd, dtype=torch.float64, requires_grad=True)
    W2 = torch.randn(E, Fd, H, dtype=torch.float64, requires_grad=True)
    B2 = torch.randn(E, H, dtype=torch.float64, requires_grad=True)
    idx = torch.randint(0, E, (T, k))
    val = torch.rand(T, k, dtype=torch.float64)
    r = gm.permute(idx, E)
    y = gm.combine(gm.grouped_ffn(gm.gather(x, r), W1, B1, W2, B2, r, "relu"), val, r)
    ref = _dense(x, idx, val, W1, B1, W2, B2, "relu")
    assert torch.allclose(y, ref, atol=1e-6)
    g = torch.randn_like(ref)
    got = torch.autograd.grad(y, (x, W1, B1, W2, B2), g)
    exp = torch.autograd.grad(ref, (x, W1, B1, W2, B2), g)
    for a, b in zip(got, exp):
        assert torch.allclose(a, b, atol=1e-6), (a - b).abs().max()


def test_moe_layer_grouped_path_cpu_reference():
    from paddle_infer_amd.incubate.nn import FusedMoELayer
    torch.manual_seed(2)
    m = FusedMoELayer(32, 64, num_expert=4, top_k=2, approximate=True)
    x = torch.randn(2, 5, 32)
    y = m(x)
    assert y.shape == x.shape and torch.isfinite(y).all()


def test_weight_only_moe_multi_transformer_close_to_float():
    from paddle_infer_amd.incubate.nn import (FusedMultiTransformerMoe,
                                              FusedMultiTransformerMoeWeightOnly)
    torch.manual_seed(3)
    kw = dict(num_expert=4, top_k=2, num_layers=2)
    ref = FusedMultiTransformerMoe(64, 64, 4, 128, **kw)
    with torch.no_grad():
        for p in ref.parameters():
            p.normal_(0, 0.05)
    q = FusedMultiTransformerMoeWeightOnly(64, 64, 4, 128, weight_dtype="int8", **kw)
    q.load_from_float(ref)
    x = torch.randn(2, 6, 64) * 0.5
    a, b = ref(x), q(x)
    assert (a - b).abs().max() < 0.05 * a.abs().max() + 1e-3
