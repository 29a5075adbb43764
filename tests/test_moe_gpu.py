"""Grouped MoE expert GEMM HIP kernels (``gemm.hip`` moe_gemm / moe_wgrad, ``infer.hip``
wo_moe_gemm) against plain PyTorch fp32 references of the same ops."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    import paddle_infer_amd  # noqa: F401
    from paddle_infer_amd.ops import _lib
    _lib.lib()
    assert _lib.has("piamd_moe_gemm") and _lib.has("piamd_moe_wgrad") and _lib.has("piamd_wo_moe_gemm")


def _close(a, b, atol, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max err {err} > {tol}"


def _routing(T, k, E, seed=0, skew=False):
    from paddle_infer_amd.ops import moe as gm
    g = torch.Generator().manual_seed(seed)
    if skew:  # one hot expert, one empty expert
        p = torch.tensor([8.0] + [1.0] * (E - 2) + [0.0])
        idx = torch.multinomial(p.expand(T, E), k, generator=g)
    else:
        idx = torch.randint(0, E, (T, k), generator=g)
    return idx.to(DEV), gm.permute(idx.to(DEV), E)


@pytest.mark.parametrize("trans_w", [False, True])
@pytest.mark.parametrize("skew", [False, True])
def test_grouped_gemm_bias_act(trans_w, skew):
    from paddle_infer_amd.ops import moe as gm
    T, k, E, K, N = 300, 2, 6, 256, 512
    idx, r = _routing(T, k, E, skew=skew)
    x = torch.randn(T, K, device=DEV).bfloat16()
    xs = gm.gather(x, r)
    w = (torch.randn(E, K, N, device=DEV) * 0.05).bfloat16()
    b = torch.randn(E, N, device=DEV).bfloat16()
    wk = w.transpose(1, 2).contiguous() if trans_w else w
    aux = torch.empty(r.rows_cap, N, device=DEV, dtype=torch.bfloat16)
    y = gm.grouped_gemm(xs, wk, r.offs, r.rows_cap, b, "gelu_tanh", trans_w=trans_w, aux=aux)
    torch.cuda.synchronize()
    offs = r.offs.tolist()
    for e in range(E):
        a0, a1 = offs[e], offs[e + 1]
        if a1 == a0:
            continue
        pre = xs[a0:a1].float() @ w[e].float() + b[e].float()
        _close(aux[a0:a1], pre, 3e-2)
        _close(y[a0:a1], F.gelu(pre, approximate="tanh"), 3e-2)


def test_grouped_ffn_training_grads():
    from paddle_infer_amd.ops import moe as gm
    T, k, E, H, Fd = 200, 2, 4, 256, 512
    idx, r = _routing(T, k, E, seed=3)
    val = torch.rand(T, k, device=DEV)
    x = torch.randn(T, H, device=DEV).bfloat16().requires_grad_(True)
    W1 = (torch.randn(E, H, Fd, device=DEV) * 0.05).bfloat16().requires_grad_(True)
    B1 = (torch.randn(E, Fd, device=DEV) * 0.1).bfloat16().requires_grad_(True)
    W2 = (torch.randn(E, Fd, H, device=DEV) * 0.05).bfloat16().requires_grad_(True)
    B2 = (torch.randn(E, H, device=DEV) * 0.1).bfloat16().requires_grad_(True)
    y = gm.combine(gm.grouped_ffn(gm.gather(x, r), W1, B1, W2, B2, r, "gelu_tanh"), val, r)
    g = torch.randn_like(y)
    got = torch.autograd.grad(y, (x, W1, B1, W2, B2), g)
    # fp32 reference on the same routing (dense per expert)
    ref_in = [t.detach().float().requires_grad_(True) for t in (x, W1, B1, W2, B2)]
    xf, W1f, B1f, W2f, B2f = ref_in
    out = torch.zeros_like(xf)
    for e in range(E):
        tok, j = (idx == e).nonzero(as_tuple=True)
        h = F.gelu(xf[tok] @ W1f[e] + B1f[e], approximate="tanh")
        out = out.index_add(0, tok, val[tok, j][:, None] * (h @ W2f[e] + B2f[e]))
    _close(y, out, 3e-2)
    exp = torch.autograd.grad(out, ref_in, g.float())
    for a, b in zip(got, exp):
        _close(a, b, 5e-2)


@pytest.mark.parametrize("bits", [16, 8, 4])
def test_grouped_weight_only(bits):
    from paddle_infer_amd.ops import moe as gm
    from paddle_infer_amd.ops.inference import weight_quantize, weight_dequantize, pack_bf16
    T, k, E, K, N = 9, 2, 8, 512, 256
    idx, _ = _routing(T, k, E, seed=5)
    r = gm.permute(idx, E, align=1)
    x = torch.randn(T, K, device=DEV).bfloat16()
    xs = gm.gather(x, r)
    w = (torch.randn(E, K, N, device=DEV) * 0.05).bfloat16()
    b = torch.randn(E, N, device=DEV).bfloat16()
    if bits == 16:
        wq, sc = torch.stack([pack_bf16(w[e]) for e in range(E)]), None
        wd = w.float()
    else:
        algo = "weight_only_int4" if bits == 4 else "weight_only_int8"
        qs = [weight_quantize(w[e], algo) for e in range(E)]
        wq, sc = torch.stack([q for q, _ in qs]), torch.stack([s for _, s in qs])
        wd = torch.stack([weight_dequantize(q, s, algo, "float32") for q, s in qs]).float()
    y = gm.grouped_weight_only_linear(xs, wq, sc, r.offs, r.rows_cap, b, bits, "relu")
    yo = gm.combine(y, torch.ones(T, k, device=DEV), r)
    ref = torch.zeros(T, N, device=DEV)
    for t in range(T):
        for j in range(k):
            e = int(idx[t, j])
            ref[t] += torch.relu(x[t].float() @ wd[e] + b[e].float())
    _close(yo, ref, 5e-2)


def test_fused_moe_layer_grouped_matches_per_expert_path(monkeypatch):
    from paddle_infer_amd.incubate import moe as M
    from paddle_infer_amd.incubate.nn import FusedMoELayer
    torch.manual_seed(7)
    m = FusedMoELayer(256, 512, num_expert=4, top_k=2)
    for p in m.parameters():
        p.data = p.data.to(DEV, torch.bfloat16)
    x = torch.randn(2, 33, 256, device=DEV).bfloat16()
    with torch.no_grad():
        got = m(x)  # grouped MFMA kernels (same bf16 gate → same routing as below)
        monkeypatch.setattr(M, "_grouped_ok", lambda *a: False)
        ref = m(x)  # per-expert hipBLASLt loop
    _close(got, ref, 5e-2)
