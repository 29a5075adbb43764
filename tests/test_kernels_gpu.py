"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    import paddle_infer_amd  # noqa: F401
    from paddle_infer_amd.ops import _lib
    _lib.lib()  # HIP path must be the one that runs


def _close(a, b, atol, rtol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max err {err} > {tol}"


@pytest.mark.parametrize("N", [256, 768, 2048, 4096])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_layernorm(N, dtype):
    from paddle_infer_amd.ops import layer_norm
    x = torch.randn(300, N, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(N, device=DEV)).to(dtype).requires_grad_()
    b = (0.1 * torch.randn(N, device=DEV)).to(dtype).requires_grad_()
    y = layer_norm(x, w, b, 1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = F.layer_norm(xr, (N,), wr, br, 1e-5)
    yr.backward(dy.float())
    at = 3e-2 if dtype == torch.bfloat16 else 1e-4
    _close(y, yr, at)
    _close(x.grad, xr.grad, at)
    _close(w.grad, wr.grad, at * 10, 3e-2)
    _close(b.grad, br.grad, at * 10, 3e-2)


def test_fused_add_layernorm():
    from paddle_infer_amd.ops import fused_add_layer_norm
    N = 2048
    x = torch.randn(4, 128, N, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn_like(x, requires_grad=True)
    xb = (0.1 * torch.randn(N, device=DEV)).bfloat16().requires_grad_()
    w = torch.ones(N, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = torch.zeros(N, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y, h = fused_add_layer_norm(x, r, w, b, 1e-5, xb, 0.0)
    dy, dh = torch.randn_like(y), torch.randn_like(h)
    torch.autograd.backward([y, h], [dy, dh])
    xr, rr, xbr, wr, br = (t.detach().float().requires_grad_() for t in (x, r, xb, w, b))
    hr = rr + xr + xbr
    yr = F.layer_norm(hr, (N,), wr, br, 1e-5)
    torch.autograd.backward([yr, hr], [dy.float(), dh.float()])
    _close(y, yr, 3e-2)
    _close(h, hr, 3e-2)
    _close(x.grad, xr.grad, 5e-2)
    _close(r.grad, rr.grad, 5e-2)
    _close(xb.grad, xbr.grad, 1.0, 3e-2)
    _close(w.grad, wr.grad, 1.0, 3e-2)


@pytest.mark.parametrize("N,rows", [(1536, 333), (2048, 1), (2048, 3001)])
def test_fused_add_layernorm_pair_backward(N, rows):
    """1024 < N <= 2048: the two-waves-per-row backward (prefetched second row, uniform trip count
    over odd row counts) against the fp32 reference, incl. the residual / x-bias gradients."""
    from paddle_infer_amd.ops import fused_add_layer_norm
    torch.manual_seed(N + rows)
    x = torch.randn(rows, N, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn_like(x, requires_grad=True)
    xb = (0.1 * torch.randn(N, device=DEV)).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(N, device=DEV)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(N, device=DEV)).bfloat16().requires_grad_()
    y, h = fused_add_layer_norm(x, r, w, b, 1e-5, xb, 0.0)
    dy, dh = torch.randn_like(y), torch.randn_like(h)
    torch.autograd.backward([y, h], [dy, dh])
    xr, rr, xbr, wr, br = (t.detach().float().requires_grad_() for t in (x, r, xb, w, b))
    hr = rr + xr + xbr
    yr = F.layer_norm(hr, (N,), wr, br, 1e-5)
    torch.autograd.backward([yr, hr], [dy.float(), dh.float()])
    _close(x.grad, xr.grad, 5e-2)
    _close(r.grad, rr.grad, 5e-2)
    _close(xb.grad, xbr.grad, 1.0, 3e-2)
    _close(w.grad, wr.grad, 1.0, 3e-2)
    _close(b.grad, br.grad, 1.0, 3e-2)


def test_fused_add_layernorm_dropout_consistent():
    from paddle_infer_amd.ops import fused_add_layer_norm
    N = 1024
    x = torch.randn(64, N, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.zeros_like(x)
    y, h = fused_add_layer_norm(x, r, None, None, 1e-5, None, 0.25)
    kept = h != 0
    frac = kept.float().mean().item()
    assert 0.7 < frac < 0.8
    _close(h[kept], (x.detach() / 0.75)[kept], 2e-2)
    h.backward(torch.ones_like(h))
    assert torch.equal(x.grad != 0, kept)


def test_dropout_masks_independent_across_calls():
    """Consecutive dropout launches draw (near-)uncorrelated masks, also under XOR-shifted indices
    (a single XOR-keyed hash round made one mask an index-permuted copy of the other)."""
    from paddle_infer_amd.ops import fused_add_layer_norm
    N, R = 2048, 512
    x = torch.ones(R, N, device=DEV, dtype=torch.bfloat16)
    masks = []
    for _ in range(4):
        _, h = fused_add_layer_norm(x, torch.zeros_like(x), None, None, 1e-5, None, 0.5)
        masks.append((h != 0).float().reshape(-1))
    idx = torch.arange(R * N, device=DEV)
    for i in range(3):
        a, b = masks[i] - masks[i].mean(), masks[i + 1] - masks[i + 1].mean()
        assert abs((a * b).mean().item() / (a.std() * b.std()).item()) < 0.01
        for d in (1, 2, 3, 7, 64, 1000):  # b read at index i ^ d
            bs = masks[i + 1][idx ^ d] - masks[i + 1].mean()
            c = (a * bs).mean().item() / (a.std() * bs.std()).item()
            assert abs(c) < 0.01, (i, d, c)


@pytest.mark.parametrize("B,Sq,Sk,Hq,Hk,D,causal", [
    (2, 256, 256, 4, 4, 128, True),
    (2, 256, 256, 4, 4, 128, False),
    (1, 200, 200, 2, 2, 128, True),
    (2, 128, 384, 4, 2, 64, True),
    (1, 333, 333, 8, 2, 64, False),
    (2, 1024, 1024, 2, 2, 128, True),
])
def test_flash_attention(B, Sq, Sk, Hq, Hk, D, causal):
    from paddle_infer_amd.ops import flash_attention, attention_reference
    torch.manual_seed(0)
    q = torch.randn(B, Sq, Hq, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Sk, Hk, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Sk, Hk, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attention(q, k, v, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = attention_reference(qr, kr, vr, causal=causal)
    orf.backward(do.float())
    _close(o, orf, 2e-2)
    _close(q.grad, qr.grad, 5e-2)
    _close(k.grad, kr.grad, 5e-2)
    _close(v.grad, vr.grad, 5e-2)


def test_flash_attention_packed():
    from paddle_infer_amd.ops import flash_attention_packed, attention_reference
    B, S, H, D = 2, 512, 4, 128
    qkv = torch.randn(B, S, 3 * H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attention_packed(qkv, H, H, causal=True)
    do = torch.randn_like(o)
    o.backward(do)
    r = qkv.detach().float().requires_grad_()
    orf = attention_reference(r[:, :, :H], r[:, :, H:2 * H], r[:, :, 2 * H:], causal=True)
    orf.backward(do.float())
    _close(o, orf, 2e-2)
    _close(qkv.grad, r.grad, 5e-2)


@pytest.mark.parametrize("V", [1000, 50304])
def test_softmax_cross_entropy(V):
    from paddle_infer_amd.ops import softmax_cross_entropy
    logits = (3 * torch.randn(257, V, device=DEV)).bfloat16().requires_grad_()
    labels = torch.randint(0, V, (257,), device=DEV)
    labels[5] = -100
    loss = softmax_cross_entropy(logits, labels)
    loss.mean().backward()
    lr = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(lr, labels, ignore_index=-100, reduction="none")
    ref.mean().backward()
    _close(loss, ref, 2e-2)
    _close(logits.grad, lr.grad, 1e-4)


@pytest.mark.parametrize("act", ["gelu", "gelu_tanh", "relu", "silu"])
def test_bias_act(act):
    from paddle_infer_amd.ops import bias_act
    x = torch.randn(512, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = (0.1 * torch.randn(1024, device=DEV)).bfloat16().requires_grad_()
    y = bias_act(x, b, act)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, br = x.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    t = xr + br
    yr = {"gelu": F.gelu(t), "gelu_tanh": F.gelu(t, approximate="tanh"), "relu": F.relu(t),
          "silu": F.silu(t)}[act]
    yr.backward(dy.float())
    _close(y, yr, 2e-2)
    _close(x.grad, xr.grad, 3e-2)
    _close(b.grad, br.grad, 0.5, 3e-2)


def test_softmax_mask():
    from paddle_infer_amd.ops import fused_softmax_mask
    x = torch.randn(2, 4, 128, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = fused_softmax_mask(x, None, 0.5, causal=True)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    s = (xr * 0.5).masked_fill(torch.ones(128, 128, device=DEV).triu(1).bool(), float("-inf"))
    yr = torch.softmax(s, -1)
    yr.backward(dy.float())
    _close(y, yr, 1e-2)
    _close(x.grad, xr.grad, 2e-2)


def test_adamw_flat():
    from paddle_infer_amd.ops import adamw_flat
    n = 10001
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV).bfloat16()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    model = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    pc, mc, vc = p.cpu().clone(), m.cpu().clone(), v.cpu().clone()
    for step in (1, 2, 3):
        adamw_flat(p, m, v, g, 1e-3, 0.9, 0.95, 1e-8, 0.1, step, model=model, static_grad_scale=0.5)
        adamw_flat(pc, mc, vc, g.cpu(), 1e-3, 0.9, 0.95, 1e-8, 0.1, step, static_grad_scale=0.5)
    _close(p.cpu(), pc, 1e-5, 1e-5)
    _close(model.cpu(), pc, 1e-2)


def test_sumsq():
    from paddle_infer_amd.ops import sumsq
    x = torch.randn(1_000_003, device=DEV).bfloat16()
    s = sumsq(x)
    ref = x.float().pow(2).sum()
    assert abs(s.item() - ref.item()) / ref.item() < 1e-4


def test_gpt_tiny_matches_fp32_cpu():
    import copy
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    torch.manual_seed(0)
    cfg = gpt_config("gpt3-tiny", dtype="float32", hidden_dropout_prob=0.0, hidden_size=256,
                     num_heads=2)
    ref = GPTForPretraining(cfg)
    cfg_b = copy.deepcopy(cfg)
    cfg_b.dtype = "bfloat16"
    with torch.device(DEV):
        m = GPTForPretraining(cfg_b)
    m.set_state_dict(ref.state_dict())
    ids = torch.randint(0, cfg.vocab_size, (2, 129))
    l_ref = ref(ids[:, :-1], labels=ids[:, 1:])
    l_gpu = m(ids[:, :-1].to(DEV), labels=ids[:, 1:].to(DEV))
    assert abs(l_ref.item() - l_gpu.item()) < 2e-2 * abs(l_ref.item())
    l_gpu.backward()
    l_ref.backward()
    g_ref = ref.gpt.layers[0].attn.qkv_proj.weight.grad
    g_gpu = m.gpt.layers[0].attn.qkv_proj.weight.grad
    _close(g_gpu.cpu(), g_ref, 5e-2 * g_ref.abs().max().item())


def test_gpt_recompute_with_kernel_dropout_matches_plain():
    """GPU: layer recompute must replay the kernel-dropout generator (seed, offset) so the
    recomputed forward and its backward use the forward's masks (torch.utils.checkpoint
    restored only torch's RNG)."""
    from paddle_infer_amd.framework import random as prand
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config

    def grads(recompute):
        cfg = gpt_config("gpt3-tiny", hidden_dropout_prob=0.1, recompute=recompute)
        torch.manual_seed(0)
        with torch.device(DEV):
            m = GPTForPretraining(cfg)
        m.train()
        ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=torch.Generator().manual_seed(1)).to(DEV)
        prand.seed(11)
        loss = m(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        return loss.detach().float(), {n: p.grad.float().clone() for n, p in m.named_parameters()
                                       if p.grad is not None}

    l0, g0 = grads(False)
    l1, g1 = grads(True)
    assert torch.allclose(l0, l1)
    for n in g0:
        _close(g1[n], g0[n], 1e-3)


@pytest.mark.parametrize("act", ["gelu", "gelu_tanh", "relu", "silu"])
def test_fp32_bias_act_on_kernel(act):
    """fp32 (Paddle's default dtype) bias + activation on the elementwise HIP kernel, forward and
    backward with the fused bias-gradient column sums, against PyTorch fp32 — no fallback."""
    from paddle_infer_amd.ops import _lib, bias_act
    _lib.FALLBACKS.clear()
    torch.manual_seed(3)
    x = torch.randn(333, 264, device=DEV, requires_grad=True)
    b = torch.randn(264, device=DEV, requires_grad=True)
    y = bias_act(x, b, act)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, br = x.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    ref = {"gelu": lambda t: F.gelu(t), "gelu_tanh": lambda t: F.gelu(t, approximate="tanh"),
           "relu": F.relu, "silu": F.silu}[act](xr + br)
    ref.backward(dy)
    _close(y, ref, 2e-5, 1e-5)
    _close(x.grad, xr.grad, 2e-5, 1e-5)
    _close(b.grad, br.grad, 2e-4, 1e-5)
    assert not _lib.FALLBACKS, _lib.FALLBACKS


def test_fp32_dropout_and_softmax_on_kernel():
    from paddle_infer_amd.ops import _lib, dropout, fused_softmax_mask
    _lib.FALLBACKS.clear()
    x = torch.ones(512, 1024, device=DEV, requires_grad=True)
    y = dropout(x, 0.3)
    kept = y != 0
    assert abs(kept.float().mean().item() - 0.7) < 0.01
    _close(y[kept], torch.full_like(y[kept], 1 / 0.7), 1e-6, 0.0)
    y.backward(torch.ones_like(y))
    assert torch.equal(x.grad != 0, kept)  # backward regenerates the same mask
    s = torch.randn(6, 40, 256, device=DEV, requires_grad=True)
    m = torch.randn(40, 256, device=DEV)
    p = fused_softmax_mask(s, m, 0.5)
    dp = torch.randn_like(p)
    p.backward(dp)
    sr = s.detach().clone().requires_grad_()
    pr = torch.softmax(sr * 0.5 + m, -1)
    pr.backward(dp)
    _close(p, pr, 1e-6, 1e-5)
    _close(s.grad, sr.grad, 1e-6, 1e-5)
    assert not _lib.FALLBACKS, _lib.FALLBACKS
