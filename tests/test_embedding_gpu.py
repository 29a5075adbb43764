"""Fused embedding HIP kernels (``embedding.hip``) against plain PyTorch fp32 references:
word + position lookup, vocab-shard masking, sort-based deterministic backward (heavy duplicates),
position gradients, and the main_grad + ready-hook path used by the flat training engine."""
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
    assert _lib.has("piamd_embedding_fwd") and _lib.has("piamd_embedding_bwd")


def _close(a, b, atol, rtol=1e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    assert err <= atol + rtol * b.abs().max().item(), err


@pytest.mark.parametrize("start,V", [(0, 1000), (500, 500)])
@pytest.mark.parametrize("with_pos", [False, True])
def test_embedding_fwd_bwd(start, V, with_pos):
    from paddle_infer_amd.ops.embedding import embedding
    B, S, H = 4, 64, 384
    ids = torch.randint(0, 1000, (B, S), device=DEV)
    ids[0, :40] = start + 7  # a long run of one token
    w = torch.randn(V, H, device=DEV).bfloat16().requires_grad_(True)
    p = torch.randn(128, H, device=DEV).bfloat16().requires_grad_(True) if with_pos else None
    y = embedding(ids, w, start, p)
    g = torch.randn_like(y)
    grads = torch.autograd.grad(y, [w] + ([p] if with_pos else []), g)
    wf = w.detach().float().requires_grad_(True)
    pf = p.detach().float().requires_grad_(True) if with_pos else None
    loc = ids - start
    ok = (loc >= 0) & (loc < V)
    ref = F.embedding(torch.where(ok, loc, 0), wf) * ok[..., None]
    if with_pos:
        ref = ref + pf[:S]
    _close(y, ref, 1e-2)
    rg = torch.autograd.grad(ref, [wf] + ([pf] if with_pos else []), g.float())
    for a, b in zip(grads, rg):
        _close(a, b, 5e-2)


def test_embedding_main_grad_and_hook():
    from paddle_infer_amd.ops.embedding import embedding
    V, H = 300, 256
    ids = torch.randint(0, V, (2, 32), device=DEV)
    w = torch.randn(V, H, device=DEV).bfloat16().requires_grad_(True)
    w.main_grad = torch.ones(V, H, device=DEV, dtype=torch.bfloat16)  # accumulates on top
    fired = []
    w._grad_ready = lambda t: fired.append(1)
    y = embedding(ids, w)
    g = torch.randn_like(y)
    y.backward(g)
    ref = torch.zeros(V, H, device=DEV).index_add_(0, ids.reshape(-1), g.reshape(-1, H).float()) + 1
    _close(w.main_grad, ref, 5e-2)
    assert fired == [1] and w.grad is None
