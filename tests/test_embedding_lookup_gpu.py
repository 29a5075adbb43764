"""paddle.nn.functional.embedding on the own kernels (embedding.hip *_dt entry points): f32 / bf16
/ fp16 tables, Paddle padding semantics (zero output rows, no gradient), deterministic sort-based
gradient, against the fp32 PyTorch reference; no library fallback."""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _no_fallback(monkeypatch):
    from paddle_infer_amd.ops import _lib
    seen = []
    monkeypatch.setattr(_lib, "fallback", lambda op, why="": seen.append(op))
    yield
    assert not seen, seen


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("pad", [None, 0, -1])
def test_embedding_lookup(dt, pad):
    import paddle_infer_amd.nn.functional as F
    torch.manual_seed(7)
    V, H = 1000, 136
    w = torch.randn(V, H, device=DEV).to(dt).requires_grad_(True)
    ids = torch.randint(0, V, (4, 257), device=DEV)
    ids[0, :7] = 0
    ids[1, 3:9] = V - 1
    ids[2, :50] = 5  # a long run of one id
    y = F.embedding(ids, w, padding_idx=pad)
    dy = torch.randn_like(y)
    y.backward(dy)
    wr = w.detach().float().requires_grad_(True)
    p = None if pad is None else (pad + V if pad < 0 else pad)
    yr = TF.embedding(ids, wr)
    if p is not None:
        yr = yr * (ids != p).unsqueeze(-1).float()
    yr.backward(dy.float())
    assert torch.equal(y.float(), yr.to(dt).float())  # a gather: exact
    tol = {torch.float32: 1e-5, torch.bfloat16: 3e-2, torch.float16: 3e-3}[dt]
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=tol * 8, rtol=tol)
    if p is not None:
        assert torch.all(w.grad[p] == 0)
    g1 = w.grad.clone()
    w.grad = None
    F.embedding(ids, w, padding_idx=pad).backward(dy)
    assert torch.equal(w.grad, g1)
