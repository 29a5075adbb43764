"""LayerNorm fold algebra (ops.gemm.ln_fold, used by the skinny GEMM's LN mode): with the folded
weight W∘γ, its row sums c1 and b2 = bias + W·β, rstd·(a·(W∘γ)ᵀ − mean·c1) + b2 equals
LN(a)·Wᵀ + bias — the identity the kernel epilogue applies (fp32 on CPU)."""
import pytest
import torch
import torch.nn.functional as F


@pytest.mark.parametrize("M,N,K,shift", [(8, 64, 128, 0.0), (5, 96, 256, 4.0), (32, 128, 64, -2.0)])
def test_ln_fold_identity(M, N, K, shift):
    from paddle_infer_amd.ops.gemm import ln_fold
    torch.manual_seed(M * N + K)
    a = torch.randn(M, K, dtype=torch.float64) * 2 + shift
    w = torch.randn(N, K, dtype=torch.float64) / K ** 0.5
    g = 1 + 0.3 * torch.randn(K, dtype=torch.float64)
    b = 0.2 * torch.randn(K, dtype=torch.float64)
    bias = torch.randn(N, dtype=torch.float64)
    wf, c1, b2 = ln_fold(w, g, b, bias)
    assert wf.dtype == w.dtype and c1.dtype == torch.float32 and b2.dtype == torch.float32
    mean = a.mean(1, keepdim=True)
    rstd = 1.0 / torch.sqrt(a.var(1, unbiased=False, keepdim=True) + 1e-5)
    got = rstd * (a @ wf.t() - mean * c1.double()) + b2.double()
    ref = F.layer_norm(a, (K,), g, b, 1e-5) @ w.t() + bias
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()


def test_ln_fold_rounded_weight_consistency():
    """c1 sums the ROUNDED folded weight, so the mean term cancels exactly against the GEMM's
    a·(W∘γ)ᵀ for a constant row (whose LayerNorm is β)."""
    from paddle_infer_amd.ops.gemm import ln_fold
    torch.manual_seed(0)
    K, N = 256, 64
    w = (torch.randn(N, K) / K ** 0.5).bfloat16()
    g = (1 + 0.3 * torch.randn(K)).bfloat16()
    b = (0.2 * torch.randn(K)).bfloat16()
    wf, c1, b2 = ln_fold(w, g, b)
    a = torch.full((1, K), 3.0)
    acc = a @ wf.float().t()
    assert torch.allclose(acc - 3.0 * c1, torch.zeros_like(acc), atol=1e-4)
    assert torch.allclose(b2, w.float() @ b.float(), atol=1e-5)
