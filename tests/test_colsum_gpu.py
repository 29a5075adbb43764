"""Column sums (bias gradients): ops.linear.colsum_into (rowsum partials + the wide column-sum
reduce) and ops.gemm.colsum_parts on many partial rows, against fp32 sums; both reduce kernels
(G ≥ 64 float4 lanes / the 4-row-group one) and ragged widths."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("rows,N", [(98304 // 16, 6144), (4096, 100), (4096, 102), (2048, 2048), (40, 8)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("acc", [False, True])
def test_colsum_into(rows, N, dt, acc):
    from paddle_infer_amd.ops.linear import colsum_into
    torch.manual_seed(rows + N)
    x = torch.randn(rows, N, device=DEV).to(dt)
    base = torch.randn(N, device=DEV).to(dt)
    out = base.clone()
    colsum_into(x, out, accumulate=acc)
    ref = x.float().sum(0) + (base.float() if acc else 0)
    tol = 1e-3 * rows ** 0.5 * (8 if dt != torch.float32 else 1)
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=1e-2)
    out2 = base.clone()
    colsum_into(x, out2, accumulate=acc)
    assert torch.equal(out, out2)  # deterministic


@pytest.mark.parametrize("G,N", [(768, 8192), (64, 36), (63, 8192), (1, 2048)])
def test_colsum_parts(G, N):
    from paddle_infer_amd.ops.gemm import colsum_parts
    torch.manual_seed(G)
    part = torch.randn(G, N, device=DEV)
    out = torch.zeros(N, device=DEV, dtype=torch.bfloat16)
    colsum_parts(part, out, accumulate=False)
    torch.testing.assert_close(out.float(), part.sum(0), atol=2e-2 * G ** 0.5, rtol=1e-2)
