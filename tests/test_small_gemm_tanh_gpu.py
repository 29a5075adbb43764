"""tanh epilogue of the skinny GEMM (act code 5, skinny kernel only) behind the `fc` program op
with activation_type tanh (the BERT pooler), against the fp32 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(1, 1024, 1024), (128, 1024, 1024), (16, 1024, 4096)])
def test_small_gemm_tanh(dt, M, N, K):
    from paddle_infer_amd.ops import gemm as G
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device=DEV).to(dt)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(dt)
    b = (0.1 * torch.randn(N, device=DEV)).to(dt)
    y = G.small_gemm(x, w, bias=b, act="tanh")
    ref = torch.tanh(x.float() @ w.float().t() + b.float())
    assert (y.float() - ref).abs().max().item() < 2e-2


def test_fc_tanh_op_uses_the_epilogue():
    from paddle_infer_amd.static import ops_registry as R
    torch.manual_seed(0)
    x = torch.randn(4, 1024, device=DEV).half()
    w = (torch.randn(1024, 768, device=DEV) / 32).half()
    b = (0.1 * torch.randn(768, device=DEV)).half()
    assert R._tanh_small_ok(x, w, b)
    y = R.REGISTRY["fc"]({"Input": [x], "W": [w], "Bias": [b]}, {"activation_type": "tanh", "in_num_col_dims": 1})["Out"]
    ref = torch.tanh(x.float() @ w.float() + b.float())
    assert (y.float() - ref).abs().max().item() < 2e-2
