"""Transposed-weight cache and linear path vs fp32 PyTorch references (the GEMM kernels themselves:
tests/test_agemm_gpu.py, tests/test_gemm_own_gpu.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max err {err} > {tol}"


@pytest.mark.parametrize("R,C", [(2048, 6144), (200, 72), (64, 8)])
def test_transpose_bf16(R, C):
    from paddle_infer_amd.ops import _lib
    w = torch.randn(R, C, device=DEV).bfloat16()
    out = torch.empty(C, R, device=DEV, dtype=torch.bfloat16)
    _lib.call("piamd_transpose_bf16", w.data_ptr(), out.data_ptr(), R, C, _lib.stream())
    assert torch.equal(out, w.t())


def test_linear_transposed_weight_cache():
    """Forward via the cached [out,in] copy == x @ W; the copy refreshes after in-place updates and
    after a flat-optimizer step (kernel writes do not bump autograd's version counter)."""
    from paddle_infer_amd.ops import linear as L
    x = torch.randn(2048, 256, device=DEV).bfloat16().requires_grad_()
    w = (0.05 * torch.randn(256, 512, device=DEV)).bfloat16().requires_grad_()
    b = torch.zeros(512, device=DEV).bfloat16().requires_grad_()
    y = L.linear(x, w, b)
    _close(y, x.float() @ w.float(), 0.02)
    y.float().sum().backward()
    _close(x.grad, torch.ones(2048, 512, device=DEV) @ w.float().t(), 0.5)
    with torch.no_grad():
        w.mul_(2.0)  # autograd-visible change
    _close(L.linear(x, w, b), x.float() @ w.float(), 0.04)
    with torch.no_grad():  # change behind autograd's back, then the epoch bump
        ptr = w.data_ptr()
        tmp = (w.float() * 0.5).bfloat16()
        from paddle_infer_amd.ops import _lib
        _lib.call("piamd_transpose_bf16", tmp.t().contiguous().data_ptr(), ptr, 512, 256, _lib.stream())
    L.bump_param_epoch()
    _close(L.linear(x, w, b), x.float() @ tmp.float(), 0.02)
