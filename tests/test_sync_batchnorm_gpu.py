"""SyncBatchNorm's GPU kernels (`batchnorm.hip` piamd_bn_local_stats / piamd_bn_fwd3 with
cross-rank partials / piamd_bn_bwd_local_sums / piamd_bn_bwd_apply_sums) at world size 1 against
the fp32 PyTorch batch norm: statistics, output, input / affine gradients, running stats."""
import pytest
import torch

from paddle_infer_amd.ops import _lib
from paddle_infer_amd.ops.batchnorm import _SyncBN

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_fallback():
    _lib.lib()
    _lib.FALLBACKS.clear()
    yield


@pytest.mark.parametrize("fmt,dtype", [("NCHW", torch.float32), ("NHWC", torch.bfloat16),
                                       ("NHWC", torch.float32)])
def test_sync_bn_kernels_match_fp32(fmt, dtype):
    torch.manual_seed(0)
    C = 64
    shape = (8, C, 14, 14) if fmt == "NCHW" else (8, 14, 14, C)
    x = (torch.randn(*shape, device="cuda") * 2 + 5).to(dtype).requires_grad_(True)
    w = torch.linspace(0.5, 1.5, C, device="cuda").requires_grad_(True)
    b = torch.linspace(-1, 1, C, device="cuda").requires_grad_(True)
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y = _SyncBN.apply(x, w, b, rm, rv, 0.9, 1e-5, None, fmt == "NHWC")
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    rmr, rvr = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    xin = xr.movedim(-1, 1) if fmt == "NHWC" else xr
    yr = torch.nn.functional.batch_norm(xin, rmr, rvr, wr, br, True, 0.1, 1e-5)
    yr = yr.movedim(1, -1) if fmt == "NHWC" else yr
    yr.backward(dy.float())
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol)
    torch.testing.assert_close(w.grad, wr.grad, rtol=tol, atol=tol * 10)
    torch.testing.assert_close(b.grad, br.grad, rtol=tol, atol=tol * 10)
    torch.testing.assert_close(rm, rmr, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(rv, rvr, rtol=1e-3, atol=1e-3)
