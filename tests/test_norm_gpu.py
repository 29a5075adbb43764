"""LayerNorm / RMSNorm HIP kernels (layernorm.hip) vs plain PyTorch fp32: fp16 / bf16 / f32,
rows up to 16384 (LLaMA-13B 5120, 65B 8192), fused residual + RMSNorm, AMP-style f32 params over
16-bit activations. Every case also asserts the op stayed on the HIP path (no recorded fallback)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _hip_only():
    import paddle_infer_amd  # noqa: F401
    from paddle_infer_amd.ops import _lib
    _lib.lib()
    _lib.FALLBACKS.clear()
    yield
    assert not _lib.FALLBACKS, f"ops left the HIP path: {_lib.FALLBACKS}"


def _close(a, b, atol, rtol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max err {err} > {tol}"


def _tol(dtype):
    return {torch.bfloat16: 3e-2, torch.float16: 4e-3, torch.float32: 1e-4}[dtype]


def _rms_ref(h, w, eps):
    return h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * w


@pytest.mark.parametrize("N", [1024, 2048, 4096, 5120, 8192, 16384])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_layernorm_dtypes_wide(N, dtype):
    from paddle_infer_amd.ops import layer_norm
    rows = 96 if N > 4096 else 300
    x = torch.randn(rows, N, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(N, device=DEV)).to(dtype).requires_grad_()
    b = (0.1 * torch.randn(N, device=DEV)).to(dtype).requires_grad_()
    y = layer_norm(x, w, b, 1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    F.layer_norm(xr, (N,), wr, br, 1e-5).backward(dy.float())
    at = _tol(dtype)
    _close(y, F.layer_norm(xr.detach(), (N,), wr.detach(), br.detach(), 1e-5), at)
    _close(x.grad, xr.grad, at)
    _close(w.grad, wr.grad, at * 10, 3e-2)
    _close(b.grad, br.grad, at * 10, 3e-2)


@pytest.mark.parametrize("N", [2048, 5120, 8192])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_rms_norm(N, dtype):
    from paddle_infer_amd.ops import rms_norm
    x = torch.randn(200, N, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(N, device=DEV)).to(dtype).requires_grad_()
    y = rms_norm(x, w, 1e-6)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr = (t.detach().float().requires_grad_() for t in (x, w))
    yr = _rms_ref(xr, wr, 1e-6)
    yr.backward(dy.float())
    at = _tol(dtype)
    _close(y, yr, at)
    _close(x.grad, xr.grad, at)
    _close(w.grad, wr.grad, at * 10, 3e-2)


@pytest.mark.parametrize("N", [4096, 5120])
def test_fused_add_rms_norm(N):
    from paddle_infer_amd.ops import fused_add_rms_norm
    dt = torch.bfloat16
    x = torch.randn(2, 64, N, device=DEV, dtype=dt, requires_grad=True)
    r = torch.randn_like(x, requires_grad=True)
    w = (1 + 0.1 * torch.randn(N, device=DEV)).to(dt).requires_grad_()
    y, h = fused_add_rms_norm(x, r, w, 1e-6)
    dy, dh = torch.randn_like(y), torch.randn_like(h)
    torch.autograd.backward([y, h], [dy, dh])
    xr, rr, wr = (t.detach().float().requires_grad_() for t in (x, r, w))
    hr = xr + rr
    yr = _rms_ref(hr, wr, 1e-6)
    torch.autograd.backward([yr, hr], [dy.float(), dh.float()])
    _close(y, yr, 3e-2)
    _close(h, hr, 3e-2)
    _close(x.grad, xr.grad, 5e-2)
    _close(r.grad, rr.grad, 5e-2)
    _close(w.grad, wr.grad, 1.0, 3e-2)


def test_fused_add_layernorm_fp16_wide_dropout_consistent():
    """fp16, N = 5120 (workgroup-per-row kernels) with dropout: h - residual is exactly
    0 or x / (1 - p), and the backward regenerates the same mask."""
    from paddle_infer_amd.ops import fused_add_layer_norm
    N, p = 5120, 0.25
    x = torch.randn(64, N, device=DEV, dtype=torch.float16, requires_grad=True)
    r = torch.zeros_like(x)
    y, h = fused_add_layer_norm(x, r, None, None, 1e-5, None, p)
    kept = h != 0
    frac = kept.float().mean().item()
    assert abs(frac - (1 - p)) < 0.02, frac
    _close(h[kept], (x.detach() / (1 - p))[kept], 2e-3)
    h.backward(torch.ones_like(h))
    g = x.grad
    nz = x.detach() != 0  # an exact fp16 zero in x is "dropped-looking" in h whatever the mask
    assert torch.equal((g != 0)[nz], kept[nz])


def test_layernorm_f32_params_bf16_activations():
    """AMP O1: LayerNorm weights stay f32 while activations are bf16 — still the HIP kernel."""
    from paddle_infer_amd.ops import layer_norm
    N = 2048
    x = torch.randn(128, N, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(N, device=DEV)).requires_grad_()
    b = (0.1 * torch.randn(N, device=DEV)).requires_grad_()
    y = layer_norm(x, w, b, 1e-5)
    assert y.dtype == torch.bfloat16
    y.float().sum().backward()
    assert w.grad.dtype == torch.float32 and b.grad.dtype == torch.float32
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    F.layer_norm(xr, (N,), wr, br, 1e-5).sum().backward()
    _close(w.grad, wr.grad, 0.5, 3e-2)
    _close(b.grad, br.grad, 0.5, 3e-2)


def test_unsupported_row_length_warns_once():
    from paddle_infer_amd.ops import layer_norm, _lib
    x = torch.randn(4, 20, device=DEV)
    with pytest.warns(RuntimeWarning, match="row length 20"):
        layer_norm(x, None, None)
    assert _lib.FALLBACKS.pop(("layer_norm", "row length 20 (kernel: multiple of 8, <= 16384)")) == 1
