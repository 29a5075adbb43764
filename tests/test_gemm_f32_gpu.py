"""fp32 GEMMs on the framework's own kernels (split-bf16 products, `ops/gemm.py gemm_nt_f32` /
`wgrad_f32` / fp32 `bmm`, and AMP O1 casting in the matmul dispatcher) against plain PyTorch fp32
references: `paddle.matmul` forward + backward, batched / transposed matmuls, fp32 `nn.Linear`
training (forward, data and weight gradients), `fc` / `matmul_v2` program ops, and `paddle.matmul`
under `paddle.amp.auto_cast` (O1). The autouse fixture asserts nothing left the HIP path."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _no_fallback():
    from paddle_infer_amd.ops import _lib
    _lib.FALLBACKS.clear()
    yield
    assert not _lib.FALLBACKS, f"ops left the HIP path: {_lib.FALLBACKS}"


def _rel(got, ref):
    got, ref = got.double(), ref.double()
    return ((got - ref).abs().max() / ref.abs().max().clamp_min(1e-12)).item()


def _r(*s, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed + sum(s))
    return torch.randn(*s, device=DEV, generator=g)


@pytest.mark.parametrize("M,N,K", [(8, 64, 128), (100, 96, 72), (300, 520, 200), (2048, 1024, 1024),
                                   (4096, 3000, 1000)])
def test_gemm_nt_f32(M, N, K):
    from paddle_infer_amd.ops.gemm import gemm_nt_f32
    a, b = _r(M, K), _r(N, K, seed=1)
    y = gemm_nt_f32(a, b)
    assert y.dtype == torch.float32 and y.shape == (M, N)
    assert _rel(y, a @ b.t()) < 1e-4


@pytest.mark.parametrize("T,K,N", [(128, 64, 64), (1000, 96, 200), (8192, 1024, 1024)])
def test_wgrad_f32(T, K, N):
    from paddle_infer_amd.ops.gemm import wgrad_f32
    x, dy = _r(T, K), _r(T, N, seed=2)
    ref = x.t() @ dy
    assert _rel(wgrad_f32(x, dy), ref) < 1e-4
    acc = _r(K, N, seed=3)
    want = acc + ref
    wgrad_f32(x, dy, out=acc)
    assert _rel(acc, want) < 1e-4


@pytest.mark.parametrize("tx,ty", [(False, False), (False, True), (True, False), (True, True)])
def test_paddle_matmul_f32_autograd(tx, ty):
    import paddle_infer_amd as paddle
    M, K, N = 257, 192, 136
    x = _r(*((K, M) if tx else (M, K))).requires_grad_()
    y = _r(*((N, K) if ty else (K, N)), seed=4).requires_grad_()
    out = paddle.matmul(x, y, transpose_x=tx, transpose_y=ty)
    xr, yr = x.detach().clone().requires_grad_(), y.detach().clone().requires_grad_()
    ref = (xr.t() if tx else xr) @ (yr.t() if ty else yr)
    assert _rel(out, ref) < 1e-4
    g = _r(M, N, seed=5)
    gx, gy = torch.autograd.grad(out, (x, y), g)
    rx, ry = torch.autograd.grad(ref, (xr, yr), g)
    assert _rel(gx, rx) < 1e-4 and _rel(gy, ry) < 1e-4


@pytest.mark.parametrize("shape_x,shape_y,ty", [((4, 100, 64), (4, 64, 72), False), ((3, 65, 48), (48, 96), False),
                                                ((2, 5, 130, 64), (2, 5, 80, 64), True)])
def test_paddle_bmm_f32(shape_x, shape_y, ty):
    import paddle_infer_amd as paddle
    x, y = _r(*shape_x), _r(*shape_y, seed=6)
    out = paddle.matmul(x, y, transpose_y=ty)
    ref = torch.matmul(x, y.transpose(-1, -2) if ty else y)
    assert out.shape == ref.shape and _rel(out, ref) < 1e-4


def test_linear_f32_training():
    import paddle_infer_amd as paddle
    torch.manual_seed(0)
    with torch.device(DEV):
        lin = paddle.nn.Linear(96, 160)
    x = _r(2, 300, 96).requires_grad_()
    y = lin(x)
    w, b = lin.weight.detach().clone().requires_grad_(), lin.bias.detach().clone().requires_grad_()
    xr = x.detach().clone().requires_grad_()
    ref = xr @ w + b
    assert _rel(y, ref) < 1e-4
    g = _r(2, 300, 160, seed=7)
    y.backward(g)
    ref.backward(g)
    assert _rel(x.grad, xr.grad) < 1e-4
    assert _rel(lin.weight.grad, w.grad) < 1e-4
    assert _rel(lin.bias.grad, b.grad) < 1e-5


def test_static_fc_matmul_v2_f32():
    from paddle_infer_amd.static.ops_registry import REGISTRY
    x, w, b = _r(64, 128), _r(128, 96, seed=8), _r(96, seed=9)
    out = REGISTRY["matmul_v2"]({"X": [x], "Y": [w]}, {"trans_x": False, "trans_y": False})["Out"]
    assert _rel(out, x @ w) < 1e-4
    out = REGISTRY["fc"]({"Input": [x], "W": [w], "Bias": [b]}, {"in_num_col_dims": 1, "activation_type": "relu"})["Out"]
    assert _rel(out, torch.relu(x @ w + b)) < 1e-4


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_paddle_matmul_amp_o1(dtype):
    import paddle_infer_amd as paddle
    x, w = _r(512, 256).requires_grad_(), _r(256, 384, seed=10).requires_grad_()
    with paddle.amp.auto_cast(level="O1", dtype=dtype):
        y = paddle.matmul(x, w)
    assert y.dtype == getattr(torch, dtype)
    dt = getattr(torch, dtype)
    ref = x.detach().to(dt).float() @ w.detach().to(dt).float()
    assert _rel(y.float(), ref) < 1e-2
    y.float().sum().backward()
    assert x.grad is not None and x.grad.dtype == torch.float32 and w.grad.dtype == torch.float32
    assert _rel(w.grad, x.detach().to(dt).float().t() @ torch.ones(512, 384, device=DEV)) < 2e-2
