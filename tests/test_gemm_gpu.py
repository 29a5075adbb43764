"""Hand-written MFMA GEMM (gemm.hip) vs fp32 PyTorch reference: all four operand layouts,
ragged M / N edges, bias+GELU epilogue with aux pre-activation, dGELU epilogue, f32 accumulate."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max err {err} > {tol}"


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (768, 1024, 512), (300, 260, 128)])
def test_gemm_layouts(ta, tb, M, N, K):
    from paddle_infer_amd.ops.gemm import gemm, supported
    a = torch.randn(K, M, device=DEV).bfloat16() if ta else torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16() if tb else torch.randn(K, N, device=DEV).bfloat16()
    if not supported(a, b, ta, tb):
        pytest.skip("shape outside the kernel contract")
    got = gemm(a, b, ta, tb)
    ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
    _close(got, ref, 0.05)


def test_gemm_epilogues():
    from paddle_infer_amd.ops.gemm import gemm
    M, N, K = 512, 768, 256
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (0.1 * torch.randn(K, N, device=DEV)).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    y = gemm(x, w, epi="bias_act", act="gelu_tanh", bias=bias, aux=aux)
    pre = x.float() @ w.float() + bias.float()
    _close(aux, pre, 0.05)
    _close(y, torch.nn.functional.gelu(pre, approximate="tanh"), 0.05)
    # dgelu epilogue: dX = (dY @ Wᵀ) ⊙ gelu'(aux)
    dy = torch.randn(M, K, device=DEV).bfloat16()
    w2 = (0.1 * torch.randn(N, K, device=DEV)).bfloat16()  # [out=N? no: W2 stored [N][K]] -> B_KC
    d = gemm(dy, w2, trans_b=True, epi="dact", act="gelu_tanh", aux=aux)
    h = aux.float().requires_grad_(True)
    g = torch.autograd.grad(torch.nn.functional.gelu(h, approximate="tanh").sum(), h)[0]
    _close(d, (dy.float() @ w2.float().t()) * g, 0.05)
    # f32 accumulate (weight gradient into main_grad): C += Aᵀ B
    acc = torch.randn(K, N, device=DEV)
    base = acc.clone()
    gemm(x, dy.new_empty(0) if False else y.new_tensor(y), trans_a=True, out=acc, accumulate=True)
    _close(acc, base + x.float().t() @ y.float(), 0.1)


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


# ---- pipelined kernel (gemm_pipe.hip) ---------------------------------------------------------
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 192), (296, 264, 320), (1032, 520, 128),
                                   (24, 1032, 256)])
def test_gemm_pipe_layouts(ta, tb, M, N, K):
    from paddle_infer_amd.ops.gemm import gemm, pipe_supported
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + K)
    a = torch.randn(K, M, device=DEV, generator=g).bfloat16() if ta else \
        torch.randn(M, K, device=DEV, generator=g).bfloat16()
    b = torch.randn(N, K, device=DEV, generator=g).bfloat16() if tb else \
        torch.randn(K, N, device=DEV, generator=g).bfloat16()
    assert pipe_supported(a, b, ta, tb)
    got = gemm(a, b, ta, tb, impl="pipe")
    ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
    _close(got, ref, 0.05)


def test_gemm_pipe_asymmetric_identity():
    """A = I, asymmetric B: catches a transposed C write (guide §3)."""
    from paddle_infer_amd.ops.gemm import gemm
    n = 256
    a = torch.eye(n, device=DEV).bfloat16()
    b = (torch.arange(n * n, device=DEV).float().view(n, n) % 251 - 125).bfloat16()
    for tb in (False, True):
        bb = b.t().contiguous() if tb else b
        got = gemm(a, bb, trans_b=tb, impl="pipe")
        assert torch.equal(got.float(), b.float())


@pytest.mark.parametrize("ks", [1, 2, 4])
@pytest.mark.parametrize("c_f32", [False, True])
def test_gemm_pipe_splitk_accumulate(ks, c_f32):
    """Weight-gradient form: C (+)= Aᵀ·B with both operands M/N-contiguous, split over K."""
    from paddle_infer_amd.ops.gemm import gemm
    T, K_in, N = 2048, 512, 768
    x = torch.randn(T, K_in, device=DEV).bfloat16()
    dy = torch.randn(T, N, device=DEV).bfloat16()
    acc = torch.randn(K_in, N, device=DEV)
    acc = acc if c_f32 else acc.bfloat16()
    base = acc.float().clone()
    gemm(x, dy, trans_a=True, out=acc, accumulate=True, ksplit=ks, impl="pipe")
    _close(acc, base + x.float().t() @ dy.float(), 0.5)


def test_gemm_pipe_epilogues():
    from paddle_infer_amd.ops.gemm import gemm
    M, N, K = 520, 768, 256
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (0.1 * torch.randn(N, K, device=DEV)).bfloat16()  # [out, in]: K-contiguous
    bias = torch.randn(N, device=DEV).bfloat16()
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    y = gemm(x, w, trans_b=True, epi="bias_act", act="gelu_tanh", bias=bias, aux=aux, impl="pipe")
    pre = x.float() @ w.float().t() + bias.float()
    _close(aux, pre, 0.05)
    _close(y, torch.nn.functional.gelu(pre, approximate="tanh"), 0.05)
    dy = torch.randn(M, K, device=DEV).bfloat16()
    w2 = (0.1 * torch.randn(K, N, device=DEV)).bfloat16()  # FFN2 weight [in=N, out=K] as [N][K]ᵀ
    d = gemm(dy, w2, epi="dact", act="gelu_tanh", aux=aux, impl="pipe")
    h = aux.float().requires_grad_(True)
    gd = torch.autograd.grad(torch.nn.functional.gelu(h, approximate="tanh").sum(), h)[0]
    _close(d, (dy.float() @ w2.float()) * gd, 0.05)
