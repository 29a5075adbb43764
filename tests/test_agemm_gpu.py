"""Assembly GEMM (`csrc/asm/gemm_gen.py`) against fp32 PyTorch references: every operand layout,
plain / accumulate / split-K / fused epilogues, edge tiles, the persistent and one-tile kernels, and
the fused MLP (bias+GELU in the FFN1 epilogue, GELU backward in the FFN2 dgrad epilogue)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b, ta, tb):
    A = a.t() if ta else a
    B = b.t() if tb else b
    return A.float() @ B.float()


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (304, 264, 192), (1000, 1008, 448),
                                   (512, 768, 512), (4352, 4104, 256)])
@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (False, False), (True, True)])
@pytest.mark.parametrize("kind", ["bf16", "bf16acc", "f32", "f32acc"])
def test_asm_gemm_layouts(M, N, K, ta, tb, kind):
    from paddle_infer_amd.ops.gemm import asm_gemm
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn((K, M) if ta else (M, K), device="cuda", generator=g).bfloat16()
    b = torch.randn((N, K) if tb else (K, N), device="cuda", generator=g).bfloat16()
    r = _ref(a, b, ta, tb)
    if kind in ("bf16acc", "f32acc"):
        c0 = torch.randn(M, N, device="cuda", generator=g)
        c = c0.bfloat16() if kind == "bf16acc" else c0.clone()
        r = r + c.float()
        asm_gemm(a, b, ta, tb, out=c, accumulate=True)
    else:
        c = asm_gemm(a, b, ta, tb, out_f32=kind == "f32")
    err = (c.float() - r).abs().max().item()
    tol = 0.01 * r.abs().max().item() if kind.startswith("bf16") else 2e-3 * K ** 0.5
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("ks,kind", [(4, "f32acc"), (2, "bf16acc")])
def test_asm_gemm_splitk_wgrad(ks, kind):
    from paddle_infer_amd.ops.gemm import asm_gemm
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(2048, 512, device="cuda", generator=g).bfloat16()
    dy = torch.randn(2048, 768, device="cuda", generator=g).bfloat16()
    out = torch.randn(512, 768, device="cuda", generator=g)
    out = out.bfloat16() if kind == "bf16acc" else out
    r = out.float() + x.float().t() @ dy.float()
    asm_gemm(x, dy, trans_a=True, out=out, accumulate=True, ksplit=ks)
    assert (out.float() - r).abs().max().item() <= 0.01 * r.abs().max().item()


@pytest.mark.parametrize("act", ["none", "gelu_tanh", "relu"])
def test_asm_gemm_fused_epilogues(act):
    from paddle_infer_amd.ops.activation import ACTS, _ref_act
    from paddle_infer_amd.ops.gemm import _act_grad_ref, asm_gemm
    g = torch.Generator(device="cuda").manual_seed(5)
    for M, N, K in ((512, 1024, 256), (304, 520, 192)):
        a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        b = (0.1 * torch.randn(N, K, device="cuda", generator=g)).bfloat16()
        bias = torch.randn(N, device="cuda", generator=g).bfloat16()
        r = a.float() @ b.float().t()
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        c = asm_gemm(a, b, trans_b=True, epi="bias_act", act=act, bias=bias, aux=aux)
        pre = (r + bias.float()).bfloat16()
        torch.testing.assert_close(aux.float(), pre.float(), rtol=0.02, atol=0.02)
        ref_c = _ref_act(pre.float(), ACTS[act])
        torch.testing.assert_close(c.float(), ref_c, rtol=0.02, atol=0.02)
        if act == "none":
            continue
        h = torch.randn(M, N, device="cuda", generator=g).bfloat16()
        d = asm_gemm(a, b, trans_b=True, epi="dact", act=act, aux=h)
        ref_d = r * _act_grad_ref(h, ACTS[act])
        torch.testing.assert_close(d.float(), ref_d, rtol=0.02, atol=0.02 * ref_d.abs().max().item())


def test_fused_mlp_matches_fp32_composition():
    from paddle_infer_amd.ops.linear import fused_mlp, fused_mlp_supported
    g = torch.Generator(device="cuda").manual_seed(11)
    T, H, Fd, O = 1024, 256, 1024, 256
    x = torch.randn(T, H, device="cuda", generator=g).bfloat16().requires_grad_(True)
    w1 = (0.05 * torch.randn(H, Fd, device="cuda", generator=g)).bfloat16().requires_grad_(True)
    b1 = (0.1 * torch.randn(Fd, device="cuda", generator=g)).bfloat16().requires_grad_(True)
    w2 = (0.05 * torch.randn(Fd, O, device="cuda", generator=g)).bfloat16().requires_grad_(True)
    assert fused_mlp_supported(x, w1, b1, w2, "gelu_tanh")
    m = fused_mlp(x, w1, b1, w2, "gelu_tanh")
    dm = torch.randn(T, O, device="cuda", generator=g).bfloat16()
    m.backward(dm)
    ref = [t.detach().float().requires_grad_(True) for t in (x, w1, b1, w2)]
    mr = torch.nn.functional.gelu(ref[0] @ ref[1] + ref[2], approximate="tanh") @ ref[3]
    mr.backward(dm.float())
    torch.testing.assert_close(m.float(), mr, rtol=0.03, atol=0.03 * mr.abs().max().item())
    for got, r in zip((x.grad, w1.grad, b1.grad, w2.grad), ref):
        torch.testing.assert_close(got.float(), r.grad, rtol=0.03, atol=0.03 * r.grad.abs().max().item())


def test_linear_training_uses_asm_and_matches():
    """paddle Linear fwd/bwd on the GPU runs the assembly kernels (no silent library fallback)."""
    import paddle_infer_amd as paddle
    from paddle_infer_amd.ops import linear as L
    assert L._GEMM_IMPL[0] == "asm"
    torch.manual_seed(0)
    lin = paddle.nn.Linear(512, 768)
    lin.to(device="cuda", dtype=torch.bfloat16)
    x = torch.randn(4, 256, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = lin(x)
    y.float().square().mean().backward()
    xr = x.detach().float().requires_grad_(True)
    wr = lin.weight.detach().float().requires_grad_(True)
    br = lin.bias.detach().float().requires_grad_(True)
    yr = xr @ wr + br
    yr.square().mean().backward()
    torch.testing.assert_close(y.float(), yr, rtol=0.02, atol=0.02)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=0.03, atol=1e-4)
    torch.testing.assert_close(lin.weight.grad.float(), wr.grad, rtol=0.03, atol=1e-3)


@pytest.mark.parametrize("act", ["gelu_tanh", "relu"])
@pytest.mark.parametrize("M,N,K", [(512, 1024, 256), (304, 520, 192), (1000, 776, 512), (2048, 1024, 128)])
def test_dact_epilogue_column_sums(act, M, N, K):
    """The *cs dact kernels: C = (A·Bᵀ) ⊙ act'(aux) unchanged, plus per-128-row-band column sums of C
    (persistent kernel: K/64 even ≥ 4; one-tile kernel otherwise; edge tiles in M and N)."""
    from paddle_infer_amd.ops.activation import ACTS
    from paddle_infer_amd.ops.gemm import _act_grad_ref, asm_gemm, colsum_parts
    g = torch.Generator(device="cuda").manual_seed(M + N)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (0.1 * torch.randn(N, K, device="cuda", generator=g)).bfloat16()
    h = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    cs = torch.full(((M + 127) // 128, N), float("nan"), device="cuda")
    d = asm_gemm(a, b, trans_b=True, epi="dact", act=act, aux=h, colsum=cs)
    ref_d = (a.float() @ b.float().t()) * _act_grad_ref(h, ACTS[act])
    torch.testing.assert_close(d.float(), ref_d, rtol=0.02, atol=0.02 * ref_d.abs().max().item())
    assert torch.isfinite(cs).all(), "every partial row / column must be written"
    bands = torch.stack([ref_d[i * 128:(i + 1) * 128].sum(0) for i in range(cs.shape[0])])
    torch.testing.assert_close(cs, bands, rtol=2e-3, atol=2e-3 * bands.abs().max().item())
    out = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
    colsum_parts(cs, out, accumulate=True)
    torch.testing.assert_close(out.float(), ref_d.sum(0), rtol=0.02, atol=0.02 * ref_d.sum(0).abs().max().item())
