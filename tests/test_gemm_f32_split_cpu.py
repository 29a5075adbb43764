"""Numerics model of the fp32 split-bf16 GEMM (`ops/gemm.py gemm_nt_f32`): x·w ≈ x_hi·w_hi +
x_lo·w_hi + x_hi·w_lo with t = bf16(t) + bf16(t − bf16(t)), emulated on the CPU exactly as the
kernel forms its operands (`piamd_split3_f32`), against fp64 — the bound the GPU tests assert."""
import pytest
import torch


def _split(t):
    hi = t.to(torch.bfloat16)
    return hi, (t - hi.float()).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (33, 70, 1000), (128, 96, 4096)])
@pytest.mark.parametrize("scale", [1.0, 1e-3, 1e4])
def test_three_product_split_error(M, N, K, scale):
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g) * scale
    w = torch.randn(N, K, generator=g)
    xh, xl = _split(x)
    wh, wl = _split(w)
    a3 = torch.cat([xh, xl, xh], 1).double()
    b3 = torch.cat([wh, wh, wl], 1).double()
    got = (a3 @ b3.t()).float()
    ref = x.double() @ w.double().t()
    rel = ((got.double() - ref).abs().max() / ref.abs().max()).item()
    assert rel < 2e-5, rel
    # the dropped x_lo·w_lo term is what the split gives up: one bf16 product alone is ~1e-2 off
    one = (xh.double() @ wh.double().t())
    assert ((one - ref).abs().max() / ref.abs().max()).item() > 50 * rel
