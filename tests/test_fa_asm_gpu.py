"""Hand-scheduled assembly flash-attention dK/dV and dQ kernels (csrc/asm/fa_gen.py, launched
from flash_attn.h `launch_bwd` through fa_asm_host.hip) against a plain PyTorch fp32 reference and
against the HIP kernels: causal / full, GQA, packed-QKV strides, several tiles per head."""
import ctypes
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _asm_loaded():
    from paddle_infer_amd.ops import _lib, attention
    _lib.lib()
    attention._fa_asm_load()
    assert _lib.lib().piamd_fa_asm_loaded() == 1
    _lib.call("piamd_fa_asm_enable", 7)
    yield
    _lib.call("piamd_fa_asm_enable", 7)


def _ref_grads(q, k, v, do, causal, scale):
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    Hq, Hk = q.shape[2], k.shape[2]
    kr = kf.transpose(1, 2).repeat_interleave(Hq // Hk, 1)
    vr = vf.transpose(1, 2).repeat_interleave(Hq // Hk, 1)
    s = qf.transpose(1, 2) @ kr.transpose(-1, -2) * scale
    if causal:
        S = s.shape[-1]
        i = torch.arange(S, device=s.device)
        s = s.masked_fill(i[None, :] > i[:, None], float("-inf"))
    o = (torch.softmax(s, -1) @ vr).transpose(1, 2)
    o.backward(do.float())
    return qf.grad, kf.grad, vf.grad


def _run(q, k, v, do, causal, scale, use_asm, with_o=False):
    from paddle_infer_amd.ops import _lib, attention
    _lib.call("piamd_fa_asm_enable", 7 if use_asm else 0)
    o, lse = attention._fwd(q, k, v, causal, scale)
    if with_o:
        torch.cuda.synchronize()
        return o, lse
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    B, S, Hq, D = q.shape
    a = attention._args(q, k, v, o, lse, causal, scale, None, 0.0, 0, 0, B, S, S, Hq, k.shape[2], D)
    applies = _lib.lib().piamd_fa_asm_applies(ctypes.byref(a))
    attention._bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale)
    torch.cuda.synchronize()
    return dq, dk, dv, applies


def _close(a, b, what):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = 4e-2 + 3e-2 * b.abs().max().item()
    assert err <= tol, f"{what}: max err {err} > {tol}"


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("B,S,Hq,Hk", [(2, 256, 4, 4), (1, 512, 4, 2), (3, 256, 2, 1), (1, 1024, 2, 2)])
def test_dkdv_asm_matches_reference(causal, B, S, Hq, Hk):
    torch.manual_seed(0)
    D = 128
    q = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, S, Hk, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, S, Hk, D, device=DEV, dtype=torch.bfloat16)
    do = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16)
    sc = 1 / math.sqrt(D)
    dq, dk, dv, applies = _run(q, k, v, do, causal, sc, True)
    assert applies == 1, "the assembly dK/dV kernel must take this shape"
    rq, rk, rv = _ref_grads(q, k, v, do, causal, sc)
    _close(dk, rk, "dk")
    _close(dv, rv, "dv")
    _close(dq, rq, "dq")
    # against the HIP dK/dV kernel (same math, different schedule)
    hq, hk, hv, ap2 = _run(q, k, v, do, causal, sc, False)
    assert ap2 == 0
    _close(dk, hk, "dk vs HIP")
    _close(dv, hv, "dv vs HIP")
    _close(dq, hq, "dq vs HIP")


def test_dkdv_asm_packed_qkv_strides():
    """q / k / v as views of one fused [B, S, 3, H, D] projection output (the GPT layout)."""
    torch.manual_seed(1)
    B, S, H, D = 2, 512, 4, 128
    qkv = torch.randn(B, S, 3, H, D, device=DEV, dtype=torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    do = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    sc = 1 / math.sqrt(D)
    from paddle_infer_amd.ops import _lib, attention
    _lib.call("piamd_fa_asm_enable", 7)
    o, lse = attention._fwd(q, k, v, True, sc)
    dqkv = torch.empty_like(qkv)
    attention._bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], True, sc)
    torch.cuda.synchronize()
    rq, rk, rv = _ref_grads(q, k, v, do, True, sc)
    _close(dqkv[:, :, 1], rk, "dk")
    _close(dqkv[:, :, 2], rv, "dv")
    _close(dqkv[:, :, 0], rq, "dq")


def test_dkdv_asm_declines_other_shapes():
    """D = 64 and Sq % 256 != 0 stay on the HIP kernels."""
    from paddle_infer_amd.ops import _lib, attention
    q = torch.randn(1, 200, 2, 128, device=DEV, dtype=torch.bfloat16)
    o = torch.empty_like(q)
    lse = torch.empty(1, 2, 200, device=DEV)
    a = attention._args(q, q, q, o, lse, True, 0.1, None, 0.0, 0, 0, 1, 200, 200, 2, 2, 128)
    assert _lib.lib().piamd_fa_asm_applies(ctypes.byref(a)) == 0
    q2 = torch.randn(1, 256, 2, 64, device=DEV, dtype=torch.bfloat16)
    a = attention._args(q2, q2, q2, q2, lse, True, 0.1, None, 0.0, 0, 0, 1, 256, 256, 2, 2, 64)
    assert _lib.lib().piamd_fa_asm_applies(ctypes.byref(a)) == 0


def _ref_fwd(q, k, v, causal, scale):
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    Hq, Hk = q.shape[2], k.shape[2]
    kf = kf.repeat_interleave(Hq // Hk, 1)
    vf = vf.repeat_interleave(Hq // Hk, 1)
    s = qf @ kf.transpose(-1, -2) * scale
    if causal:
        S = s.shape[-1]
        i = torch.arange(S, device=s.device)
        s = s.masked_fill(i[None, :] > i[:, None], float("-inf"))
    return (torch.softmax(s, -1) @ vf).transpose(1, 2), torch.logsumexp(s, -1)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("B,S,Hq,Hk", [(2, 256, 4, 4), (1, 512, 4, 2), (1, 1024, 2, 2)])
def test_fwd_asm_matches_reference(causal, B, S, Hq, Hk):
    """Assembly forward (O and lse) against fp32 PyTorch and the HIP forward kernel."""
    torch.manual_seed(3)
    D = 128
    q = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, S, Hk, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, S, Hk, D, device=DEV, dtype=torch.bfloat16)
    sc = 1 / math.sqrt(D)
    o, lse = _run(q, k, v, None, causal, sc, True, with_o=True)
    ro, rl = _ref_fwd(q, k, v, causal, sc)
    _close(o, ro, "o")
    torch.testing.assert_close(lse, rl, rtol=1e-3, atol=2e-3)
    ho, hl = _run(q, k, v, None, causal, sc, False, with_o=True)
    _close(o, ho, "o vs HIP")
    torch.testing.assert_close(lse, hl, rtol=1e-3, atol=2e-3)


@pytest.mark.parametrize("causal", [True, False])
def test_fwd8_asm_matches_reference(causal):
    """The 8-wave forward variant (256 queries per workgroup; piamd_fa_fwd_nw(8))."""
    from paddle_infer_amd.ops import _lib
    _lib.call("piamd_fa_fwd_nw", 8)
    try:
        test_fwd_asm_matches_reference(causal, 1, 1024, 2, 2)
        test_fwd_asm_matches_reference(causal, 2, 512, 4, 2)
    finally:
        _lib.call("piamd_fa_fwd_nw", 4)
