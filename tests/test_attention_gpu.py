"""Flash attention MFMA kernel (flash_attn.h) vs a plain PyTorch fp32 reference: bf16 / fp16,
head dims 64 / 80 (padded to 96) / 96 / 128, causal, GQA, additive + bool masks, and in-kernel
attention dropout (mask recovered from the kernel itself, then checked fwd + bwd)."""
import math

import pytest
import torch

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


def _close(a, b, atol, rtol=2e-2, what=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"{what} max err {err} > {tol}"


def _ref(q, k, v, causal, scale, mask=None, drop_keep=None, p=0.0):
    """fp32 attention on [B, S, H, D]; drop_keep: [B, H, Sq, Sk] bool dropout mask."""
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    Hq, Hk = qf.shape[1], kf.shape[1]
    if Hk != Hq:
        kf = kf.repeat_interleave(Hq // Hk, 1)
        vf = vf.repeat_interleave(Hq // Hk, 1)
    s = qf @ kf.transpose(-1, -2) * scale
    if mask is not None:
        s = s.masked_fill(~mask, float("-inf")) if mask.dtype == torch.bool else s + mask.float()
    if causal:
        Sq, Sk = s.shape[-2], s.shape[-1]
        i = torch.arange(Sq, device=s.device)[:, None]
        j = torch.arange(Sk, device=s.device)[None, :]
        s = s.masked_fill(j > i + (Sk - Sq), float("-inf"))
    pr = torch.softmax(s, -1).nan_to_num(0.0)
    if drop_keep is not None:
        pr = pr * drop_keep / (1 - p)
    return (pr @ vf).transpose(1, 2)


def _run(q, k, v, fn, dtype, D):
    qq, kk, vv = (t.detach().clone().requires_grad_() for t in (q, k, v))
    o = fn(qq, kk, vv)
    do = torch.randn_like(o)
    o.backward(do)
    return o, do, qq.grad, kk.grad, vv.grad


def _check(o, do, grads, q, k, v, ref_fn, dtype):
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = ref_fn(qr, kr, vr)
    orf.backward(do.float())
    at = 2e-2 if dtype == torch.bfloat16 else 4e-3
    _close(o, orf, at, what="o")
    for g, gr, n in zip(grads, (qr.grad, kr.grad, vr.grad), "qkv"):
        _close(g, gr, at * 2, 3e-2, what=f"d{n}")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [64, 80, 96, 128])
@pytest.mark.parametrize("causal", [False, True])
def test_flash_dtypes_headdims(dtype, D, causal):
    from paddle_infer_amd.ops import flash_attention
    torch.manual_seed(0)
    B, Sq, Sk, Hq, Hk = 2, 200, 200, 4, 2
    q = torch.randn(B, Sq, Hq, D, device=DEV, dtype=dtype)
    k = torch.randn(B, Sk, Hk, D, device=DEV, dtype=dtype)
    v = torch.randn(B, Sk, Hk, D, device=DEV, dtype=dtype)
    sc = 1 / math.sqrt(D)
    o, do, *g = _run(q, k, v, lambda a, b, c: flash_attention(a, b, c, causal, sc), dtype, D)
    _check(o, do, g, q, k, v, lambda a, b, c: _ref(a, b, c, causal, sc), dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", ["full", "bcast", "bool", "odd_sk"])
def test_flash_additive_mask(dtype, shape):
    from paddle_infer_amd.ops import flash_attention
    torch.manual_seed(1)
    B, Sq, H, D = 2, 160, 4, 128
    Sk = 190 if shape == "odd_sk" else 160
    q = torch.randn(B, Sq, H, D, device=DEV, dtype=dtype)
    k = torch.randn(B, Sk, H, D, device=DEV, dtype=dtype)
    v = torch.randn(B, Sk, H, D, device=DEV, dtype=dtype)
    if shape == "bool":
        mask = torch.rand(B, 1, Sq, Sk, device=DEV) > 0.3
        mask[..., 0] = True
    elif shape == "bcast":
        mask = (torch.randn(1, 1, Sq, Sk, device=DEV) * 2).to(dtype)
    else:
        mask = (torch.randn(B, H, Sq, Sk, device=DEV) * 2).to(dtype)
        mask[:, :, :, -7:] = float("-inf")
    sc = 1 / math.sqrt(D)
    o, do, *g = _run(q, k, v, lambda a, b, c: flash_attention(a, b, c, False, sc, attn_mask=mask),
                     dtype, D)
    _check(o, do, g, q, k, v, lambda a, b, c: _ref(a, b, c, False, sc, mask), dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
def test_flash_dropout_matches_reference_with_kernel_mask(dtype, causal):
    """V = identity reveals the kernel's dropout mask (o[q, key] = P * keep / (1-p) for Sk <= D);
    the same RNG state then drives a real call whose fwd + bwd must equal the fp32 reference
    under that mask — i.e. forward, dK/dV and dQ kernels regenerate one identical mask."""
    from paddle_infer_amd.framework import random as R
    from paddle_infer_amd.ops import flash_attention
    torch.manual_seed(2)
    B, S, H, D, p = 2, 128, 2, 128, 0.3
    q = torch.randn(B, S, H, D, device=DEV, dtype=dtype)
    k = torch.randn(B, S, H, D, device=DEV, dtype=dtype)
    v = torch.randn(B, S, H, D, device=DEV, dtype=dtype)
    eye = torch.eye(S, D, device=DEV, dtype=dtype)[None, :, None, :].expand(B, S, H, D).contiguous()
    sc = 1 / math.sqrt(D)
    st = R.get_rng_state()
    oid = flash_attention(q, k, eye, causal, sc, dropout_p=p)
    keep = (oid.float() != 0).permute(0, 2, 1, 3)[..., :S]  # [B, H, Sq, Sk]
    if causal:
        allowed = torch.ones(S, S, device=DEV).tril().bool()
        assert not keep[..., ~allowed].any()
        frac = keep[..., allowed].float().mean().item()
    else:
        frac = keep.float().mean().item()
    assert abs(frac - (1 - p)) < 0.03, frac
    R.set_rng_state(st)
    o, do, *g = _run(q, k, v, lambda a, b, c: flash_attention(a, b, c, causal, sc, dropout_p=p),
                     dtype, D)
    _check(o, do, g, q, k, v, lambda a, b, c: _ref(a, b, c, causal, sc, None, keep, p), dtype)
    # a fresh call (next RNG offset) draws a different mask
    oid2 = flash_attention(q, k, eye, causal, sc, dropout_p=p)
    keep2 = (oid2.float() != 0).permute(0, 2, 1, 3)[..., :S]
    assert (keep2 != keep).float().mean().item() > 0.2


def test_sdpa_mask_dropout_eval_is_identity_of_dropout():
    from paddle_infer_amd.nn import functional as F
    torch.manual_seed(3)
    q = torch.randn(2, 64, 4, 64, device=DEV, dtype=torch.bfloat16)
    mask = torch.randn(2, 1, 64, 64, device=DEV).bfloat16()
    a = F.scaled_dot_product_attention(q, q, q, mask, dropout_p=0.5, training=False)
    b = F.scaled_dot_product_attention(q, q, q, mask, dropout_p=0.0)
    assert torch.equal(a, b)


def test_varlen_masked_single_launch_matches_reference():
    from paddle_infer_amd.incubate.nn.functional import variable_length_memory_efficient_attention
    torch.manual_seed(4)
    B, H, S, D = 3, 4, 96, 128
    q = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16)
    lq = torch.tensor([96, 50, 7], device=DEV, dtype=torch.int32)
    mask = (torch.randn(B, 1, S, S, device=DEV)).bfloat16()
    for causal in (False, True):
        o = variable_length_memory_efficient_attention(q, k, v, lq, lq, mask, None, causal)
        for b in range(B):
            n = int(lq[b])
            r = _ref(q[b:b + 1, :, :n].transpose(1, 2), k[b:b + 1, :, :n].transpose(1, 2),
                     v[b:b + 1, :, :n].transpose(1, 2), causal, 1 / math.sqrt(D),
                     mask[b:b + 1, :, :n, :n]).transpose(1, 2)
            _close(o[b:b + 1, :, :n], r, 2e-2)
            assert n == S or o[b, :, n:].abs().max().item() == 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D,causal,masked", [(256, True, False), (256, False, True), (192, True, False)])
def test_flash_wide_head_dims(dtype, D, causal, masked):
    """Head dims 129..256: the wide forward kernel (D = 256, narrower heads zero-padded) and the
    backward from its log-sum-exp on the own batched assembly GEMMs — no op leaves the HIP path
    (the autouse fixture)."""
    from paddle_infer_amd.ops import _lib, flash_attention
    torch.manual_seed(1)
    B, Sq, Sk, Hq, Hk = 2, 150, 150, 4, 2
    q = torch.randn(B, Sq, Hq, D, device=DEV, dtype=dtype)
    k = torch.randn(B, Sk, Hk, D, device=DEV, dtype=dtype)
    v = torch.randn(B, Sk, Hk, D, device=DEV, dtype=dtype)
    mask = torch.randn(B, 1, Sq, Sk, device=DEV, dtype=dtype) if masked else None
    sc = 1 / math.sqrt(D)
    o, do, *g = _run(q, k, v, lambda a, b, c: flash_attention(a, b, c, causal, sc, attn_mask=mask),
                     dtype, D)
    _check(o, do, g, q, k, v, lambda a, b, c: _ref(a, b, c, causal, sc, mask), dtype)
