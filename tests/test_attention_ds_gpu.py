"""Stored-dS flash-attention backward (flash_attn.h: bwd_dkdv_kernel<..., DS> writes dS,
bwd_dq_ds_kernel reads it back) against the recomputing dQ kernel and the fp32 reference: causal
with Sq == Sk, Sq > Sk and Sq < Sk (bottom-right aligned), odd lengths, GQA, additive mask,
dropout, head dims 64 / 96 / 128, bf16 and fp16."""
import math

import pytest
import torch

from test_attention_gpu import _check, _close, _ref, _run

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


def _both(monkeypatch, fn):
    from paddle_infer_amd.ops import attention as A
    monkeypatch.setattr(A, "DS_MAX_BYTES", 0)
    ref = fn()
    monkeypatch.setattr(A, "DS_MAX_BYTES", 8 << 30)
    return ref, fn()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [64, 96, 128])
@pytest.mark.parametrize("causal,Sq,Sk", [(True, 256, 256), (True, 300, 300), (True, 200, 330),
                                          (True, 330, 200), (False, 190, 250)])
def test_stored_ds_matches_recompute(monkeypatch, dtype, D, causal, Sq, Sk):
    from paddle_infer_amd.ops import flash_attention
    torch.manual_seed(3)
    B, Hq, Hk = 2, 4, 2
    q = torch.randn(B, Sq, Hq, D, device=DEV, dtype=dtype)
    k = torch.randn(B, Sk, Hk, D, device=DEV, dtype=dtype)
    v = torch.randn(B, Sk, Hk, D, device=DEV, dtype=dtype)
    sc = 1 / math.sqrt(D)
    f = lambda a, b, c: flash_attention(a, b, c, causal, sc)  # noqa: E731
    torch.manual_seed(4)
    (o0, do0, *g0), (o1, do1, *g1) = _both(monkeypatch, lambda: (torch.manual_seed(4), _run(q, k, v, f, dtype, D))[1])
    assert torch.equal(o0, o1) and torch.equal(do0, do1)
    # dK / dV come from the same kernel either way; dQ from the stored 16-bit dS (the values the
    # recomputing kernel also rounds to before its MFMA)
    assert torch.equal(g0[1], g1[1]) and torch.equal(g0[2], g1[2])
    _close(g1[0], g0[0], 1e-2 if dtype == torch.bfloat16 else 2e-3, 1e-2, what="dq ds vs recompute")
    _check(o1, do1, g1, q, k, v, lambda a, b, c: _ref(a, b, c, causal, sc), dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_stored_ds_mask_and_dropout(monkeypatch, dtype):
    from paddle_infer_amd.framework import random as R
    from paddle_infer_amd.ops import flash_attention
    torch.manual_seed(5)
    B, S, H, D, p = 2, 192, 4, 128, 0.2
    q = torch.randn(B, S, H, D, device=DEV, dtype=dtype)
    k = torch.randn(B, S, H, D, device=DEV, dtype=dtype)
    v = torch.randn(B, S, H, D, device=DEV, dtype=dtype)
    mask = (torch.randn(B, H, S, S, device=DEV) * 2).to(dtype)
    sc = 1 / math.sqrt(D)
    st = R.get_rng_state()

    def run():
        R.set_rng_state(st)
        torch.manual_seed(6)
        return _run(q, k, v, lambda a, b, c: flash_attention(a, b, c, True, sc, attn_mask=mask, dropout_p=p),
                    dtype, D)

    (o0, _, *g0), (o1, _, *g1) = _both(monkeypatch, run)
    assert torch.equal(o0, o1)
    assert torch.equal(g0[1], g1[1]) and torch.equal(g0[2], g1[2])
    _close(g1[0], g0[0], 1e-2 if dtype == torch.bfloat16 else 2e-3, 1e-2, what="dq ds vs recompute")


def test_ds_bytes_layout():
    from paddle_infer_amd.ops.attention import _ds_bytes
    # B96 S1024 H16 (the GPT-3 1.3B bench step): 32 x 32 blocks of 2 KiB per (batch, head)
    assert _ds_bytes(96, 16, 1024, 1024) == 96 * 16 * 32 * 32 * 2048
    assert _ds_bytes(1, 1, 970, 130) == 1 * 1 * 32 * 8 * 2048
