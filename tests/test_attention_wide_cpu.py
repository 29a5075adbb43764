"""The wide-head (D > 128) attention backward (`ops.attention._bwd_wide_own`: batched GEMMs on the
framework's assembly kernel on the GPU, the same contract in PyTorch on the CPU): from O and the
log-sum-exp it matches autograd through the reference (causal, GQA, additive mask, query chunks,
sequence / head-dim padding)."""
import math

import pytest
import torch

from paddle_infer_amd.ops.attention import _bwd_wide_own, attention_reference


@pytest.mark.parametrize("causal,hq,hk,masked,chunk,S", [
    (True, 4, 4, False, 1 << 30, 150), (False, 4, 2, True, 5000, 150), (True, 6, 2, True, 300000, 150),
    (True, 2, 1, True, 5000, 300)])
def test_chunked_backward_matches_autograd(causal, hq, hk, masked, chunk, S):
    torch.manual_seed(0)
    B, Sq, Sk, D = 2, S, S, 200
    q = torch.randn(B, Sq, hq, D, dtype=torch.float64, requires_grad=True)
    k = torch.randn(B, Sk, hk, D, dtype=torch.float64, requires_grad=True)
    v = torch.randn(B, Sk, hk, D, dtype=torch.float64, requires_grad=True)
    mask = torch.randn(B, 1, Sq, Sk, dtype=torch.float64) if masked else None
    scale = 1 / math.sqrt(D)
    o = attention_reference(q, k, v, causal, scale, mask)
    do = torch.randn_like(o)
    o.backward(do)
    # forward log-sum-exp as the kernel writes it: [B, Hq, Sq], natural log
    kf = k.detach().transpose(1, 2).repeat_interleave(hq // hk, 1)
    s = torch.matmul(q.detach().transpose(1, 2), kf.transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask
    if causal:
        i, j = torch.arange(Sq)[:, None], torch.arange(Sk)[None, :]
        s = s.masked_fill(j > i + (Sk - Sq), float("-inf"))
    lse = torch.logsumexp(s, -1)
    dq, dk, dv = _bwd_wide_own(q.detach(), k.detach(), v.detach(), o.detach(), lse, do, causal,
                              scale, mask, chunk_bytes=chunk)
    for a, b in ((dq, q.grad), (dk, k.grad), (dv, v.grad)):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=2e-5)  # reference computes in f32
