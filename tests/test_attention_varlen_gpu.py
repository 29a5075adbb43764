"""Variable-length (packed, cu_seqlens) flash attention (``flash_attn.hip`` varlen entry points)
against a per-sequence fp32 PyTorch reference: forward, backward, GQA, causal, ragged lengths,
and the padded ``variable_length_memory_efficient_attention`` API on top of it."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _close(a, b, atol, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    assert err <= atol + rtol * b.abs().max().item(), err


def _ref(q, k, v, cu_q, cu_k, causal, scale):
    from paddle_infer_amd.ops.attention import attention_reference
    cq, ck = cu_q.tolist(), cu_k.tolist()
    outs = []
    for i in range(len(cq) - 1):
        outs.append(attention_reference(q[cq[i]:cq[i + 1]][None].float(), k[ck[i]:ck[i + 1]][None].float(),
                                        v[ck[i]:ck[i + 1]][None].float(), causal, scale)[0])
    return torch.cat(outs, 0)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("hq,hk", [(4, 4), (4, 2)])
def test_varlen_fwd_bwd(D, causal, hq, hk):
    from paddle_infer_amd.ops import flash_attention_varlen
    torch.manual_seed(0)
    lens = [1, 200, 37, 129, 64]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = sum(lens)
    q = torch.randn(T, hq, D, device=DEV).bfloat16().requires_grad_(True)
    k = torch.randn(T, hk, D, device=DEV).bfloat16().requires_grad_(True)
    v = torch.randn(T, hk, D, device=DEV).bfloat16().requires_grad_(True)
    scale = 1.0 / math.sqrt(D)
    o = flash_attention_varlen(q, k, v, cu, cu, max(lens), max(lens), causal, scale)
    qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = _ref(qf, kf, vf, cu, cu, causal, scale)
    _close(o, ref, 2e-2)
    g = torch.randn_like(ref)
    got = torch.autograd.grad(o, (q, k, v), g.bfloat16())
    exp = torch.autograd.grad(ref, (qf, kf, vf), g)
    for a, b in zip(got, exp):
        _close(a, b, 5e-2)


def test_varlen_cross_lengths_and_padded_api():
    from paddle_infer_amd.incubate.nn.functional import variable_length_memory_efficient_attention
    from paddle_infer_amd.ops.attention import attention_reference
    torch.manual_seed(1)
    B, H, S, D = 3, 4, 96, 128
    q = torch.randn(B, H, S, D, device=DEV).bfloat16()
    k = torch.randn(B, H, S, D, device=DEV).bfloat16()
    v = torch.randn(B, H, S, D, device=DEV).bfloat16()
    lq = torch.tensor([96, 10, 50], device=DEV, dtype=torch.int32)
    lk = torch.tensor([96, 70, 50], device=DEV, dtype=torch.int32)
    out = variable_length_memory_efficient_attention(q, k, v, lq, lk, causal=True)
    for b in range(B):
        sq, sk = int(lq[b]), int(lk[b])
        r = attention_reference(q[b:b + 1, :, :sq].transpose(1, 2), k[b:b + 1, :, :sk].transpose(1, 2),
                                v[b:b + 1, :, :sk].transpose(1, 2), True).transpose(1, 2)
        _close(out[b:b + 1, :, :sq], r, 2e-2)
        assert out[b, :, sq:].abs().max().item() == 0.0 if sq < S else True
