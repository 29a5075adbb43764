"""Device Viterbi decoding (csrc/kernels/viterbi.hip, one launch) against the framework's CPU
dynamic programme (text.viterbi_decode on CPU tensors) — scores and paths, with and without the
BOS / EOS tags, ragged lengths."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bos_eos", [True, False])
@pytest.mark.parametrize("B,T,N", [(4, 17, 6), (3, 64, 40), (2, 5, 300)])
def test_viterbi_device_matches_cpu(bos_eos, B, T, N):
    from paddle_infer_amd.text import viterbi_decode
    g = torch.Generator().manual_seed(B * 1000 + T + N)
    pot = torch.randn(B, T, N, generator=g)
    trans = torch.randn(N, N, generator=g)
    lengths = torch.randint(1, T + 1, (B,), generator=g)
    lengths[0] = T
    s_ref, p_ref = viterbi_decode(pot, trans, lengths, bos_eos)
    s, p = viterbi_decode(pot.cuda(), trans.cuda(), lengths.cuda(), bos_eos)
    torch.testing.assert_close(s.cpu(), s_ref, rtol=1e-5, atol=1e-4)
    assert p.shape == p_ref.shape
    assert torch.equal(p.cpu(), p_ref)
