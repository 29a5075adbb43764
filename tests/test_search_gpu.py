"""beam_search_softmax HIP kernels (``search.hip``) against the PyTorch reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("beam", [1, 4, 8, 16])
@pytest.mark.parametrize("step", [0, 3])
@pytest.mark.parametrize("early_stop,penalty,fuse,dtype", [
    (False, 0.0, True, torch.float32), (True, 1.2, True, torch.float32),
    (False, 0.0, False, torch.float32), (True, 0.0, True, torch.bfloat16)])
def test_beam_search_softmax_matches_reference(beam, step, early_stop, penalty, fuse, dtype):
    from paddle_infer_amd.ops.search import beam_search_softmax
    torch.manual_seed(beam * 10 + step)
    bs, V, ms, md = 3, 50304, 16, 8
    R = bs * beam
    logits = torch.randn(R, V) * 3
    if not fuse:
        logits = torch.log_softmax(logits, -1)
    logits = logits.to(dtype).float().to(dtype)
    kw = dict(cum_scores=torch.randn(R), sequence_lengths=torch.randint(1, ms, (R,), dtype=torch.int32),
              stop_flags=torch.rand(R) < 0.25, end_ids=torch.tensor([2], dtype=torch.int32),
              step_ids=torch.full((R,), step, dtype=torch.int32),
              last_cache_ids=torch.randint(0, V, (R, md), dtype=torch.int32),
              last_beam_offsets=torch.randint(0, beam, (bs, beam, ms + md), dtype=torch.int32))
    if step == 0:
        kw["stop_flags"][:] = False
    args = dict(beam_size=beam, max_seq_len=ms, max_dec_len=md, fuse_softmax=fuse,
                early_stop=early_stop, length_penalty=penalty)
    ref = beam_search_softmax(logits, **kw, **args)
    got = beam_search_softmax(logits.cuda(), **{k: v.cuda() for k, v in kw.items()}, **args)
    names = ["ids", "cum", "cache", "offs", "parent", "stop", "sl", "st"]
    for n, a, b in zip(names, got, ref):
        a = a.cpu()
        if n == "cum":
            assert torch.allclose(a.float(), b.float(), atol=2e-3, rtol=1e-4), (n, a, b)
        else:
            assert torch.equal(a.to(b.dtype), b), (n, a, b)
