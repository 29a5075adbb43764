"""beam_search_softmax semantics (reference `test_beam_search_softmax_op`-style): first step
expands only beam 0, log-softmax + running score, finished beams, early stop, history rewrite."""
import math

import torch

from paddle_infer_amd.ops.search import beam_search_softmax


def _inputs(bs=2, beam=3, V=11, max_seq=4, max_dec=5, step=1, seed=0):
    g = torch.Generator().manual_seed(seed)
    R = bs * beam
    return dict(
        logits=torch.randn(R, V, generator=g),
        cum_scores=torch.randn(R, generator=g),
        sequence_lengths=torch.full((R,), 3, dtype=torch.int32),
        stop_flags=torch.zeros(R, dtype=torch.bool),
        end_ids=torch.tensor([0], dtype=torch.int32),
        step_ids=torch.full((R,), step, dtype=torch.int32),
        last_cache_ids=torch.randint(0, V, (R, max_dec), generator=g, dtype=torch.int32),
        last_beam_offsets=torch.randint(0, beam, (bs, beam, max_seq + max_dec), generator=g,
                                        dtype=torch.int32),
        beam_size=beam, max_seq_len=max_seq, max_dec_len=max_dec)


def test_scores_and_parents_match_bruteforce():
    kw = _inputs()
    ids, cum, cache, offs, parent, stop, sl, st = beam_search_softmax(**kw)
    lp = torch.log_softmax(kw["logits"].double(), -1)
    beam = kw["beam_size"]
    for b in range(2):
        cand = (kw["cum_scores"][b * beam:(b + 1) * beam, None].double() + lp[b * beam:(b + 1) * beam]).reshape(-1)
        top = cand.topk(beam)
        for j in range(beam):
            o = b * beam + j
            assert math.isclose(float(cum[o]), float(top.values[j]), rel_tol=1e-5, abs_tol=1e-5)
            assert int(parent[o]) == int(top.indices[j]) // lp.shape[1]
            assert int(ids[o]) == int(top.indices[j]) % lp.shape[1]
            # history rewritten from the parent, this step's token at position `step`
            src = b * beam + int(parent[o])
            assert int(cache[o, 1]) == int(ids[o])
            assert int(cache[o, 0]) == int(kw["last_cache_ids"][src, 0])
            assert int(offs[b, j, 3]) == int(parent[o])


def test_first_step_uses_beam_zero_only():
    kw = _inputs(step=0)
    ids, cum, *_ , parent, stop, sl, st = beam_search_softmax(**kw)
    assert (parent == 0).all()


def test_finished_beam_early_stop_keeps_slot():
    kw = _inputs()
    kw["stop_flags"][1] = True
    ids, cum, cache, offs, parent, stop, sl, st = beam_search_softmax(**kw, early_stop=True)
    assert int(ids[1]) == 0 and int(parent[1]) == 1
    assert math.isclose(float(cum[1]), float(kw["cum_scores"][1]), rel_tol=1e-6)
    assert bool(stop[1])
    # the other slots of batch 0 come from live beams only
    assert int(parent[0]) != 1 and int(parent[2]) != 1
