"""Strided conv data gradient helpers (ops/conv.py): the one-gather phase sub-filters against the
slice + flip construction they replace, for 1×1 / 3×3 / 7×7 filters, stride 2 and mixed strides,
padding and dilation; tapless phases are absent."""
import pytest
import torch


@pytest.mark.parametrize("K,C,R,S,st,pad,dil", [(64, 32, 3, 3, (2, 2), (1, 1), (1, 1)),
                                                 (16, 8, 1, 1, (2, 2), (0, 0), (1, 1)),
                                                 (8, 4, 7, 7, (2, 2), (3, 3), (1, 1)),
                                                 (8, 4, 3, 3, (2, 1), (2, 1), (2, 1)),
                                                 (4, 4, 5, 3, (3, 2), (2, 1), (1, 1))])
def test_phase_filters_match_slices(K, C, R, S, st, pad, dil):
    from paddle_infer_amd.ops import conv as oc
    torch.manual_seed(K + R)
    w = torch.randn(K, C, R, S)
    subs = oc._phase_filters(w, st, pad, dil)
    seen = 0
    for ph in range(st[0]):
        for pw in range(st[1]):
            th = oc._phase_taps(R, st[0], pad[0], dil[0], ph)
            tw = oc._phase_taps(S, st[1], pad[1], dil[1], pw)
            if th is None or tw is None:
                assert (ph, pw) not in subs
                continue
            ref = oc._take_ap(oc._take_ap(w, 2, th[0]), 3, tw[0]).permute(1, 2, 3, 0).contiguous()
            got = subs[(ph, pw)]
            assert got.is_contiguous() and torch.equal(got, ref), (ph, pw)
            seen += 1
    assert seen == len(subs) > 0
