"""Native token-window loader (csrc/runtime/dataloader.cc): determinism, rank sharding, epoch
coverage, resume. Data: a synthetic arange token file (window start identifies the sample)."""
import numpy as np
import pytest
import torch

from paddle_infer_amd.io import TokenDataLoader, write_token_file

S, B = 16, 4


@pytest.fixture
def tokfile(tmp_path):
    p = str(tmp_path / "tok.bin")
    write_token_file(p, np.arange(S * 64 + 1) % 60000)  # 64 windows
    return p


def _starts(batch):
    assert (batch[:, 1:] - batch[:, :-1] == 1).all()  # contiguous windows (+ shifted label)
    return [int(x) for x in batch[:, 0]]


def test_epoch_covers_all_windows_once(tokfile):
    L = TokenDataLoader(tokfile, S, B, seed=7)
    assert L.batches_per_epoch == 16
    seen = []
    for _ in range(16):
        seen += _starts(next(L))
    assert sorted(seen) == [i * S for i in range(64)]
    nxt = _starts(next(L))  # epoch 2 is a different permutation
    assert len(set(nxt)) == B
    L.close()


def test_deterministic_and_resume(tokfile):
    a = TokenDataLoader(tokfile, S, B, seed=3)
    seq = [next(a) for _ in range(6)]
    st = a.state_dict()
    after = next(a)
    b = TokenDataLoader(tokfile, S, B, seed=3)
    for x in seq[:3]:
        assert torch.equal(x, next(b))
    b.set_state_dict(st)
    assert torch.equal(after, next(b))
    c = TokenDataLoader(tokfile, S, B, seed=3, start_batch=6)
    assert torch.equal(after, next(c))
    d = TokenDataLoader(tokfile, S, B, seed=4)
    assert not torch.equal(seq[0], next(d))


def test_ranks_disjoint(tokfile):
    world = 4
    per = []
    for r in range(world):
        L = TokenDataLoader(tokfile, S, B, seed=11, rank=r, world_size=world)
        assert L.batches_per_epoch == 4
        s = []
        for _ in range(4):
            s += _starts(next(L))
        per.append(set(s))
    allw = set().union(*per)
    assert sum(len(x) for x in per) == len(allw) == 64


def test_uint32_tokens_and_errors(tmp_path):
    p = str(tmp_path / "t32.bin")
    write_token_file(p, np.arange(S * 8 + 1) + 100000, dtype=np.int32)
    L = TokenDataLoader(p, S, 2, dtype=np.int32)
    b = next(L)
    assert int(b.min()) >= 100000
    with pytest.raises(ValueError):
        TokenDataLoader(p, S, 64, dtype=np.int32)  # fewer windows than one batch
    with pytest.raises(FileNotFoundError):
        TokenDataLoader(str(tmp_path / "missing.bin"), S, 2)


@pytest.mark.gpu
def test_cuda_prefetch_path(tokfile):
    L = TokenDataLoader(tokfile, S, B, seed=5, device="cuda:0")
    H = TokenDataLoader(tokfile, S, B, seed=5)
    for _ in range(5):
        g = next(L)
        assert g.is_cuda
        assert torch.equal(g.cpu(), next(H))
