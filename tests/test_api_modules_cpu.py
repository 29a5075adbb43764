"""Paddle API modules beyond the core (reference `python/paddle/{fft,signal,distribution,sparse,
geometric,text,audio,regularizer,reader,hub,sysconfig,quantization}`, `nn/quant`,
`incubate/{autograd,optimizer,asp,tensor}`): numerics against numpy / scipy / closed forms."""
import math
import os

import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle


def test_fft_matches_numpy():
    x = np.random.RandomState(0).randn(4, 16)
    t = torch.from_numpy(x)
    np.testing.assert_allclose(paddle.fft.fft(t).numpy(), np.fft.fft(x), atol=1e-10)
    np.testing.assert_allclose(paddle.fft.rfft2(t, norm="ortho").numpy(), np.fft.rfft2(x, norm="ortho"), atol=1e-10)
    np.testing.assert_allclose(paddle.fft.ihfft(t).numpy(), np.fft.ihfft(x), atol=1e-10)
    np.testing.assert_allclose(paddle.fft.fftshift(t).numpy(), np.fft.fftshift(x))
    np.testing.assert_allclose(paddle.fft.fftfreq(8, 0.5).numpy(), np.fft.fftfreq(8, 0.5))
    with pytest.raises(ValueError):
        paddle.fft.fft(t, norm="bad")


def test_signal_frame_overlap_add_stft_roundtrip():
    x = torch.arange(10.0)
    f = paddle.signal.frame(x, 4, 2)
    assert f.shape == (4, 4) and torch.equal(f[:, 1], torch.tensor([2.0, 3, 4, 5]))
    assert paddle.signal.frame(x.reshape(10, 1), 4, 2, axis=0).shape == (4, 4, 1)
    oa = paddle.signal.overlap_add(torch.ones(4, 3), 2)
    assert torch.equal(oa, torch.tensor([1.0, 1, 2, 2, 2, 2, 1, 1]))
    s = torch.randn(2, 512, dtype=torch.float64)
    w = torch.hann_window(64, dtype=torch.float64)
    spec = paddle.signal.stft(s, 64, 16, window=w)
    back = paddle.signal.istft(spec, 64, 16, window=w, length=512)
    assert torch.allclose(back, s, atol=1e-8)


def test_distributions():
    D = paddle.distribution
    n = D.Normal(torch.tensor([0.0, 1.0]), torch.tensor([1.0, 2.0]))
    assert n.sample([5]).shape == (5, 2)
    assert torch.allclose(n.log_prob(torch.tensor([0.0, 1.0])),
                          torch.tensor([-0.5 * math.log(2 * math.pi), -0.5 * math.log(2 * math.pi) - math.log(2)]))
    kl = D.kl_divergence(D.Normal(0.0, 1.0), D.Normal(1.0, 2.0))
    assert abs(float(kl) - (math.log(2) + (1 + 1) / 8 - 0.5)) < 1e-6
    u = D.Uniform(0.0, 2.0)
    assert float(u.log_prob(torch.tensor(3.0))) == float("-inf")
    c = D.Categorical(torch.tensor([1.0, 3.0]))
    assert abs(float(c.probs(torch.tensor(1))) - 0.75) < 1e-6
    b = D.Beta(2.0, 3.0)
    assert abs(float(b.mean) - 0.4) < 1e-6
    t = D.TransformedDistribution(D.Normal(0.0, 1.0), [D.ExpTransform()])
    assert abs(float(t.log_prob(torch.tensor(1.0))) - float(D.Normal(0.0, 1.0).log_prob(torch.tensor(0.0)))) < 1e-6
    a = D.AffineTransform(torch.tensor(1.0), torch.tensor(2.0))
    assert float(a.inverse(a.forward(torch.tensor(3.0)))) == 3.0

    @D.register_kl(D.Beta, D.Beta)
    def _kl(p, q):
        return torch.tensor(42.0)
    assert float(D.kl_divergence(b, b)) == 42.0


def test_sparse_ops():
    sp = paddle.sparse
    x = sp.sparse_coo_tensor([[0, 1, 2], [1, 0, 2]], [4.0, 9.0, 16.0], [3, 3])
    assert torch.equal(sp.sqrt(x).to_dense(), torch.tensor([[0, 2.0, 0], [3, 0, 0], [0, 0, 4]]))
    d = torch.randn(3, 2)
    assert torch.allclose(sp.matmul(x, d), x.to_dense() @ d)
    csr = sp.sparse_csr_tensor([0, 1, 2, 3], [1, 0, 2], [4.0, 9.0, 16.0], [3, 3])
    assert torch.equal(csr.to_dense(), x.to_dense())
    assert torch.equal(sp.add(x, x).to_dense(), 2 * x.to_dense())
    m = sp.masked_matmul(torch.ones(3, 4), torch.ones(4, 3), x)
    assert torch.equal(m.to_dense(), 4 * (x.to_dense() != 0).float())
    assert torch.equal(sp.transpose(x, [1, 0]).to_dense(), x.to_dense().t())
    y = sp.nn.ReLU()(sp.sparse_coo_tensor([[0, 1], [0, 1]], [-1.0, 2.0], [2, 2]))
    assert torch.equal(y.to_dense(), torch.tensor([[0.0, 0], [0, 2]]))


def test_geometric_and_incubate_segments():
    G = paddle.geometric
    x = torch.tensor([[1.0, 2], [3, 4], [5, 6]])
    src, dst = torch.tensor([0, 1, 2, 0]), torch.tensor([1, 2, 1, 0])
    assert torch.equal(G.send_u_recv(x, src, dst, "max"), torch.tensor([[1.0, 2], [5, 6], [3, 4]]))
    assert torch.equal(G.send_u_recv(x, src, dst, "mean"), torch.tensor([[1.0, 2], [3, 4], [3, 4]]))
    assert torch.equal(G.send_uv(x, x, src, dst, "mul")[0], torch.tensor([3.0, 8]))
    seg = torch.tensor([0, 0, 1])
    assert torch.equal(paddle.incubate.segment_sum(x, seg), torch.tensor([[4.0, 6], [5, 6]]))
    s, d, nodes = G.reindex_graph(torch.tensor([0, 5]), torch.tensor([5, 9, 0]), torch.tensor([2, 1]))
    assert s.tolist() == [1, 2, 0] and d.tolist() == [0, 0, 1] and nodes.tolist() == [0, 5, 9]
    row, colptr = torch.tensor([1, 2, 0, 2, 0]), torch.tensor([0, 2, 4, 5])
    nb, cnt = G.sample_neighbors(row, colptr, torch.tensor([0, 1]), sample_size=1)
    assert cnt.tolist() == [1, 1]


def test_text_viterbi_bruteforce():
    torch.manual_seed(0)
    B, T, N = 2, 4, 3
    pot, trans = torch.randn(B, T, N), torch.randn(N, N)
    lengths = torch.tensor([4, 2])
    scores, paths = paddle.text.viterbi_decode(pot, trans, lengths, include_bos_eos_tag=False)
    import itertools
    for b in range(B):
        L = int(lengths[b])
        best = max(itertools.product(range(N), repeat=L),
                   key=lambda p: sum(pot[b, t, p[t]] for t in range(L)) + sum(trans[p[t], p[t + 1]] for t in range(L - 1)))
        assert paths[b, :L].tolist() == list(best)


def test_audio_features_against_formulas(tmp_path):
    A = paddle.audio
    assert abs(A.functional.hz_to_mel(1000.0) - 15.0) < 1e-9
    assert abs(A.functional.mel_to_hz(A.functional.hz_to_mel(3000.0)) - 3000.0) < 1e-6
    fb = A.functional.compute_fbank_matrix(16000, 512, 40)
    assert fb.shape == (40, 257) and (fb >= 0).all()
    dct = A.functional.create_dct(13, 40)
    assert torch.allclose(dct.t() @ dct, torch.eye(13), atol=1e-5)
    x = torch.randn(2, 4000)
    assert A.features.MFCC(sr=16000, n_mfcc=13)(x).shape[1] == 13
    f = os.path.join(tmp_path, "a.wav")
    A.save(f, x[:1].clamp(-1, 1), 16000)
    w, sr = A.load(f)
    assert sr == 16000 and torch.allclose(w, x[:1].clamp(-1, 1), atol=1e-4)


def test_reader_decorators_and_misc():
    r = lambda: iter(range(7))  # noqa: E731
    assert list(paddle.batch(r, 3)()) == [[0, 1, 2], [3, 4, 5], [6]]
    R = paddle.reader
    assert list(R.firstn(R.map_readers(lambda a: a * 2, r), 3)()) == [0, 2, 4]
    assert sorted(R.shuffle(r, 3)()) == list(range(7))
    assert list(R.buffered(r, 2)()) == list(range(7))
    assert list(R.compose(r, r)())[1] == (1, 1)
    assert os.path.exists(os.path.join(paddle.sysconfig.get_include(), "common.h"))
    assert paddle.regularizer.L2Decay(0.1)._coeff == 0.1


def test_hub_local(tmp_path):
    (tmp_path / "hubconf.py").write_text("def tiny(k=1):\n    '''doc'''\n    return k * 2\n")
    assert "tiny" in paddle.hub.list(str(tmp_path), source="local")
    assert paddle.hub.load(str(tmp_path), "tiny", source="local", k=3) == 6
    with pytest.raises(RuntimeError):
        paddle.hub.list("x/y", source="github")


def test_incubate_autograd_optimizer_asp():
    ia = paddle.incubate.autograd
    J = ia.Jacobian(lambda a: a ** 2, torch.tensor([1.0, 3.0]))
    assert torch.equal(J[:], torch.diag(torch.tensor([2.0, 6.0])))
    H = ia.Hessian(lambda a: (a ** 3).sum(), torch.tensor([1.0, 2.0]))
    assert torch.equal(H[:], torch.diag(torch.tensor([6.0, 12.0])))
    _, g = ia.vjp(lambda a: a * 3, torch.ones(2))
    assert torch.equal(g, torch.full((2,), 3.0))
    ok, n, xopt, f, grad = paddle.incubate.optimizer.minimize_lbfgs(lambda x: ((x - 2) ** 2).sum(), torch.zeros(3))
    assert torch.allclose(xopt, torch.full((3,), 2.0), atol=1e-4)
    lin = paddle.nn.Linear(8, 8)
    opt = paddle.incubate.asp.decorate(paddle.optimizer.SGD(0.1, parameters=lin.parameters()))
    lin2 = paddle.nn.Linear(8, 8)
    paddle.incubate.asp.prune_model(lin2, mask_algo="mask_2d_greedy")
    assert 0.375 <= paddle.incubate.asp.calculate_density(lin2.weight) <= 0.5
    paddle.incubate.asp.prune_model(lin, mask_algo="mask_1d")
    assert paddle.incubate.asp.calculate_density(lin.weight) == 0.5
    lin(torch.randn(4, 8)).sum().backward()
    opt.step()
    w = lin.weight.detach().t().reshape(8, 2, 4)
    assert ((w != 0).sum(-1) <= 2).all()
    la = paddle.incubate.LookAhead(paddle.optimizer.SGD(0.1, parameters=lin.parameters()), 0.5, 2)
    for _ in range(2):
        lin(torch.randn(4, 8)).sum().backward()
        la.step()
        la.clear_grad()


def test_quantization_qat_and_ptq():
    from paddle_infer_amd.quantization import (ImperativeQuantAware, ImperativePTQ, PTQConfig,
                                               AbsmaxQuantizer, PerChannelAbsmaxQuantizer)
    m = paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.ReLU(), paddle.nn.Linear(16, 4))
    x = torch.randn(6, 8)
    ref = m(x)
    q = ImperativeQuantAware(weight_quantize_type="channel_wise_abs_max",
                             activation_quantize_type="abs_max").quantize(m)
    y = q(x)
    assert type(q[0]).__name__ == "QuantizedLinear"
    assert (y - ref).abs().max() < 0.1 * ref.abs().max() + 0.05
    y.sum().backward()  # straight-through gradients reach the weights
    assert q[0].weight.grad is not None
    m2 = paddle.nn.Sequential(paddle.nn.Linear(8, 16))
    ptq = ImperativePTQ(PTQConfig(AbsmaxQuantizer(), PerChannelAbsmaxQuantizer()))
    mm = ptq.quantize(m2)
    mm(x)
    ptq.convert(mm)
    assert abs(mm[0]._quant_in_threshold[0] - float(x.abs().max())) < 1e-6
    fq = paddle.nn.quant.fake_quant_dequant(torch.tensor([0.5, -1.0]), torch.tensor(1.0), 8)
    assert torch.allclose(fq, torch.tensor([64 / 127, -1.0]))
