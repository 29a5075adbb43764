"""RNN cells / drivers / beam search (reference `python/paddle/nn/layer/rnn.py`,
`fluid/layers/rnn.py`; tests modelled on `unittests/rnn/test_rnn_nets.py`, `test_rnn_cells.py`,
`test_rnn_decode_api.py`): each cell against PyTorch's fp32 RNN of the same gate layout, masking by
``sequence_length``, BiRNN / multi-layer state layout, gather_tree and a BeamSearchDecoder run."""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import nn

torch.manual_seed(0)


def _copy_into_torch(cell, tmod, suffix="_l0"):
    with torch.no_grad():
        getattr(tmod, "weight_ih" + suffix).copy_(cell.weight_ih)
        getattr(tmod, "weight_hh" + suffix).copy_(cell.weight_hh)
        getattr(tmod, "bias_ih" + suffix).copy_(cell.bias_ih)
        getattr(tmod, "bias_hh" + suffix).copy_(cell.bias_hh)


@pytest.mark.parametrize("kind", ["lstm", "gru", "rnn_tanh", "rnn_relu"])
def test_single_layer_matches_torch(kind):
    B, T, I, H = 3, 7, 5, 6
    if kind == "lstm":
        ours, ref = nn.LSTM(I, H), torch.nn.LSTM(I, H, batch_first=True)
    elif kind == "gru":
        ours, ref = nn.GRU(I, H), torch.nn.GRU(I, H, batch_first=True)
    else:
        act = kind.split("_")[1]
        ours, ref = nn.SimpleRNN(I, H, activation=act), torch.nn.RNN(I, H, nonlinearity=act, batch_first=True)
    _copy_into_torch(ours.layers[0].cell, ref)
    x = torch.randn(B, T, I)
    y, st = ours(x)
    y_ref, st_ref = ref(x)
    torch.testing.assert_close(y, y_ref, atol=1e-5, rtol=1e-5)
    if kind == "lstm":
        torch.testing.assert_close(st[0], st_ref[0], atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(st[1], st_ref[1], atol=1e-5, rtol=1e-5)
    else:
        torch.testing.assert_close(st, st_ref, atol=1e-5, rtol=1e-5)


def test_bidirect_multilayer_lstm_matches_torch():
    B, T, I, H, L = 2, 5, 4, 3, 2
    ours = nn.LSTM(I, H, num_layers=L, direction="bidirect")
    ref = torch.nn.LSTM(I, H, num_layers=L, bidirectional=True, batch_first=True)
    for l in range(L):
        _copy_into_torch(ours.layers[l].cell_fw, ref, f"_l{l}")
        _copy_into_torch(ours.layers[l].cell_bw, ref, f"_l{l}_reverse")
    x = torch.randn(B, T, I)
    h0, c0 = torch.randn(2 * L, B, H), torch.randn(2 * L, B, H)
    y, (h, c) = ours(x, (h0, c0))
    y_ref, (h_ref, c_ref) = ref(x, (h0, c0))
    assert y.shape == (B, T, 2 * H) and h.shape == (2 * L, B, H)
    torch.testing.assert_close(y, y_ref, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(h, h_ref, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(c, c_ref, atol=1e-5, rtol=1e-5)


def test_sequence_length_masks_padding():
    """Outputs past each sequence's length are zero and the final state is the state at its last
    valid step — identical to running the unpadded sequence alone."""
    I, H, T = 4, 5, 6
    gru = nn.GRU(I, H, direction="bidirect")
    x = torch.randn(2, T, I)
    lens = torch.tensor([6, 3])
    y, h = gru(x, sequence_length=lens)
    assert torch.all(y[1, 3:] == 0)
    y1, h1 = gru(x[1:2, :3])
    torch.testing.assert_close(y[1:2, :3], y1, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(h[:, 1:2], h1, atol=1e-5, rtol=1e-5)


def test_time_major_and_cells():
    cell = nn.LSTMCell(3, 4)
    x = torch.randn(2, 3)
    h, (h2, c2) = cell(x)
    assert h.shape == (2, 4) and torch.equal(h, h2) and c2.shape == (2, 4)
    rnn = nn.RNN(nn.GRUCell(3, 4), time_major=True)
    y, s = rnn(torch.randn(5, 2, 3))
    assert y.shape == (5, 2, 4) and s.shape == (2, 4)
    init = cell.get_initial_states(x, init_value=0.5)
    assert all(torch.all(t == 0.5) for t in init)


def test_rnn_backward_flows():
    lstm = nn.LSTM(3, 4, num_layers=2)
    x = torch.randn(2, 5, 3, requires_grad=True)
    y, _ = lstm(x)
    y.sum().backward()
    assert x.grad is not None and lstm.layers[0].cell.weight_hh.grad.abs().sum() > 0


def test_gather_tree_matches_manual_backtrace():
    ids = torch.tensor([[[2, 2], [6, 1]], [[3, 9], [6, 1]], [[0, 1], [9, 0]]])
    parents = torch.tensor([[[0, 0], [1, 1]], [[1, 0], [1, 0]], [[0, 0], [0, 1]]])
    out = paddle.nn.functional.gather_tree(ids, parents)
    # batch 0, final beam 0: t2 id 0 (parent 0) → t1 beam 0 id 3 (parent 1) → t0 beam 1 id 2
    assert out[:, 0, 0].tolist() == [2, 3, 0]
    # batch 1, final beam 1: t2 id 0 (parent 1) → t1 beam 1 id 1 (parent 0) → t0 beam 0 id 6
    assert out[:, 1, 1].tolist() == [6, 1, 0]


class _CountCell(nn.RNNCellBase):
    """A deterministic 'cell': logits prefer token (input + 1) % V, end token after 3 steps."""
    V = 6

    def forward(self, inputs, states):
        logits = torch.full((inputs.shape[0], self.V), -5.0)
        logits[torch.arange(inputs.shape[0]), (inputs + 1) % self.V] = 5.0
        logits[:, 5] = torch.where(states[:, 0] >= 2, 10.0, -10.0)
        return logits, states + 1

    @property
    def state_shape(self):
        return (1,)


def test_beam_search_decoder_dynamic_decode():
    dec = nn.BeamSearchDecoder(_CountCell(), start_token=0, end_token=5, beam_size=2)
    init = torch.zeros(3, 1)
    out, states, lengths = nn.dynamic_decode(dec, init, max_step_num=10, return_length=True)
    assert out.shape[0] == 3 and out.shape[2] == 2  # [B, T, beam]
    best = out[:, :, 0]
    assert best[0].tolist()[:3] == [1, 2, 5] and set(best[0].tolist()[3:]) <= {5}  # end-padded
    assert bool(states["finished"].all())
    assert lengths[:, 0].tolist() == [3, 3, 3]


def test_layer_api_names():
    for n in ["RNNCellBase", "SimpleRNNCell", "LSTMCell", "GRUCell", "RNN", "BiRNN", "SimpleRNN",
              "LSTM", "GRU", "BeamSearchDecoder", "dynamic_decode"]:
        assert hasattr(nn, n), n
    np.testing.assert_equal(nn.LSTM(2, 3).layers[0].cell.weight_ih.shape, [12, 2])
