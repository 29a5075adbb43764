"""RNN on the GPU: the ``rnn`` program op (one input-projection GEMM per layer/direction, sync-free
masked writes) and the dygraph LSTM (cell projections on the own split-bf16 fp32 GEMMs) against
PyTorch's fp32 CPU RNN."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["LSTM", "GRU"])
def test_rnn_op_gpu_matches_torch(mode):
    from paddle_infer_amd.static.ops_registry import REGISTRY
    torch.manual_seed(0)
    T, B, I, Hs, L = 9, 4, 48, 64, 2
    net = (torch.nn.LSTM if mode == "LSTM" else torch.nn.GRU)(I, Hs, num_layers=L, bidirectional=True)
    x = torch.randn(T, B, I)
    lens = torch.tensor([9, 5, 1, 7])
    h0, c0 = torch.randn(2 * L, B, Hs), torch.randn(2 * L, B, Hs)
    ws, bs = [], []
    for l in range(L):
        for d in range(2):
            sfx = f"_l{l}" + ("_reverse" if d else "")
            ws += [getattr(net, "weight_ih" + sfx).detach().cuda(), getattr(net, "weight_hh" + sfx).detach().cuda()]
            bs += [getattr(net, "bias_ih" + sfx).detach().cuda(), getattr(net, "bias_hh" + sfx).detach().cuda()]
    pre = [h0.cuda(), c0.cuda()] if mode == "LSTM" else [h0.cuda()]
    out = REGISTRY["rnn"]({"Input": [x.cuda()], "WeightList": ws + bs, "PreState": pre,
                           "SequenceLength": [lens.cuda()]},
                          {"mode": mode, "hidden_size": Hs, "num_layers": L, "is_bidirec": True, "is_test": True})
    packed = torch.nn.utils.rnn.pack_padded_sequence(x, lens, enforce_sorted=False)
    with torch.no_grad():
        ro, _ = net(packed, (h0, c0) if mode == "LSTM" else h0)
    ro, _ = torch.nn.utils.rnn.pad_packed_sequence(ro, total_length=T)
    # split-bf16 fp32 GEMMs: ~1e-5 relative per product
    torch.testing.assert_close(out["Out"].cpu(), ro, rtol=2e-4, atol=2e-4)


def test_dygraph_lstm_gpu_forward_backward():
    from paddle_infer_amd import nn
    torch.manual_seed(1)
    B, T, I, H = 4, 6, 64, 128
    ours, ref = nn.LSTM(I, H), torch.nn.LSTM(I, H, batch_first=True)
    cell = ours.layers[0].cell
    with torch.no_grad():
        for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
            getattr(ref, n + "_l0").copy_(getattr(cell, n))
    ours = ours.cuda()
    x = torch.randn(B, T, I)
    y, _ = ours(x.cuda())
    y_ref, _ = ref(x)
    torch.testing.assert_close(y.cpu(), y_ref, rtol=2e-4, atol=2e-4)
    y.sum().backward()
    y_ref.sum().backward()
    torch.testing.assert_close(cell.weight_hh.grad.cpu(), ref.weight_hh_l0.grad, rtol=2e-3, atol=2e-3)
