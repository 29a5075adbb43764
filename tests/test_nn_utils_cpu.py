"""paddle.nn.utils: weight_norm / remove_weight_norm, spectral_norm, parameters_to_vector /
vector_to_parameters against fp32 compositions of the reference formulas
(`python/paddle/nn/utils/*.py`)."""
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd.nn import utils as U


@pytest.mark.parametrize("dim", [0, 1, None])
def test_weight_norm_forward_grad_and_remove(dim):
    torch.manual_seed(0)
    conv = paddle.nn.Conv2D(3, 5, 3)
    w0 = conv.weight.detach().clone()
    x = torch.randn(2, 3, 8, 8)
    y0 = conv(x)
    U.weight_norm(conv, dim=dim)
    names = dict(conv.named_parameters())
    assert "weight_g" in names and "weight_v" in names and "weight" not in names
    d = -1 if dim is None else dim
    if d == -1:
        assert conv.weight_g.numel() == 1
    else:
        assert conv.weight_g.shape == (w0.shape[d],)
    y1 = conv(x)
    torch.testing.assert_close(y1, y0, rtol=1e-5, atol=1e-5)  # g initialised to ‖w‖
    with torch.no_grad():
        conv.weight_g.mul_(2.0)
    y2 = conv(x)
    torch.testing.assert_close(y2 - conv.bias.view(1, -1, 1, 1), 2 * (y0 - conv.bias.view(1, -1, 1, 1)),
                               rtol=1e-4, atol=1e-4)
    y2.sum().backward()
    assert conv.weight_g.grad is not None and conv.weight_v.grad is not None
    U.remove_weight_norm(conv)
    names = dict(conv.named_parameters())
    assert "weight" in names and "weight_g" not in names
    torch.testing.assert_close(conv(x), y2.detach(), rtol=1e-4, atol=1e-4)


def test_spectral_norm_divides_by_top_singular_value():
    torch.manual_seed(0)
    lin = paddle.nn.Linear(6, 4)
    w = lin.weight.detach().clone()  # [in, out]; dim defaults to 1 for Linear
    U.spectral_norm(lin, n_power_iterations=30)
    lin.train()
    x = torch.randn(3, 6)
    y = lin(x)
    sigma = torch.linalg.matrix_norm(w.t(), ord=2)
    torch.testing.assert_close(y - lin.bias, x @ (w / sigma), rtol=1e-3, atol=1e-3)
    assert "weight_orig" in dict(lin.named_parameters())
    lin.eval()
    torch.testing.assert_close(lin(x), y.detach(), rtol=1e-4, atol=1e-4)  # no iteration in eval


def test_parameters_vector_roundtrip():
    a = paddle.nn.Linear(10, 15)
    b = paddle.nn.Linear(10, 15)
    v = U.parameters_to_vector(a.parameters())
    assert v.shape == (10 * 15 + 15,)
    U.vector_to_parameters(v, b.parameters())
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q)
    assert all(hasattr(paddle.nn.utils, n) for n in U.__all__)
