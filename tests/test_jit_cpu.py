"""paddle.jit tests (CPU): to_static keeps dygraph numerics and exposes a concrete program;
jit.save → jit.load round trip (dynamic batch dim), TracedLayer, Predictor over a jit-saved model.
Parity model: reference `unittests/dygraph_to_static/test_save_load.py`, `test_jit_save_load.py`,
`test_traced_layer_err_msg.py`."""
import numpy as np
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import jit, nn
from paddle_infer_amd.static import InputSpec


class Net(nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(8, 16)
        self.ln = nn.LayerNorm(16)
        self.fc2 = nn.Linear(16, 4)

    def forward(self, x):
        return self.fc2(nn.functional.gelu(self.ln(self.fc1(x))))


def test_jit_save_load_round_trip(tmp_path):
    paddle.seed(0)
    net = Net()
    net.eval()
    x = torch.randn(3, 8)
    ref = net(x)
    path = str(tmp_path / "net" / "model")
    jit.save(net, path, input_spec=[InputSpec([None, 8], "float32", "x")])
    loaded = jit.load(path)
    torch.testing.assert_close(loaded(x), ref)
    assert loaded(torch.randn(7, 8)).shape == (7, 4)  # symbolic batch dim
    types = [op.type for op in loaded.program().global_block().ops]
    assert "layer_norm" in types and "matmul_v2" in types and "linear" not in types  # Paddle op types only


def test_to_static_layer_and_function():
    net = Net()
    net.eval()
    snet = jit.to_static(net, input_spec=[InputSpec([None, 8])])
    x = torch.randn(2, 8)
    out = snet(x)
    assert out.shape == (2, 4)
    prog = snet._static_function.main_program
    assert len(prog.global_block().ops) >= 4

    @jit.to_static
    def f(a, b):
        return a * 2 + b
    torch.testing.assert_close(f(torch.ones(2), torch.ones(2)), torch.full((2,), 3.0))
    assert f.rollback()(torch.ones(1), torch.zeros(1)).item() == 2.0


def test_traced_layer_and_predictor(tmp_path):
    net = Net()
    net.eval()
    x = torch.randn(4, 8)
    out, traced = jit.TracedLayer.trace(net, [x])
    got = traced([x])[0]
    torch.testing.assert_close(got, out)
    traced.save_inference_model(str(tmp_path / "traced" / "inference"))
    from paddle_infer_amd import inference as pinf
    pred = pinf.create_predictor(pinf.Config(str(tmp_path / "traced")))
    res = pred.run([x])[0]
    np.testing.assert_allclose(res.numpy(), out.detach().numpy(), rtol=1e-5, atol=1e-6)
