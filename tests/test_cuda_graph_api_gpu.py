"""paddle.device.cuda.graphs (reference `python/paddle/device/cuda/graphs.py:38`): capture of the
framework's own HIP kernels into a hipGraph, replay on new inputs, against eager fp32."""
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import ops
from paddle_infer_amd.ops.linear import linear as _linear

pytestmark = pytest.mark.gpu


def _fn(x, w, g, b):
    h = _linear(x, w)                       # own GEMM
    return ops.layer_norm(h, g, b, 1e-5)              # own LayerNorm kernel


def test_cuda_graph_capture_replay_matches_eager():
    from paddle_infer_amd.device.cuda.graphs import CUDAGraph
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(256, 512, device=dev, dtype=torch.bfloat16)
    w = torch.randn(512, 768, device=dev, dtype=torch.bfloat16) * 0.05
    g = torch.ones(768, device=dev, dtype=torch.bfloat16)
    b = torch.zeros(768, device=dev, dtype=torch.bfloat16)
    with torch.no_grad():
        _fn(x, w, g, b)  # warm-up: weight caches, kernel load
        torch.cuda.synchronize()
        graph = CUDAGraph()
        graph.capture_begin()
        out = _fn(x, w, g, b)
        graph.capture_end()
        for _ in range(2):
            x.copy_(torch.randn_like(x))
            graph.replay()
            torch.cuda.synchronize()
            ref = torch.nn.functional.layer_norm(x.float() @ w.float(), (768,), g.float(), b.float(), 1e-5)
            torch.testing.assert_close(out.float(), ref, rtol=3e-2, atol=3e-2)
    graph.reset()


def test_wrap_cuda_graph_layer():
    from paddle_infer_amd.device.cuda.graphs import wrap_cuda_graph
    torch.manual_seed(0)
    lin = paddle.nn.Linear(256, 128).to("cuda").astype("bfloat16")
    lin.eval()
    wrapped = wrap_cuda_graph(lin)
    with torch.no_grad():
        for i in range(4):
            x = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16)
            y = wrapped(x)
            ref = x.float() @ lin.weight.float() + lin.bias.float()
            torch.testing.assert_close(y.float(), ref, rtol=3e-2, atol=3e-2)
    assert lin.forward.graph is not None and lin.forward.calls == 4
