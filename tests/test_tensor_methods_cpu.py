"""Paddle-signature Tensor methods (framework/tensor_patch.py): the Paddle form of each method
(axis=, a permutation list, an index tensor first, num_or_sections, transpose flags) gives the
reference Paddle result, while the torch form of the same method keeps torch's meaning — and a
to_static trace of Paddle-form calls still lowers to reference Paddle op types."""
import numpy as np
import torch

import paddle_infer_amd as paddle  # noqa: F401  (installs the adapters)


def test_paddle_forms():
    x = torch.arange(24.).reshape(2, 3, 4)
    n = x.numpy()
    assert x.transpose([0, 2, 1]).shape == (2, 4, 3)
    np.testing.assert_array_equal(x.sum(axis=1).numpy(), n.sum(1))
    np.testing.assert_array_equal(x.mean(axis=[1, 2], keepdim=True).numpy(), n.mean((1, 2), keepdims=True))
    np.testing.assert_array_equal(x.max(axis=2).numpy(), n.max(2))
    np.testing.assert_array_equal(x.min(axis=0).numpy(), n.min(0))
    assert x.flatten(start_axis=1, stop_axis=2).shape == (2, 12)
    assert x.unsqueeze([0, 4]).shape == (1, 2, 3, 4, 1)
    assert x.unsqueeze(-1).squeeze(axis=[-1]).shape == (2, 3, 4)
    assert [t.shape[1] for t in x.split(3, axis=1)] == [1, 1, 1]
    assert [t.shape[2] for t in x.split([1, -1], axis=2)] == [1, 3]
    idx = torch.tensor([2, 0])
    np.testing.assert_array_equal(x.gather(idx, axis=1).numpy(), n[:, [2, 0]])
    np.testing.assert_array_equal(x.index_select(idx, axis=2).numpy(), n[:, :, [2, 0]])
    np.testing.assert_allclose(x.matmul(x, transpose_y=True).numpy(), n @ n.transpose(0, 2, 1))
    np.testing.assert_array_equal(x.argmax(axis=-1).numpy(), n.argmax(-1))
    np.testing.assert_array_equal(x.cumsum(axis=1).numpy(), n.cumsum(1))
    np.testing.assert_array_equal(x.sort(axis=-1, descending=True).numpy(), -np.sort(-n, -1))
    np.testing.assert_array_equal(x.flip(axis=[1]).numpy(), n[:, ::-1])
    assert x.topk(2, axis=1)[0].shape == (2, 2, 4)
    np.testing.assert_array_equal(x.scale(2.0, 1.0).numpy(), n * 2 + 1)
    np.testing.assert_array_equal(x.scale(2.0, 1.0, bias_after_scale=False).numpy(), (n + 1) * 2)


def test_torch_forms_unchanged():
    x = torch.arange(24.).reshape(2, 3, 4)
    assert x.transpose(0, 1).shape == (3, 2, 4)
    assert x.max(1).values.shape == (2, 4)  # torch: (values, indices)
    assert [t.shape[2] for t in x.split(2, 2)] == [2, 2]  # torch: split SIZE
    assert x.gather(1, torch.zeros(2, 1, 4, dtype=torch.long)).shape == (2, 1, 4)
    assert x.index_select(2, torch.tensor([0])).shape == (2, 3, 1)
    assert x.flatten(1).shape == (2, 12)
    v, i = x.sort(-1)
    assert v.shape == i.shape == x.shape


def test_static_trace_of_paddle_forms_lowers():
    import paddle_infer_amd.nn as nn
    from paddle_infer_amd import jit
    from paddle_infer_amd.static import InputSpec
    import tempfile
    import os

    class M(nn.Layer):
        def forward(self, x):
            y = x.transpose([0, 2, 1]).sum(axis=-1)
            return y.unsqueeze([1]).flatten(start_axis=1)

    with tempfile.TemporaryDirectory() as td:
        jit.save(M(), os.path.join(td, "m"), input_spec=[InputSpec([2, 3, 4], "float32", "x")])
        from paddle_infer_amd.onnx import load_paddle_model
        desc, _ = load_paddle_model(os.path.join(td, "m"))
    types = [o["type"] for o in desc["blocks"][0]["ops"]]
    assert "transpose2" in types and "reduce_sum" in types and "unsqueeze2" in types


def test_torch_keyword_gather_index_select_unchanged():
    """The Paddle-signature adapters must not capture torch keyword calls (process-wide patch)."""
    import paddle_infer_amd  # noqa: F401
    x = torch.arange(12.).reshape(3, 4)
    idx = torch.tensor([[0, 1], [2, 3], [1, 1]])
    torch.testing.assert_close(x.gather(dim=1, index=idx), torch.gather(x, 1, idx))
    torch.testing.assert_close(x.gather(1, idx), torch.gather(x, 1, idx))
    i1 = torch.tensor([3, 0])
    torch.testing.assert_close(x.index_select(dim=1, index=i1), torch.index_select(x, 1, i1))
    torch.testing.assert_close(x.index_select(1, i1), torch.index_select(x, 1, i1))
    # Paddle forms still work
    torch.testing.assert_close(x.gather(torch.tensor([2, 0])), x[[2, 0]])
    torch.testing.assert_close(x.index_select(i1, axis=1), x[:, [3, 0]])
    torch.testing.assert_close(x.gather(index=torch.tensor([1]), axis=0), x[[1]])
