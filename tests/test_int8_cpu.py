"""Activation-quantised int8 linear (reference `fused_multi_transformer_int8_op`,
`llm_int8_linear`) on CPU: per-token / static quantisation, dequantising GEMM contract,
FusedMultiTransformerINT8 close to its float original."""
import torch

from paddle_infer_amd.ops import inference as I


def test_quantize_rows_roundtrip():
    x = torch.randn(7, 256) * 3
    q, s = I.quantize_rows(x)
    assert q.dtype == torch.int8 and (q.abs() <= 127).all()
    assert torch.allclose(q.float() * s[:, None], x, atol=(s.max() / 2 + 1e-6).item())
    q2, s2 = I.quantize_rows(x, 0.05)
    assert torch.all(s2 == 0.05)


def test_int8_linear_close_to_float():
    torch.manual_seed(0)
    x = torch.randn(5, 256)
    w = torch.randn(256, 128) * 0.05
    b = torch.randn(128)
    wq, ws = I.weight_quantize(w, "llm.int8")
    assert wq.shape == (128, 256) and wq.dtype == torch.int8
    y = I.int8_linear(x, wq, ws, b.bfloat16(), act="relu")
    ref = torch.relu(x @ w + b)
    assert (y.float() - ref).abs().max() < 0.05 * ref.abs().max()


def test_llm_int8_outliers():
    torch.manual_seed(1)
    x = torch.randn(4, 256)
    x[:, 3] = 40.0  # outlier feature → bf16 path
    w = torch.randn(256, 64) * 0.05
    wq, ws = I.weight_quantize(w, "llm.int8")
    y = I.llm_int8_linear(x, wq, None, ws, threshold=6.0)
    ref = x @ w
    assert (y.float() - ref).abs().max() < 0.05 * ref.abs().max()


def test_fused_multi_transformer_int8_close_to_float():
    from paddle_infer_amd.incubate.nn import FusedMultiTransformer, FusedMultiTransformerINT8
    torch.manual_seed(2)
    ref = FusedMultiTransformer(256, 4, 512, num_layers=2)
    with torch.no_grad():
        for p in ref.parameters():
            if p.dim() > 1:
                p.normal_(0, 0.03)
    q = FusedMultiTransformerINT8(256, 4, 512, num_layers=2).load_from_float(ref)
    x = torch.randn(2, 5, 256) * 0.5
    a, b = ref(x), q(x)
    assert (a - b).abs().max() < 0.05 * a.abs().max() + 1e-3
