"""int8 × int8 MFMA GEMM (``gemm.hip`` gemm_i8) and row quantisation against exact/fp32 PyTorch
references; the INT8 fused multi-transformer on the GPU against its CPU run."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N,K", [(1, 256, 128), (300, 512, 384), (1024, 768, 2048), (33, 260, 256)])
def test_gemm_i8_exact(M, N, K):
    from paddle_infer_amd.ops import inference as I
    torch.manual_seed(M)
    xq = torch.randint(-127, 128, (M, K), dtype=torch.int8)
    wq = torch.randint(-127, 128, (N, K), dtype=torch.int8)
    xs = torch.rand(M) * 0.01 + 1e-3
    ws = torch.rand(N) * 0.01 + 1e-3
    b = torch.randn(N).bfloat16()
    got = I.int8_gemm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), b.to(DEV), "relu").cpu()
    acc = xq.long() @ wq.long().t()  # exact int32 accumulation
    ref = torch.relu(acc.double() * xs.double()[:, None] * ws.double()[None, :] + b.double())
    assert torch.allclose(got.double(), ref, rtol=1e-2, atol=1e-2), (got.double() - ref).abs().max()


def test_quantize_rows_gpu_matches_cpu():
    from paddle_infer_amd.ops import inference as I
    x = (torch.randn(77, 512) * 4).bfloat16()
    q, s = I.quantize_rows(x.to(DEV))
    qr, sr = I.quantize_rows(x.float())
    assert torch.allclose(s.cpu(), sr, rtol=1e-5)
    assert (q.cpu().int() - qr.int()).abs().max() <= 1
    q2, _ = I.quantize_rows(x.to(DEV), 0.04)
    q2r, _ = I.quantize_rows(x.float(), 0.04)
    assert (q2.cpu().int() - q2r.int()).abs().max() <= 1


def test_fused_multi_transformer_int8_gpu():
    from paddle_infer_amd.incubate.nn import FusedMultiTransformer, FusedMultiTransformerINT8
    torch.manual_seed(3)
    ref = FusedMultiTransformer(256, 4, 512, num_layers=2)
    with torch.no_grad():
        for p in ref.parameters():
            if p.dim() > 1:
                p.normal_(0, 0.03)
    q = FusedMultiTransformerINT8(256, 4, 512, num_layers=2).load_from_float(ref)
    x = torch.randn(2, 40, 256) * 0.5
    cpu = q(x)
    qg = q.to(DEV)
    for n, p in qg.named_parameters():
        if p.dtype == torch.float32 and "scale" not in n or "ln" in n:
            p.data = p.data.to(torch.bfloat16) if "ln" not in n else p.data
    got = qg(x.to(DEV).bfloat16())
    assert (got.float().cpu() - cpu).abs().max() < 0.05 * cpu.abs().max() + 2e-2
