"""Deferred LayerNorm (inference/ln_defer.py + gemm_small.hip): fp16 / bf16 LN fold with the row
statistics written out, the residual epilogue that applies a deferred LayerNorm, and the BERT
Predictor at few rows with the deferral on vs off vs the fp32 dygraph model."""
import os
import tempfile

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(128, 3072, 1024), (128, 4096, 1024), (20, 512, 512)])
def test_ln_fold_stats_out(dt, M, N, K):
    from paddle_infer_amd.ops import gemm as G
    torch.manual_seed(M + N)
    x = (torch.randn(M, K, device=DEV) * 1.5 + torch.randn(M, 1, device=DEV)).to(dt)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(dt)
    gamma = (1 + 0.2 * torch.randn(K, device=DEV)).to(dt)
    beta = (0.1 * torch.randn(K, device=DEV)).to(dt)
    bias = (0.1 * torch.randn(N, device=DEV)).to(dt)
    wf, c1, b2 = G.ln_fold(w, gamma, beta, bias)
    st = torch.full((M, 2), float("nan"), device=DEV)
    y = G.small_gemm(x, wf, act="gelu", ln=(c1, b2, 1e-5), ln_stats=st)
    h = F.layer_norm(x.float(), (K,), gamma.float(), beta.float(), 1e-5)
    ref = F.gelu(h @ w.float().t() + bias.float())
    err = (y.float() - ref).abs().max().item()
    assert err <= 2e-2 + 1e-2 * ref.abs().max().item(), err
    mean = x.float().mean(1)
    rstd = torch.rsqrt(x.float().var(1, unbiased=False) + 1e-5)
    torch.testing.assert_close(st[:, 0], mean, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(st[:, 1], rstd, atol=1e-3, rtol=2e-3)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(128, 1024, 1024), (128, 1024, 4096), (16, 1024, 4096)])
def test_resid_ln_epilogue(dt, M, N, K):
    """out = x·wᵀ + bias + LN(h) with LN's statistics supplied (split-K and B-deep configs)."""
    from paddle_infer_amd.ops import gemm as G
    torch.manual_seed(K + M)
    x = torch.randn(M, K, device=DEV).to(dt)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(dt)
    bias = (0.1 * torch.randn(N, device=DEV)).to(dt)
    h = (2 * torch.randn(M, N, device=DEV) + 0.5).to(dt)
    g = (1 + 0.2 * torch.randn(N, device=DEV)).to(dt)
    b = (0.1 * torch.randn(N, device=DEV)).to(dt)
    mean = h.float().mean(1)
    rstd = torch.rsqrt(h.float().var(1, unbiased=False) + 1e-12)
    st = torch.stack([mean, rstd], 1).contiguous()
    y = G.small_gemm(x, w, bias=bias, resid=h, resid_ln=(st, g, b))
    ref = x.float() @ w.float().t() + bias.float() + F.layer_norm(h.float(), (N,), g.float(), b.float(), 1e-12)
    err = (y.float() - ref).abs().max().item()
    assert err <= 2e-2 + 1e-2 * ref.abs().max().item(), err


def _bert_predictor(model, seq, dt):
    from paddle_infer_amd import inference as pinf, jit
    from paddle_infer_amd.static import InputSpec
    d = tempfile.mkdtemp(prefix="lndefer_")
    st = jit.to_static(model, input_spec=[InputSpec([None, seq], "int64", "input_ids")])
    jit.save(st, os.path.join(d, "model"))
    c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
    c.enable_use_gpu(1024, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Half if dt == torch.float16 else pinf.PrecisionType.Bfloat16)
    c.enable_hip_graph(True)
    return pinf.create_predictor(c)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_bert_predictor_ln_defer(dt):
    from paddle_infer_amd.inference import ln_defer
    from paddle_infer_amd.models.bert import BertModel, bert_config
    torch.manual_seed(0)
    cfg = bert_config("bert-large", num_hidden_layers=3, hidden_size=1024, num_attention_heads=16,
                      intermediate_size=4096, vocab_size=1000)
    model = BertModel(cfg)
    model.eval()
    seq, B = 128, 1
    pred = _bert_predictor(model, seq, dt)
    assert pred.pass_stats.get("ln_defer_pass") == 5  # 2 per layer; the last output is fetched
    ids = torch.randint(0, 1000, (B, seq))

    def run():
        h = pred.get_input_handle(pred.get_input_names()[0])
        h.copy_from_cpu(ids.numpy())
        pred.run()
        return torch.from_numpy(pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()).float()

    calls = []
    orig = ln_defer.linear

    def spy(*a, **k):
        y = orig(*a, **k)
        calls.append(y is not None)
        return y
    ln_defer.linear = spy
    try:
        on = run()
    finally:
        ln_defer.linear = orig
    assert calls and all(calls), calls  # every deferred LayerNorm was folded (none materialised)
    with torch.no_grad():
        ref = model(ids)
    ref = (ref[0] if isinstance(ref, (tuple, list)) else ref).float()
    err = (on - ref).abs().max().item()
    assert err <= 6e-2 + 2e-2 * ref.abs().max().item(), err
