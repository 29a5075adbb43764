"""LayerNorm fold in the skinny MFMA GEMM (gemm_small.hip LN mode, ops.gemm.ln_fold): the row
statistics come from the raw rows inside the GEMM and the epilogue applies
rstd·(acc − mean·c1) + b2. Checked against the plain PyTorch fp32 reference LN → linear (+ act,
+ residual), over tile configs that split K over 1 / 2 / 4 waves, partial row tiles and a large row
mean; and the serving-batch decode layer stack with the fold on vs off."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N,K,cfg", [(32, 6144, 2048, None), (32, 8192, 2048, None),
                                       (20, 512, 1024, (2, 1, 1, 2)), (8, 256, 512, (1, 2, 2, 1)),
                                       (64, 1024, 2048, (4, 1, 4, 2)), (48, 768, 768, (1, 4, 1, 2))])
@pytest.mark.parametrize("act", ["none", "gelu"])
def test_small_gemm_ln_fold(M, N, K, cfg, act):
    from paddle_infer_amd.ops import gemm as G
    torch.manual_seed(M + N + K)
    x = (torch.randn(M, K, device=DEV) * 1.5 + torch.randn(M, 1, device=DEV) * 3).bfloat16()
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    gamma = (1 + 0.2 * torch.randn(K, device=DEV)).bfloat16()
    beta = (0.1 * torch.randn(K, device=DEV)).bfloat16()
    bias = (0.1 * torch.randn(N, device=DEV)).bfloat16()
    resid = torch.randn(M, N, device=DEV).bfloat16()
    wf, c1, b2 = G.ln_fold(w, gamma, beta, bias)
    full = None if cfg is None else (*cfg, 1)
    y = G.small_gemm(x, wf, act=act, resid=resid, cfg=full, ln=(c1, b2, 1e-5))
    h = F.layer_norm(x.float(), (K,), gamma.float(), beta.float(), 1e-5)
    ref = h @ w.float().t() + bias.float()
    if act == "gelu":
        ref = F.gelu(ref)
    ref = ref + resid.float()
    err = (y.float() - ref).abs().max().item()
    assert err <= 3e-2 + 2e-2 * ref.abs().max().item(), err


def test_serving_decode_ln_fold_matches_layernorm_path():
    """GPT-style pre-LN decode at 32 rows through multi_transformer_forward: LN-folded projections
    (no LayerNorm launches) vs the same stack with explicit LayerNorm passes."""
    from paddle_infer_amd.incubate.nn import functional as IF
    torch.manual_seed(0)
    E, H, F_, nl, B, S = 1024, 16, 4096, 2, 32, 96
    D = E // H

    def lin(i, o):
        return IF._Linear((torch.randn(i, o, device=DEV) / i ** 0.5).bfloat16()).prepack()

    layers = []
    for _ in range(nl):
        layers.append(dict(ln_scale=(1 + 0.1 * torch.randn(E, device=DEV)).bfloat16(),
                           ln_bias=(0.1 * torch.randn(E, device=DEV)).bfloat16(),
                           qkv=lin(E, 3 * E), qkv_bias=(0.1 * torch.randn(3 * E, device=DEV)).bfloat16(),
                           out=lin(E, E), out_bias=(0.1 * torch.randn(E, device=DEV)).bfloat16(),
                           ffn_ln_scale=(1 + 0.1 * torch.randn(E, device=DEV)).bfloat16(),
                           ffn_ln_bias=(0.1 * torch.randn(E, device=DEV)).bfloat16(),
                           ffn1=lin(E, F_), ffn1_bias=(0.1 * torch.randn(F_, device=DEV)).bfloat16(),
                           ffn2=lin(F_, E), ffn2_bias=(0.1 * torch.randn(E, device=DEV)).bfloat16()))
    assert layers[0]["qkv"].ln_fold_ok(B, "none") and layers[0]["ffn1"].ln_fold_ok(B, "gelu")
    x = torch.randn(B, 1, E, device=DEV).bfloat16()
    lens = torch.full((B,), 40, dtype=torch.int32, device=DEV)
    pos = lens - 1

    def run(fold):
        IF.LN_FOLD = fold
        try:
            torch.manual_seed(1)
            caches = [(torch.randn(B, H, S, D, device=DEV).bfloat16(),
                       torch.randn(B, H, S, D, device=DEV).bfloat16()) for _ in range(nl)]
            return IF.multi_transformer_forward(x, layers, H, caches=caches, pos=pos, lens=lens,
                                                decode=True, activation="gelu").float()
        finally:
            IF.LN_FOLD = True

    on, off = run(True), run(False)
    assert len(layers[0]["qkv"].lnf) == 1 and len(layers[0]["ffn1"].lnf) == 1
    err = (on - off).abs().max().item()
    assert err <= 5e-2 + 2e-2 * off.abs().max().item(), err
