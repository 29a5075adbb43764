"""Focused NT asm GEMM check (ping-pong kernel when PIAMD_AGEMM_PP=1): dtypes × split-K × epilogue."""
import sys
import torch
sys.path.insert(0, ".")
from paddle_infer_amd.ops.gemm import asm_gemm

torch.manual_seed(0)
for M, N, K in ((2048, 3072, 1024), (512, 512, 512), (256, 256, 256), (300, 520, 512)):
    for dt in (torch.bfloat16, torch.float16):
        a = (0.5 * torch.randn(M, K, device="cuda")).to(dt)
        b = (0.05 * torch.randn(N, K, device="cuda")).to(dt)
        bias = torch.randn(N, device="cuda").to(dt)
        ref = a.float() @ b.float().t()
        for ks in (1, 2, 4):
            if K % (64 * ks) or K // ks < 256:
                continue
            for kind in ("plain", "f32", "biasnx"):
                if kind == "biasnx" and ks > 1:
                    continue
                if kind == "plain":
                    c = asm_gemm(a, b, trans_b=True, ksplit=ks).float()
                    r = ref
                elif kind == "f32":
                    c = asm_gemm(a, b, trans_b=True, ksplit=ks, out_f32=True)
                    r = ref
                else:
                    c = asm_gemm(a, b, trans_b=True, epi="bias_act", act="none", bias=bias).float()
                    r = ref + bias.float()
                err = (c - r).abs().max().item()
                bad = (c - r).abs() > 0.05 * r.abs().max()
                rows = bad.any(1).nonzero().flatten()
                cols = bad.any(0).nonzero().flatten()
                print(M, N, K, str(dt)[6:], "ks", ks, kind, "err %.4f" % err,
                      "bad rows", rows[:4].tolist(), len(rows), "cols", cols[:4].tolist(), len(cols), flush=True)
