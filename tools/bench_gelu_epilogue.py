"""Inference FFN1: hipBLASLt GEMM with the bias+GELU epilogue (``torch._addmm_activation``,
tanh-form GELU like the reference's ``fused_gemm_epilogue`` / CUBLASLT_EPILOGUE_GELU_BIAS) vs
GEMM + the HIP bias-act kernel, on BERT-Large / GPT-1.3B shapes. No aux output (inference only).

  python tools/bench_gelu_epilogue.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import paddle_infer_amd  # noqa: E402,F401
from paddle_infer_amd.ops import bias_act  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda", 0)
    for T, H, F in [(16384, 1024, 4096), (4096, 1024, 4096), (32768, 2048, 8192), (2048, 2048, 8192)]:
        x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(F, H, device=dev, dtype=torch.bfloat16) * H ** -0.5)  # [out, in]
        b = torch.randn(F, device=dev, dtype=torch.bfloat16) * 0.1
        wt = w.t()
        ref = torch.nn.functional.gelu(x.float() @ wt.float() + b.float(), approximate="tanh")
        y_ep = torch._addmm_activation(b, x, wt, use_gelu=True)
        y_k = bias_act(torch.mm(x, wt), b, "gelu_tanh")
        t_ep = timeit(lambda: torch._addmm_activation(b, x, wt, use_gelu=True))
        t_k = timeit(lambda: bias_act(torch.mm(x, wt), b, "gelu_tanh"))
        t_mm = timeit(lambda: torch.mm(x, wt))
        print(json.dumps({"T": T, "H": H, "F": F, "epilogue_ms": round(t_ep, 4),
                          "mm_plus_biasact_ms": round(t_k, 4), "mm_only_ms": round(t_mm, 4),
                          "epilogue_err": round((y_ep.float() - ref).abs().max().item(), 4),
                          "kernel_err": round((y_k.float() - ref).abs().max().item(), 4)}), flush=True)


if __name__ == "__main__":
    main()
