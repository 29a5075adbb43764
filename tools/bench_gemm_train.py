"""gemm.hip against hipBLASLt on the GPT-3 1.3B training GEMMs at T = 32768 tokens
(micro-batch 32 × 1024). A deep-prefetch main-loop variant measured with this tool gained nothing
(`profiles/gemm_pipeline_ab_r1.txt`).

  fwd   y[T,N]  = x[T,K] · Wᵀ  (W stored [N,K]: TN, both operands K-contiguous)
  wgrad W[K,N] += xᵀ · dy      (x [T,K], dy [T,N]: NT, both operands T-strided; bf16 main_grad)

Prints one JSON line per (shape, pass, impl) with TFLOP/s and the max error vs hipBLASLt.

  python tools/bench_gemm_pipe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    from paddle_infer_amd.ops.gemm import gemm
    T = int(os.environ.get("T", 32768))
    for K, N in [(2048, 6144), (2048, 2048), (2048, 8192), (8192, 2048)]:
        x = torch.randn(T, K, device="cuda").bfloat16()
        dy = torch.randn(T, N, device="cuda").bfloat16() * 0.1
        w = (0.02 * torch.randn(N, K, device="cuda")).bfloat16()
        fl = 2.0 * T * K * N
        ref_f = torch.mm(x, w.t())
        ref_w = torch.mm(x.t(), dy)
        mg = torch.zeros(K, N, device="cuda", dtype=torch.bfloat16)
        cases = [
            ("fwd", "hipblaslt", lambda: torch.mm(x, w.t()), None),
            ("wgrad", "hipblaslt", lambda: mg.addmm_(x.t(), dy), None),
        ]
        cases.append(("fwd", "piamd", lambda: gemm(x, w, trans_b=True), None))
        cases.append(("wgrad", "piamd", lambda: gemm(x, dy, trans_a=True, out=mg, accumulate=True), None))
        for pas, impl, fn, _ in cases:
            err = None
            if impl != "hipblaslt":
                if pas == "fwd":
                    err = (fn().float() - ref_f.float()).abs().max().item()
                else:
                    mg.zero_()
                    fn()
                    err = (mg.float() - ref_w.float()).abs().max().item()
            ms = timeit(fn)
            print(json.dumps({"K": K, "N": N, "T": T, "pass": pas, "impl": impl, "ms": round(ms, 4),
                              "tflops": round(fl / ms / 1e9, 1),
                              "max_err": None if err is None else round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
