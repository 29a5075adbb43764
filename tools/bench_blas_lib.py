"""hipBLASLt vs rocBLAS (torch.backends.cuda.preferred_blas_library) on the GPT-3 1.3B training
GEMMs (T = 65536 tokens): fwd x·Wtᵀ, dgrad dy·Wᵀ, wgrad main_grad(fp32) += xᵀ·dy (addmm_)."""
import json
import sys

import torch


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    dt = torch.bfloat16
    for name, K, N in [("qkv", 2048, 6144), ("out", 2048, 2048), ("ffn1", 2048, 8192), ("ffn2", 8192, 2048)]:
        x = torch.randn(T, K, device="cuda", dtype=dt)
        dy = torch.randn(T, N, device="cuda", dtype=dt)
        w = torch.randn(K, N, device="cuda", dtype=dt)
        wt = w.t().contiguous()
        mg = torch.zeros(K, N, device="cuda", dtype=torch.float32)
        mgb = torch.zeros(K, N, device="cuda", dtype=dt)
        flops = 2 * T * K * N
        row = {"gemm": name}
        for lib in ("cublaslt", "cublas"):
            torch.backends.cuda.preferred_blas_library(lib)
            for p, fn in (("fwd", lambda: torch.mm(x, wt.t())), ("dgrad", lambda: torch.mm(dy, w.t())),
                          ("wgrad_f32", lambda: mg.addmm_(x.t(), dy)),
                          ("wgrad_bf16", lambda: mgb.addmm_(x.t(), dy))):
                try:
                    us = timeit(fn)
                    row[f"{p}_{'lt' if lib == 'cublaslt' else 'roc'}_TF"] = round(flops / us / 1e6, 1)
                except Exception as e:  # noqa: BLE001
                    row[f"{p}_{lib}"] = repr(e)[:60]
        print(json.dumps(row), flush=True)
        del x, dy, w, wt, mg, mgb


if __name__ == "__main__":
    main()
