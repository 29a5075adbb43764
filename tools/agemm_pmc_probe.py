"""Run the assembly GEMM on a long-K square problem in both layouts (for rocprofv3 --pmc passes):
nt = A[M,K]·B[N,K]ᵀ (ds_read_b128 fragments), tn = A[K,M]ᵀ·B[K,N] (ds_read_b64_tr_b16)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import paddle_infer_amd  # noqa: F401
    from paddle_infer_amd.ops.gemm import asm_gemm
    M = N = 4096
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    g = torch.Generator(device="cuda").manual_seed(0)
    for ta, tb in ((False, True), (True, False)):
        a = torch.randn((K, M) if ta else (M, K), device="cuda", generator=g).bfloat16()
        b = torch.randn((N, K) if tb else (K, N), device="cuda", generator=g).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            asm_gemm(a, b, ta, tb, out=c)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
