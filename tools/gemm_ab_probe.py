"""A/B probe: the assembly GEMM against hipBLASLt (torch.mm) on one shape, random bf16 operands,
interleaved rounds in one process (rocprofv3 target for per-kernel PMC passes, and a wall-clock
A/B printed as JSON lines).

  python tools/gemm_ab_probe.py --M 98304 --N 2048 --K 2048 --layout nt --iters 20 --rounds 3
layout: "nt" = A[M,K]·B[N,K]ᵀ (forward / data gradient), "tn" = A[K,M]ᵀ·B[K,N] (weight gradient).
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=98304)
    ap.add_argument("--N", type=int, default=2048)
    ap.add_argument("--K", type=int, default=2048)
    ap.add_argument("--layout", default="nt")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--impls", default="asm,hipblaslt")
    a = ap.parse_args()
    import paddle_infer_amd  # noqa: F401
    from paddle_infer_amd.ops.gemm import asm_gemm
    ta, tb = a.layout[0] == "t", a.layout[1] == "t"
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(*((a.K, a.M) if ta else (a.M, a.K)), device="cuda", generator=g).bfloat16()
    B = torch.randn(*((a.N, a.K) if tb else (a.K, a.N)), device="cuda", generator=g).bfloat16()
    C = torch.empty(a.M, a.N, device="cuda", dtype=torch.bfloat16)
    Aop = A.t() if ta else A
    Bop = B.t() if tb else B

    def run(impl):
        if impl == "hipblaslt":
            torch.mm(Aop, Bop, out=C)
        else:
            asm_gemm(A, B, ta, tb, out=C)

    impls = a.impls.split(",")
    for impl in impls:
        for _ in range(3):
            run(impl)
    torch.cuda.synchronize()
    flop = 2.0 * a.M * a.N * a.K
    times = {i: [] for i in impls}
    for _ in range(a.rounds):
        for impl in impls:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run(impl)
            e1.record()
            torch.cuda.synchronize()
            times[impl].append(e0.elapsed_time(e1) / a.iters)
    base = statistics.median(times[impls[-1]])
    for impl in impls:
        ms = statistics.median(times[impl])
        print(json.dumps({"M": a.M, "N": a.N, "K": a.K, "layout": a.layout, "impl": impl,
                          "ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1),
                          "vs_last": round(base / ms, 3)}))


if __name__ == "__main__":
    main()
