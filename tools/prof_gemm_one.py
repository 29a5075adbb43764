"""Run one GEMM configuration repeatedly (rocprofv3 target for per-kernel counters).

  python tools/prof_gemm_one.py --M 65536 --N 2048 --K 8192 --layout nt --impl pipe --iters 20
layout: two letters for A and B storage: n = K-contiguous ([M][K] / [N][K]), t = M/N-contiguous.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--N", type=int, default=2048)
    ap.add_argument("--K", type=int, default=8192)
    ap.add_argument("--layout", default="nn")
    ap.add_argument("--impl", default="pipe")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ksplit", type=int, default=0)
    a = ap.parse_args()
    from paddle_infer_amd.ops.gemm import gemm
    ta, tb = a.layout[0] == "t", a.layout[1] == "n"
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(*((a.K, a.M) if ta else (a.M, a.K)), device="cuda", generator=g).bfloat16()
    B = torch.randn(*((a.N, a.K) if tb else (a.K, a.N)), device="cuda", generator=g).bfloat16()
    C = torch.empty(a.M, a.N, device="cuda", dtype=torch.bfloat16)
    for _ in range(a.iters):
        if a.impl == "hipblaslt":
            torch.mm(A.t() if ta else A, B.t() if tb else B, out=C)
        else:
            gemm(A, B, ta, tb, out=C, impl=a.impl, ksplit=a.ksplit or None)
    torch.cuda.synchronize()
    t = 2.0 * a.M * a.N * a.K
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        if a.impl == "hipblaslt":
            torch.mm(A.t() if ta else A, B.t() if tb else B, out=C)
        else:
            gemm(A, B, ta, tb, out=C, impl=a.impl, ksplit=a.ksplit or None)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(f"{a.impl} {a.layout} M{a.M} N{a.N} K{a.K}: {ms:.4f} ms {t / ms / 1e9:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
