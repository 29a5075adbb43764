"""Own MFMA GEMMs (gemm_pipe.hip) against hipBLASLt on every GPT-3 1.3B training GEMM.

T tokens per step (default 65536 = micro-batch 64 × seq 1024, the bench.py config). For each
projection (K_in → N_out) the three training products, in the layouts the training path uses:

  fwd    y[T,N]   = x[T,K] · Wtᵀ          Wt = [N,K] (cached transposed weight; both K-contiguous)
  dgrad  dx[T,K]  = dy[T,N] · Wᵀ          W  = [K,N] (Paddle layout = [N][K]ᵀ, both K-contiguous)
  wgrad  W[K,N]  += xᵀ · dy               x, dy token-major (both operands M/N-contiguous), bf16
                                          main_grad accumulate

plus the LM head (V = 50304). Variants are timed in interleaved rounds in ONE process (guide
§5.4 rule 24); the median over rounds is printed with the max error vs hipBLASLt.

  python tools/bench_gemm_train.py [--T 65536] [--rounds 5] [--only fwd,dgrad,wgrad]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--shapes", default="qkv,out,ffn1,ffn2,head")
    args = ap.parse_args()
    from paddle_infer_amd.ops.gemm import gemm, pick_ksplit
    T = args.T
    shapes = {"qkv": (2048, 6144), "out": (2048, 2048), "ffn1": (2048, 8192), "ffn2": (8192, 2048),
              "head": (2048, 50304)}
    passes = args.only.split(",")
    gen = torch.Generator(device="cuda").manual_seed(0)
    for name in args.shapes.split(","):
        K, N = shapes[name]
        x = torch.randn(T, K, device="cuda", generator=gen).bfloat16()
        dy = (0.1 * torch.randn(T, N, device="cuda", generator=gen)).bfloat16()
        w = (0.02 * torch.randn(K, N, device="cuda", generator=gen)).bfloat16()
        wt = w.t().contiguous()
        mg = torch.zeros(K, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * K * N
        cases = []
        if "fwd" in passes:
            ref = torch.mm(x, wt.t())
            cases += [("fwd", "hipblaslt", lambda: torch.mm(x, wt.t()), ref, None),
                      ("fwd", "pipe", lambda: gemm(x, wt, trans_b=True, impl="pipe"), ref, None)]
        if "dgrad" in passes:
            ref = torch.mm(dy, w.t())
            cases += [("dgrad", "hipblaslt", lambda: torch.mm(dy, w.t()), ref, None),
                      ("dgrad", "pipe", lambda: gemm(dy, w, trans_b=True, impl="pipe"), ref, None)]
        if "wgrad" in passes:
            ref = torch.mm(x.t().float(), dy.float())
            ks = pick_ksplit(K, N, T)
            cases += [("wgrad", "hipblaslt", lambda: mg.addmm_(x.t(), dy), ref, "mg"),
                      ("wgrad", f"pipe_ks{ks}",
                       lambda: gemm(x, dy, trans_a=True, out=mg, accumulate=True, impl="pipe"), ref,
                       "mg")]
        errs = {}
        for pas, impl, fn, ref, kind in cases:
            if kind == "mg":
                mg.zero_()
                fn()
                got = mg
            else:
                got = fn()
            torch.cuda.synchronize()
            errs[(pas, impl)] = (got.float() - ref.float()).abs().max().item()
            for _ in range(2):
                fn()
        times = {(c[0], c[1]): [] for c in cases}
        for _ in range(args.rounds):
            for pas, impl, fn, _, _ in cases:
                times[(pas, impl)].append(timeit(fn, args.iters))
        for (pas, impl), ts in times.items():
            ms = statistics.median(ts)
            print(json.dumps({"shape": name, "T": T, "K": K, "N": N, "pass": pas, "impl": impl,
                              "ms": round(ms, 4), "min_ms": round(min(ts), 4),
                              "tflops": round(fl / ms / 1e9, 1),
                              "max_err": round(errs[(pas, impl)], 4)}), flush=True)
        del x, dy, w, wt, mg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
