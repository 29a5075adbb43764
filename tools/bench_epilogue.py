"""Assembly-GEMM fused epilogue cost: C = act(A·Bᵀ + bias) at a BERT-Large FFN1 shape, per
activation (none / bias / bias+GELU(erf) / bias+GELU(tanh) / bias+ReLU), fp16 and bf16.

  python tools/bench_epilogue.py [--M 16384 --N 4096 --K 1024]
Prints one JSON line per (dtype, epilogue): median ms over --iters launches."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    from paddle_infer_amd.ops.gemm import gemm_nt
    for dt in (torch.float16, torch.bfloat16):
        x = torch.randn(a.M, a.K, device="cuda").to(dt)
        w = (torch.randn(a.N, a.K, device="cuda") * 0.03).to(dt)
        b = torch.randn(a.N, device="cuda").to(dt)
        for name, bias, act in (("plain", None, "none"), ("bias", b, "none"), ("bias_gelu_erf", b, "gelu"),
                                ("bias_gelu_tanh", b, "gelu_tanh"), ("bias_relu", b, "relu")):
            for _ in range(3):
                gemm_nt(x, w, bias=bias, act=act)
            ts = []
            for _ in range(a.iters):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gemm_nt(x, w, bias=bias, act=act)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            ms = ts[len(ts) // 2]
            print(json.dumps({"dtype": str(dt).split(".")[-1], "epilogue": name, "M": a.M, "N": a.N, "K": a.K,
                              "ms": round(ms, 4), "tflops": round(2 * a.M * a.N * a.K / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
