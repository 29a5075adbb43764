"""hipBLASLt (torch) vs gemm.hip on every GEMM of a GPT-1.3B training step, for both weight
storage layouts ([in,out] = Paddle's, and [out,in]). Random normal operands (DVFS-honest).
Prints one JSON line per (shape, pass, layout, impl)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    return e0.elapsed_time(e1) / iters


def main():
    from paddle_infer_amd.ops.gemm import gemm
    T = int(os.environ.get("T", 32768))
    shapes = [(2048, 6144), (2048, 2048), (2048, 8192), (8192, 2048), (2048, 50304)]
    for K, N in shapes:
        x = torch.randn(T, K, device="cuda").bfloat16()
        w = (0.02 * torch.randn(K, N, device="cuda")).bfloat16()
        wt = w.t().contiguous()
        dy = torch.randn(T, N, device="cuda").bfloat16()
        mg = torch.zeros(K, N, device="cuda", dtype=torch.bfloat16)
        mgt = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * K * N
        cases = [
            ("fwd", "w_in_out", lambda: torch.mm(x, w)),
            ("fwd", "w_out_in", lambda: torch.mm(x, wt.t())),
            ("dgrad", "w_in_out", lambda: torch.mm(dy, w.t())),
            ("dgrad", "w_out_in", lambda: torch.mm(dy, wt)),
            ("wgrad_acc", "w_in_out", lambda: mg.addmm_(x.t(), dy)),
            ("wgrad_acc", "w_out_in", lambda: mgt.addmm_(dy.t(), x)),
            ("wgrad", "w_in_out", lambda: torch.mm(x.t(), dy)),
            ("wgrad", "w_out_in", lambda: torch.mm(dy.t(), x)),
        ]
        if N % 256 == 0:
            cases += [
                ("fwd", "w_in_out/piamd", lambda: gemm(x, w)),
                ("dgrad", "w_in_out/piamd", lambda: gemm(dy, w, trans_b=True)),
                ("fwd", "w_out_in/piamd", lambda: gemm(x, wt, trans_b=True)),
            ]
        for p, lay, fn in cases:
            ms = timeit(fn)
            print(json.dumps({"K": K, "N": N, "T": T, "pass": p, "layout": lay, "ms": round(ms, 4),
                              "tflops": round(fl / ms / 1e9, 1)}), flush=True)
        del x, w, wt, dy, mg, mgt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
