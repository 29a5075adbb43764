"""GEMM microbenchmark: hand-written gemm.hip vs torch.matmul (hipBLASLt) on the GPT-1.3B training
shapes (T = 16384 tokens). Prints one JSON line per (shape, layout, impl) with TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
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
    T = int(os.environ.get("T", 16384))
    shapes = [(2048, 6144), (2048, 2048), (2048, 8192), (8192, 2048)]  # (K_in, N_out) of x @ W
    rows = []
    for K, N in shapes:
        x = torch.randn(T, K, device="cuda").bfloat16()
        w = (0.02 * torch.randn(K, N, device="cuda")).bfloat16()
        dy = torch.randn(T, N, device="cuda").bfloat16()
        dw = torch.zeros(K, N, device="cuda")
        fl = 2.0 * T * K * N
        cases = {
            "fwd_NN": (lambda: gemm(x, w), lambda: torch.matmul(x, w)),
            "dgrad_TN": (lambda: gemm(dy, w, trans_b=True), lambda: torch.matmul(dy, w.t())),
            "wgrad_f32acc": (lambda: gemm(x, dy, trans_a=True, out=dw, accumulate=True),
                             lambda: dw.addmm_(x.t().float(), dy.float()) if False else torch.matmul(x.t(), dy, out=None)),
        }
        for name, (ours, ref) in cases.items():
            for impl, fn in (("piamd", ours), ("hipblaslt", ref)):
                ms = timeit(fn)
                r = {"K": K, "N": N, "T": T, "case": name, "impl": impl, "ms": round(ms, 4),
                     "tflops": round(fl / ms / 1e9, 1)}
                print(json.dumps(r), flush=True)
                rows.append(r)
    out = os.environ.get("OUT")
    if out:
        with open(out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
