"""Weight-gradient GEMM layout A/B on hipBLASLt for the GPT-3 1.3B shapes (T = 65536 tokens):
(a) main_grad.addmm_(x^T, dy)  (b) mm(x^T, dy) into a temp + add  (c) mm(dy^T, x) (transposed
product, the NT kernel family) + add of its transpose. Interleaved rounds, median ms."""
import json
import sys

import torch

T = 65536
SHAPES = {"qkv": (2048, 6144), "out": (2048, 2048), "ffn1": (2048, 8192), "ffn2": (8192, 2048)}


def main(dtype_name="bfloat16"):
    dt = getattr(torch, dtype_name)
    res = {}
    for name, (IN, OUT) in SHAPES.items():
        x = torch.randn(T, IN, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, OUT, device="cuda", dtype=torch.bfloat16)
        mg = torch.zeros(IN, OUT, device="cuda", dtype=dt)
        tmp = torch.empty(IN, OUT, device="cuda", dtype=torch.bfloat16)
        tmpt = torch.empty(OUT, IN, device="cuda", dtype=torch.bfloat16)
        fns = {
            "a_addmm": lambda: mg.addmm_(x.t(), dy),
            "b_mm_add": lambda: mg.add_(torch.mm(x.t(), dy, out=tmp)),
            "c_mmT_add": lambda: mg.add_(torch.mm(dy.t(), x, out=tmpt).t()),
        }
        times = {k: [] for k in fns}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        for _ in range(5):
            for k, f in fns.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(3):
                    f()
                e.record()
                e.synchronize()
                times[k].append(s.elapsed_time(e) / 3)
        flops = 2 * T * IN * OUT
        res[name] = {k: {"ms": round(sorted(v)[2], 3), "tflops": round(flops / sorted(v)[2] / 1e9, 1)}
                     for k, v in times.items()}
        print(json.dumps({name: res[name], "main_grad": dtype_name}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "bfloat16")
