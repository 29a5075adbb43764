"""Small-M inference linears (BERT-Large batch 1: M = 128 tokens) — hipBLASLt NN (Paddle [K, N]
weight), hipBLASLt TN (cached [N, K] weight) and the packed-weight MFMA stream kernel (wo_gemm,
bf16) per shape; weights rotated over > 768 MB so each call streams from HBM."""
import json
import sys

import torch

sys.path.insert(0, ".")
import paddle_infer_amd  # noqa: F401,E402
from paddle_infer_amd.ops import inference as I  # noqa: E402
from tools.bench_gemv import timeit  # noqa: E402


def main():
    for dt in (torch.float16, torch.bfloat16):
        for M in (128, 256, 512):
            for K, N in [(1024, 3072), (1024, 1024), (1024, 4096), (4096, 1024)]:
                R = max(2, (768 << 20) // (K * N * 2))
                ws = [(torch.randn(K, N, device="cuda") * 0.02).to(dt) for _ in range(R)]
                wts = [w.t().contiguous() for w in ws]
                b = torch.randn(N, device="cuda").to(dt)
                x = torch.randn(M, K, device="cuda").to(dt)
                it = iter(range(10 ** 9))
                r = {"dtype": str(dt).split(".")[-1], "M": M, "K": K, "N": N}
                r["nn_us"] = round(timeit(lambda: torch.addmm(b, x, ws[next(it) % R])), 2)
                r["tn_us"] = round(timeit(lambda: torch.addmm(b, x, wts[next(it) % R].t())), 2)
                if dt == torch.bfloat16:
                    wps = [I.pack_bf16(w) for w in ws]
                    r["packed_us"] = round(timeit(lambda: I.packed_linear(x, wps[next(it) % R], b)), 2)
                    del wps
                print(json.dumps(r), flush=True)
                del ws, wts


if __name__ == "__main__":
    main()
