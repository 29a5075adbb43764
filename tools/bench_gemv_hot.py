"""Decode GEMV (wo_gemm, packed bf16, M=1) with weights streamed from HBM (rotated over > MALL)
vs resident in the 256 MB Infinity Cache (same weight every call): how much a MALL prefetch of the
next layer's weights could save per GEMV."""
import json
import sys

import torch

sys.path.insert(0, ".")
import paddle_infer_amd  # noqa: F401,E402
from paddle_infer_amd.ops import inference as I  # noqa: E402
from tools.bench_gemv import timeit  # noqa: E402


def main():
    for K, N in [(2048, 6144), (2048, 2048), (2048, 8192), (8192, 2048)]:
        w = (torch.randn(K, N, device="cuda") * 0.02).bfloat16()
        R = max(2, (768 << 20) // (K * N * 2))
        wps = [I.pack_bf16(w) for _ in range(R)]
        x = torch.randn(1, K, device="cuda").bfloat16()
        it = iter(range(10 ** 9))
        cold = timeit(lambda: I.packed_linear(x, wps[next(it) % R]))
        hot = timeit(lambda: I.packed_linear(x, wps[0]))
        print(json.dumps({"K": K, "N": N, "MB": round(K * N * 2 / 2 ** 20, 1), "cold_us": round(cold, 2),
                          "hot_us": round(hot, 2)}), flush=True)


if __name__ == "__main__":
    main()
