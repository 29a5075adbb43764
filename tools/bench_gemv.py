"""Decode GEMV (packed-bf16 / int8 / int4 weight-stream MFMA kernel, ``infer.hip`` wo_gemm) at
GPT-3 1.3B shapes: time per call and achieved HBM bandwidth for each split-K factor, to pick the
split heuristic (``ops.inference._split_k``)."""
import json
import sys

import torch

sys.path.insert(0, ".")
import paddle_infer_amd  # noqa: F401,E402
from paddle_infer_amd.ops import inference as I  # noqa: E402


def timeit(fn, it=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3  # us


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--ks", type=int, nargs="+", default=[1, 2, 4, 8, 16, 32])
    a = ap.parse_args()
    shapes = [(2048, 6144), (2048, 2048), (2048, 8192), (8192, 2048)]
    orig = I._split_k
    rows = []
    for M in a.M:
        for K, N in shapes:
            w = (torch.randn(K, N, device="cuda") * 0.02).bfloat16()
            # rotate over enough copies (> 256 MB MALL) that every call streams from HBM
            R = max(2, (768 << 20) // (K * N * 2))
            wps = [I.pack_bf16(w) for _ in range(R)]
            it = iter(range(10 ** 9))
            x = torch.randn(M, K, device="cuda").bfloat16()
            for KS in a.ks:
                if (K // 16) % KS:
                    continue
                I._split_k = lambda tiles, kb, KS=KS: KS
                try:
                    us = timeit(lambda: I.packed_linear(x, wps[next(it) % R]))
                except Exception as e:  # noqa: BLE001
                    us = float("nan")
                rows.append({"M": M, "K": K, "N": N, "KS": KS, "us": round(us, 2),
                             "TBps": round(K * N * 2 / us / 1e6, 3)})
                print(json.dumps(rows[-1]), flush=True)
            I._split_k = orig
            rows.append({"M": M, "K": K, "N": N, "KS": "auto",
                         "us": round(timeit(lambda: I.packed_linear(x, wps[next(it) % R])), 2)})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
