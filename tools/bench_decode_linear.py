"""Serving-batch linears (GPT-3 1.3B shapes, M = decode rows): the packed weight-stream GEMV
(``packed_linear``, infer.hip wo_gemm) against the skinny MFMA GEMM (``gemm_small.hip``, best of a
small config sweep) and the dispatcher's default (``gemm_nt``), weights streamed from HBM.

  python tools/bench_decode_linear.py --M 8 16 32 64"""
import argparse
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from paddle_infer_amd.ops import gemm as G  # noqa: E402
from paddle_infer_amd.ops import inference as I  # noqa: E402


def timeit(fn, it=50):
    for _ in range(3):
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
    return e0.elapsed_time(e1) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[8, 16, 32, 64])
    a = ap.parse_args()
    for M in a.M:
        for K, N in ((2048, 6144), (2048, 2048), (2048, 8192), (8192, 2048)):
            R = max(2, (768 << 20) // (K * N * 2))
            ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(min(R, 24))]
            wps = [I.pack_bf16(w.t().contiguous()) for w in ws]
            ctr = itertools.count()
            x = torch.randn(M, K, device="cuda").bfloat16()
            ref = (x.float() @ ws[0].float().t())
            row = {"M": M, "K": K, "N": N}
            row["packed_us"] = round(timeit(lambda: I.packed_linear(x, wps[next(ctr) % len(wps)])), 2)
            best = None
            for cfg in [(1, 1, 1, 1, 1), (1, 2, 1, 1, 1), (2, 1, 1, 1, 1), (2, 2, 1, 1, 1), (1, 2, 1, 2, 1),
                        (2, 2, 1, 2, 1), (1, 1, 1, 1, 2), (1, 2, 1, 1, 2), (2, 2, 1, 1, 2), (4, 2, 1, 1, 1),
                        (2, 4, 1, 1, 1), (4, 1, 1, 1, 1)]:
                if 16 * cfg[0] > 2 * max(M, 16):
                    continue
                try:
                    out = G.small_gemm(x, ws[0], cfg=cfg)
                except Exception:  # noqa: BLE001
                    continue
                if (out.float() - ref).abs().max().item() > 0.05 * ref.abs().max().item():
                    continue
                t = timeit(lambda: G.small_gemm(x, ws[next(ctr) % len(ws)], cfg=cfg))
                if best is None or t < best[0]:
                    best = (t, cfg)
            row["small_us"], row["small_cfg"] = round(best[0], 2), str(best[1])
            row["default_us"] = round(timeit(lambda: G.gemm_nt(x, ws[next(ctr) % len(ws)])), 2)
            row["TBps_best"] = round(K * N * 2 / min(row["packed_us"], row["small_us"]) / 1e6, 3)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
