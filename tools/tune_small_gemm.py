"""Sweep the skinny MFMA GEMM's (mb, nb, wn, ks) on few-row shapes and compare with the assembly
GEMM and hipBLASLt (torch.matmul): prints one JSON line per shape with the best config.

Shapes: BERT-Large inference linears at M = 128 (batch 1 × seq 128), GPT-1.3B prefill / small-batch
projections, decode-batch rows.

  python tools/tune_small_gemm.py [--dtype fp16] [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from paddle_infer_amd.ops import gemm as G  # noqa: E402

SHAPES = [(M, N, K) for M in (128,) for N, K in ((3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096))] + \
         [(M, N, K) for M in (16, 32, 64, 256) for N, K in ((3072, 1024), (1024, 4096))] + \
         [(M, N, K) for M in (128, 256, 512) for N, K in ((6144, 2048), (2048, 2048), (8192, 2048), (2048, 8192))]


def bench(fn, iters, reps=3):
    """Device time per call: ``iters`` calls captured in one hipGraph, replayed (no host launch
    overhead — the way the Predictor / decode loop run them)."""
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        st, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        t = st.elapsed_time(e) * 1e3 / iters
        best = t if best is None else min(best, t)
    del g
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default="all", help="all | bert (the four M = 128 BERT-Large linears) | M,N,K;...")
    args = ap.parse_args()
    shapes = SHAPES
    if args.shapes == "bert":
        shapes = SHAPES[:4]
    elif args.shapes != "all":
        shapes = [tuple(int(v) for v in t.split(",")) for t in args.shapes.split(";")]
    dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    # weights rotated over > 512 MB so each call reads them from HBM, as in a real forward
    for M, N, K in shapes:
        nw = max(2, (512 << 20) // (N * K * 2))
        ws = [torch.randn(N, K, device="cuda", dtype=dt) * 0.05 for _ in range(min(nw, 64))]
        a = torch.randn(M, K, device="cuda", dtype=dt)
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % len(ws)
            return ws[it[0]]
        res = {}
        ref = a.float() @ ws[0].float().t()
        for mb, nb in sorted(G._SG_SHAPES):
            if 16 * mb > 2 * max(M, 16):
                continue
            for wn in (1, 2, 4):
              # depth: A ring | B ring << 4 (B-deep variants: A depth 1, wn 1)
              for depth in ((1, 2, 0x21, 0x41, 0x81) if wn == 1 else (1, 2)):
                for ks in (1, 2, 4, 8):
                    if ks > K // 64 // 2:
                        continue
                    cfg = (mb, nb, wn, depth, ks)
                    out = G.small_gemm(a, ws[0], cfg=cfg)
                    err = (out.float() - ref).abs().max().item()
                    if err > 0.05 * ref.abs().max().item():
                        res[str(cfg)] = "WRONG"
                        continue
                    res[str(cfg)] = bench(lambda: G.small_gemm(a, nxt(), cfg=cfg), args.iters)
        good = {k: v for k, v in res.items() if v != "WRONG"}
        best = min(good, key=good.get)
        heur = G.small_cfg(M, N, K)
        t_heur = bench(lambda: G.small_gemm(a, nxt(), cfg=heur), args.iters)
        t_blas = bench(lambda: torch.matmul(a, nxt().t()), args.iters)
        t_asm, asm_ks = None, None
        if K >= 128:
            for ks in (1, 2, 4, 8):
                if K % (64 * ks) or K // ks < 128:
                    continue
                t = bench(lambda: G.asm_gemm(a, nxt(), trans_b=True, ksplit=ks), args.iters)
                if t_asm is None or t < t_asm:
                    t_asm, asm_ks = t, ks
        wrong = [k for k, v in res.items() if v == "WRONG"]
        print(json.dumps({"M": M, "N": N, "K": K, "best": best, "best_us": round(good[best], 2),
                          "heuristic": str(heur), "heur_us": round(t_heur, 2),
                          "hipblaslt_us": round(t_blas, 2), "asm_us": round(t_asm, 2) if t_asm else None,
                          "asm_ks": asm_ks,
                          "top5": sorted(((round(v, 2), k) for k, v in good.items()))[:5],
                          "wrong": wrong}), flush=True)


if __name__ == "__main__":
    main()
