"""Skinny-GEMM LayerNorm fold: kernel time per tile config at the serving-batch decode shapes,
LN mode vs the plain kernel of the same config (and the plain default + a separate LayerNorm).
Prints one JSON line per (shape, config)."""
import argparse
import json

import torch


def timeit(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    from paddle_infer_amd import ops
    from paddle_infer_amd.ops import gemm as G
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="32x6144x2048,32x8192x2048,8x6144x2048,64x6144x2048")
    a = ap.parse_args()
    cfgs = [(1, 1, 1, 2), (1, 2, 1, 2), (1, 4, 1, 2), (2, 1, 1, 2), (2, 2, 1, 2), (2, 4, 1, 2),
            (2, 2, 2, 2), (2, 2, 1, 1), (1, 2, 2, 2), (4, 1, 1, 2), (4, 2, 1, 2)]
    for sh in a.shapes.split(","):
        M, N, K = map(int, sh.split("x"))
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        g = torch.ones(K, device="cuda").bfloat16()
        b = torch.zeros(K, device="cuda").bfloat16()
        wf, c1, b2 = G.ln_fold(w, g, b, None)
        base = G.small_cfg(M, N, K)
        t_sep = timeit(lambda: G.small_gemm(ops.layer_norm(x, g, b, 1e-5), w))
        print(json.dumps({"M": M, "N": N, "K": K, "default_cfg": str(base),
                          "ln_launch_plus_default_us": round(t_sep, 2)}), flush=True)
        for c in cfgs:
            mb, nb, wn, d = c
            if 16 * mb > max(16, M) * 2:
                continue
            t_ln = timeit(lambda: G.small_gemm(x, wf, cfg=(*c, 1), ln=(c1, b2, 1e-5)))
            t_pl = timeit(lambda: G.small_gemm(x, w, cfg=(*c, 1)))
            print(json.dumps({"M": M, "N": N, "K": K, "cfg": str(c), "ln_us": round(t_ln, 2),
                              "plain_us": round(t_pl, 2)}), flush=True)


if __name__ == "__main__":
    main()
