"""Micro-benchmark: our MFMA flash attention vs torch SDPA (ROCm flash/aotriton) on the same
random bf16 data. Prints TFLOP/s for fwd and fwd+bwd (causal FLOPs counted as half)."""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_infer_amd  # noqa: E402,F401
from paddle_infer_amd.ops import flash_attention  # noqa: E402


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8,1024,16,128;4,2048,16,128;2,4096,16,128;8,1024,32,64")
    ap.add_argument("--causal", type=int, default=1)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--dropout", type=float, default=0.0)
    ap.add_argument("--mask", type=int, default=0, help="additive [1, 1, S, S] mask")
    ap.add_argument("--no-sdpa", action="store_true")
    args = ap.parse_args()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    out = []
    for s in args.shapes.split(";"):
        B, S, H, D = map(int, s.split(","))
        q = torch.randn(B, S, H, D, device="cuda", dtype=dt, requires_grad=True)
        mask = torch.randn(1, 1, S, S, device="cuda").to(dt) if args.mask else None
        kw = dict(causal=bool(args.causal), attn_mask=mask, dropout_p=args.dropout)
        k = torch.randn_like(q, requires_grad=True)
        v = torch.randn_like(q, requires_grad=True)
        do = torch.randn_like(q)
        flops = 4 * B * H * S * S * D * (0.5 if args.causal else 1.0)
        ours_f = timeit(lambda: flash_attention(q, k, v, **kw))

        def ours_fb():
            o = flash_attention(q, k, v, **kw)
            o.backward(do)
        ours_fb_t = timeit(ours_fb)
        if args.no_sdpa:
            print(json.dumps(dict(shape=s, causal=args.causal, dtype=args.dtype, dropout=args.dropout,
                                  mask=args.mask, ours_fwd_tflops=round(flops / ours_f / 1e12, 1),
                                  ours_fwdbwd_tflops=round(3.5 * flops / ours_fb_t / 1e12, 1),
                                  ours_fwd_ms=round(ours_f * 1e3, 3),
                                  ours_fwdbwd_ms=round(ours_fb_t * 1e3, 3))), flush=True)
            continue
        qt, kt, vt = (t.detach().transpose(1, 2).contiguous().requires_grad_() for t in (q, k, v))
        dot = do.transpose(1, 2).contiguous()
        sd = torch.nn.functional.scaled_dot_product_attention
        ref_f = timeit(lambda: sd(qt, kt, vt, is_causal=bool(args.causal)))

        def ref_fb():
            o = sd(qt, kt, vt, is_causal=bool(args.causal))
            o.backward(dot)
        ref_fb_t = timeit(ref_fb)
        r = dict(shape=s, causal=args.causal,
                 ours_fwd_tflops=round(flops / ours_f / 1e12, 1),
                 ours_fwdbwd_tflops=round(3.5 * flops / ours_fb_t / 1e12, 1),
                 sdpa_fwd_tflops=round(flops / ref_f / 1e12, 1),
                 sdpa_fwdbwd_tflops=round(3.5 * flops / ref_fb_t / 1e12, 1),
                 ours_fwd_ms=round(ours_f * 1e3, 3), ours_fwdbwd_ms=round(ours_fb_t * 1e3, 3),
                 sdpa_fwd_ms=round(ref_f * 1e3, 3), sdpa_fwdbwd_ms=round(ref_fb_t * 1e3, 3))
        print(json.dumps(r), flush=True)
        out.append(r)


if __name__ == "__main__":
    main()
