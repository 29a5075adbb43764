"""Fused add+LayerNorm microbenchmark (forward and backward of ``ops.norm.fused_add_layer_norm``
as used by the GPT block: bf16, bias + dropout + residual). Prints one JSON line with per-call
times and the effective HBM bandwidth of each pass. ``PIAMD_KERNEL_LIB`` selects another build
of the kernel library for A/B runs."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_infer_amd  # noqa: E402,F401
from paddle_infer_amd.ops.norm import fused_add_layer_norm, fused_add_rms_norm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32768)
    ap.add_argument("--hidden", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "f32"])
    ap.add_argument("--rms", action="store_true", help="fused residual + RMSNorm instead of LayerNorm")
    a = ap.parse_args()
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "f32": torch.float32}[a.dtype]
    dev = torch.device("cuda")
    R, N = a.rows, a.hidden
    x = torch.randn(R, N, device=dev, dtype=dt, requires_grad=True)
    res = torch.randn(R, N, device=dev, dtype=dt, requires_grad=True)
    w = torch.ones(N, device=dev, dtype=dt, requires_grad=True)
    b = torch.zeros(N, device=dev, dtype=dt, requires_grad=True)
    xb = torch.zeros(N, device=dev, dtype=dt, requires_grad=True)
    dy = torch.randn(R, N, device=dev, dtype=dt)
    dh = torch.randn(R, N, device=dev, dtype=dt)

    def fwd():
        if a.rms:
            return fused_add_rms_norm(x, res, w, x_bias=xb, dropout_p=a.dropout, training=True)
        return fused_add_layer_norm(x, res, w, b, x_bias=xb, dropout_p=a.dropout, training=True)

    def bwd(y, h):
        for t in (x, res, w, b, xb):  # no leaf-grad accumulation kernels inside the timing
            t.grad = None
        torch.autograd.backward([y, h], [dy, dh])

    for _ in range(3):
        y, h = fwd()
        bwd(y, h)
    torch.cuda.synchronize()
    tf = tb = 0.0
    for _ in range(a.iters):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        y, h = fwd()
        e1.record()
        bwd(y, h)
        e2.record()
        torch.cuda.synchronize()
        tf += e0.elapsed_time(e1)
        tb += e1.elapsed_time(e2)
    tf, tb = tf / a.iters, tb / a.iters
    el = R * N * x.element_size()
    # fwd: x, residual in; y, h out. bwd: dy, h, dh in; dres, dx out (dropout > 0)
    print(json.dumps({"rows": R, "hidden": N, "dtype": a.dtype, "rms": a.rms, "dropout": a.dropout, "fwd_ms": round(tf, 4),
                      "bwd_ms": round(tb, 4), "fwd_TBps": round(4 * el / tf / 1e9, 2),
                      "bwd_TBps": round(5 * el / tb / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
