"""Bias + activation microbenchmark (``ops.bias_act`` forward and backward on the GPT FFN shape:
[tokens, 4h] bf16, tanh GELU). One JSON line; run under ``rocprofv3 --kernel-trace --stats`` for
per-kernel times. ``PIAMD_KERNEL_LIB`` selects another kernel-library build for A/B runs."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_infer_amd  # noqa: E402,F401
from paddle_infer_amd.ops import bias_act  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32768)
    ap.add_argument("--cols", type=int, default=8192)
    ap.add_argument("--act", default="gelu_tanh")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda")
    x = torch.randn(a.rows, a.cols, device=dev, dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(a.cols, device=dev, dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(a.rows, a.cols, device=dev, dtype=torch.bfloat16)
    tf = tb = 0.0
    for it in range(a.iters + 3):
        x.grad = b.grad = None
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        y = bias_act(x, b, a.act)
        e1.record()
        y.backward(dy)
        e2.record()
        torch.cuda.synchronize()
        if it >= 3:
            tf += e0.elapsed_time(e1)
            tb += e1.elapsed_time(e2)
    tf, tb = tf / a.iters, tb / a.iters
    el = a.rows * a.cols * 2
    print(json.dumps({"rows": a.rows, "cols": a.cols, "act": a.act, "fwd_ms": round(tf, 4),
                      "bwd_ms": round(tb, 4), "fwd_TBps": round(2 * el / tf / 1e9, 2),
                      "bwd_TBps": round(3 * el / tb / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
