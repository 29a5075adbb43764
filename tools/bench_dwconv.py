"""Depthwise 3x3 conv kernels (csrc/kernels/conv_dw.hip) at the 17 MobileNetV2 layer shapes
(batch 128, 224x224 input, bf16 NHWC): weight-gradient time per layer, plus the bytes it must read.

  python tools/bench_dwconv.py [--batch 128]
Prints one JSON line per layer and a total."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

# (H, C, stride) of MobileNetV2's depthwise convs at 224x224 input
LAYERS = [(112, 32, 1), (112, 96, 2), (56, 144, 1), (56, 144, 2), (28, 192, 1), (28, 192, 1),
          (28, 192, 2), (14, 384, 1), (14, 384, 1), (14, 384, 1), (14, 384, 1), (14, 576, 1),
          (14, 576, 1), (14, 576, 2), (7, 960, 1), (7, 960, 1), (7, 960, 1)]


def timed(fn, iters):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from paddle_infer_amd.ops.conv import _direct, _direct_wgrad
    tot = tot_f = 0.0
    for H, C, s in LAYERS:
        OH = (H + 2 - 3) // s + 1
        x = torch.randn(a.batch, H, H, C, device="cuda").bfloat16()
        dy = torch.randn(a.batch, OH, OH, C, device="cuda").bfloat16()
        ms = timed(lambda: _direct_wgrad(x, dy, 3, 3, (s, s), (1, 1), (1, 1), C, C, groups=C), a.iters)
        tot += ms
        w = torch.randn(3, 3, 1, C, device="cuda").bfloat16()
        msf = timed(lambda: _direct(x, w, None, OH, OH, C, 3, 3, (s, s), (1, 1), (1, 1), 1, 1, False), a.iters)
        tot_f += msf
        gb = (x.numel() + dy.numel()) * 2 / 1e9
        print(json.dumps({"H": H, "C": C, "stride": s, "wgrad_ms": round(ms, 4), "fwd_ms": round(msf, 4),
                          "min_bytes_GB": round(gb, 3), "GBps": round(gb / ms * 1e3, 1)}), flush=True)
    print(json.dumps({"total_wgrad_ms": round(tot, 3), "total_fwd_ms": round(tot_f, 3)}))


if __name__ == "__main__":
    main()
