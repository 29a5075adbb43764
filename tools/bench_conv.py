"""Implicit-GEMM NHWC conv (``ops/conv.py``) vs the library (MIOpen) channels_last bf16 conv at
ResNet-50 shapes (batch 64): forward time and achieved TFLOP/s of each."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from paddle_infer_amd.ops import conv as CV  # noqa: E402
from paddle_infer_amd.ops.conv import conv2d_nhwc  # noqa: E402

SHAPES = [  # H, C, K, R, stride, pad
    (56, 64, 64, 1, 1, 0), (56, 64, 64, 3, 1, 1), (56, 64, 256, 1, 1, 0), (56, 256, 64, 1, 1, 0),
    (28, 128, 128, 3, 1, 1), (28, 128, 512, 1, 1, 0), (28, 512, 128, 1, 1, 0),
    (14, 256, 256, 3, 1, 1), (14, 256, 1024, 1, 1, 0), (14, 1024, 256, 1, 1, 0),
    (7, 512, 512, 3, 1, 1), (7, 512, 2048, 1, 1, 0), (7, 2048, 512, 1, 1, 0),
    (56, 128, 128, 3, 2, 1), (28, 256, 256, 3, 2, 1),
]


def timeit(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    for H, C, K, R, st, pad in SHAPES:
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(K, C, R, R, device="cuda") * 0.05).bfloat16()
        xcl = x.permute(0, 3, 1, 2)
        wcl = w.contiguous(memory_format=torch.channels_last)
        OH = (H + 2 * pad - R) // st + 1
        flop = 2 * N * OH * OH * K * C * R * R
        ours = timeit(lambda: conv2d_nhwc(x, w, None, st, pad))
        M, nk = N * OH * OH, R * R * C // 64
        sweep = {}
        for tn in (64, 128, 256):
            for ks in (1, 2, 4, 8):
                if ks > nk or (tn > 64 and K <= tn // 2):
                    continue
                CV.PLAN_OVERRIDE = (tn, ks)
                sweep[f"{tn}/{ks}"] = round(timeit(lambda: conv2d_nhwc(x, w, None, st, pad)), 1)
        CV.PLAN_OVERRIDE = None
        lib = timeit(lambda: F.conv2d(xcl, wcl, None, st, pad))
        print(json.dumps({"H": H, "C": C, "K": K, "R": R, "st": st, "ours_us": round(ours, 1),
                          "miopen_us": round(lib, 1), "ours_TF": round(flop / ours / 1e6, 1),
                          "miopen_TF": round(flop / lib / 1e6, 1),
                          "speedup": round(lib / ours, 2),
                          "plan": "%d/%d" % CV._plan(M, K, nk), "sweep": sweep}), flush=True)


if __name__ == "__main__":
    main()
