"""Streaming floor of MI355X for the weight sizes of decode / small-batch GEMVs: device time of
reading N bytes once (a column-sum over a [rows, 2048] bf16 tensor: torch's reduce and the
framework's colsum) and of a device copy, at 4-256 MB, graph-timed with rotating buffers (> MALL),
next to the packed GEMV (M = 1 / 32) at the same byte counts. Tells how far a short kernel is from
its ramp floor.

  python tools/bench_stream_floor.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from paddle_infer_amd.ops import inference as I  # noqa: E402


def timeit(fn, it=40):
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
    for mb in (4, 8, 16, 25, 33, 64, 128, 256):
        n = mb << 20
        rows = n // (2048 * 2)
        R = max(2, (1024 << 20) // n)
        bufs = [torch.randn(rows, 2048, device="cuda").bfloat16() for _ in range(min(R, 16))]
        outs = [torch.empty_like(b) for b in bufs[:2]]
        it = iter(range(10 ** 9))
        row = {"MB": mb}
        row["sum_us"] = round(timeit(lambda: bufs[next(it) % len(bufs)].sum(0)), 2)
        row["copy_us"] = round(timeit(lambda: outs[0].copy_(bufs[next(it) % len(bufs)])), 2)
        # packed GEMV with the same weight bytes: K = 2048, N = rows
        if rows % 32 == 0:
            wps = [I.pack_bf16(b.t().contiguous()) for b in bufs[:min(len(bufs), 8)]]
            for M in (1, 32):
                x = torch.randn(M, 2048, device="cuda").bfloat16()
                row[f"gemv_m{M}_us"] = round(timeit(lambda: I.packed_linear(x, wps[next(it) % len(wps)])), 2)
        row["sum_TBps"] = round(n / row["sum_us"] / 1e6, 2)
        row["copy_TBps_rw"] = round(2 * n / row["copy_us"] / 1e6, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
