"""fft.hip (LDS Stockham) vs rocFFT (torch.fft) on batched complex64 rows, interleaved rounds."""
import json
import sys

import torch

sys.path.insert(0, ".")
from paddle_infer_amd.ops import fft as F  # noqa: E402


def main():
    for N, rows in ((64, 1 << 16), (256, 1 << 14), (1024, 1 << 13), (4096, 1 << 11)):
        x = torch.randn(rows, N, dtype=torch.complex64, device="cuda")
        fns = {"piamd": lambda: F._pow2(x, False), "rocfft": lambda: torch.fft.fft(x)}
        t = {k: [] for k in fns}
        for f in fns.values():
            f()
        for _ in range(5):
            for k, f in fns.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    f()
                e.record()
                e.synchronize()
                t[k].append(s.elapsed_time(e) / 10)
        gb = 2 * x.numel() * 8 / 1e9
        res = {k: {"us": round(sorted(v)[2] * 1e3, 1), "GB/s": round(gb / (sorted(v)[2] / 1e3), 0)}
               for k, v in t.items()}
        print(json.dumps({"N": N, "rows": rows, **res}), flush=True)


if __name__ == "__main__":
    main()
