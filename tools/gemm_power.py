"""Clock / power side by side for the assembly GEMM and hipBLASLt on the same operands: each
kernel runs back-to-back for a few seconds while a sampler thread polls `rocm-smi --showclocks
--showpower --json`; prints TFLOP/s with the median SCLK and socket power seen under it.

  python tools/gemm_power.py [M,N,K] [seconds]
"""
import json
import os
import re
import subprocess
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_infer_amd  # noqa: E402,F401
from paddle_infer_amd.ops import gemm  # noqa: E402


def smi_sample():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--json"], capture_output=True,
                             text=True, timeout=5).stdout
        d = json.loads(out)
    except Exception:
        return None
    card = next(iter(d.values())) if d else {}
    sclk = pwr = None
    for k, v in card.items():
        kl = k.lower()
        if "sclk" in kl and sclk is None:
            m = re.search(r"(\d+)\s*mhz", str(v).lower())
            if m:
                sclk = int(m.group(1))
        if "power" in kl and "socket" in kl or ("average graphics package power" in kl):
            try:
                pwr = float(re.findall(r"[\d.]+", str(v))[0])
            except (IndexError, ValueError):
                pass
    return sclk, pwr


def run(fn, secs, flops):
    samples, stop = [], threading.Event()

    def sampler():
        while not stop.is_set():
            s = smi_sample()
            if s:
                samples.append(s)
            time.sleep(0.1)

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    th = threading.Thread(target=sampler)
    th.start()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < secs:
        for _ in range(10):
            fn()
        n += 10
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stop.set()
    th.join()
    sc = sorted(s[0] for s in samples if s[0])
    pw = sorted(s[1] for s in samples if s[1])
    return dict(tflops=round(flops * n / dt / 1e12, 1), ms=round(dt / n * 1e3, 4),
                sclk_mhz_median=sc[len(sc) // 2] if sc else None,
                power_w_median=pw[len(pw) // 2] if pw else None, samples=len(samples))


def main():
    M, N, K = map(int, (sys.argv[1] if len(sys.argv) > 1 else "8192,8192,8192").split(","))
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    flops = 2.0 * M * N * K
    res = {"shape": [M, N, K]}
    res["asm"] = run(lambda: gemm.asm_gemm(a, b, trans_b=True, out=c), secs, flops)
    res["hipblaslt"] = run(lambda: torch.matmul(a, b.t(), out=c), secs, flops)
    res["asm_again"] = run(lambda: gemm.asm_gemm(a, b, trans_b=True, out=c), secs, flops)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
