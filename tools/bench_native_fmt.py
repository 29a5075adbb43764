"""fused_multi_transformer decode latency: the native C++ engine (C API in process, no Python inside
the engine; and `pd_infer_run` eager / hipGraph) against the Python Predictor, on a GPT-1.3B-width
program (E 2048, 16 heads, FFN 8192; --layers of them, random weights) at batch 1.

  python tools/bench_native_fmt.py --layers 4 --steps 64
Prints one JSON line per engine: median ms per decode step (caches resident, TimeStep advanced)."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--E", type=int, default=2048)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--maxs", type=int, default=512)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--steps", type=int, default=64)
    a = ap.parse_args()
    from fmt_wire import write_fmt_program
    from native_capi import PD_PRECISION_BFLOAT16, Predictor
    from paddle_infer_amd import inference as pinf
    from paddle_infer_amd.incubate.nn import FusedMultiTransformer
    torch.manual_seed(0)
    E, H, L = a.E, a.heads, a.layers
    D = E // H
    layer = FusedMultiTransformer(E, H, 4 * E, num_layers=L)
    layer.eval()
    for p in layer.parameters():
        p.data.mul_(0.02 / max(p.data.std().item(), 1e-6) if p.dim() > 1 else 1.0)
    tmp = tempfile.mkdtemp()
    dec = os.path.join(tmp, "dec")
    write_fmt_program(layer, dec, True, L, E)
    del layer
    dev = torch.device("cuda")
    res = {}

    # Python Predictor
    c = pinf.Config(dec + ".pdmodel", dec + ".pdiparams")
    c.enable_use_gpu(256, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Bfloat16)
    pp = pinf.create_predictor(c)
    caches = [torch.zeros(2, 1, H, a.maxs, D, dtype=torch.bfloat16, device=dev) for _ in range(L)]
    x = torch.randn(1, 1, E, device=dev).to(torch.bfloat16)
    pp.get_input_handle("x").share_external_data(x)
    for i, cc in enumerate(caches):
        pp.get_input_handle(f"cache_kv.{i}").share_external_data(cc)
    ms = []
    for t in range(a.steps):
        pp.get_input_handle("time_step").copy_from_cpu(np.array([a.prompt + t], dtype=np.int32))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pp.run()
        pp.get_output_handle("out").to_torch()
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
    res["python_predictor"] = float(np.median(ms[4:]))
    del pp

    # native engine, C API in process (eager)
    nd = Predictor(dec, 0, PD_PRECISION_BFLOAT16)
    caches_n = [torch.zeros_like(cc) for cc in caches]
    torch.cuda.synchronize()
    nd.share("x", x)
    for i, cc in enumerate(caches_n):
        nd.share(f"cache_kv.{i}", cc)
    ms = []
    for t in range(a.steps):
        nd.feed("time_step", np.array([a.prompt + t], dtype=np.int32))
        t0 = time.perf_counter()
        nd.run()
        nd.fetch_float("out", (1, 1, E))
        ms.append((time.perf_counter() - t0) * 1e3)
    res["native_capi_eager"] = float(np.median(ms[4:]))
    nd.close()

    # pd_infer_run (C++ driver), eager and hipGraph, caches fed once and kept resident
    run = os.path.join(ROOT, "paddle_infer_amd", "_lib", "pd_infer_run")
    args = []
    feeds = {"x": np.random.RandomState(0).randn(1, 1, E).astype(np.float32),
             "time_step": np.array([a.prompt], dtype=np.int32)}
    for i in range(L):
        feeds[f"cache_kv.{i}"] = np.zeros((2, 1, H, a.maxs, D), dtype=np.float32)
    for n, arr in feeds.items():
        f = os.path.join(tmp, f"in_{n}.bin")
        arr.tofile(f)
        args += ["--input", n, str(arr.dtype), ",".join(map(str, arr.shape)), f]
    for mode in ("eager", "graph"):
        cmd = [run, dec + ".pdmodel", dec + ".pdiparams", "--gpu", "0", "--precision", "bf16", "--step-input",
               "time_step", "--warmup", "4", "--repeat", str(a.steps), "--output-dir", tmp] + args
        if mode == "graph":
            cmd.append("--graph")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(r.stderr + r.stdout, file=sys.stderr)
            raise SystemExit(1)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("run_ms")][0]
        res[f"pd_infer_run_{mode}"] = float(line.split()[1])
    print(json.dumps({"model": f"FMT E{E} H{H} L{L}", "batch": 1, "maxs": a.maxs,
                      "ms_per_step": {k: round(v, 4) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
