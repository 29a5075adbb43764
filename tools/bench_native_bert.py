"""BERT-Large fp16 inference latency: the Python Predictor (hipGraph) vs the native C++ predictor
(`pd_infer_run --graph`, no Python) on the same IR-optimised model, per batch size.

  python tools/bench_native_bert.py [--batches 1,32,128] [--dtype fp16]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from paddle_infer_amd import inference as pinf, jit  # noqa: E402
from paddle_infer_amd.models.bert import BertModel, bert_config  # noqa: E402
from paddle_infer_amd.static import InputSpec  # noqa: E402

RUN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "paddle_infer_amd", "_lib", "pd_infer_run")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,32,128")
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    torch.manual_seed(0)
    m = BertModel(bert_config("bert-large"))
    m.eval()
    d = tempfile.mkdtemp(prefix="nbert_")
    jit.save(jit.to_static(m, input_spec=[InputSpec([None, 128], "int64", "input_ids")]), os.path.join(d, "model"))
    c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
    c.enable_use_gpu(1024, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Half if a.dtype == "fp16" else pinf.PrecisionType.Bfloat16)
    c.enable_hip_graph(True)
    c.enable_save_optim_model(True)
    c.set_optim_cache_dir(d)
    p = pinf.create_predictor(c)
    pre = os.path.join(d, "_optimized")
    for B in [int(b) for b in a.batches.split(",")]:
        ids = np.random.RandomState(B).randint(1, 30000, size=(B, 128)).astype("int64")
        h = p.get_input_handle(p.get_input_names()[0])
        h.share_external_data(torch.from_numpy(ids).cuda())
        for _ in range(3):
            p.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            p.run()
        torch.cuda.synchronize()
        py_ms = (time.perf_counter() - t0) / a.iters * 1e3
        ref = p.get_output_handle(p.get_output_names()[0]).copy_to_cpu().astype(np.float32)
        f = os.path.join(d, f"ids_{B}.bin")
        ids.tofile(f)
        r = subprocess.run([RUN, pre + ".pdmodel", pre + ".pdiparams", "--gpu", "0", "--graph", "--warmup", "3",
                            "--repeat", str(a.iters), "--input", "input_ids", "int64", f"{B},128", f,
                            "--output-dir", d], capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(r.stderr[-2000:], file=sys.stderr)
            sys.exit(1)
        nat_ms = float([ln.split()[1] for ln in r.stdout.splitlines() if ln.startswith("run_ms")][0])
        out0 = np.fromfile(os.path.join(d, "0.bin"), dtype=np.float32).reshape(ref.shape)
        print(json.dumps({"model": "bert-large", "dtype": a.dtype, "batch": B, "seq": 128,
                          "python_predictor_ms": round(py_ms, 3), "native_ms": round(nat_ms, 3),
                          "native_vs_python": round(py_ms / nat_ms, 3),
                          "native_seq_per_s": round(B / nat_ms * 1e3, 1),
                          "max_abs_diff": float(np.abs(out0 - ref).max())}), flush=True)


if __name__ == "__main__":
    main()
