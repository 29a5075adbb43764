"""BERT-Large inference through the Paddle Inference API (BASELINE.json config 4).

Path measured: dygraph ``BertModel`` → ``jit.save`` (Paddle-wire ``.pdmodel`` + ``.pdiparams``) →
``inference.Config`` + IR fusion passes + 16-bit mixed precision + hipGraph capture →
``Predictor.run``. Reference path: `paddle/fluid/inference/api/analysis_predictor.cc` with the GPU
pass list of `paddle_pass_builder.cc` and `enable_use_gpu` + fp16 (`exp_enable_use_gpu_fp16`).

Synthetic token ids, random-init BERT-Large weights (24 layers, hidden 1024, 16 heads, FFN 4096,
vocab 30522). The 16-bit dtype is bf16: every hand-written MI355X kernel is bf16-native (same
width / bandwidth as fp16, wider exponent); ``--dtype fp16`` runs BASELINE config 4 as written
(fp16 LayerNorm / softmax / flash-attention / bias-act kernels). Reports sequences/s per batch size for
(a) the Predictor (passes + hipGraph) and (b) the same model run eagerly in dygraph bf16, and the
max |Predictor − fp32 dygraph| on the final hidden states.

  python tools/bench_bert_infer.py [--seq 128] [--batches 1,8,32,128] [--iters 20]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import paddle_infer_amd  # noqa: E402,F401
from paddle_infer_amd import inference as pinf  # noqa: E402
from paddle_infer_amd import jit  # noqa: E402
from paddle_infer_amd.models.bert import BertModel, bert_config  # noqa: E402
from paddle_infer_amd.static import InputSpec  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-large")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--batches", default="1,8,32,128")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--predictor-only", action="store_true",
                    help="skip the fp32 reference and the eager timing (clean rocprof traces)")
    a = ap.parse_args()
    h16 = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    torch.manual_seed(0)
    cfg = bert_config(a.model)
    dev = torch.device("cuda", 0)
    model = BertModel(cfg)
    model.eval()
    d = tempfile.mkdtemp(prefix="bert_infer_")
    st = jit.to_static(model, input_spec=[InputSpec([None, a.seq], "int64", "input_ids")])
    jit.save(st, os.path.join(d, "model"))
    c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
    c.enable_use_gpu(1024, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Half if a.dtype == "fp16"
                                 else pinf.PrecisionType.Bfloat16)
    c.enable_hip_graph(not a.no_graph)
    pred = pinf.create_predictor(c)
    fused = {k: v for k, v in getattr(pred, "pass_stats", {}).items() if v}
    ops = [o.type for o in pred.program.global_block().ops]

    model_gpu = model.to(dev)
    ref32 = None
    model_bf = BertModel(cfg)
    model_bf.set_state_dict(model.state_dict())
    model_bf = model_bf.to(dev).to(h16)
    model_bf.eval()
    results = []
    for B in [int(b) for b in a.batches.split(",")]:
        ids = torch.randint(1, cfg.vocab_size, (B, a.seq), device=dev)
        h = pred.get_input_handle(pred.get_input_names()[0])
        h.share_external_data(ids)
        pred.run()
        out = pred.get_output_handle(pred.get_output_names()[0]).to_torch()
        if a.predictor_only:
            t_pred = timeit(lambda: pred.run(), a.iters)
            print(json.dumps({"model": a.model, "batch": B, "seq": a.seq, "dtype": a.dtype,
                              "predictor_ms": round(t_pred * 1e3, 3),
                              "predictor_seq_per_s": round(B / t_pred, 1)}), flush=True)
            continue
        with torch.no_grad():
            ref32 = model_gpu(ids)[0]
        err = (out.float() - ref32).abs().max().item()
        t_pred = timeit(lambda: pred.run(), a.iters)
        with torch.no_grad():
            t_eager = timeit(lambda: model_bf(ids), a.iters)
        r = {"model": a.model, "batch": B, "seq": a.seq, "dtype": a.dtype,
             "predictor_ms": round(t_pred * 1e3, 3), "predictor_seq_per_s": round(B / t_pred, 1),
             "eager_ms": round(t_eager * 1e3, 3), "eager_seq_per_s": round(B / t_eager, 1),
             "speedup_vs_eager": round(t_eager / t_pred, 2), "max_abs_err_vs_fp32": round(err, 4),
             "hip_graph": not a.no_graph}
        results.append(r)
        print(json.dumps(r), flush=True)
    print(json.dumps({"passes_fired": fused, "op_types": sorted(set(ops))}), flush=True)


if __name__ == "__main__":
    main()
