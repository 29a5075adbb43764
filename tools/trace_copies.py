"""Where do a Predictor run's copy / cast kernels come from? Runs a (shortened) BERT-Large fp16
Predictor eagerly under torch.profiler with Python stacks and prints every aten copy-like op with
its call count per run and the innermost framework frames.

  python tools/trace_copies.py [--layers 2] [--batch 128] [--dtype fp16]
"""
import argparse
import collections
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from paddle_infer_amd import inference as pinf, jit  # noqa: E402
from paddle_infer_amd.models.bert import BertModel, bert_config  # noqa: E402
from paddle_infer_amd.static import InputSpec  # noqa: E402

COPY_OPS = ("aten::copy_", "aten::to", "aten::_to_copy", "aten::contiguous", "aten::clone",
            "aten::cat", "aten::index_put_", "aten::zeros", "aten::fill_")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--runs", type=int, default=2)
    a = ap.parse_args()
    cfg = bert_config("bert-large")
    cfg.num_hidden_layers = a.layers
    torch.manual_seed(0)
    m = BertModel(cfg)
    m.eval()
    d = tempfile.mkdtemp(prefix="trace_copies_")
    jit.save(jit.to_static(m, input_spec=[InputSpec([None, 128], "int64", "input_ids")]),
             os.path.join(d, "model"))
    c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
    c.enable_use_gpu(1024, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Half if a.dtype == "fp16" else pinf.PrecisionType.Bfloat16)
    c.enable_hip_graph(False)
    pred = pinf.create_predictor(c)
    ids = torch.randint(1, cfg.vocab_size, (a.batch, 128), device="cuda")
    pred.get_input_handle(pred.get_input_names()[0]).share_external_data(ids)
    for _ in range(2):
        pred.run()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(a.runs):
            pred.run()
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name in COPY_OPS:
            frames = [f for f in (ev.stack or []) if "paddle_infer_amd" in f or "tools/" in f][:4]
            sites[(ev.name, " <- ".join(frames))] += 1
    for (name, where), n in sites.most_common(40):
        print(f"{n / a.runs:6.1f}/run  {name:18s} {where}")
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))


if __name__ == "__main__":
    main()
