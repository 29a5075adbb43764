"""Where do a Predictor run's device copies / casts come from? Runs one BERT-Large fp16 Predictor
step (no hipGraph) under a TorchDispatchMode that records every aten op that moves data without
computing (copy_, _to_copy, clone, contiguous copies, cat, …) with its shapes and the innermost
framework frames of the Python stack.

  python tools/trace_copies.py [--batch 128 --layers 24]"""
import argparse
import collections
import os
import sys
import tempfile
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

MOVERS = ("copy_", "_to_copy", "clone", "cat", "index_select", "index", "expand_copy", "_copy_from",
          "constant_pad_nd", "fill_", "zero_", "zeros", "new_zeros", "masked_fill", "where")


class _Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.cnt = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if any(name == m or name.startswith(m) for m in MOVERS):
            shapes = [tuple(a.shape) + (str(a.dtype).replace("torch.", ""),) for a in args
                      if isinstance(a, torch.Tensor)][:3]
            fr = [f for f in traceback.extract_stack() if "paddle_infer_amd" in f.filename][-3:]
            where = " <- ".join(f"{f.filename.split('paddle_infer_amd/')[-1]}:{f.lineno}" for f in reversed(fr))
            self.cnt[(name, str(shapes)[:100], where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--layers", type=int, default=24)
    a = ap.parse_args()
    from paddle_infer_amd import inference as pinf, jit
    from paddle_infer_amd.models.bert import BertModel, bert_config
    from paddle_infer_amd.static import InputSpec
    cfg = bert_config("bert-large", num_hidden_layers=a.layers)
    m = BertModel(cfg).eval()
    d = tempfile.mkdtemp()
    jit.save(jit.to_static(m, input_spec=[InputSpec([None, 128], "int64", "input_ids")]), os.path.join(d, "model"))
    c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
    c.enable_use_gpu(1024, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Half)
    c.enable_hip_graph(False)
    p = pinf.create_predictor(c)
    ids = torch.randint(1, cfg.vocab_size, (a.batch, 128), device="cuda")
    p.get_input_handle(p.get_input_names()[0]).share_external_data(ids)
    for _ in range(2):
        p.run()
    torch.cuda.synchronize()
    rec = _Rec()
    with rec:
        p.run()
    torch.cuda.synchronize()
    print(f"# data-moving aten ops in one run ({a.layers} layers, batch {a.batch}):")
    for (n, shp, st), k in rec.cnt.most_common(40):
        print(f"{k:4d}  {n:16s} {shp}\n        {st}")


if __name__ == "__main__":
    main()
