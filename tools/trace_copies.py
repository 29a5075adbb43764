"""Where do a Predictor run's device copies come from? Profiles one BERT-Large fp16 Predictor run
(no hipGraph) with torch.profiler and prints each aten copy / cast with its shapes and the
innermost framework frames of its Python stack.

  python tools/trace_copies.py [--batch 128 --layers 24]"""
import argparse
import collections
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


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
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        p.run()
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::_to_copy", "aten::contiguous", "aten::clone", "aten::cat"):
            st = [f for f in (ev.stack or []) if "paddle_infer_amd" in f][:3]
            cnt[(ev.name, str(ev.input_shapes)[:90], " <- ".join(s.split("paddle_infer_amd/")[-1] for s in st))] += 1
    for (n, shp, st), k in cnt.most_common(25):
        print(f"{k:4d}  {n:16s} {shp}\n        {st}")


if __name__ == "__main__":
    main()
