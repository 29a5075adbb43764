"""Which ATen kernels does one BERT Predictor run still launch, and from where? Runs the
Predictor eagerly (no hipGraph) under a TorchDispatchMode and prints the device ops with the
innermost framework frames (tools/trace_aten_step.py does the same for a training step).

  python tools/trace_aten_predictor.py [--batch 1] [--dtype fp16]"""
import argparse
import collections
import os
import sys
import tempfile
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_aten_step import _NOKERNEL  # noqa: E402


class _Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.cnt = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__.split(".")[0]
        if any(isinstance(a, torch.Tensor) and a.is_cuda for a in args) and name not in _NOKERNEL:
            fr = [f for f in traceback.extract_stack() if "paddle_infer_amd" in f.filename][-2:]
            where = " <- ".join(f"{f.filename.split('paddle_infer_amd/')[-1]}:{f.lineno}" for f in reversed(fr))
            self.cnt[(name, where)] += 1
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtype", default="fp16")
    a = ap.parse_args()
    import paddle_infer_amd  # noqa: F401
    from paddle_infer_amd import inference as pinf, jit
    from paddle_infer_amd.models.bert import BertModel, bert_config
    from paddle_infer_amd.static import InputSpec
    torch.manual_seed(0)
    m = BertModel(bert_config("bert-large"))
    m.eval()
    d = tempfile.mkdtemp()
    jit.save(jit.to_static(m, input_spec=[InputSpec([None, 128], "int64", "input_ids")]), os.path.join(d, "model"))
    c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
    c.enable_use_gpu(1024, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Half if a.dtype == "fp16" else pinf.PrecisionType.Bfloat16)
    c.enable_hip_graph(False)
    pred = pinf.create_predictor(c)
    ids = torch.randint(0, 30000, (a.batch, 128))
    h = pred.get_input_handle(pred.get_input_names()[0])
    for _ in range(2):
        h.copy_from_cpu(ids.numpy())
        pred.run()
    torch.cuda.synchronize()
    rec = _Rec()
    with rec:
        pred.run()
    torch.cuda.synchronize()
    print(f"# aten ops launching device work in one BERT-Large Predictor run (batch {a.batch}): {sum(rec.cnt.values())}")
    for (n, st), k in rec.cnt.most_common(30):
        print(f"{k:4d}  {n:28s} {st}")


if __name__ == "__main__":
    main()
