"""Which PyTorch (ATen) kernels does a training step still launch, and from where? Runs one
ResNet / MobileNet training step (tools/bench_resnet.build) under a TorchDispatchMode that records
every aten op that launches a device kernel — everything except views / metadata and the
framework's own HIP kernels (those are ctypes launches, invisible here) — with the innermost
framework frames of the Python stack.

  python tools/trace_aten_step.py [--model resnet50 --batch 128]"""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

_NOKERNEL = ("view", "_unsafe_view", "as_strided", "t", "transpose", "permute", "expand", "slice",
             "select", "unsqueeze", "squeeze", "alias", "detach", "empty", "empty_like",
             "empty_strided", "_to_copy_noop", "lift_fresh", "unbind", "split", "chunk", "reshape",
             "_reshape_alias", "new_empty", "new_empty_strided", "is_same_size", "_local_scalar_dense",
             "sym_size", "sym_stride", "set_", "resize_", "contiguous")


class _Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.cnt = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__.split(".")[0]
        dev = any(isinstance(a, torch.Tensor) and a.is_cuda for a in args)
        if dev and name not in _NOKERNEL:
            fr = [f for f in traceback.extract_stack() if "paddle_infer_amd" in f.filename][-2:]
            where = " <- ".join(f"{f.filename.split('paddle_infer_amd/')[-1]}:{f.lineno}" for f in reversed(fr))
            if not where:  # no framework frame (autograd engine): show the operands instead
                where = "; ".join(f"{tuple(a.shape)}/{a.stride()}/{str(a.dtype)[6:]}" for a in args
                                  if isinstance(a, torch.Tensor))[:150]
            self.cnt[(name, where)] += 1
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from bench_resnet import build
    step = build(a.batch, True, 0.1, model=a.model)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    rec = _Rec()
    with rec:
        step()
    torch.cuda.synchronize()
    print(f"# aten ops launching device work in one {a.model} training step (batch {a.batch}): "
          f"{sum(rec.cnt.values())}")
    for (n, st), k in rec.cnt.most_common(45):
        print(f"{k:4d}  {n:28s} {st}")


if __name__ == "__main__":
    main()
