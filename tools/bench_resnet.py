"""ResNet-50 training step (channels_last, bf16 autocast) images/s through the framework's own
training API: ``paddle.vision.models.resnet50`` + ``paddle.DataParallel`` +
``paddle.optimizer.Momentum`` (merged multi-tensor update kernel) with the convolutions on the MFMA
implicit-GEMM kernels (``ops/conv.py``: forward, data gradient, weight gradient) — or, for the A/B,
on the library (MIOpen) path.

Reference parity: the reference's ResNet-50 benchmark (`python/paddle/vision/models/resnet.py`,
BASELINE config "ResNet-50 bf16 paddle.DataParallel"). Multi-GPU: launch under torchrun (one
rank per GPU, RCCL); images/s is the whole-job aggregate (max step time over ranks).

``--parity N``: N same-seed steps on a fixed batch for both conv paths, printing both loss curves."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import paddle_infer_amd as paddle  # noqa: E402
from paddle_infer_amd.ops import conv as CV  # noqa: E402
from paddle_infer_amd.vision import models as VM  # noqa: E402


def _setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import paddle_infer_amd.distributed as dist
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_parallel_env()
    return world


def build(batch, hip_conv, lr, res=224, seed=0, model="resnet50", static_grads=False):
    CV.HIP_CONV = hip_conv
    torch.manual_seed(seed)
    m = getattr(VM, model)(num_classes=1000).cuda().to(memory_format=torch.channels_last)
    model = paddle.DataParallel(m)
    opt = paddle.optimizer.Momentum(learning_rate=lr, momentum=0.9, parameters=m.parameters(),
                                    weight_decay=1e-4)
    g = torch.Generator(device="cuda").manual_seed(1234 + int(os.environ.get("RANK", "0")))
    x = torch.randn(batch, 3, res, res, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device="cuda", generator=g)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        # graph replay needs the gradient buffers (and the merged optimizer's pointer table) to
        # stay put: zero them in place instead of releasing them
        opt.clear_grad(set_to_zero=static_grads)
        return loss
    return step


def graphed(step, warmup=3):
    """The whole training step (forward, backward, optimizer update, gradient zeroing) captured
    once into a hipGraph and replayed: the ~1k kernel launches of a step leave the host. The
    warm-up runs eagerly on a side stream first (autotuned conv plans, optimizer state and the
    gradient buffers exist before capture; the graph reuses those static tensors)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warmup):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss = step()

    def replay():
        g.replay()
        return loss
    return replay


def run(batch, steps, hip_conv, world, lr=0.02, model="resnet50", graph=False):
    # lr 0.02 (momentum 0.9, no warm-up): the timed steps keep training on the fixed synthetic
    # batch (loss falls below ln 1000); lr 0.1 without warm-up diverged there (loss 11.7, r2)
    step = build(batch, hip_conv, lr=lr, model=model, static_grads=graph)
    if graph:
        step = graphed(step)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = t.item()
    return {"model": model, "hip_conv": hip_conv, "hipgraph": graph, "batch_per_gpu": batch, "n_gpus": world,
            "ms_per_step": round(dt * 1e3, 2), "images_per_s": round(batch * world / dt, 1),
            "loss": round(loss.item(), 3), "lr": lr, "optimizer": "paddle.optimizer.Momentum (merged)",
            "wrapper": "paddle.DataParallel"}


def parity(steps, batch=32, res=112, lr=0.02):
    curves = {}
    for hc in (False, True):
        step = build(batch, hc, lr=lr, res=res)
        curves[hc] = [round(step().item(), 4) for _ in range(steps)]
    CV.HIP_CONV = True
    return {"parity_steps": steps, "batch": batch, "res": res, "lr": lr,
            "library_conv": curves[False], "hip_conv": curves[True]}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mode", choices=["both", "hip", "lib"], default="hip")
    ap.add_argument("--parity", type=int, default=0)
    ap.add_argument("--model", default="resnet50", help="any paddle.vision.models constructor")
    ap.add_argument("--graph", action="store_true", help="replay the step as one captured hipGraph")
    a = ap.parse_args()
    world = _setup()
    if a.parity:
        print(json.dumps(parity(a.parity)), flush=True)
    else:
        for hc in {"both": (False, True), "hip": (True,), "lib": (False,)}[a.mode]:
            r = run(a.batch, a.steps, hc, world, model=a.model, graph=a.graph)
            if int(os.environ.get("RANK", "0")) == 0:
                print(json.dumps(r), flush=True)
