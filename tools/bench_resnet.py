"""ResNet-50 training step (channels_last, bf16 autocast, SGD momentum) images/s with the
convolutions on the MFMA implicit-GEMM kernel (``ops/conv.py``) vs the library (MIOpen) path.
Reference parity: the reference's ResNet-50 benchmark (`python/paddle/vision/models/resnet.py`)."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import paddle_infer_amd  # noqa: E402,F401
from paddle_infer_amd.ops import conv as CV  # noqa: E402
from paddle_infer_amd.vision.models import resnet50  # noqa: E402


def run(batch, steps, hip_conv):
    CV.HIP_CONV = hip_conv
    torch.manual_seed(0)
    m = resnet50(num_classes=1000).cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(batch, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"hip_conv": hip_conv, "batch": batch, "ms_per_step": round(dt * 1e3, 2),
            "images_per_s": round(batch / dt, 1), "loss": round(loss.item(), 3)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mode", choices=["both", "hip", "lib"], default="both")
    a = ap.parse_args()
    for hc in {"both": (False, True), "hip": (True,), "lib": (False,)}[a.mode]:
        print(json.dumps(run(a.batch, a.steps, hc)), flush=True)
