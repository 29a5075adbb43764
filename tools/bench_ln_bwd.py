"""LayerNorm backward throughput at the GPT-1.3B training shape (fused add + LN, bf16, rows x 2048):
ms per backward and effective HBM GB/s (reads h, dy, dres_in; writes dres). Env PIAMD_LN_BWD_PAIR
selects the two-waves-per-row kernel (default) or the wave-per-row one (0)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_infer_amd.ops import fused_add_layer_norm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=98304)
    ap.add_argument("--N", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    x = torch.randn(a.rows, a.N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn_like(x, requires_grad=True)
    xb = torch.zeros(a.N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(a.N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    b = torch.zeros(a.N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y, h = fused_add_layer_norm(x, r, w, b, 1e-5, xb, 0.0)
    dy, dh = torch.randn_like(y), torch.randn_like(h)
    for _ in range(3):
        torch.autograd.backward([y, h], [dy, dh], retain_graph=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        torch.autograd.backward([y, h], [dy, dh], retain_graph=True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    gb = 4 * a.rows * a.N * 2 / 1e9
    print(json.dumps({"rows": a.rows, "N": a.N, "pair": os.environ.get("PIAMD_LN_BWD_PAIR", "1"),
                      "bwd_ms": round(ms, 4), "eff_GBps": round(gb / ms * 1e3, 1)}))


if __name__ == "__main__":
    main()
