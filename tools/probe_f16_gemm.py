"""Data dependence of the assembly GEMM's speed (BERT-Large FFN1 shape, 16384x4096x1024): fp16 random
vs fp16 values that are exactly bf16 (fewer toggling mantissa bits) vs zeros, and bf16.

  python tools/probe_f16_gemm.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from paddle_infer_amd.ops.gemm import gemm_nt
def t(fn, it=30):
    for _ in range(3): fn()
    ts=[]
    for _ in range(it):
        a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize(); ts.append(a.elapsed_time(b))
    ts.sort(); return ts[len(ts)//2]
M,N,K=16384,4096,1024
for name, mk in [("f16 randn", lambda s: torch.randn(s, device="cuda").half()),
                 ("f16 bf16-representable", lambda s: torch.randn(s, device="cuda").bfloat16().half()),
                 ("f16 zeros", lambda s: torch.zeros(s, device="cuda").half()),
                 ("bf16 randn", lambda s: torch.randn(s, device="cuda").bfloat16()),
                 ("bf16 zeros", lambda s: torch.zeros(s, device="cuda").bfloat16())]:
    x=mk((M,K)); w=mk((N,K))*0.03
    print(json.dumps({"case": name, "ms": round(t(lambda: gemm_nt(x, w)), 4)}), flush=True)
