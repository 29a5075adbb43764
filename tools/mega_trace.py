"""Phase timeline of the single-launch decode step (csrc/kernels/decode_mega.hip).

Runs a GPT-1.3B-shaped generator (random init) at batch 1 (or --batch 2 / 4), records the per-workgroup wall-clock
(100 MHz) at every phase start and grid-barrier arrival, and prints per phase kind: the median
and max in-phase work, the barrier release latency (first release − last arrival) and the
phase period. Usage: python tools/mega_trace.py [--layers 24] [--prompt 128] [--batch 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KINDS = ["qkv", "attn", "out", "ffn1", "ffn2"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1)
    args = ap.parse_args()
    os.environ.setdefault("PIAMD_DECODE_MEGA", "1")
    import paddle_infer_amd as paddle
    from paddle_infer_amd.inference.generation import GPTGenerator
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    paddle.seed(1)
    cfg = gpt_config("gpt3-1.3b", num_layers=args.layers, hidden_dropout_prob=0.0)
    m = GPTForPretraining(cfg).cuda().to(torch.bfloat16).eval()
    B = args.batch
    gen = GPTGenerator(m, max_batch=B, max_seq_len=1024, use_hip_graph=False)
    ids = torch.randint(0, cfg.vocab_size, (B, args.prompt), device="cuda")
    logits = gen.prefill(ids, torch.full((B,), args.prompt, device="cuda"))
    pos = torch.full((B,), args.prompt, dtype=torch.int32, device="cuda")
    nl = args.layers
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = []
    for step in range(args.steps):
        tok = logits.argmax(-1)
        if step == args.steps - 1:
            gen._mega[B].trace = torch.zeros(256, 5 * nl, 4, dtype=torch.int64, device="cuda")
        ev[0].record()
        logits = gen.decode(tok, pos)
        ev[1].record()
        torch.cuda.synchronize()
        times.append(ev[0].elapsed_time(ev[1]))
        pos += 1
    gen._mega[B].check()
    tr = gen._mega[B].trace.cpu().double() * 10.0 / 1000.0  # 100 MHz ticks -> µs
    start, pro, gem, arrive = tr[:, :, 0], tr[:, :, 1], tr[:, :, 2], tr[:, :, 3]
    t0 = start[:, 0].min()
    res = {k: {"prologue": 0.0, "gemv": 0.0, "epilogue": 0.0, "work_med": 0.0, "work_max": 0.0,
              "barrier": 0.0, "period": 0.0} for k in KINDS}
    nph = 5 * nl
    for p in range(nph - 1):
        k = KINDS[p % 5]
        work = arrive[:, p] - start[:, p]
        if k != "attn":
            res[k]["prologue"] += (pro[:, p] - start[:, p]).median().item() / nl
            res[k]["gemv"] += (gem[:, p] - pro[:, p]).median().item() / nl
            res[k]["epilogue"] += (arrive[:, p] - gem[:, p]).median().item() / nl
        res[k]["work_med"] += work.median().item() / nl
        res[k]["work_max"] += work.max().item() / nl
        res[k]["barrier"] += (start[:, p + 1].min() - arrive[:, p].max()).item() / nl
        res[k]["period"] += (start[:, p + 1].median() - start[:, p].median()).item() / nl
    # attention workgroups (the first nb·Hq·nsplit) against the others in the out phase: the
    # former queue their FFN1 DMA only there
    mg = gen._mega[B]
    na = mg.nb * mg.HQ * mg.nsplit
    for grp, sl in (("attn_wgs", slice(0, na)), ("other_wgs", slice(na, 256))):
        if sl.start >= sl.stop:
            continue
        o = {"pro": 0.0, "gemv": 0.0, "epi": 0.0}
        for p in range(2, nph - 1, 5):
            o["pro"] += (pro[sl, p] - start[sl, p]).median().item() / nl
            o["gemv"] += (gem[sl, p] - pro[sl, p]).median().item() / nl
            o["epi"] += (arrive[sl, p] - gem[sl, p]).median().item() / nl
        res.setdefault("out_split", {})[grp] = {k: round(v, 2) for k, v in o.items()}
    total = (start[:, nph - 1].max() - t0).item()
    print(json.dumps({"out_phase_by_group": res.pop("out_split", {}), "nsplit": mg.nsplit}))
    print(json.dumps({"layers": nl, "batch": B, "step_ms_eager": sorted(times)[len(times) // 2],
                      "kernel_span_us_to_last_phase": round(total, 1)}))
    for k in KINDS:
        print(json.dumps({"phase": k, **{n: round(v, 2) for n, v in res[k].items()}}))


if __name__ == "__main__":
    main()
