"""Serving benchmark: GPT prefill + KV-cached decode on one MI355X.

Reports prefill tokens/s and decode tokens/s (batch × generated tokens / decode time) for the
fused multi-transformer path, with/without hipGraph replay and with weight-only int8/int4.
Random-init weights of the named GPT preset, synthetic prompts.

  python tools/bench_generate.py --model gpt3-1.3b --batch 1 8 32 --prompt 128 --gen 128
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt3-1.3b")
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8, 32])
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--modes", nargs="+", default=["graph", "eager", "int8", "int4"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import paddle_infer_amd as paddle
    from paddle_infer_amd.inference.generation import GPTGenerator
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    paddle.seed(0)
    cfg = gpt_config(a.model, hidden_dropout_prob=0.0, max_position_embeddings=max(2048, a.prompt + a.gen))
    with torch.device("cuda"):
        model = GPTForPretraining(cfg)
    model = model.cuda().to(torch.bfloat16).eval()
    rows = []
    for mode in a.modes:
        gen = GPTGenerator(model, max_batch=max(a.batch), max_seq_len=a.prompt + a.gen + 8,
                           use_hip_graph=(mode != "eager"),
                           weight_only=mode if mode in ("int8", "int4") else None,
                           prepack=(mode != "graph_blaslt"))
        for B in a.batch:
            ids = torch.randint(0, cfg.vocab_size, (B, a.prompt), device="cuda")
            lens = torch.full((B,), a.prompt, device="cuda")
            gen.generate(ids, lens, max_new_tokens=4)  # warm-up + graph capture
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                gen.prefill(ids, lens)
            torch.cuda.synchronize()
            t_pre = (time.perf_counter() - t0) / 3
            tok = torch.zeros(B, dtype=torch.long, device="cuda")
            pos = torch.full((B,), a.prompt, dtype=torch.int32, device="cuda")
            gen.decode(tok, pos)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.gen):
                logits = gen.decode(tok, pos + i)
                tok = logits.argmax(-1)
            torch.cuda.synchronize()
            t_dec = time.perf_counter() - t0
            # end-to-end greedy generate(): prefill + (gen - 1) decode steps with the token choice
            # (inside the captured step for graph modes)
            gen.generate(ids, lens, max_new_tokens=a.gen)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gen.generate(ids, lens, max_new_tokens=a.gen)
            torch.cuda.synchronize()
            t_gen = time.perf_counter() - t0
            r = {"mode": mode, "batch": B, "prompt": a.prompt, "gen": a.gen,
                 "generate_decode_ms_per_step": round((t_gen - t_pre) / max(1, a.gen - 1) * 1e3, 4),
                 "prefill_ms": round(t_pre * 1e3, 3),
                 "prefill_tok_s": round(B * a.prompt / t_pre, 1),
                 "decode_ms_per_step": round(t_dec / a.gen * 1e3, 4),
                 "decode_tok_s": round(B * a.gen / t_dec, 1)}
            mega = gen._mega.get(B)
            if mega:
                r["mega_decode"] = True
                r["mega_timeouts"] = int(mega.err.item())
            print(json.dumps(r), flush=True)
            rows.append(r)
        del gen
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
