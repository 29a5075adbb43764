#!/usr/bin/env python
"""Headline benchmark: GPT-3 1.3B hybrid-parallel pre-training throughput (tokens/s, whole job).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (one rank per GPU, RCCL). W untimed steps, then EXACTLY K timed steps
bracketed by barrier + device synchronize; the max elapsed over ranks is reported by rank 0 as one
JSON line. Synthetic token ids and random-init weights of the real GPT-3 1.3B architecture
(24 layers, hidden 2048, 16 heads, FFN 8192, vocab 50304, seq 1024); bf16 compute with fp32
master weights + AdamW states; every timed step is a full forward + backward + gradient
collectives + optimizer update.

Everything goes through the Fleet API users call: ``fleet.init`` (hybrid_configs dp / mp / pp /
sharding degrees) → ``fleet.distributed_model`` → ``fleet.distributed_optimizer(paddle AdamW +
ClipGradByGlobalNorm)``; on the GPU the optimizer is the fused flat-buffer engine (bucketed
reduce-scatter / all-reduce overlapped with backward, one AdamW launch per parameter group).

Parallelism: ``--tp`` model-parallel degree, ``--pp`` pipeline degree (GPTForPretrainingPipe,
1F1B; ``--vpp`` virtual chunks per rank = interleaved 1F1B; ``--accumulate`` micro-batches per
step), ``--sharding-degree`` a separate ZeRO axis (the rest is dp), ``--sharding`` ZeRO stage on
that axis (default 1 over dp: sharded optimizer states; 3 = ZeRO-3 per-block parameter shards,
composable with ``--pp`` / ``--tp`` — BASELINE config 5 is ``--model gpt3-13b --pp 2
--sharding-degree 4 --sharding 3`` on 8 GPUs; ``--offload 1`` keeps its optimizer states on the host).
Weak scaling: the per-GPU micro batch is fixed as N grows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

METRIC = "tokens/sec (node) GPT-3 1.3B Fleet hybrid-parallel at 1/2/4/8 MI355X"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt3-1.3b")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--num-layers", type=int, default=0, help="override the model's layer count (rehearsals)")
    ap.add_argument("--micro-batch", type=int, default=96,
                    help="sequences per data-parallel rank (96 x 1024 tokens: ~177 GB of the "
                         "288 GB HBM3E; amortises the optimizer step and the gradient collectives: "
                         "128.9k / 130.1k / 130.5k tok/s at 64 / 96 / 128 on one MI355X, "
                         "profiles/bench_mb_sweep_r2.txt — 96 keeps >100 GB free for the multi-GPU "
                         "collective buffers; at 8 GPUs the global batch is 768 x 1024 = 0.79M tokens, "
                         "GPT-3 1.3B used 1M)")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--pp", type=int, default=1)
    ap.add_argument("--vpp", type=int, default=1, help="virtual pipeline chunks per rank (interleaved 1F1B)")
    ap.add_argument("--accumulate", type=int, default=0,
                    help="pipeline micro-batches per step (default 2 x pp); --micro-batch is split")
    ap.add_argument("--sharding-degree", type=int, default=1)
    ap.add_argument("--sharding", type=int, default=1, help="ZeRO stage (0 = plain all-reduce DP)")
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--offload", type=int, default=0, help="ZeRO-3: f32 master / moments in pinned host memory")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--recompute", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo + the ops' CPU reference paths (rehearses the multi-rank driver "
                         "command without a GPU; not a performance number)")
    ap.add_argument("--tuned-gemm", type=int, default=0,
                    help="replay the in-tree TunableOp GEMM table (paddle_infer_amd/tuning)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {args.gpus}", file=sys.stderr)
    on_gpu = args.device == "cuda"
    # the package installs the framework's auto-growth allocator at import: it must come before
    # the first HIP call of the process (set_device initialises the caching allocator otherwise)
    import paddle_infer_amd as pia
    from paddle_infer_amd.framework import allocator as pia_alloc
    if on_gpu:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if on_gpu:
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")

    from paddle_infer_amd.incubate import autotune
    tuned = autotune.use_tuned_gemms() if args.tuned_gemm else False
    from paddle_infer_amd.distributed import fleet
    from paddle_infer_amd.models.gpt import (GPTForPretraining, GPTForPretrainingPipe, gpt_config,
                                             gpt_flops_per_token)
    from paddle_infer_amd.framework import random as prand

    tp, pp, shd = args.tp, args.pp, args.sharding_degree
    assert world % (tp * pp * shd) == 0, f"world {world} not divisible by tp*pp*sharding"
    dp = world // (tp * pp * shd)
    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": dp, "mp_degree": tp, "pp_degree": pp,
                               "sharding_degree": shd}
    stage3 = args.sharding == 3
    if args.sharding:
        # ZeRO on the sharding axis (or over dp when there is none); stage 3 composes with pp / tp
        strategy.sharding = shd == 1 and dp > 1
        strategy.sharding_configs = {"stage": args.sharding, "offload": bool(args.offload)}
    strategy.fuse_grad_size_in_MB = args.bucket_mb
    acc = args.accumulate or (2 * pp if pp > 1 else 1)
    acc = max(1, min(acc, args.micro_batch))
    assert args.micro_batch % acc == 0, "--micro-batch must split into --accumulate micro-batches"
    strategy.pipeline_configs = {"accumulate_steps": acc, "micro_batch_size": max(1, args.micro_batch // acc)}
    fleet.init(is_collective=True, strategy=strategy)
    hcg = fleet.get_hybrid_communicate_group()
    mp_group = hcg.get_model_parallel_group() if tp > 1 else None
    prand.model_parallel_random_seed(1234, hcg.get_model_parallel_rank(), hcg.get_stage_id())

    over = {"num_layers": args.num_layers} if args.num_layers else {}
    cfg = gpt_config(args.model, max_position_embeddings=max(args.seq, 1024),
                     hidden_dropout_prob=args.dropout, recompute=args.recompute, **over)
    with torch.device(device):
        if pp > 1:
            net = GPTForPretrainingPipe(cfg, mp_group=mp_group,
                                        num_virtual_pipeline_stages=args.vpp if args.vpp > 1 else None)
        else:
            net = GPTForPretraining(cfg, mp_group=mp_group)
    net.train()
    decay = {getattr(p, "pd_name", None) for p in net.parameters() if p.dim() > 1}
    opt = pia.optimizer.AdamW(learning_rate=1e-4, beta1=0.9, beta2=0.95, epsilon=1e-8,
                              parameters=list(net.parameters()), weight_decay=0.1,
                              grad_clip=pia.nn.ClipGradByGlobalNorm(1.0),
                              apply_decay_param_fun=lambda n: n in decay)
    n_params = sum(p.numel() for p in net.parameters())  # before ZeRO-3 releases the blocks
    model = fleet.distributed_model(net)
    opt = fleet.distributed_optimizer(opt)
    if world > 1:
        t = torch.tensor([n_params], device=device, dtype=torch.float64)
        if pp > 1:  # each stage holds its own layers (a tied table counted on both ends)
            dist.all_reduce(t, group=hcg.get_pipe_parallel_group())
        if tp > 1:
            dist.all_reduce(t, group=hcg.get_model_parallel_group())
        n_params = int(t.item())

    mb, S = args.micro_batch, args.seq
    gen = torch.Generator(device=device)
    gen.manual_seed(1000 + hcg.get_data_parallel_rank() * shd + hcg.get_sharding_parallel_rank())
    ids = torch.randint(0, cfg.vocab_size, (mb, S + 1), device=device, generator=gen)
    x, y = ids[:, :-1].contiguous(), ids[:, 1:].contiguous()
    flat = getattr(opt, "_flat", None)

    def step():
        if pp > 1:
            return model.train_batch([x, y], opt)
        loss = model(x, labels=y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        return loss

    for _ in range(args.warmup):
        loss = step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    if flat is not None:
        flat.wait_params()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())

    tokens = args.steps * dp * shd * mb * S
    tps = tokens / elapsed
    ms = elapsed / args.steps * 1e3
    flops_tok = gpt_flops_per_token(cfg, S)
    tflops_gpu = tps * flops_tok / world / 1e12
    par = ((f"tp{tp}" if tp > 1 else "") + (f"pp{pp}" if pp > 1 else "") + (f"v{args.vpp}" if args.vpp > 1 else "")
           + (f"sh{shd}" if shd > 1 else "") + f"dp{dp}"
           + (f"_zero{args.sharding}" if (dp * shd > 1 and args.sharding) else ""))
    if rank == 0:
        print(json.dumps({
            "metric": METRIC if args.model == "gpt3-1.3b" else f"tokens/sec {args.model} training",
            "value": round(tps, 1), "unit": "tokens/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random token ids, random-init weights)",
            "config": {"model": "GPT-3 1.3B" if args.model == "gpt3-1.3b" else args.model,
                       "global_batch": dp * shd * mb, "seq_len": S, "parallelism": par,
                       "micro_batch_per_dp_rank": mb, "params": n_params,
                       "hidden_dropout": args.dropout, "attention_dropout": 0.0,
                       "optimizer": "AdamW fp32 master", "grad_clip": 1.0,
                       "api": "fleet.init/distributed_model/distributed_optimizer"
                       + (" (sharding stage 3)" if stage3 else ""),
                       **({"pp_micro_batches": acc} if pp > 1 else {})},
            "tflops_per_gpu": round(tflops_gpu, 1), "final_loss": round(final_loss, 4),
            "tuned_gemm_table": bool(tuned),
            "allocator": "auto_growth" if pia_alloc.active() else "torch_caching",
            # the framework allocator's own peak when it is active (torch.cuda's is routed to it)
            "peak_mem_gb": round((pia_alloc.stats(local_rank)["peak_allocated"] if pia_alloc.active()
                                  else torch.cuda.max_memory_allocated()) / 2 ** 30, 1) if on_gpu else None,
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
