#!/bin/bash
# Serving refresh: GPT-1.3B batch-32 decode / prefill, BERT-Large fp16 Predictor batch 1 / 128.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/bench_generate.py --batch 32 --prompt 128 --gen 64 --modes graph > gpurun_out/r4s_gen32.log 2>&1 || { tail -20 gpurun_out/r4s_gen32.log; exit 1; }
grep "^{" gpurun_out/r4s_gen32.log | cut -c1-300
timeout -k 10 400 python tools/bench_bert_infer.py --batches 1,128 --predictor-only > gpurun_out/r4s_bert.log 2>&1 || { tail -20 gpurun_out/r4s_bert.log; exit 1; }
grep "^{" gpurun_out/r4s_bert.log | cut -c1-300
