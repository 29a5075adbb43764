#!/bin/bash
# Decode (GPT-1.3B, fp16/bf16 graph mode): batch 1 and 32 at prompt 128 and 1024.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 128 1024; do
  timeout -k 10 280 python tools/bench_generate.py --batch 1 32 --prompt $p --gen 128 --modes graph > gpurun_out/r6_dec_$p.log 2>&1 || { tail -20 gpurun_out/r6_dec_$p.log; exit 1; }
  grep '^{' gpurun_out/r6_dec_$p.log
done
