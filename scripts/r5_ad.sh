#!/bin/bash
# GPT-3 13B full training step on one MI355X (BASELINE config 5's model; 288 GB holds the unsharded state).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_ad
mkdir -p $OUT
for mb in ${MBS:-2 4}; do
  timeout -k 10 600 python -u bench.py --model gpt3-13b --seq 2048 --micro-batch $mb --recompute --steps 4 --warmup 2 > $OUT/b13_mb$mb.log 2>&1 || { tail -30 $OUT/b13_mb$mb.log; exit 1; }
  grep "^{" $OUT/b13_mb$mb.log | cut -c1-600
done
