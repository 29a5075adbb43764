#!/bin/bash
# Decode GEMV vs rows (M = 1 / 8 / 16 / 32) and split-K: where batch-32 decode loses bandwidth.
set -o pipefail
OUT=gpurun_out/r5_h
mkdir -p $OUT
timeout -k 10 300 python3 tools/bench_gemv.py --M 1 8 16 32 --ks 1 2 4 8 > $OUT/gemv.jsonl 2>&1 || { echo "gemv failed"; tail -20 $OUT/gemv.jsonl; exit 1; }
grep '^{' $OUT/gemv.jsonl
