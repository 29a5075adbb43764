#!/bin/bash
# Serving-batch linears: packed GEMV vs skinny MFMA GEMM at M = 8-64 (GPT-1.3B shapes).
set -o pipefail
OUT=gpurun_out/r5_p
mkdir -p $OUT
timeout -k 10 400 python3 tools/bench_decode_linear.py --M 8 16 32 64 > $OUT/lin.jsonl 2>&1 || { echo "bench failed"; tail -20 $OUT/lin.jsonl; exit 1; }
grep '^{' $OUT/lin.jsonl
