#!/bin/bash
# int8 weight-only single-launch decode + the skinny-GEMM depth-4 sweep at M = 128 (BERT-Large b1).
set -o pipefail
bash scripts/r5_j.sh || exit 1
OUT=gpurun_out/r5_k
mkdir -p $OUT
timeout -k 10 600 python3 tools/tune_small_gemm.py --only-m 128 > $OUT/tune128.jsonl 2>&1 || { echo "tune failed"; tail -20 $OUT/tune128.jsonl; exit 1; }
grep '^{' $OUT/tune128.jsonl | cut -c1-260
