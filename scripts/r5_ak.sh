#!/bin/bash
# LN-fold skinny GEMM tile-config sweep at the decode shapes.
set -o pipefail
OUT=gpurun_out/r5_ak
mkdir -p $OUT
PYTHONPATH=$PWD timeout -k 10 300 python3 tools/bench_ln_fold.py > $OUT/sweep.log 2>&1 || { tail -20 $OUT/sweep.log; exit 1; }
grep '^{' $OUT/sweep.log
