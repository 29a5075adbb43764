#!/bin/bash
# BERT inference: fused-epilogue GEMM cost and the Predictor's device-copy call sites.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_epilogue.py > gpurun_out/r4b_epi.log 2>&1 || { tail -20 gpurun_out/r4b_epi.log; exit 1; }
grep "^{" gpurun_out/r4b_epi.log
timeout -k 10 300 python tools/trace_copies.py > gpurun_out/r4b_copies.log 2>&1 || { tail -20 gpurun_out/r4b_copies.log; exit 1; }
tail -60 gpurun_out/r4b_copies.log
