#!/bin/bash
# Skinny GEMM sweep with the B-deep (weight stream issued up front) variants at the BERT M = 128 shapes.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/tune_small_gemm.py --shapes bert --iters 40 > gpurun_out/r6_sg.log 2>&1 || { tail -20 gpurun_out/r6_sg.log; exit 1; }
cat gpurun_out/r6_sg.log
