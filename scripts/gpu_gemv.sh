#!/bin/bash
# Decode GEMV sweep + generation bench + batch-1 decode kernel profile.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-nt}
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_gemv.py > gpurun_out/gemv_$TAG.log 2>&1 || { tail -20 gpurun_out/gemv_$TAG.log; exit 1; }
grep '"M": 1,' gpurun_out/gemv_$TAG.log | head -30
bash scripts/decode_prof.sh $TAG
