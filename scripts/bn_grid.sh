#!/bin/bash
# BN statistics/reduction grid sweep on the ResNet-50 training step (eager), then a kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for G in "65536,512" "32768,1024" "16384,2048" "32768,2048" "8192,2048"; do
  PIAMD_BN_GRID=$G timeout -k 10 200 python tools/bench_resnet.py --steps 10 > gpurun_out/bn_grid_$G.log 2>&1 || { tail -10 gpurun_out/bn_grid_$G.log; exit 1; }
  echo "$G $(grep '^{' gpurun_out/bn_grid_$G.log | cut -c1-160)"
done
