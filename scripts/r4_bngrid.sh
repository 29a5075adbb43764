#!/bin/bash
# BN statistics / backward-reduction grid sweep (PIAMD_BN_GRID) on the ResNet-50 training step.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for G in "65536,512" "32768,1024" "16384,2048" "65536,2048" "32768,2048"; do
PIAMD_BN_GRID=$G timeout -k 10 300 python tools/bench_resnet.py --model resnet50 --steps 10 > gpurun_out/r4bn_$G.log 2>&1 || { tail -20 gpurun_out/r4bn_$G.log; exit 1; }
echo "grid $G $(grep '^{' gpurun_out/r4bn_$G.log | cut -c60-150)"
done
