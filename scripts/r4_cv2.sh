#!/bin/bash
# Conv forward pipeline depth A/B (PIAMD_CONV_STAGES) on ResNet-50 / MobileNetV2 training steps.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for R in 1 2; do
for S in 2 3; do
for M in resnet50 mobilenet_v2; do
PIAMD_CONV_STAGES=$S timeout -k 10 300 python tools/bench_resnet.py --model $M --steps 10 > gpurun_out/r4cv2_${M}_$S.log 2>&1 || { tail -20 gpurun_out/r4cv2_${M}_$S.log; exit 1; }
echo "stages $S $(grep '^{' gpurun_out/r4cv2_${M}_$S.log | cut -c1-160)"
done
done
done
