#!/bin/bash
# BN backward with the x-derived ReLU mask: BN / conv-net tests, then ResNet-50 with BN grid options.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $(grep -ln "batch_norm\|BatchNorm" tests/*gpu*.py) > gpurun_out/r4bn2_tests.log 2>&1 || { tail -30 gpurun_out/r4bn2_tests.log; exit 1; }
tail -1 gpurun_out/r4bn2_tests.log
for G in "65536,512" "32768,1024" "16384,2048"; do
PIAMD_BN_GRID=$G timeout -k 10 300 python tools/bench_resnet.py --model resnet50 --steps 10 > gpurun_out/r4bn2_$G.log 2>&1 || { tail -20 gpurun_out/r4bn2_$G.log; exit 1; }
echo "grid $G $(grep '^{' gpurun_out/r4bn2_$G.log | cut -c60-150)"
done
