#!/bin/bash
# Implicit-GEMM conv forward with a 3-stage LDS pipeline: conv tests + ResNet-50 / MobileNetV2 step.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_any_gpu.py tests/test_conv_bwd_gpu.py tests/test_conv_gpu.py > gpurun_out/r4cv_tests.log 2>&1 || { tail -30 gpurun_out/r4cv_tests.log; exit 1; }
tail -1 gpurun_out/r4cv_tests.log
for M in resnet50 mobilenet_v2; do
timeout -k 10 300 python tools/bench_resnet.py --model $M --steps 10 > gpurun_out/r4cv_$M.log 2>&1 || { tail -20 gpurun_out/r4cv_$M.log; exit 1; }
grep "^{" gpurun_out/r4cv_$M.log | cut -c1-250
done
