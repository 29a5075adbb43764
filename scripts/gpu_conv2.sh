#!/bin/bash
# Transposed conv tests, ResNet-50 / MobileNetV2 throughput, ResNet-50 kernel profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_conv_any_gpu.py > gpurun_out/conv_any2.log 2>&1 || { tail -40 gpurun_out/conv_any2.log; exit 1; }
tail -2 gpurun_out/conv_any2.log
timeout -k 10 300 python tools/bench_resnet.py --steps 10 > gpurun_out/resnet.log 2>&1 || { tail -20 gpurun_out/resnet.log; exit 1; }
cat gpurun_out/resnet.log
timeout -k 10 300 python tools/bench_resnet.py --steps 10 --model mobilenet_v2 --mode both > gpurun_out/mbv2.log 2>&1 || { tail -20 gpurun_out/mbv2.log; exit 1; }
cat gpurun_out/mbv2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet -o run -- python tools/bench_resnet.py --steps 3 > gpurun_out/prof_resnet.log 2>&1 || { tail -20 gpurun_out/prof_resnet.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mbv2 -o run -- python tools/bench_resnet.py --steps 3 --model mobilenet_v2 > gpurun_out/prof_mbv2.log 2>&1 || { tail -20 gpurun_out/prof_mbv2.log; exit 1; }
ls gpurun_out/prof_resnet gpurun_out/prof_mbv2
