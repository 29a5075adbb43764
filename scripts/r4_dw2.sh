#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_any_gpu.py tests/test_conv_bwd_gpu.py tests/test_conv_gpu.py > gpurun_out/r4dw2_tests.log 2>&1 || { tail -30 gpurun_out/r4dw2_tests.log; exit 1; }
tail -1 gpurun_out/r4dw2_tests.log
timeout -k 10 300 python tools/bench_dwconv.py > gpurun_out/r4dw2.log 2>&1 || { tail -20 gpurun_out/r4dw2.log; exit 1; }
grep "^{" gpurun_out/r4dw2.log
timeout -k 10 300 python tools/bench_resnet.py --model mobilenet_v2 --steps 10 > gpurun_out/r4dw2_mbv2.log 2>&1 || { tail -20 gpurun_out/r4dw2_mbv2.log; exit 1; }
grep "^{" gpurun_out/r4dw2_mbv2.log | cut -c1-300
