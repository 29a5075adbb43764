#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pool_gpu.py tests/test_batchnorm_gpu.py tests/test_conv_any_gpu.py > gpurun_out/r4pool_tests.log 2>&1 || { tail -30 gpurun_out/r4pool_tests.log; exit 1; }
tail -1 gpurun_out/r4pool_tests.log
timeout -k 10 300 python tools/bench_dwconv.py > gpurun_out/r4pool_dw.log 2>&1 || { tail -20 gpurun_out/r4pool_dw.log; exit 1; }
tail -1 gpurun_out/r4pool_dw.log
for M in resnet50 resnet50 mobilenet_v2; do
timeout -k 10 300 python tools/bench_resnet.py --model $M --steps 10 > gpurun_out/r4pool_$M.log 2>&1 || { tail -20 gpurun_out/r4pool_$M.log; exit 1; }
echo "$(grep '^{' gpurun_out/r4pool_$M.log | cut -c1-200)"
done
