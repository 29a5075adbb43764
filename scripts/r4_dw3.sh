#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_any_gpu.py > gpurun_out/r4dw3_tests.log 2>&1 || { tail -30 gpurun_out/r4dw3_tests.log; exit 1; }
tail -1 gpurun_out/r4dw3_tests.log
for V in 4 8; do
  echo "== V $V"
  PIAMD_DW3_V=$V timeout -k 10 300 python tools/bench_dwconv.py > gpurun_out/r4dw3_$V.log 2>&1 || { tail -20 gpurun_out/r4dw3_$V.log; exit 1; }
  grep "^{" gpurun_out/r4dw3_$V.log | cut -c1-110
done
timeout -k 10 300 python tools/bench_resnet.py --model mobilenet_v2 --steps 10 > gpurun_out/r4dw3_mbv2.log 2>&1 || { tail -20 gpurun_out/r4dw3_mbv2.log; exit 1; }
grep "^{" gpurun_out/r4dw3_mbv2.log | cut -c1-300
