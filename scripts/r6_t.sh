#!/bin/bash
# Conv->conv gradient join (downsampling blocks): GPU tests + ResNet-50 A/B + ATen trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_join_gpu.py tests/test_conv_gpu.py tests/test_conv_bwd_gpu.py tests/test_conv_bn_stats_gpu.py > gpurun_out/r6t_tests.log 2>&1 || { tail -40 gpurun_out/r6t_tests.log; exit 1; }
tail -2 gpurun_out/r6t_tests.log
for j in 1 0; do
  PIAMD_RES_JOIN=$j timeout -k 10 240 python tools/bench_resnet.py --mode hip --batch 128 --steps 20 > gpurun_out/r6t_rn_$j.log 2>&1 || { tail -20 gpurun_out/r6t_rn_$j.log; exit 1; }
  echo "RES_JOIN=$j"; grep '^{' gpurun_out/r6t_rn_$j.log
done
bash scripts/r6_r.sh
