#!/bin/bash
# Conv wgrad in the channels_last parameter layout: conv GPU tests + ResNet-50 step + ATen census.
set -o pipefail
OUT=gpurun_out/r5_o
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_conv_bwd_gpu.py tests/test_conv_any_gpu.py > $OUT/tests.log 2>&1 || { echo "conv tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 tools/bench_resnet.py --model resnet50 --steps 20 > $OUT/rn50.log 2>&1 || { echo "bench failed"; tail -20 $OUT/rn50.log; exit 1; }
grep '^{' $OUT/rn50.log | tail -1 | cut -c1-200
timeout -k 10 300 python3 tools/trace_aten_step.py > $OUT/aten_rn50.txt 2>&1 || { echo "aten trace failed"; tail -20 $OUT/aten_rn50.txt; exit 1; }
head -12 $OUT/aten_rn50.txt
