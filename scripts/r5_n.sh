#!/bin/bash
# Device runtime tests + conv tests (one-launch filter prep) + ResNet-50 step A/B (prep on / off).
set -o pipefail
bash scripts/r5_m.sh || exit 1
OUT=gpurun_out/r5_n
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_conv_bwd_gpu.py tests/test_conv_any_gpu.py tests/test_batchnorm_gpu.py > $OUT/tests.log 2>&1 || { echo "conv tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for P in 1 0; do
  PIAMD_CONV_WPREP=$P timeout -k 10 300 python3 tools/bench_resnet.py --model resnet50 --steps 20 > $OUT/rn50_prep$P.log 2>&1 || { echo "bench failed"; tail -20 $OUT/rn50_prep$P.log; exit 1; }
  echo "prep=$P $(grep '^{' $OUT/rn50_prep$P.log | tail -2 | cut -c1-250)"
done
timeout -k 10 300 python3 tools/trace_aten_step.py > $OUT/aten_rn50.txt 2>&1 || { echo "aten trace failed"; tail -20 $OUT/aten_rn50.txt; exit 1; }
head -40 $OUT/aten_rn50.txt
