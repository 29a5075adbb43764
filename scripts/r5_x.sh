#!/bin/bash
# Conv-epilogue BN statistics: tests, then ResNet-50 with the fusion on / off.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_x
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_conv_bn_stats_gpu.py tests/test_conv_gpu.py tests/test_batchnorm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PIAMD_CONV_BN_STATS=1 timeout -k 10 400 python -u tools/bench_resnet.py --model resnet50 --steps 20 > $OUT/rn50_on.log 2>&1 || { tail -30 $OUT/rn50_on.log; exit 1; }
grep "^{" $OUT/rn50_on.log | cut -c1-300
PIAMD_CONV_BN_STATS=0 timeout -k 10 400 python -u tools/bench_resnet.py --model resnet50 --steps 20 > $OUT/rn50_off.log 2>&1 || { tail -30 $OUT/rn50_off.log; exit 1; }
grep "^{" $OUT/rn50_off.log | cut -c1-300
