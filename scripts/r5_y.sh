#!/bin/bash
# Kernel census of ResNet-50 with the conv-epilogue BN statistics on / off.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_y
mkdir -p $OUT
for mode in 1 0; do
  PIAMD_CONV_BN_STATS=$mode timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/p$mode -o run -- python3 tools/bench_resnet.py --model resnet50 --steps 5 > $OUT/rn50_$mode.log 2>&1 || { tail -20 $OUT/rn50_$mode.log; exit 1; }
  python3 tools/rocpd_stats.py $(find $OUT/p$mode -name "*.db" | head -1) --top 30 > $OUT/stats_$mode.txt 2>&1
  rm -rf $OUT/p$mode
  head -25 $OUT/stats_$mode.txt
done
