#!/bin/bash
# BN statistics / backward-reduction grid sweep (PIAMD_BN_GRID = elems_per_block,max_blocks) on ResNet-50.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_z
mkdir -p $OUT
for g in 65536,512 32768,1024 16384,2048 65536,2048 131072,256; do
  PIAMD_BN_GRID=$g timeout -k 10 300 python -u tools/bench_resnet.py --model resnet50 --steps 20 > $OUT/rn50_$g.log 2>&1 || { tail -20 $OUT/rn50_$g.log; exit 1; }
  echo "$g $(grep '^{' $OUT/rn50_$g.log | cut -c100-200)"
done
