#!/bin/bash
# Attention split count at batch 1 (PIAMD_MEGA_NSPLIT) on the MFMA single-launch kernel.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_ae
mkdir -p $OUT
for ns in 4 8 16; do
  PIAMD_MEGA_NSPLIT=$ns timeout -k 10 200 python -u tools/mega_trace.py --batch 1 > $OUT/trace_ns$ns.log 2>&1 || { tail -30 $OUT/trace_ns$ns.log; exit 1; }
  echo "nsplit=$ns $(grep '^{' $OUT/trace_ns$ns.log | sed -n 2p)"
done
for ns in 8 16; do
  PIAMD_MEGA_NSPLIT=$ns timeout -k 10 300 python -u tools/bench_generate.py --batch 1 --gen 128 --modes graph > $OUT/gen_ns$ns.log 2>&1 || { tail -30 $OUT/gen_ns$ns.log; exit 1; }
  echo "nsplit=$ns $(grep '^{' $OUT/gen_ns$ns.log | cut -c1-120)"
done
