#!/bin/bash
# FFN2-slice touch during the attention phase (late_dma bit 2) A/B on the batch-1 / 4-row kernel.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_decode_mega_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for ld in 1 5; do
  for b in 1 4; do
    PIAMD_MEGA_LATE_DMA=$ld timeout -k 10 200 python -u tools/mega_trace.py --batch $b > $OUT/trace_b${b}_$ld.log 2>&1 || { tail -30 $OUT/trace_b${b}_$ld.log; exit 1; }
    echo "late_dma=$ld batch=$b"; grep "^{" $OUT/trace_b${b}_$ld.log | sed -n 2,7p
  done
done
