#!/bin/bash
# FFN2 touch default (batch 1) vs off: tests + greedy generate A/B (two runs each, interleaved).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_ac
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_decode_mega_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for ld in 5 1; do
    PIAMD_MEGA_LATE_DMA=$ld timeout -k 10 300 python -u tools/bench_generate.py --batch 1 --gen 128 --modes graph > $OUT/gen_${ld}_$r.log 2>&1 || { tail -30 $OUT/gen_${ld}_$r.log; exit 1; }
    echo "late_dma=$ld run=$r $(grep '^{' $OUT/gen_${ld}_$r.log | cut -c1-140)"
  done
done
