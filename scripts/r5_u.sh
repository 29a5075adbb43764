#!/bin/bash
# FFN1-head placement A/B (late_dma bit 1) on the MFMA batch-1 kernel and the batched kernels.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_u
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_decode_mega_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for ld in 1 3; do
  PIAMD_MEGA_LATE_DMA=$ld PIAMD_MEGA_MFMA=1 timeout -k 10 200 python -u tools/mega_trace.py --batch 1 > $OUT/trace_b1m_$ld.log 2>&1 || { tail -30 $OUT/trace_b1m_$ld.log; exit 1; }
  grep "^{" $OUT/trace_b1m_$ld.log | head -3
  PIAMD_MEGA_LATE_DMA=$ld timeout -k 10 200 python -u tools/mega_trace.py --batch 4 > $OUT/trace_b4_$ld.log 2>&1 || { tail -30 $OUT/trace_b4_$ld.log; exit 1; }
  grep "^{" $OUT/trace_b4_$ld.log | head -3
done
PIAMD_MEGA_MFMA=1 timeout -k 10 300 python -u tools/bench_generate.py --batch 1 2 4 --gen 64 --modes eager > $OUT/gen_mega.log 2>&1 || { tail -30 $OUT/gen_mega.log; exit 1; }
grep "^{" $OUT/gen_mega.log
