#!/bin/bash
# Batched / MFMA single-launch decode: numerics, phase timelines at 1 / 2 / 4 rows, generate bench.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_t
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_decode_mega_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -3
PIAMD_MEGA_LOADER=0 timeout -k 10 200 python -u tools/mega_trace.py --batch 1 > $OUT/trace_b1.log 2>&1 || { tail -30 $OUT/trace_b1.log; exit 1; }
grep "^{" $OUT/trace_b1.log
PIAMD_MEGA_MFMA=1 timeout -k 10 200 python -u tools/mega_trace.py --batch 1 > $OUT/trace_b1m.log 2>&1 || { tail -30 $OUT/trace_b1m.log; exit 1; }
grep "^{" $OUT/trace_b1m.log
for b in 2 4; do
  timeout -k 10 200 python -u tools/mega_trace.py --batch $b > $OUT/trace_b$b.log 2>&1 || { tail -30 $OUT/trace_b$b.log; exit 1; }
  grep "^{" $OUT/trace_b$b.log
done
timeout -k 10 300 python -u tools/bench_generate.py --batch 1 2 4 --gen 64 --modes eager > $OUT/gen_mega.log 2>&1 || { tail -30 $OUT/gen_mega.log; exit 1; }
grep "^{" $OUT/gen_mega.log
