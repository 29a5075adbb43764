#!/bin/bash
# MFMA-default single-launch decode: tests, phase timelines at 1 / 2 / 4 rows, generate bench.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_v
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_decode_mega_gpu.py tests/test_infer_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for b in 1 2 4; do
  timeout -k 10 200 python -u tools/mega_trace.py --batch $b > $OUT/trace_b$b.log 2>&1 || { tail -30 $OUT/trace_b$b.log; exit 1; }
  grep "^{" $OUT/trace_b$b.log
done
timeout -k 10 500 python -u tools/bench_generate.py --batch 1 2 4 8 --gen 64 --modes graph eager > $OUT/gen.log 2>&1 || { tail -30 $OUT/gen.log; exit 1; }
grep "^{" $OUT/gen.log
