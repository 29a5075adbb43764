#!/bin/bash
# Batched single-launch decode: numerics vs the per-op path, then batch 1/2/4 decode latency with
# the batched kernel and with the per-op path.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_s
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_decode_mega_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -3
timeout -k 10 300 python -u tools/bench_generate.py --batch 1 2 4 --gen 64 --modes eager > $OUT/gen_mega.log 2>&1 || { tail -30 $OUT/gen_mega.log; exit 1; }
grep "^{" $OUT/gen_mega.log
PIAMD_DECODE_MEGA=0 timeout -k 10 300 python -u tools/bench_generate.py --batch 2 4 --gen 64 --modes graph > $OUT/gen_perop.log 2>&1 || { tail -30 $OUT/gen_perop.log; exit 1; }
grep "^{" $OUT/gen_perop.log
