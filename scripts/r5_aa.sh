#!/bin/bash
# int4 weight-only single-launch decode: tests + generate bench (int4 / int8 / bf16 graph).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_aa
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_decode_mega_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 500 python -u tools/bench_generate.py --batch 1 4 --gen 64 --modes int4 int8 graph > $OUT/gen.log 2>&1 || { tail -30 $OUT/gen.log; exit 1; }
grep "^{" $OUT/gen.log
