#!/bin/bash
# int8 weight-only single-launch decode on MFMA: tests + generate bench (int8 / bf16 graph).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r5_w
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_decode_mega_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python -u tools/bench_generate.py --batch 1 --gen 64 --modes int8 graph > $OUT/gen.log 2>&1 || { tail -30 $OUT/gen.log; exit 1; }
grep "^{" $OUT/gen.log
PIAMD_MEGA_MFMA=0 timeout -k 10 400 python -u tools/bench_generate.py --batch 1 --gen 64 --modes int8 > $OUT/gen_valu.log 2>&1 || { tail -30 $OUT/gen_valu.log; exit 1; }
grep "^{" $OUT/gen_valu.log
