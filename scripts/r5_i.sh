#!/bin/bash
# Decode GEMV with the x rows staged in LDS (XM 2) and the pre-LN prologue for up to 32 rows (XM 1):
# correctness (GEMV GPU tests) + the rows / split-K / LN-fusion A/B at serving batch sizes.
set -o pipefail
OUT=gpurun_out/r5_i
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_infer_kernels_gpu.py tests/test_batchnorm_gpu.py tests/test_rnn_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 tools/bench_gemv_rows.py --M 8 16 32 64 > $OUT/rows.jsonl 2>&1 || { echo "bench failed"; tail -20 $OUT/rows.jsonl; exit 1; }
grep '^{' $OUT/rows.jsonl
