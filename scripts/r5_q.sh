#!/bin/bash
# Serving-batch linears on the skinny GEMM: inference GPU tests + batch 8 / 32 generate.
set -o pipefail
OUT=gpurun_out/r5_q
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_infer_kernels_gpu.py tests/test_decode_mega_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python3 tools/bench_generate.py --batch 8 32 --prompt 128 --gen 32 --modes graph > $OUT/gen.log 2>&1 || { echo "gen failed"; tail -20 $OUT/gen.log; exit 1; }
grep '^{' $OUT/gen.log
